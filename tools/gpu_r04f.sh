set -o pipefail
bash tools/profile_cfg.sh r04f C5 1 || exit 1
BURN=spin VARIANTS="single replicated leader leader_trace" ROUNDS=2 bash tools/rehearse_ranks.sh C4 r04f 8 || exit 1
