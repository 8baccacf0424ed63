# round 6, final tree: rocprofv3 trace + PMC passes and the bench line of C4 and of C5's first chromosome
# (tools/profile_cfg.sh), then rank 0 of an 8-GPU C4 job rehearsed (leader layout, 2 rounds)
set -o pipefail
bash tools/profile_cfg.sh r06c C4 || exit 1
bash tools/profile_cfg.sh r06c C5 1 || exit 1
VARIANTS=leader ROUNDS=2 timeout -k 10 400 bash tools/rehearse_ranks.sh C4 r06c_c4 8 || exit 1
