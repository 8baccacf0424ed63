set -o pipefail
mkdir -p gpurun_out/r04l
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r04l/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r04l/tests.log; exit 1; }
tail -2 gpurun_out/r04l/tests.log
BURN=spin VARIANTS="single leader" ROUNDS=1 bash tools/rehearse_ranks.sh C4 r04l 8 || exit 1
bash tools/profile_cfg.sh r04l C5 1 || exit 1
