set -o pipefail
mkdir -p gpurun_out/r04e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r04e/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r04e/tests.log; exit 1; }
tail -2 gpurun_out/r04e/tests.log
bash tools/profile_cfg.sh r04e C4 || exit 1
timeout -k 10 60 ./tools/hostread_probe/hostread_probe > gpurun_out/r04e/hostread.txt 2>&1 || exit 1
cat gpurun_out/r04e/hostread.txt
