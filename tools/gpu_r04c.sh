set -o pipefail
mkdir -p gpurun_out/r04c
FSCL_AMD_LIBDIR=$PWD/fscl_amd/_build_rhot timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "matches_golden or full_size_configs or window_sum or fixture and not C5_chr_p10000" > gpurun_out/r04c/tests_hot.log 2>&1 || { echo HOT_TESTS_FAILED; tail -30 gpurun_out/r04c/tests_hot.log; exit 1; }
tail -2 gpurun_out/r04c/tests_hot.log
bash tools/ab_hot.sh r04c 2 || exit 1
