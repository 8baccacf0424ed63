# 1024-thread workgroups (4 waves/SIMD, 112 VGPRs, no spills, 160 KB LDS: twice the coefficient window) vs HEAD: interleaved A/B at C4 and C2, plus a parity subset with the variant
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02ar
mkdir -p $OUT
FSCL_AMD_LIBDIR=$R/fscl_amd/_build_pwg timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "golden and not cli or full_size or pipelined" > $OUT/gputest_wg.log 2>&1 || exit 1
timeout -k 10 600 bash tools/gpu_ab2.sh 3 "wg:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_pwg" "head:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_phead" > $OUT/ab_c4.txt 2>&1 || exit 1
mv gpurun_out/ab2 $OUT/ab2_c4
BENCH_ARGS="--config C2" timeout -k 10 400 bash tools/gpu_ab2.sh 3 "wg:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_pwg" "head:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_phead" > $OUT/ab_c2.txt 2>&1 || exit 1
mv gpurun_out/ab2 $OUT/ab2_c2
