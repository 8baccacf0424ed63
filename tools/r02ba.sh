# mid-branch test only in trips that are not all-far (vs HEAD): parity subset, interleaved A/B at C4 and C2
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02ba
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "golden and not cli or full_size or pipelined or tiny" > $OUT/gputest.log 2>&1 || exit 1
timeout -k 10 600 bash tools/gpu_ab2.sh 3 "midin:FSCL_AMD_DEVICE=0" "head:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_phead" > $OUT/ab_c4.txt 2>&1 || exit 1
mv gpurun_out/ab2 $OUT/ab2_c4
BENCH_ARGS="--config C2" timeout -k 10 400 bash tools/gpu_ab2.sh 3 "midin:FSCL_AMD_DEVICE=0" "head:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_phead" > $OUT/ab_c2.txt 2>&1 || exit 1
mv gpurun_out/ab2 $OUT/ab2_c2
