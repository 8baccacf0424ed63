# machine-scheduler strategies for the device build (max-ilp, max-memory-clause) vs the default build's iterative-ilp: interleaved A/B at C4 and C2
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02ay
mkdir -p $OUT
V="ilp:FSCL_AMD_DEVICE=0 maxilp:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_pmaxilp memclause:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_pmemclause"
timeout -k 10 600 bash tools/gpu_ab2.sh 2 $V > $OUT/ab_c4.txt 2>&1 || exit 1
mv gpurun_out/ab2 $OUT/ab2_c4
BENCH_ARGS="--config C2" timeout -k 10 400 bash tools/gpu_ab2.sh 2 $V > $OUT/ab_c2.txt 2>&1 || exit 1
mv gpurun_out/ab2 $OUT/ab2_c2
