# occupancy / workgroup-shape variants of the same source vs HEAD (interleaved A/B, -p 20): C4 and C2
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02as
mkdir -p $OUT
V="head:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_phead"
for n in w512x8 w640x5 w512x6 w768u1; do V="$V $n:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_p$n"; done
timeout -k 10 700 bash tools/gpu_ab2.sh 2 $V > $OUT/ab_c4.txt 2>&1 || exit 1
mv gpurun_out/ab2 $OUT/ab2_c4
BENCH_ARGS="--config C2" timeout -k 10 500 bash tools/gpu_ab2.sh 2 $V > $OUT/ab_c2.txt 2>&1 || exit 1
mv gpurun_out/ab2 $OUT/ab2_c2
