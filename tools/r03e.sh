# A/B: interleaved site array (new) vs round-2 HEAD (phead), and the look-ahead issued at the trip start (pnxe)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03e
timeout -k 10 900 bash tools/gpu_ab2.sh 3 "c4head:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_phead" "c4new:FSCL_AMD_AB=1" "c4nxe:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_pnxe" > gpurun_out/r03e/ab_c4.log 2>&1 || exit 1
BENCH_ARGS="--config C2" timeout -k 10 600 bash tools/gpu_ab2.sh 2 "c2head:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_phead" "c2new:FSCL_AMD_AB=1" "c2nxe:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_pnxe" > gpurun_out/r03e/ab_c2.log 2>&1 || exit 1
cat gpurun_out/r03e/ab_c4.log gpurun_out/r03e/ab_c2.log
