set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/vp gpurun_out/r03d
timeout -k 10 120 ./tools/vmem_probe/vmem_probe > gpurun_out/vp/plain2.txt 2>&1 || exit 1
bash tools/measure.sh r03d tests || exit 1
timeout -k 10 900 bash tools/gpu_ab2.sh 2 "c4head:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_phead" "c4new:FSCL_AMD_AB=1" > gpurun_out/r03d/ab_c4.log 2>&1 || exit 1
BENCH_ARGS="--config C2" timeout -k 10 600 bash tools/gpu_ab2.sh 2 "c2head:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_phead" "c2new:FSCL_AMD_AB=1" > gpurun_out/r03d/ab_c2.log 2>&1 || exit 1
cat gpurun_out/vp/plain2.txt gpurun_out/r03d/ab_c4.log gpurun_out/r03d/ab_c2.log
