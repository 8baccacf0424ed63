# A/B timing of kernel build variants (development aid): bash tools/gpu_ab.sh variant...
set -e
mkdir -p gpurun_out
for v in "$@"; do
  FSCL_AMD_LIBDIR=$PWD/fscl_amd/$v timeout -k 10 200 python bench.py --steps 1 --warmup 1 --n-permute 20 --no-cpu-baseline > gpurun_out/ab_$v.json 2>/dev/null
done
