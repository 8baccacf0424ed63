# fused long walks: correctness of the fused build on a few GPU tests, then C2 / C4 (-p 20) per variant
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02t
mkdir -p $OUT
FSCL_AMD_LIBDIR=$R/fscl_amd/_build_fmax3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread -k "golden or full_size or c2_scale" > $OUT/gputest.log 2>&1
echo "tests rc=$?" >> $OUT/gputest.log
for cfg in C2 C4; do
  for v in _build_nofuse _build_fmax3 _build_fmax2; do
    FSCL_AMD_LIBDIR=$R/fscl_amd/$v timeout -k 10 300 python3 bench.py --config $cfg --n-permute 20 --warmup 1 --steps 2 --no-cpu-baseline > $OUT/${cfg}$v.json || exit 1
  done
done
