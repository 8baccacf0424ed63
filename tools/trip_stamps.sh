# per-trip phase stamps of the term loop (FSCLG_TRIP_STAMPS build, fscl_amd/_build_pstamp), C4 and C2 at -p 20
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03f
for c in C4 C2; do
  FSCL_AMD_LIBDIR=$R/fscl_amd/_build_pstamp timeout -k 10 300 python bench.py --config $c --n-permute 20 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r03f/$c.json 2> gpurun_out/r03f/$c.err || exit 1
  grep -A2 "trip stamps" gpurun_out/r03f/$c.err
done
