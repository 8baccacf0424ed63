# round 6: which half of the site-major change breaks g2_grid50k: golden tests on the default build (grid
# anchored at the nearest site + site-major dealing), anc (grid only), smo (dealing only), wm (neither)
set -o pipefail
mkdir -p gpurun_out/r6k
for v in _build_wm _build_anc _build_smo _build; do
  FSCL_AMD_LIBDIR=$PWD/fscl_amd/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "golden" --timeout 200 --timeout-method thread > gpurun_out/r6k/gt$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/r6k/gt$v.log)"
  [ $rc -gt 1 ] && exit $rc
done
exit 0
