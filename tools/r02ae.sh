# drop-in search_maxalpha with split members per point: parity test + per-call probe (1 vs 8 members)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02ae
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k "dropin or golden" > $OUT/gputest.log 2>&1 || exit 1
FSCLG_POINTS_SPLIT=1 timeout -k 10 120 python -u tools/dropin_probe.py > $OUT/probe_g1.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/dropin_probe.py > $OUT/probe_g8.txt 2>&1 || exit 1
