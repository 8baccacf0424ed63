# round 6 (re-entry): GPU suite on the current tree, then band mode against the walk-window path on
# C5 one chromosome (band is the default there) and on the C4 job (walk window the default there)
set -o pipefail
mkdir -p gpurun_out/r6g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6g/gputest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6g/gputest.log; exit 1; }
tail -1 gpurun_out/r6g/gputest.log
B=fscl_amd/_build
AB_LIMIT=300 bash tools/ab.sh g_c5chr 1 "--config C5 --chromosomes 1 --steps 1 --warmup 0" old=$B,FSCLG_BAND_TH=-1 band=$B || exit 1
AB_LIMIT=300 bash tools/ab.sh g_c4 1 "--config C4 --steps 2 --warmup 1" base=$B band=$B,FSCLG_BAND_TH=16 || exit 1
