# round 6: band mode's BandLds moved to the dynamic LDS (reserved only in band mode): band GPU tests, then
# the C4 job (walk-window path, K back to 10) and C5 one chromosome (band default against the walk window)
set -o pipefail
mkdir -p gpurun_out/r6h
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "band or golden" --timeout 300 --timeout-method thread > gpurun_out/r6h/gputest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6h/gputest.log; exit 1; }
tail -1 gpurun_out/r6h/gputest.log
B=fscl_amd/_build
AB_LIMIT=300 bash tools/ab.sh h_c4 2 "--config C4 --steps 2 --warmup 1" base=$B || exit 1
AB_LIMIT=300 bash tools/ab.sh h_c5chr 1 "--config C5 --chromosomes 1 --steps 1 --warmup 0" old=$B,FSCLG_BAND_TH=-1 band=$B || exit 1
