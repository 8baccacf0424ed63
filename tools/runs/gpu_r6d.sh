# round 6: GPU suite, then C5 one-chromosome job A/B (walk-window path vs band mode, the default there)
set -o pipefail
mkdir -p gpurun_out/r6d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6d/gputest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6d/gputest.log; exit 1; }
tail -2 gpurun_out/r6d/gputest.log
AB_LIMIT=300 bash tools/ab.sh c5chr 1 "--config C5 --chromosomes 1 --steps 1 --warmup 0" old=fscl_amd/_build,FSCLG_BAND_TH=-1 band=fscl_amd/_build || exit 1
