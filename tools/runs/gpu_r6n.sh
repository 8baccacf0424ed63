# round 6: GPU suite on 2048-site segments (the default now), then the C4 job with 1024 / 2048 / 4096
set -o pipefail
mkdir -p gpurun_out/r6n
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6n/gputest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6n/gputest.log; exit 1; }
tail -1 gpurun_out/r6n/gputest.log
B=fscl_amd/_build
AB_LIMIT=300 bash tools/ab.sh n_c4 2 "--config C4 --steps 2 --warmup 1" s2k=$B s1k=fscl_amd/_build_s1k s4k=fscl_amd/_build_s4k || exit 1
