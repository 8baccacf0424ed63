# round 6: GPU suite on the dynamic split dealing, then the C4 rank-0-of-8 phase breakdown and timing
set -o pipefail
mkdir -p gpurun_out/r6f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6f/gputest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6f/gputest.log; exit 1; }
tail -1 gpurun_out/r6f/gputest.log
TAG=r6f bash tools/runs/gpu_r6e.sh
