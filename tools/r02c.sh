set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02c_gputest.log 2>&1 && \
timeout -k 10 400 bash tools/scale_sim.sh C4 r02c 8 > gpurun_out/r02c_sim.log 2>&1
