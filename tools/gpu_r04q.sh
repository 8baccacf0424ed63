set -o pipefail
mkdir -p gpurun_out/r04q
# the GPU suite on the submit path without hash maps, then r04p's host profile again
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04q/pytest.log 2>&1 || { tail -30 gpurun_out/r04q/pytest.log; exit 1; }
tail -3 gpurun_out/r04q/pytest.log
bash tools/gpu_r04p.sh && cp -r gpurun_out/r04p/. gpurun_out/r04q/
