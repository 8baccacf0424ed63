set -o pipefail
mkdir -p gpurun_out/r04s
# the GPU suite with the window-range memo, r04p's host profile, then r04r's depth A/B on the whole C5 job
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04s/pytest.log 2>&1 || { tail -30 gpurun_out/r04s/pytest.log; exit 1; }
tail -1 gpurun_out/r04s/pytest.log
bash tools/gpu_r04p.sh && cp -r gpurun_out/r04p/. gpurun_out/r04s/ && bash tools/gpu_r04r.sh
