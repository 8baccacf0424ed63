set -o pipefail
for n in 8 40; do for sp in 1 8; do
  echo "$(FSCL_AMD_SPLIT=$sp timeout -k 10 120 python3 tools/split_probe.py $n 2>/dev/null | tail -1)"; done; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02h_gputest.log 2>&1 && \
bash tools/r02e.sh
