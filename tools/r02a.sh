set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02a_gputest.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r02a_bench_c2.json 2> gpurun_out/r02a_bench_c2.err
