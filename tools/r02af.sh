# full GPU suite after throughput mode, split drop-in and the CLI rank path; default bench
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02af
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 1
