# round-2 measurement of the final build (per-trial window sums, ms block interface): GPU suite,
# default bench (C4), rocprofv3 trace + PMC passes on C4 -p 100 (SQ_INSTS_VMEM_WR: scratch spill stores)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02ac
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 1
timeout -k 10 1300 bash tools/profile.sh r02ac_c4_p100 --config C4 --n-permute 100 --warmup 1 --steps 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
