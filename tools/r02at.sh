# final round-2 measurement pass (mid-branch trip path): GPU suite, default bench (C4, CPU baseline),
# C2/C3 bench lines, rocprofv3 trace + PMC passes on C4 -p 100, 2/4/8-GPU C4 rehearsal
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02at
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 1
timeout -k 10 300 python -u bench.py --config C2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
timeout -k 10 300 python -u bench.py --config C3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 1
timeout -k 10 1300 bash tools/profile.sh r02at_c4_p100 --config C4 --n-permute 100 --warmup 1 --steps 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
timeout -k 10 600 bash tools/scale_sim.sh C4 r02at 2 4 8 > $OUT/sim.log 2>&1
