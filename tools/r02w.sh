# round-2 measurement pass: GPU suite, bench lines (C4 default, C2, C3, C5 early prune), rocprofv3
# trace + PMC passes on C4 -p 100, 8-GPU rehearsal of the C4 job
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02w
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 1
timeout -k 10 300 python -u bench.py --config C2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
timeout -k 10 300 python -u bench.py --config C3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 1
timeout -k 10 600 python -u bench.py --config C5 --n-permute 200 --warmup 0 --steps 1 > $OUT/bench_c5_p200.json 2> $OUT/bench_c5_p200.err || exit 1
timeout -k 10 1300 bash tools/profile.sh r02w_c4_p100 --config C4 --n-permute 100 --warmup 1 --steps 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
timeout -k 10 400 bash tools/scale_sim.sh C4 r02w 2 4 8 > $OUT/sim.log 2>&1
