# two bisection levels per alpha search (lookahead): parity subset, C4 bench with/without,
# C2 bench with/without, 8-GPU C4 rehearsal with/without
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02aj
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "golden or oracle or pipelined or throughput" > $OUT/gputest.log 2>&1 || exit 1
for la in 1 0; do
  FSCLG_LOOKAHEAD=$la timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 > $OUT/bench_c4_la$la.json 2> $OUT/bench_c4_la$la.err || exit 1
  FSCLG_LOOKAHEAD=$la timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 2 > $OUT/bench_c2_la$la.json 2> $OUT/bench_c2_la$la.err || exit 1
  FSCLG_LOOKAHEAD=$la timeout -k 10 400 bash tools/scale_sim.sh C4 r02aj_la$la 8 > $OUT/sim_la$la.log 2>&1 || exit 1
done
