# One measurement pass on the GPU box (replaces round 2's one-off tools/r02*.sh wrappers):
#   bash tools/measure.sh <tag> [steps...]
# steps (run in order, each under its own time limit, the pass stops at the first failure):
#   tests        the -m gpu suite
#   smoke        __graft_entry__.smoke()
#   bench[:CFG]  bench.py (default C4 with the CPU baseline) -> <tag>/bench_<cfg>.json
#   prof[:CFG]   tools/profile.sh on exactly the bench job (1 step, 0 warmup): trace + PMC passes
#   sim[:CFG]    tools/scale_sim.sh rehearsal of 2/4/8 GPUs (needs fscl_amd/_build_rehearsal)
#   ab:<N>:<spec...>  tools/gpu_ab2.sh interleaved A/B (spec as gpu_ab2.sh takes it, ';'-separated)
# Outputs under gpurun_out/<tag>/; copy what is judged into profiles/.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for step in "$@"; do
  kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  echo "[measure] $step $(date +%T)"
  case $kind in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
             > $OUT/gputest.log 2>&1 || { tail -30 $OUT/gputest.log; exit 1; } ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1 ;;
    bench) cfg=${arg:-C4}; extra=""; [ "$cfg" != "C4" ] && extra="--no-cpu-baseline"
           [ -n "$BENCH_CPU" ] && extra=""
           timeout -k 10 1000 python -u bench.py --config $cfg $extra $BENCH_ARGS > $OUT/bench_${cfg,,}.json \
             2> $OUT/bench_${cfg,,}.err || { tail -20 $OUT/bench_${cfg,,}.err; exit 1; } ;;
    prof)  cfg=${arg:-C4}
           timeout -k 10 1500 bash tools/profile.sh ${TAG}_${cfg,,} --config $cfg --warmup 0 --steps 1 --no-cpu-baseline \
             $BENCH_ARGS > $OUT/prof_${cfg,,}.log 2>&1 || exit 1 ;;
    sim)   cfg=${arg:-C4}
           timeout -k 10 900 bash tools/scale_sim.sh $cfg $TAG 2 4 8 > $OUT/sim_${cfg,,}.log 2>&1 || exit 1 ;;
    ab)    n=${arg%%:*}; specs=${arg#*:}; IFS=';' read -ra S <<< "$specs"
           timeout -k 10 1500 bash tools/gpu_ab2.sh $n "${S[@]}" > $OUT/ab.log 2>&1 || exit 1; cat $OUT/ab.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[measure] done $(date +%T)"
