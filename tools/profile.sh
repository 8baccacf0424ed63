# rocprofv3 evidence for the bench's dominant kernel (run on the GPU box):
#   [PASSES="trace fetch write sq f64 mem tcc"] bash tools/profile.sh <tag> [bench args...]
# kernel-trace + stats in one pass, then one pass per PMC counter group (never combined with tracing);
# PASSES selects a subset (a long job's passes can then go in separate calls, same output directory).
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/prof_$TAG
# PROF_TMP=1 (long jobs): the raw passes go to /tmp, and only the reduced summaries and the bench lines are
# copied under gpurun_out/ -- a pass killed at the call's limit then leaves nothing large behind there
FINAL=$OUT
[ -n "$PROF_TMP" ] && OUT=/tmp/prof_$TAG
mkdir -p $OUT $FINAL
cd /tmp && export TMPDIR=/tmp
LIM=${PROF_LIMIT:-400}
for p in ${PASSES:-trace fetch write sq f64 mem tcc}; do
  case $p in
    trace) args="--kernel-trace --stats" ;;
    fetch) args="--pmc FETCH_SIZE" ;;
    write) args="--pmc WRITE_SIZE" ;;
    sq)    args="--pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE" ;;
    f64)   args="--pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VMEM_WR SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE" ;;
    mem)   args="--pmc TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE GRBM_COUNT" ;;
    tcc)   args="--pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCP_PENDING_STALL_CYCLES_sum" ;;
    *) echo "unknown pass $p"; exit 2 ;;
  esac
  echo "[profile] $p $(date +%T)"
  timeout -k 10 $LIM rocprofv3 $args --output-format csv -d $OUT/$p -o run -- python3 $R/bench.py "$@" > $OUT/bench_$p.json 2> $FINAL/$p.err
done
# REDUCE=1: summarize on the box (tools/prof_summary.py) and drop the raw CSVs, which for a long job exceed
# what a call may bring back; partial summaries of separate calls merge with tools/prof_merge.py
if [ -n "$REDUCE" ]; then
  python3 $R/tools/prof_summary.py $OUT $OUT/partial_$(echo ${PASSES:-all} | tr ' ' '_') > /dev/null
  for p in ${PASSES:-trace fetch write sq f64 mem tcc}; do rm -rf $OUT/$p; done
fi
[ "$OUT" != "$FINAL" ] && cp $OUT/partial_* $OUT/bench_*.json $FINAL/ 2>/dev/null
echo done
