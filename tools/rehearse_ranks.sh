# Rehearsal of the driver's real 8-rank SCALE shape on one GPU (rehearsal build, run on the GPU box):
#   bash tools/rehearse_ranks.sh <config> <tag> [W]
# Records the job's batches once, then replays rank 0 of W three ways, each with the CPUs the
# other W-1 ranks would take on this box's cgroup kept busy by spinning processes (a rank's main
# thread spins in the exchanges), since the replay itself runs rank 0 alone:
#   single  one process driving W GPUs (bench.py --gpus W without a launcher): every spare CPU
#           speculates for the one host process, no other ranks;
#   replicated  one process per GPU, each rank building its own permutations
#           (FSCL_AMD_PERM_LEADER=0): rank 0 gets usable/W - 1 speculation threads, and the other
#           ranks' main and speculation threads take the rest;
#   leader  one process per GPU with the node leader's permutation pool (the default): rank 0
#           speculates on usable - W threads, the other ranks' main threads take W - 1 CPUs.
# The exchange latency the replay does not pay is measured separately (tools/shm_latency.py).
set -o pipefail
CFG=$1; TAG=$2; W=${3:-8}
R=${GRAFT_REPO_ROOT:-$PWD}
export FSCL_AMD_LIBDIR=$R/fscl_amd/_build_rehearsal
OUT=$R/gpurun_out/ranks_$TAG
mkdir -p $OUT
REC=/tmp/fscl_sim_ranks_$TAG.bin
U=$(python3 -c "import sys; sys.path.insert(0, '$R'); import bench; print(bench.cpu_info()['usable_cpus'])")
echo "usable CPUs: $U, W=$W"
if [ "${WARM:-1}" = 1 ]; then  # warm caches (to a file: a long silent step looks hung to gpurun); WARM=0 skips it (C5)
  timeout -k 10 900 python3 -u $R/bench.py --config $CFG --warmup 0 --steps 1 --no-cpu-baseline > $OUT/warm.log 2>&1
fi
if [ "${REUSE:-0}" = 1 ] && [ -s $REC ]; then  # REUSE=1: replay the recording an earlier call of this tag left
  echo "reusing $REC"
else
  FSCL_AMD_SIM=record:$REC timeout -k 10 900 python3 -u $R/bench.py --config $CFG --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w1_record.json 2> $OUT/w1_record.err || exit 1
fi
burn() {  # $1 spinning processes (BURN=yield: spinning with sched_yield, as the ranks' exchange waits do
          # after 4096 spins), each time-limited; their pids in BURN_PIDS
  BURN_PIDS=""
  local code="while True: pass"
  [ "${BURN:-spin}" = yield ] && code="import os
while True: os.sched_yield()"
  for i in $(seq $1); do
    timeout -k 5 600 python3 -c "$code" &
    BURN_PIDS="$BURN_PIDS $!"
  done
}
unburn() { for p in $BURN_PIDS; do kill $p 2>/dev/null; done; wait $BURN_PIDS 2>/dev/null; BURN_PIDS=""; }
run() {  # <name> <burners> <round> [env ...]: the replay sizes its threads as the product would for that env
  burn $2
  local P=""  # PROF=1: the replay under rocprofv3's kernel trace (per-kernel durations in $OUT/prof_<name>)
  [ -n "$PROF" ] && P="rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$1_$3 -o run --"
  (cd /tmp && env TMPDIR=/tmp LOCAL_WORLD_SIZE=$W ${@:4} FSCL_AMD_SIM=replay:$REC:$W:0 timeout -k 10 900 $P python3 -u $R/bench.py --config $CFG --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w${W}_$1_$3.json 2> $OUT/w${W}_$1_$3.err)
  local rc=$?
  unburn
  [ $rc -eq 0 ] || exit 1
  echo "$1 ($2 busy CPUs beside; ${@:4}) round $3: $(python3 -c "import json;d=json.load(open('$OUT/w${W}_$1_$3.json'));s=d['stats'];print(round(d['ms_per_step']), 'ms/job; blocked on batches', round(s['wait_s'],3), 's; spec threads', s['spec_threads'], 'hits', s['spec_hits'], '/', s['trials'], 'claimed', s.get('spec_claimed'), 'wait', round(s['spec_wait_s'],3), 's; main-thread perm', round(s['host_perm_s'],3), 'null', round(s['host_null_s'],3), 's; plan', s.get('plan_mode'), 'rank hist', s.get('spec_rank'))")"
}
PER=$((U / W)); [ $PER -lt 1 ] && PER=1
for r in $(seq ${ROUNDS:-2}); do
  for v0 in ${VARIANTS:-single replicated leader leader_norefine}; do
    # <variant>@VAR=x,VAR2=y: the variant with extra environment (e.g. leader@FSCLG_SPLIT_BUDGET=512)
    v=${v0%%@*}; X=""; [ "$v" != "$v0" ] && X=${v0#*@}; X=${X//,/ }
    if [ -n "$X" ]; then
      N=$(echo "${v}_${X##*/}" | tr ' =' '_-')
      case $v in
        single) run $N 0 $r LOCAL_WORLD_SIZE=1 FSCL_AMD_PERM_LEADER=0 $X ;;
        leader) run $N $((W - 1)) $r $X ;;
        *) echo "no extra environment for $v"; exit 1 ;;
      esac
      continue
    fi
    case $v in
      # one process driving W GPUs: every spare CPU speculates for it, no other ranks
      single) run single 0 $r LOCAL_WORLD_SIZE=1 FSCL_AMD_PERM_LEADER=0 ;;
      # one process per GPU, each building its own permutations: the others' main + worker threads busy
      replicated) run replicated $(( (W - 1) * PER )) $r FSCL_AMD_PERM_LEADER=0 ;;
      # the node leader's permutations (the default): the others' main threads busy
      leader) run leader $((W - 1)) $r ;;
      leader_norefine) run leader_norefine $((W - 1)) $r FSCLG_SPEC_REFINE=0 ;;
      single_norefine) run single_norefine 0 $r LOCAL_WORLD_SIZE=1 FSCL_AMD_PERM_LEADER=0 FSCLG_SPEC_REFINE=0 ;;
      # the leader with its per-trial trace (FSCL_AMD_TRIAL_TRACE: bulk wait, permutation, null sums +
      # upload + cell lists, submit, blocking wait, flush, in microseconds per trial)
      leader_trace) run leader_trace $((W - 1)) $r FSCL_AMD_TRIAL_TRACE=$OUT/trials_leader_$r.txt ;;
      # the leader oversubscribing: a worker on every CPU but its main thread
      leader_all) run leader_all $((W - 1)) $r FSCL_AMD_SPEC=$((U - 1)) ;;
    esac
  done
done
rm -f $REC
