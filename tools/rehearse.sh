# Rehearsal of W-GPU parity-mode jobs on one GPU (rehearsal build): record the job's batches once, then replay as
# rank 0 of W.  Usage: bash tools/rehearse.sh <config> <tag> "<W list>" [spec-thread counts for the largest W]
# e.g. bash tools/rehearse.sh C4 r03p "2 4 8" "1"   (the default speculation share, plus W=8 with 1 thread)
set -o pipefail
CFG=$1; TAG=$2; WS=$3; SPECS=${4:-}
R=${GRAFT_REPO_ROOT:-$PWD}
export FSCL_AMD_LIBDIR=$R/fscl_amd/_build_rehearsal
OUT=$R/gpurun_out/sim_$TAG
mkdir -p $OUT
REC=/tmp/fscl_sim_$TAG.bin
EXTRA=${BENCH_EXTRA:-}
FSCL_AMD_SIM=record:$REC timeout -k 10 900 python3 -u $R/bench.py --config $CFG --warmup 0 --steps 1 --no-cpu-baseline $EXTRA > $OUT/w1_record.json 2> $OUT/w1_record.err || exit 1
echo "W=1 $(python3 -c "import json;d=json.load(open('$OUT/w1_record.json'));print(round(d['ms_per_step']), d['stats']['spec_threads'])")"
for W in $WS; do
  FSCL_AMD_SIM=replay:$REC:$W:0 timeout -k 10 900 python3 -u $R/bench.py --config $CFG --warmup 0 --steps 1 --no-cpu-baseline $EXTRA > $OUT/w${W}_replay.json 2> $OUT/w${W}.err || exit 1
  echo "W=$W $(python3 -c "import json;d=json.load(open('$OUT/w${W}_replay.json'));s=d['stats'];print(round(d['ms_per_step']), 'spec', s['spec_threads'], 'wait', round(s['wait_s'],2), 'window_ms', round(s['window_ms']))")"
done
LW=${WS##* }
for n in $SPECS; do
  FSCL_AMD_SPEC=$n FSCL_AMD_SIM=replay:$REC:$LW:0 timeout -k 10 900 python3 -u $R/bench.py --config $CFG --warmup 0 --steps 1 --no-cpu-baseline $EXTRA > $OUT/w${LW}_spec$n.json 2> $OUT/w${LW}_spec$n.err || exit 1
  echo "W=$LW spec=$n $(python3 -c "import json;d=json.load(open('$OUT/w${LW}_spec$n.json'));print(round(d['ms_per_step']))")"
done
rm -f $REC
