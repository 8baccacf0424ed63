# member-private combine: GPU suite, split probe trace, C4 W=8 rehearsal (rank 0)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02v
mkdir -p $OUT
rm -f $OUT/ev_*.bin
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1 || exit 1
rm -f /tmp/ct.bin
FSCL_AMD_LIBDIR=$R/fscl_amd/_build_itrace FSCLG_CELL_TRACE=/tmp/ct.bin FSCLG_INST_TRACE_FILE=$OUT/ev_s8.bin FSCL_AMD_SPLIT=8 timeout -k 10 120 python3 $R/tools/split_probe.py 8 > $OUT/probe_s8.txt 2>&1 || exit 1
REC=/tmp/fscl_rec_c4.bin
FSCL_AMD_SIM=record:$REC timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w1.json || exit 1
FSCL_AMD_TRIAL_TRACE=$OUT/tt_w8.txt FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w8.json
rm -f $REC
for cfg in C2 C4; do
  timeout -k 10 300 python3 bench.py --config $cfg --n-permute 20 --warmup 1 --steps 2 --no-cpu-baseline > $OUT/${cfg}.json || exit 1
done
