# blocking-batch wave priority: C4 one GPU (bench), C4 8-GPU rehearsal, with and without
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02ab
mkdir -p $OUT
REC=/tmp/fscl_rec_c4.bin
for v in prio noprio; do
  if [ $v = noprio ]; then export FSCLG_NO_PRIO=1; else unset FSCLG_NO_PRIO; fi
  timeout -k 10 300 python3 bench.py --warmup 1 --steps 2 --no-cpu-baseline > $OUT/w1_$v.json || exit 1
  FSCL_AMD_SIM=record:$REC timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > /dev/null || exit 1
  FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w8_$v.json || exit 1
  rm -f $REC
done
