# split-cell sizing sweep on the C4 W=8 replay (rank 0): members per cell and workgroup budget
set -o pipefail
mkdir -p gpurun_out/r02n
REC=/tmp/fscl_rec_c4.bin
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r02n/gputest.log 2>&1
FSCL_AMD_SIM=record:$REC timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02n/w1.json || exit 1
for cfg in "8 256" "4 256" "2 256" "8 128" "8 448" "1 256"; do
  set -- $cfg
  FSCL_AMD_SPLIT=$1 FSCLG_SPLIT_BUDGET=$2 FSCL_AMD_TRIAL_TRACE=gpurun_out/r02n/tt_$1_$2.txt FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02n/w8_$1_$2.json || break
done
rm -f $REC
