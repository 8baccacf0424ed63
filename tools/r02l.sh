# speculation sweep on the C4 W=8 replay: worker threads 0/2/4/8/15
set -o pipefail
mkdir -p gpurun_out/r02l
REC=/tmp/fscl_rec_c4.bin
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r02l/gputest.log 2>&1 || exit 1
FSCL_AMD_SIM=record:$REC timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02l/w1.json || exit 1
for sp in 0 2 4 8 15; do
  FSCL_AMD_SPEC=$sp FSCL_AMD_TRIAL_TRACE=gpurun_out/r02l/tt_w8_s$sp.txt FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02l/w8_s$sp.json || break
done
rm -f $REC
