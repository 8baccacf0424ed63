# per-trial trace (could-draw points, draws, timings) of the C4 job at W=1 and of rank 0 of a W=8 replay
set -o pipefail
mkdir -p gpurun_out/r02j
REC=/tmp/fscl_rec_c4.bin
FSCL_AMD_SIM=record:$REC FSCL_AMD_TRIAL_TRACE=gpurun_out/r02j/tt_w1.txt timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02j/w1.json && \
FSCL_AMD_TRIAL_TRACE=gpurun_out/r02j/tt_w8.txt FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02j/w8.json
rm -f $REC
