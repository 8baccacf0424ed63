# speculative permutations: full GPU suite, then the C4 trial trace at W=1 and rank 0 of a W=8 replay
set -o pipefail
mkdir -p gpurun_out/r02k
REC=/tmp/fscl_rec_c4.bin
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r02k/gputest.log 2>&1 && \
FSCL_AMD_SIM=record:$REC FSCL_AMD_TRIAL_TRACE=gpurun_out/r02k/tt_w1.txt timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02k/w1.json && \
FSCL_AMD_TRIAL_TRACE=gpurun_out/r02k/tt_w8.txt FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02k/w8.json && \
FSCL_AMD_SPEC=0 FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02k/w8_nospec.json
rm -f $REC
