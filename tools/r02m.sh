# cell trace with phase timing of rank 0 of the C4 W=8 replay (latency of the tail's blocking batches)
set -o pipefail
mkdir -p gpurun_out/r02m
REC=/tmp/fscl_rec_c4.bin
FSCL_AMD_SIM=record:$REC timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02m/w1.json && \
FSCL_AMD_LIBDIR=$GRAFT_REPO_ROOT/fscl_amd/_build_phase FSCLG_CELL_TRACE=gpurun_out/r02m/ct_w8.bin FSCL_AMD_TRIAL_TRACE=gpurun_out/r02m/tt_w8.txt FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02m/w8.json
rm -f $REC
FSCL_AMD_SIM=record:$REC timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > /dev/null && \
FSCL_AMD_SPLIT=4 FSCL_AMD_LIBDIR=$GRAFT_REPO_ROOT/fscl_amd/_build_phase FSCLG_CELL_TRACE=gpurun_out/r02m/ct_w8_s4.bin FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02m/w8_s4.json
rm -f $REC
