set -o pipefail
mkdir -p gpurun_out/r02e
REC=/tmp/fscl_rec_c4.bin
FSCL_AMD_SIM=record:$REC FSCL_AMD_TRIAL_TRACE=gpurun_out/r02e/tt_w1.txt timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02e/record.json
for sp in 1 8; do
  FSCL_AMD_SPLIT=$sp FSCL_AMD_TRIAL_TRACE=gpurun_out/r02e/tt_w8_s$sp.txt FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02e/w8_s$sp.json
done
rm -f $REC
