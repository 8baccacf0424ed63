# Rehearse a W-GPU job on one GPU with the W-way batch / trial split recorded by one process that
# drives W contexts on the GPU (both permutation modes; throughput mode shards whole trials):
#   bash tools/scale_sim_tp.sh <config> <tag> <mode> W
# 1. record: one process, W contexts on GPU 0, every batch's results (FSCL_AMD_SIM=record);
# 2. replay as rank 0 of W: evaluate only rank 0's share (its trials, in throughput mode), take the
#    rest from the recording (rank 0's own results checked bit for bit), and time it.
set -e
export FSCL_AMD_LIBDIR=${GRAFT_REPO_ROOT:-$PWD}/fscl_amd/_build_rehearsal
CFG=$1; TAG=$2; MODE=$3; W=$4
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/simtp_$TAG
mkdir -p $OUT
REC=/tmp/fscl_simtp_$TAG.bin
FSCL_AMD_SIM=record:$REC timeout -k 10 400 python3 $R/bench.py --config $CFG --warmup 0 --steps 1 --no-cpu-baseline --permute-mode $MODE --contexts $W > $OUT/w${W}_record.json
FSCL_AMD_SIM=replay:$REC:$W:0 timeout -k 10 300 python3 $R/bench.py --config $CFG --warmup 0 --steps 1 --no-cpu-baseline --permute-mode $MODE > $OUT/w${W}_replay.json
echo "mode=$MODE W=$W $(python3 -c "import json;d=json.load(open('$OUT/w${W}_replay.json'));print(d['value'], d['ms_per_step'], d['stats']['wait_s'], d['stats']['gp_evals'], d['config']['units_per_step'])")"
rm -f $REC
