# Rehearse the W-GPU strong-scaling job on one GPU (run on the GPU box):
#   bash tools/scale_sim.sh <config> <tag> [W ...]
# 1. record every batch's results of the whole job on one GPU (FSCL_AMD_SIM=record);
# 2. for each W: replay as rank 0 of W -- evaluate only rank 0's share of every batch, take
#    the other shares from the recording (rank 0's own share is checked bit for bit) -- and
#    time it: the job time of one rank of a W-GPU run, minus the real exchange latency.
set -e
# the rehearsal hook lives only in the test build: python -m fscl_amd.build --rehearsal (in the container)
export FSCL_AMD_LIBDIR=${GRAFT_REPO_ROOT:-$PWD}/fscl_amd/_build_rehearsal
CFG=$1; TAG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/sim_$TAG
mkdir -p $OUT
REC=/tmp/fscl_sim_$TAG.bin
FSCL_AMD_SIM=record:$REC timeout -k 10 300 python3 $R/bench.py --config $CFG --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w1_record.json
for W in "$@"; do
  FSCL_AMD_SIM=replay:$REC:$W:0 timeout -k 10 300 python3 $R/bench.py --config $CFG --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w${W}_replay.json
  echo "W=$W $(python3 -c "import json;d=json.load(open('$OUT/w${W}_replay.json'));print(d['value'], d['ms_per_step'], d['stats']['wait_s'], d['stats']['host_perm_s'], d['stats']['gp_evals'])")"
done
rm -f $REC
