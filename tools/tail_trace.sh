# rank 0 of an 8-GPU C4 parity job, rehearsed on one GPU (rehearsal build), with the blocking batches' cell trace
# and the trial trace: bash tools/tail_trace.sh <tag>
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$PWD}
export FSCL_AMD_LIBDIR=$R/fscl_amd/_build_${VARIANT:-rehearsal}
OUT=$R/gpurun_out/tail_$TAG
mkdir -p $OUT
REC=/tmp/fscl_sim_$TAG.bin
FSCL_AMD_SIM=record:$REC timeout -k 10 600 python3 -u $R/bench.py --config C4 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w1.json 2> $OUT/w1.err || exit 1
FSCLG_CELL_TRACE=/tmp/ct_$TAG.bin FSCL_AMD_TRIAL_TRACE=$OUT/trials.txt FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 600 python3 -u $R/bench.py --config C4 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w8.json 2> $OUT/w8.err || exit 1
python3 $R/tools/tail_cells.py /tmp/ct_$TAG.bin > $OUT/tail_cells.txt
cat $OUT/tail_cells.txt
python3 -c "import json;d=json.load(open('$OUT/w8.json'));print('w8 ms', round(d['ms_per_step']))"
rm -f $REC /tmp/ct_$TAG.bin
