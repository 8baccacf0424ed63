# members per split cell by cost (default) vs uniform (FSCLG_SPLIT_UNIFORM=1): the parity tests that run split
# launches, then rank 0 of an 8-GPU C4 parity job rehearsed on one GPU, alternating, with the blocking batches'
# cell trace.  bash tools/ab_split.sh <tag> [rounds]
set -o pipefail
TAG=$1; ROUNDS=${2:-2}
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/split_$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "split or pipelined or full_genomes or two_devices or two_ranks" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
export FSCL_AMD_LIBDIR=$R/fscl_amd/_build_rehearsal
REC=/tmp/fscl_sim_$TAG.bin
FSCL_AMD_SIM=record:$REC timeout -k 10 600 python3 -u $R/bench.py --config C4 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w1.json 2> $OUT/w1.err || exit 1
for r in $(seq $ROUNDS); do
  for v in uniform cost; do
    E=""; [ $v = uniform ] && E="FSCLG_SPLIT_UNIFORM=1"
    env $E FSCLG_CELL_TRACE=/tmp/ct_${TAG}_$v.bin FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 600 python3 -u $R/bench.py --config C4 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w8_${v}_$r.json 2> $OUT/w8_${v}_$r.err || exit 1
    echo "$v $r: $(python3 -c "import json;d=json.load(open('$OUT/w8_${v}_$r.json'));s=d['stats'];print(round(d['ms_per_step']), 'ms/job wait', round(s['wait_s'],3), d['parity']['jobs_identical'] if 'jobs_identical' in d['parity'] else d['parity'])")"
    python3 $R/tools/tail_cells.py /tmp/ct_${TAG}_$v.bin > $OUT/tail_${v}_$r.txt; rm -f /tmp/ct_${TAG}_$v.bin
    sed -n 2,5p $OUT/tail_${v}_$r.txt
  done
done
rm -f $REC
