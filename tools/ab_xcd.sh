# A/B of FSCLG_XCD_ORDER (chromosome-major cells within an XCD's class) on this tree's build:
#   bash tools/ab_xcd.sh <tag> <rounds> [bench args for the C5 leg]
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
C5ARGS=${*:-"--config C5 --chromosomes 4 --seed 55 --n-permute 300"}
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/abxcd_$TAG
mkdir -p $OUT
for r in $(seq $ROUNDS); do
  for v in 0 1; do
    FSCLG_XCD_ORDER=$v timeout -k 10 300 python3 $R/bench.py $C5ARGS --steps 1 --warmup 0 --no-cpu-baseline > $OUT/c5_${v}_$r.json 2> $OUT/c5_${v}_$r.err || exit 1
    echo "c5 order=$v $r: $(python3 -c "import json;d=json.load(open('$OUT/c5_${v}_$r.json'));r=d['roofline'];print(round(d['ms_per_step']), 'ms/job', round(r['terms_per_s']/1e9,1), 'Gterms/s', round(r['avg_launch_ms'],2), 'ms/launch')")"
  done
done
for r in $(seq $ROUNDS); do
  for v in 0 1; do
    FSCLG_XCD_ORDER=$v timeout -k 10 300 python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c4_${v}_$r.json 2> $OUT/c4_${v}_$r.err || exit 1
    echo "c4 order=$v $r: $(python3 -c "import json;d=json.load(open('$OUT/c4_${v}_$r.json'));r=d['roofline'];print(round(d['ms_per_step']), 'ms/job', round(r['terms_per_s']/1e9,1), 'Gterms/s', d['parity']['jobs_identical'], 'of', d['parity']['jobs_checked'])")"
  done
done
