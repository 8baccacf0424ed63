# A/B of the two-level (hot-row) LDS coefficient cache build (fscl_amd/_build_rhot, -DFSCLG_HOTROWS) against the
# default build, alternating, on the C4 job (full-job parity in the bench line), 4 C5 chromosomes and C2:
#   bash tools/ab_hot.sh <tag> <rounds>
set -o pipefail
TAG=$1; ROUNDS=$2
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/abhot_$TAG
mkdir -p $OUT
line() { python3 -c "import json;d=json.load(open('$1'));r=d['roofline'];s=d['stats'];p=d.get('parity',{});print(round(d['ms_per_step']), 'ms/job', round(r['terms_per_s']/1e9,1), 'Gterms/s', round(r['avg_launch_ms'],2), 'ms/launch; window', s['cache_n_iv'], 'iv x', s['cache_n_rows'], 'rows, cover', round(s['cache_cover'],3), '; parity', p.get('jobs_identical'), '/', p.get('jobs_checked'))"; }
for r in $(seq $ROUNDS); do
  for v in _build _build_rhot; do
    for cfg in "--config C4 --steps 1 --warmup 1" "--config C5 --chromosomes 4 --n-permute 300 --steps 1 --warmup 0" "--config C2 --steps 2 --warmup 1"; do
      c=$(echo $cfg | awk '{print $2}')
      FSCL_AMD_LIBDIR=$R/fscl_amd/$v timeout -k 10 300 python3 $R/bench.py $cfg --no-cpu-baseline > $OUT/${c}_${v}_$r.json 2> $OUT/${c}_${v}_$r.err || exit 1
      echo "$c $v $r: $(line $OUT/${c}_${v}_$r.json)"
    done
  done
done
