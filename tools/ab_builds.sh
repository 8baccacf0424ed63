# build A/B: rank 0 of an 8-GPU C4 parity job rehearsed on one GPU, then the C4 job at one GPU, alternating
# between two in-tree builds (fscl_amd/_build_<variant>, each built with -DFSCL_AMD_REHEARSAL; names starting
# with r or p travel to the GPU box).  bash tools/ab_builds.sh <tag> <rounds> <variant A> <variant B>
set -o pipefail
TAG=$1; ROUNDS=$2; VA=$3; VB=$4
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/abb_$TAG
mkdir -p $OUT
for v in $VA $VB; do
  FSCL_AMD_LIBDIR=$R/fscl_amd/_build_$v FSCL_AMD_SIM=record:/tmp/fscl_sim_${TAG}_$v.bin timeout -k 10 300 python3 -u $R/bench.py --config C4 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w1_$v.json 2> $OUT/w1_$v.err || exit 1
  echo "w1 $v: $(python3 -c "import json;d=json.load(open('$OUT/w1_$v.json'));print(round(d['ms_per_step']), 'ms/job', d['parity']['jobs_identical'], 'of', d['parity']['jobs_checked'])")"
done
for r in $(seq $ROUNDS); do
  for v in $VA $VB; do
    FSCL_AMD_LIBDIR=$R/fscl_amd/_build_$v FSCL_AMD_SIM=replay:/tmp/fscl_sim_${TAG}_$v.bin:8:0 timeout -k 10 300 python3 -u $R/bench.py --config C4 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w8_${v}_$r.json 2> $OUT/w8_${v}_$r.err || exit 1
    echo "w8 $v $r: $(python3 -c "import json;d=json.load(open('$OUT/w8_${v}_$r.json'));s=d['stats'];print(round(d['ms_per_step']), 'ms/job wait', round(s['wait_s'],3))")"
  done
done
rm -f /tmp/fscl_sim_${TAG}_*.bin
for r in $(seq $ROUNDS); do
  for v in $VA $VB; do
    FSCL_AMD_LIBDIR=$R/fscl_amd/_build_$v timeout -k 10 300 python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c4_${v}_$r.json 2> $OUT/c4_${v}_$r.err || exit 1
    echo "c4 $v $r: $(python3 -c "import json;d=json.load(open('$OUT/c4_${v}_$r.json'));print(round(d['ms_per_step']), 'ms/job', d['parity']['jobs_identical'], 'of', d['parity']['jobs_checked'])")"
  done
done
