# environment A/B on this tree's build: rank 0 of an 8-GPU C4 parity job rehearsed on one GPU (rehearsal build),
# then the C4 job at one GPU, alternating.  bash tools/ab_env.sh <tag> <rounds> "<env A>" "<env B>"
# (an env list like "FSCLG_SPINWAIT=1", or "-" for none)
set -o pipefail
TAG=$1; ROUNDS=$2; EA=$3; EB=$4
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/abenv_$TAG
mkdir -p $OUT
# one recording per variant (a variant may change the batches, e.g. FSCL_AMD_DEPTH)
for v in A B; do
  E=$EA; [ $v = B ] && E=$EB; [ "$E" = "-" ] && E="FSCL_AMD_AB=1"
  env $E FSCL_AMD_LIBDIR=$R/fscl_amd/_build_${VARIANT:-rehearsal} FSCL_AMD_SIM=record:/tmp/fscl_sim_${TAG}_$v.bin timeout -k 10 600 python3 -u $R/bench.py --config C4 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w1_$v.json 2> $OUT/w1_$v.err || exit 1
done
for r in $(seq $ROUNDS); do
  for v in A B; do
    E=$EA; [ $v = B ] && E=$EB; [ "$E" = "-" ] && E="FSCL_AMD_AB=1"
    env $E FSCL_AMD_LIBDIR=$R/fscl_amd/_build_${VARIANT:-rehearsal} FSCL_AMD_TRIAL_TRACE=$OUT/trials_${v}_$r.txt FSCL_AMD_SIM=replay:/tmp/fscl_sim_${TAG}_$v.bin:8:0 timeout -k 10 600 python3 -u $R/bench.py --config C4 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w8_${v}_$r.json 2> $OUT/w8_${v}_$r.err || exit 1
    echo "w8 $v ($E) $r: $(python3 -c "import json;d=json.load(open('$OUT/w8_${v}_$r.json'));s=d['stats'];print(round(d['ms_per_step']), 'ms/job wait', round(s['wait_s'],3), 'spec_wait', round(s['spec_wait_s'],3))")"
  done
done
rm -f /tmp/fscl_sim_${TAG}_A.bin /tmp/fscl_sim_${TAG}_B.bin
for r in $(seq $ROUNDS); do
  for v in A B; do
    E=$EA; [ $v = B ] && E=$EB; [ "$E" = "-" ] && E="FSCL_AMD_AB=1"
    env $E timeout -k 10 600 python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c4_${v}_$r.json 2> $OUT/c4_${v}_$r.err || exit 1
    echo "c4 $v $r: $(python3 -c "import json;d=json.load(open('$OUT/c4_${v}_$r.json'));print(round(d['ms_per_step']), 'ms/job', d['parity']['jobs_identical'], 'of', d['parity']['jobs_checked'])")"
  done
done
