set -o pipefail
mkdir -p gpurun_out/r04d
# the split cells' speculative refine walks at one GPU (the C4 job), alternating
for r in 1 2; do
  for v in 1 0; do
    FSCLG_SPEC_REFINE=$v timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r04d/c4_spec${v}_$r.json 2> gpurun_out/r04d/c4_spec${v}_$r.err || exit 1
    echo "c4 spec_refine=$v $r: $(python3 -c "import json;d=json.load(open('gpurun_out/r04d/c4_spec${v}_$r.json'));print(round(d['ms_per_step']), 'ms/job', round(d['roofline']['terms_per_s']/1e9,1), 'Gterms/s', d['parity']['jobs_identical'], 'of', d['parity']['jobs_checked'])")"
  done
done
bash tools/profile_cfg.sh r04d C3 || exit 1
bash tools/profile_cfg.sh r04d C2 || exit 1
