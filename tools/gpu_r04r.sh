set -o pipefail
mkdir -p gpurun_out/r04r
# the whole C5 job (10 000 permutations) at pipeline depths 4 (the default), 6 and 3: the tail's
# trials have ~1.3 device rounds of cells each, and a shallower blocking class (depth 3: points
# with permute_p + queued >= 17) moves cells into the bulk batches that fill the rounds' gaps
for k in ${DEPTHS:-4 3 6}; do
  FSCL_AMD_DEPTH=$k FSCL_AMD_TRIAL_TRACE=$PWD/gpurun_out/r04r/trials_k$k.txt timeout -k 10 400 python3 -u bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04r/c5_k$k.json 2> gpurun_out/r04r/c5_k$k.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r04r/c5_k$k.json'));print('depth $k', round(d['ms_per_step']/1e3,1), 's', round(d['value']), d['parity'].get('identical'))"
done
