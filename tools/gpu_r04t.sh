set -o pipefail
mkdir -p gpurun_out/r04t
# the whole C5 job with the blocking batch split at larger batch sizes (FSCLG_SPLIT_BUDGET: members =
# budget / cells, at most 8; 256 by default keeps every member of every cell co-resident): the tail's
# ~550 blocking cells per trial are ~1.1 device rounds of one workgroup each
for b in 1200 2400 256; do
  FSCLG_SPLIT_BUDGET=$b FSCL_AMD_TRIAL_TRACE=$PWD/gpurun_out/r04t/trials_b$b.txt timeout -k 10 400 python3 -u bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04t/c5_b$b.json 2> gpurun_out/r04t/c5_b$b.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r04t/c5_b$b.json'));s=d['stats'];print('budget $b', round(d['ms_per_step']/1e3,1), 's', round(d['value']), d['parity'].get('identical'), 'split retries', s.get('n_split_retry'))"
done
