set -o pipefail
mkdir -p gpurun_out/r04x
# one-GPU C4: the tail's blocking batches hold ~300-430 cells of one workgroup each (the default budget of
# 256 workgroups splits only batches of <= 128 cells) while a quarter of the slots idle; larger budgets
# give them 2-3 members per cell, whose members may then wait for each other's slots
for r in 1 2; do
for b in 256 512 768 1024 2048; do
  FSCLG_SPLIT_BUDGET=$b timeout -k 10 300 python3 -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r04x/c4_b${b}_$r.json 2> gpurun_out/r04x/c4_b${b}_$r.err || { tail -5 gpurun_out/r04x/c4_b${b}_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r04x/c4_b${b}_$r.json'));p=d['parity'];s=d['stats'];print('budget $b round $r', round(d['ms_per_step']), 'ms/job', round(d['value']), 'identical', p.get('jobs_identical'), '/', p.get('jobs_checked'), 'split retries', s.get('n_split_retry'))"
done
done
