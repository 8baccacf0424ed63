set -o pipefail
mkdir -p gpurun_out/r04m
# the whole C5 job (22 chromosomes, 10 000 permutations): one timed job, initial scan checked against the
# C5_full digest, CPU baseline on the box's cores
timeout -k 10 900 python3 -u bench.py --config C5 --steps 1 --warmup 0 > gpurun_out/r04m/bench_c5.json 2> gpurun_out/r04m/bench_c5.err || { tail -5 gpurun_out/r04m/bench_c5.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04m/bench_c5.json'));s=d['stats'];print('c5', round(d['ms_per_step']), 'ms/job', round(d['value']), 'units/s; merged', s['n_merged'], '; parity', d['parity'])" | cut -c1-600
