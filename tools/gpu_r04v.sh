set -o pipefail
mkdir -p gpurun_out/r04u
# r04u's remainder: the whole C5 job (one timed job) with its CPU baseline, and the 8-rank C4 rehearsal
timeout -k 10 900 python3 -u bench.py --config C5 --steps 1 --warmup 0 > gpurun_out/r04u/bench_c5.json 2> gpurun_out/r04u/bench_c5.err || { tail -5 gpurun_out/r04u/bench_c5.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04u/bench_c5.json'));print('C5', round(d['ms_per_step']/1e3,1), 's', round(d['value']), d['parity'].get('identical'), d['cpu_baseline'].get('gpu_over_cpu'))"
VARIANTS="single leader" ROUNDS=1 bash tools/rehearse_ranks.sh C4 r04u 8 > gpurun_out/r04u/ranks.log 2>&1 || { tail -20 gpurun_out/r04u/ranks.log; exit 1; }
cat gpurun_out/r04u/ranks.log
