set -o pipefail
mkdir -p gpurun_out/r04u
# final round-4 lines on this tree: C4 (the bench default) profiled and benched, the whole C5 job
# benched with its CPU baseline, and the 8-rank C4 rehearsal (single process vs node leader)
bash tools/profile_cfg.sh r04u C4 > gpurun_out/r04u/c4.log 2>&1 || { tail -20 gpurun_out/r04u/c4.log; exit 1; }
tail -1 gpurun_out/r04u/c4.log
cp profiles/r04u_c4_summary.json profiles/r04u_c4_kernel_stats.csv gpurun_out/r04u/ && cp gpurun_out/final_r04u/bench_c4.json gpurun_out/r04u/
timeout -k 10 600 python3 -u bench.py --config C5 > gpurun_out/r04u/bench_c5.json 2> gpurun_out/r04u/bench_c5.err || { tail -20 gpurun_out/r04u/bench_c5.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04u/bench_c5.json'));print('C5', round(d['ms_per_step']/1e3,1), 's', round(d['value']), d['parity'].get('identical'), d['cpu_baseline'].get('gpu_over_cpu'))"
VARIANTS="single leader" ROUNDS=1 bash tools/rehearse_ranks.sh C4 r04u 8 > gpurun_out/r04u/ranks.log 2>&1 || { tail -20 gpurun_out/r04u/ranks.log; exit 1; }
cat gpurun_out/r04u/ranks.log
