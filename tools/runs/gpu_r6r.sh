# round 6, final tree: GPU suite, smoke, the whole C5 job's bench line (citing profiles/r06c_c5_summary.json),
# then rank 0 of an 8-GPU C5 job rehearsed (leader layout)
set -o pipefail
mkdir -p gpurun_out/r6r
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6r/gputest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6r/gputest.log; exit 1; }
tail -1 gpurun_out/r6r/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6r/smoke.log 2>&1 || { tail -20 gpurun_out/r6r/smoke.log; exit 1; }
tail -1 gpurun_out/r6r/smoke.log
timeout -k 10 500 python -u bench.py --config C5 --steps 1 --warmup 0 > gpurun_out/r6r/bench_c5.json 2> gpurun_out/r6r/bench_c5.err || { tail -20 gpurun_out/r6r/bench_c5.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r6r/bench_c5.json'));print('C5', round(d['ms_per_step']), 'ms', round(d['value']), d['parity'].get('identical'))"
WARM=0 VARIANTS=leader ROUNDS=1 timeout -k 10 600 bash tools/rehearse_ranks.sh C5 r06c_c5 8 || exit 1
# for the record (not the default): split segments of 2048 sites against 1024 on the C5 one-chromosome job
AB_LIMIT=300 bash tools/ab.sh r_c5chr 1 "--config C5 --chromosomes 1 --steps 1 --warmup 0" base=fscl_amd/_build ss2k=fscl_amd/_build_ss2k || exit 1
