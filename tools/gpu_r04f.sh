set -o pipefail
mkdir -p gpurun_out/r04f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r04f/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r04f/tests.log; exit 1; }
tail -2 gpurun_out/r04f/tests.log
BURN=spin VARIANTS="single leader leader_trace" ROUNDS=1 bash tools/rehearse_ranks.sh C4 r04f 8 || exit 1
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r04f/c4.json 2> gpurun_out/r04f/c4.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r04f/c4.json'));print('c4', round(d['ms_per_step']), 'ms/job', round(d['roofline']['terms_per_s']/1e9,1), 'Gterms/s', d['parity']['jobs_identical'], 'of', d['parity']['jobs_checked'])"
bash tools/profile_cfg.sh r04f C5 1 || exit 1
