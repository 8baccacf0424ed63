set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r04b/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r04b/tests.log; exit 1; }
tail -3 gpurun_out/r04b/tests.log
timeout -k 10 240 python bench.py --config C5 --chromosomes 1 --seed 55 --n-permute 10000 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04b/c5chr.json 2> gpurun_out/r04b/c5chr.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r04b/c5chr.json'));print('c5chr', d['ms_per_step'], d['value'])"
timeout -k 10 120 python tools/shm_latency.py 8 3000 344 > gpurun_out/r04b/shm_latency8.json || exit 1
cat gpurun_out/r04b/shm_latency8.json
bash tools/rehearse_ranks.sh C4 r04b 8 || exit 1
bash tools/ab_xcd.sh r04b 2 || exit 1
