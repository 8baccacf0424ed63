set -o pipefail
mkdir -p gpurun_out/r04z
# the submit's window check restored (per-batch range memo): GPU suite, host profile, whole C5 job
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04z/pytest.log 2>&1 || { tail -30 gpurun_out/r04z/pytest.log; exit 1; }
tail -1 gpurun_out/r04z/pytest.log
bash tools/gpu_r04p.sh && cp -r gpurun_out/r04p/. gpurun_out/r04z/
timeout -k 10 400 python3 -u bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04z/c5.json 2> gpurun_out/r04z/c5_full.err || { tail -5 gpurun_out/r04z/c5_full.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04z/c5.json'));print('C5', round(d['ms_per_step']/1e3,1), 's', round(d['value']), d['parity'].get('identical'))"
