set -o pipefail
mkdir -p gpurun_out/r04i
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "window or windowed or fixture or mixed or C5" > gpurun_out/r04i/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r04i/tests.log; exit 1; }
tail -2 gpurun_out/r04i/tests.log
for r in 1 2; do
  for v in 0 1; do
    FSCLG_WINDOW_TREE=$v timeout -k 10 300 python3 bench.py --config C5 --chromosomes 1 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04i/c5_tree${v}_$r.json 2> gpurun_out/r04i/c5_tree${v}_$r.err || exit 1
    echo "c5chr1 tree=$v $r: $(python3 -c "import json;d=json.load(open('gpurun_out/r04i/c5_tree${v}_$r.json'));s=d['stats'];print(round(d['ms_per_step']), 'ms/job; window_ms', round(s['window_ms']), '; parity', d['parity']['jobs_identical'], 'of', d['parity']['jobs_checked'])")"
  done
done
