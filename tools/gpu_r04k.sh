set -o pipefail
mkdir -p gpurun_out/r04k
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r04k/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r04k/tests.log; exit 1; }
tail -2 gpurun_out/r04k/tests.log
for r in 1 2; do
  for e in FSCL_AMD_NO_MERGE=1 FSCL_AMD_AB=1; do
    env $e timeout -k 10 300 python3 bench.py --config C5 --chromosomes 1 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04k/c5_${e%%=*}_$r.json 2> gpurun_out/r04k/c5_${e%%=*}_$r.err || exit 1
    echo "c5chr1 $e $r: $(python3 -c "import json;d=json.load(open('gpurun_out/r04k/c5_${e%%=*}_$r.json'));s=d['stats'];print(round(d['ms_per_step']), 'ms/job; merged', s['n_merged'], '; parity', d['parity']['jobs_identical'], 'of', d['parity']['jobs_checked'])")"
  done
done
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r04k/c4.json 2> gpurun_out/r04k/c4.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r04k/c4.json'));print('c4', round(d['ms_per_step']), 'ms/job merged', d['stats']['n_merged'], d['parity']['jobs_identical'], 'of', d['parity']['jobs_checked'])"
