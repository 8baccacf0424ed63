# chunked window null sums (default) vs the sequential kernel (FSCLG_WINDOW_CHUNK=0): the windowed parity tests,
# then C5 x 4 chromosomes at 300 permutations with each, window kernel time and job time
set -o pipefail
OUT=gpurun_out/ab_windows
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 600 --timeout-method thread -k "C5 or windowed or window" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
for r in $(seq ${AB_ROUNDS:-2}); do
  for v in chunk seq chunk2; do
    E=""; [ $v = seq ] && E="FSCLG_WINDOW_CHUNK=0"; [ $v = chunk2 ] && E="FSCLG_WINDOW_CHUNK=2"
    env $E timeout -k 10 600 python bench.py --config C5 --chromosomes 4 --n-permute 300 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/c5_${v}_$r.json 2> $OUT/c5_${v}_$r.err || exit 1
    python3 -c "import json;d=json.load(open('$OUT/c5_${v}_$r.json'));s=d['stats'];print('$v', round(d['ms_per_step']), 'ms/job, window_ms', round(s['window_ms']), 'busy', round(d['roofline']['busy_ms']))"
  done
done
