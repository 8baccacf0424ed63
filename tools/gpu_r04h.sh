set -o pipefail
mkdir -p gpurun_out/r04h
# C5's one-chromosome early-prune job (10 000 permutations): the blocking batch's split budget and the
# speculative refine walks, alternating
for r in 1 2; do
  for e in "FSCL_AMD_AB=1" "FSCLG_SPLIT_BUDGET=512" "FSCLG_SPEC_REFINE=1"; do
    env $e timeout -k 10 300 python3 bench.py --config C5 --chromosomes 1 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04h/c5_${e%%=*}_$r.json 2> gpurun_out/r04h/c5_${e%%=*}_$r.err || exit 1
    echo "c5chr1 $e $r: $(python3 -c "import json;d=json.load(open('gpurun_out/r04h/c5_${e%%=*}_$r.json'));s=d['stats'];print(round(d['ms_per_step']), 'ms/job; blocked', round(s['wait_s'],2), 's; window_ms', round(s['window_ms']), '; parity', d['parity']['jobs_identical'], 'of', d['parity']['jobs_checked'])")"
  done
done
