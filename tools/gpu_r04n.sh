set -o pipefail
mkdir -p gpurun_out/r04n
# C5's one-chromosome tail with up to 16 members per split cell and a 448-workgroup budget (this process
# alone on the GPU), against the default, alternating; parity of every job against the fixture
for r in 1 2; do
  for v in base s16; do
    if [ $v = base ]; then E="FSCL_AMD_AB=1"; L=$PWD/fscl_amd/_build; else E="FSCLG_SPLIT_BUDGET=448"; L=$PWD/fscl_amd/_build_rsplit16; fi
    env $E FSCL_AMD_LIBDIR=$L timeout -k 10 300 python3 bench.py --config C5 --chromosomes 1 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04n/c5_${v}_$r.json 2> gpurun_out/r04n/c5_${v}_$r.err || exit 1
    echo "c5chr1 $v $r: $(python3 -c "import json;d=json.load(open('gpurun_out/r04n/c5_${v}_$r.json'));s=d['stats'];print(round(d['ms_per_step']), 'ms/job; merged', s['n_merged'], '; parity', d['parity']['jobs_identical'], 'of', d['parity']['jobs_checked'])")"
  done
done
