# band mode diagnosis (round 6): per-phase timing (FSCLG_PHASE_TIMING build, FSCLG_CELL_TRACE) of the
# walk-window path (BAND_TH=-1) against band mode, C4 initial scan
set -o pipefail
mkdir -p gpurun_out/r6c
for v in old band; do
  E="FSCLG_BAND_TH=16"; [ $v = old ] && E="FSCLG_BAND_TH=-1"
  env $E FSCL_AMD_LIBDIR=fscl_amd/_build_phase FSCLG_CELL_TRACE=gpurun_out/r6c/ct_$v.bin timeout -k 10 200 python3 bench.py --config C4 --n-permute 0 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r6c/phase_$v.json 2> gpurun_out/r6c/phase_$v.err || exit 1
done
echo ok
