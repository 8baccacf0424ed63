# where a C4 cell's time goes (FSCLG_PHASE_TIMING build) and how full the workgroup slots are
# over each launch (FSCLG_CELL_TRACE), C4 at 20 permutations
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02am
mkdir -p $OUT
FSCL_AMD_LIBDIR=$R/fscl_amd/_build_phase FSCLG_CELL_TRACE=$OUT/ct_c4.bin timeout -k 10 300 python -u bench.py --n-permute 20 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 tools/cell_trace.py $OUT/ct_c4.bin > $OUT/cell_trace.txt 2>&1
