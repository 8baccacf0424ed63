# BASELINE configs[4] at full size with the final round-2 kernel (mid-branch trip path): C5 (5.0M SNPs,
# n=400, 50k cells, 10 000 permutations, early prune), one GPU; the trial trace keeps gpurun_out growing
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02az
mkdir -p $OUT
FSCL_AMD_TRIAL_TRACE=$OUT/tt_c5.txt timeout -k 10 1100 python -u bench.py --config C5 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/c5_full.json 2> $OUT/c5_full.err
