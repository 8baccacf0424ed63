# BASELINE configs[4] at full size after the two-level bisection: C5 (5.0M SNPs, n=400, 50k cells,
# 10 000 permutations, early prune), one GPU; the trial trace keeps gpurun_out growing (as r02z).
# First the bisection look-ahead fallback tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02al
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "lookahead" > $OUT/gputest.log 2>&1 || exit 1
FSCL_AMD_TRIAL_TRACE=$OUT/tt_c5.txt timeout -k 10 1100 python -u bench.py --config C5 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/c5_full.json 2> $OUT/c5_full.err
