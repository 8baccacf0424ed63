# window null sums: active ranges (this build) vs every window (previous build), C5 x 4 chromosomes -p 2000
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02y
mkdir -p $OUT
FSCL_AMD_LIBDIR=$R/fscl_amd/_build_head timeout -k 10 600 python -u bench.py --config C5 --chromosomes 4 --n-permute 2000 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/head.json 2> $OUT/head.err || exit 1
FSCL_AMD_TRIAL_TRACE=$OUT/tt_new.txt timeout -k 10 600 python -u bench.py --config C5 --chromosomes 4 --n-permute 2000 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/new.json 2> $OUT/new.err
