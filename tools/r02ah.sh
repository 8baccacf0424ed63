# trials in flight (row slots) vs C4 job time: L2 footprint of the slots' site arrays
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02ah
mkdir -p $OUT
for k in 2 3 4 6; do
  FSCL_AMD_DEPTH=$k timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 > $OUT/bench_k$k.json 2> $OUT/bench_k$k.err || exit 1
done
