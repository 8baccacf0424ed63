# kernel trace of the C5 x 4 job at 300 permutations: window_null_kernel durations and overlap
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02aa
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --config C5 --chromosomes 4 --n-permute 300 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
