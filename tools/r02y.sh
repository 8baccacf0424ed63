# window null-sum kernel with LDS null rows: GPU suite, C5 x 4 chromosomes -p 2000, C5 -p 200
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02y2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --config C5 --chromosomes 4 --n-permute 2000 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/c5x4.json 2> $OUT/c5x4.err || exit 1
timeout -k 10 600 python -u bench.py --config C5 --n-permute 200 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/c5_p200.json 2> $OUT/c5_p200.err
