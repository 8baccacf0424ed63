# final tree: full GPU suite, smoke(), and bench.py's multi-rank path (2 ranks on the one GPU, gloo)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02bb
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
FSCL_AMD_DEVICE=0 FSCL_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_w2.json 2> $OUT/bench_w2.err || exit 1
