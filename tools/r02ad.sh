# throughput permutation mode: GPU tests (oracle restatement, depths, two devices, CLI, two ranks),
# C4 bench in throughput mode beside parity mode, C5 at 200 permutations in both modes
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02ad
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "throughput or pipelined" > $OUT/gputest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --permute-mode throughput --no-cpu-baseline > $OUT/bench_c4_tp.json 2> $OUT/bench_c4_tp.err || exit 1
timeout -k 10 600 python -u bench.py --config C5 --n-permute 200 --warmup 0 --steps 1 --no-cpu-baseline --permute-mode throughput > $OUT/bench_c5_p200_tp.json 2> $OUT/bench_c5_p200_tp.err || exit 1
