# the driver's round-end commands on the final tree: smoke(), then bench.py exactly as the driver runs it
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02aw
mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
( time timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err ) 2> $OUT/time.txt || exit 1
