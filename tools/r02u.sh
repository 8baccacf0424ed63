# wave-parallel argmax / refine setup: GPU suite, split probe trace, C2 / C4 throughput
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02u
mkdir -p $OUT
rm -f $OUT/ev_*.bin
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1 || exit 1
for sp in 8; do
  rm -f /tmp/ct.bin
  FSCL_AMD_LIBDIR=$R/fscl_amd/_build_itrace FSCLG_CELL_TRACE=/tmp/ct.bin FSCLG_INST_TRACE_FILE=$OUT/ev_s$sp.bin FSCL_AMD_SPLIT=$sp timeout -k 10 120 python3 $R/tools/split_probe.py 8 > $OUT/probe_s$sp.txt 2>&1 || exit 1
done
for cfg in C2 C4; do
  timeout -k 10 300 python3 bench.py --config $cfg --n-permute 20 --warmup 1 --steps 2 --no-cpu-baseline > $OUT/${cfg}.json || exit 1
done
