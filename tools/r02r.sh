# split-cell probe: members 4/8 and wider trips (U=4 at 4 waves per SIMD), per-event trace
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02r
mkdir -p $OUT
rm -f $OUT/ev_*.bin
for cfg in "_build_itrace 8" "_build_itrace 4" "_build_u4 8" "_build_u4 4"; do
  set -- $cfg
  rm -f /tmp/ct.bin
  FSCL_AMD_LIBDIR=$R/fscl_amd/$1 FSCLG_CELL_TRACE=/tmp/ct.bin FSCLG_INST_TRACE_FILE=$OUT/ev$1_$2.bin FSCL_AMD_SPLIT=$2 timeout -k 10 120 python3 $R/tools/split_probe.py 8 > $OUT/probe$1_$2.txt 2>&1 || exit 1
done
