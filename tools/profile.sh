# rocprofv3 evidence for the bench's dominant kernel (run on the GPU box):
#   bash tools/profile.sh <tag> [bench args...]
# kernel-trace + stats in one pass, then one pass per PMC counter group (never combined with tracing).
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py "$@" > $OUT/bench_trace.json 2> $OUT/trace.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py "$@" > $OUT/bench_fetch.json 2> $OUT/fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py "$@" > $OUT/bench_write.json 2> $OUT/write.err
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 $R/bench.py "$@" > $OUT/bench_sq.json 2> $OUT/sq.err
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VMEM_WR SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE --output-format csv -d $OUT/f64 -o run -- python3 $R/bench.py "$@" > $OUT/bench_f64.json 2> $OUT/f64.err
echo done
