# instruction-fetch counters of the main kernel (C4 -p 20): is the term loop waiting on the instruction cache?
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03g
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_IFETCH_LEVEL GRBM_GUI_ACTIVE" "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --n-permute 20 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_p$i.json 2> $OUT/p$i.err
  echo "group $i rc=$?"
done
