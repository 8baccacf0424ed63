# PMC of one 8-cell launch: split (8 members per cell) vs one workgroup per cell (tools/split_probe.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02p
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for sp in 8 1; do
  FSCL_AMD_SPLIT=$sp timeout -k 10 120 python3 $R/tools/split_probe.py 8 > $OUT/probe_s$sp.txt 2>&1 || exit 1
  FSCL_AMD_SPLIT=$sp timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $OUT/sq_s$sp -o run -- python3 $R/tools/split_probe.py 8 > /dev/null 2>&1 || exit 1
  FSCL_AMD_SPLIT=$sp timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/tcc_s$sp -o run -- python3 $R/tools/split_probe.py 8 > /dev/null 2>&1 || exit 1
  FSCL_AMD_SPLIT=$sp timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES --output-format csv -d $OUT/sq2_s$sp -o run -- python3 $R/tools/split_probe.py 8 > /dev/null 2>&1 || exit 1
done
