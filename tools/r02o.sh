# split cells: register budget (no spills) and the combine's agent-scope fences, C4 W=8 replay (rank 0)
set -o pipefail
mkdir -p gpurun_out/r02o
R=$GRAFT_REPO_ROOT
REC=/tmp/fscl_rec_c4.bin
FSCL_AMD_SIM=record:$REC timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02o/w1.json || exit 1
for v in _build _build_norel _build_noacq _build_nofence; do
  FSCL_AMD_LIBDIR=$R/fscl_amd/$v FSCL_AMD_TRIAL_TRACE=gpurun_out/r02o/tt$v.txt FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02o/w8$v.json || break
done
rm -f $REC
