# 8-GPU C4 rehearsal (rank 0 of 8, FSCL_AMD_SIM) vs trials in flight K: the blocking batch
# holds the points with permute_p + queued >= 20 - K
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02ai
mkdir -p $OUT
for k in 2 3 4; do
  FSCL_AMD_DEPTH=$k timeout -k 10 400 bash tools/scale_sim.sh C4 r02ai_k$k 8 > $OUT/sim_k$k.log 2>&1 || exit 1
done
