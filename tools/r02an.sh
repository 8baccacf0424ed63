# 8-GPU rehearsal of C4 in both permutation modes, recorded with 8 contexts on the one GPU
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02an
mkdir -p $OUT
timeout -k 10 800 bash tools/scale_sim_tp.sh C4 r02an_tp throughput 8 > $OUT/tp8.log 2>&1 || exit 1
timeout -k 10 800 bash tools/scale_sim_tp.sh C4 r02an_par parity 8 > $OUT/par8.log 2>&1 || exit 1
timeout -k 10 800 bash tools/scale_sim_tp.sh C4 r02an_tp4 throughput 4 > $OUT/tp4.log 2>&1 || exit 1
timeout -k 10 800 bash tools/scale_sim_tp.sh C4 r02an_tp2 throughput 2 > $OUT/tp2.log 2>&1 || exit 1
