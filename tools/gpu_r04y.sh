set -o pipefail
# rank 0 of the 8-rank C4 shape with the other ranks' main threads yielding (BURN=yield): the node
# leader at its default 8 speculation workers against 15 (a worker on every CPU but its own main thread)
BURN=yield VARIANTS="leader leader_all" ROUNDS=2 bash tools/rehearse_ranks.sh C4 r04y 8 > gpurun_out/r04y_ranks.log 2>&1 || { tail -20 gpurun_out/r04y_ranks.log; exit 1; }
cat gpurun_out/r04y_ranks.log
