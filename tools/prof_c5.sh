# rocprofv3 passes of the whole C5 job (one GPU, 10 000 permutations) in separate calls, reduced on the box:
#   PASSES="trace fetch" bash tools/prof_c5.sh <tag>      (then merge the partials: tools/prof_merge.py)
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$PWD}
REDUCE=1 PROF_LIMIT=${PROF_LIMIT:-560} bash $R/tools/profile.sh ${TAG}_c5 --config C5 --steps 1 --warmup 0 --no-cpu-baseline \
  > $R/gpurun_out/prof_c5_${TAG}_$(echo $PASSES | tr ' ' '_').log 2>&1 || { tail -20 $R/gpurun_out/prof_c5_${TAG}_*.log; exit 1; }
ls $R/gpurun_out/prof_${TAG}_c5/
