# rocprofv3 evidence (trace + PMC passes, reduced on the box) for one configuration's bench job, then that
# configuration's bench line citing it (run on the GPU box):
#   bash tools/profile_cfg.sh <tag> <config> [chromosomes]
# The summary lands in profiles/<tag>_<config>[chr<N>]_summary.json, the name bench.py looks for.
set -o pipefail
TAG=$1; CFG=$2; NCHR=${3:-}
c=$(echo $CFG | tr A-Z a-z)
EXTRA=""
if [ -n "$NCHR" ]; then c=${c}chr$NCHR; EXTRA="--chromosomes $NCHR"; fi
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/final_$TAG
mkdir -p $OUT
REDUCE=1 bash $R/tools/profile.sh ${TAG}_$c --config $CFG $EXTRA --steps 1 --warmup 0 --no-cpu-baseline > $OUT/profile_$c.log 2>&1 || { tail -20 $OUT/profile_$c.log; exit 1; }
cp $R/gpurun_out/prof_${TAG}_$c/partial_all_summary.json $R/profiles/${TAG}_${c}_summary.json
cp $R/gpurun_out/prof_${TAG}_$c/partial_all_kernel_stats.csv $R/profiles/${TAG}_${c}_kernel_stats.csv
cd $R
timeout -k 10 900 python -u bench.py --config $CFG $EXTRA > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; exit 1; }
cat $OUT/bench_$c.json
