# PMC passes for the dominant kernel (run on the GPU box): bash tools/pmc.sh <tag> [bench args...]
# one rocprofv3 --pmc pass per counter group, never combined with tracing
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py "$@" > $OUT/bench_p$i.json 2> $OUT/p$i.err
done < ${PMC_GROUPS:-$R/tools/pmc_groups.txt}
echo done
