# round 6, final tree: rocprofv3 PMC passes of the whole C5 job, one reduced pass at a time with the raw
# output in /tmp (the first try of three passes in one call hit the call's limit with ~80 MB of raw CSVs)
set -o pipefail
for p in sq tcc mem; do
  PROF_TMP=1 PASSES=$p PROF_LIMIT=700 bash tools/prof_c5.sh r06c || exit 1
done
