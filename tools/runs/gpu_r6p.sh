# round 6, final tree: rocprofv3 passes of the whole C5 job (10 000 permutations), first call
set -o pipefail
PASSES="trace fetch write" PROF_LIMIT=600 bash tools/prof_c5.sh r06c || exit 1
