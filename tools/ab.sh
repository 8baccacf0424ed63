# A/B of builds and/or environments on one GPU, alternating legs (run on the GPU box):
#   bash tools/ab.sh <tag> <rounds> "<bench.py args>" name=<build dir>[,ENV=V...] ...
# e.g. bash tools/ab.sh coef 2 "--config C4 --steps 2 --warmup 1" base=fscl_amd/_build exp=fscl_amd/_build_exlds
# A leg's exit status 1 (bench.py's parity failure) is accepted when ABLATION=1 (timing ablations whose
# results are wrong on purpose); any other failure ends the script.
set -o pipefail
TAG=$1; ROUNDS=$2; ARGS=$3; shift 3
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/ab_$TAG
mkdir -p $OUT
for r in $(seq $ROUNDS); do
  for leg in "$@"; do
    name=${leg%%=*}; rest=${leg#*=}
    lib=${rest%%,*}; envs=""; [ "$rest" != "$lib" ] && envs=$(echo ${rest#*,} | tr ',' ' ')
    env $envs FSCL_AMD_LIBDIR=$R/$lib timeout -k 10 ${AB_LIMIT:-400} python3 -u $R/bench.py $ARGS --no-cpu-baseline \
      > $OUT/${name}_$r.json 2> $OUT/${name}_$r.err
    rc=$?
    if [ $rc -ne 0 ] && ! { [ $rc -eq 1 ] && [ -n "$ABLATION" ]; }; then echo "leg $name round $r: exit $rc"; exit $rc; fi
    python3 - $OUT/${name}_$r.json $name $r <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
p = d.get("parity", {})
par = f"{p.get('jobs_identical')}/{p.get('jobs_checked')}" if "jobs_checked" in p else p.get("identical", p.get("scope"))
rf = d.get("roofline", {})
print(f"{sys.argv[2]:10s} r{sys.argv[3]} {d['ms_per_step']:10.2f} ms/step  {d['value']:12.1f} {d['unit'][:12]}  "
      f"{rf.get('terms_per_s', 0) / 1e9:7.1f} Gterms/s  launch {rf.get('avg_launch_ms', 0):.3f} ms  parity {par}", flush=True)
PY
  done
done
