# Timing ablations (development aid): kernel terms/s of the initial scan (-p 0), per build dir.
#   bash tools/ablate.sh <config> name:libdir ...
set -e
C=$1; shift
mkdir -p gpurun_out/abl
for r in 1 2; do
  for cfg in "$@"; do
    name=${cfg%%:*}; lib=${cfg#*:}
    FSCL_AMD_LIBDIR=$lib timeout -k 10 200 python bench.py --config $C --steps 3 --warmup 1 --n-permute 0 --no-cpu-baseline \
      > gpurun_out/abl/${C}_${name}_$r.json 2>/dev/null
  done
done
python - $C "$@" <<'PY'
import json, sys, glob
C = sys.argv[1]
for cfg in sys.argv[2:]:
    name = cfg.split(":")[0]
    v = [json.load(open(f))["roofline"]["terms_per_s"] / 1e9 for f in sorted(glob.glob(f"gpurun_out/abl/{C}_{name}_*.json"))]
    print(f"{C} {name:8s} Gterms/s {[round(x, 1) for x in v]}")
PY
