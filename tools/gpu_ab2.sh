# Interleaved A/B of configurations (development aid), R rounds each, same box:
#   bash tools/gpu_ab2.sh R "name:ENV=val ..." "name2:FSCL_AMD_LIBDIR=... " ...
# Each run: bench.py --steps 1 --warmup 1 --n-permute 20 $BENCH_ARGS; prints avg launch ms per config.
set -e
R=$1; shift
mkdir -p gpurun_out/ab2
for r in $(seq 1 $R); do
  for cfg in "$@"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env $envs timeout -k 10 200 python bench.py --steps 1 --warmup 1 --n-permute 20 --no-cpu-baseline ${BENCH_ARGS:-} \
      > gpurun_out/ab2/${name}_$r.json 2>/dev/null
  done
done
python - "$@" <<'PY'
import json, sys, glob, statistics
for cfg in sys.argv[1:]:
    name = cfg.split(":")[0]
    v = [json.load(open(f))["roofline"]["avg_launch_ms"] for f in sorted(glob.glob(f"gpurun_out/ab2/{name}_*.json"))]
    print(f"{name:12s} avg_launch_ms min {min(v):.2f} median {statistics.median(v):.2f}  runs {[round(x, 2) for x in v]}")
PY
