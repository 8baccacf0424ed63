# split-cell workgroup budget for the blocking batch at one GPU (FSCLG_SPLIT_BUDGET 256 default / 512 / 1024), full C4 job, interleaved x2
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02bc
mkdir -p $OUT
for r in 1 2; do
  for b in 256 512 1024; do
    FSCLG_SPLIT_BUDGET=$b timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/c4_b${b}_$r.json 2>/dev/null || exit 1
  done
done
python - <<'PY'
import json, glob
for b in (256, 512, 1024):
    v = [json.load(open(f))["ms_per_step"] for f in sorted(glob.glob(f"gpurun_out/r02bc/c4_b{b}_*.json"))]
    print(b, [round(x) for x in v])
PY
