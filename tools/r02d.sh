# split / CU-reservation experiment on the C4 rehearsal (record once, replay W=1 and W=8 per setting)
set -o pipefail
mkdir -p gpurun_out/r02d
R=$GRAFT_REPO_ROOT
REC=/tmp/fscl_rec_c4.bin
FSCL_AMD_SIM=record:$REC timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02d/record.json
for cfg in "1 0" "8 0" "8 4" "8 8" "1 4"; do
  set -- $cfg
  for W in 1 8; do
    FSCL_AMD_SPLIT=$1 FSCLG_RESERVE=$2 FSCL_AMD_SIM=replay:$REC:$W:0 timeout -k 10 300 python3 bench.py --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/r02d/s$1_r$2_w$W.json
    echo "split=$1 reserve=$2 W=$W $(python3 -c "import json;d=json.load(open('gpurun_out/r02d/s$1_r$2_w$W.json'));s=d['stats'];print(round(d['value']), round(d['ms_per_step']), round(s['wait_s'],2), round(d['roofline']['busy_ms']))")"
  done
done
rm -f $REC
