# round 6: the split cells' phase breakdown on this tree (C4 rank 0 of 8, rehearsed),
# then the C4 rank-0-of-8 rehearsal time with the plain rehearsal build
set -o pipefail
TAG=${TAG:-r6e}
VARIANT=rphase bash tools/tail_trace.sh $TAG || exit 1
R=$PWD
REC=/tmp/fscl_sim_r6e2.bin
export FSCL_AMD_LIBDIR=$R/fscl_amd/_build_rehearsal
FSCL_AMD_SIM=record:$REC timeout -k 10 300 python3 -u bench.py --config C4 --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/tail_$TAG/w1_plain.json 2>/dev/null || exit 1
for i in 1 2; do
  FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 300 python3 -u bench.py --config C4 --warmup 0 --steps 1 --no-cpu-baseline > gpurun_out/tail_$TAG/w8_plain_$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/tail_$TAG/w8_plain_$i.json'));print('w8 plain ms', round(d['ms_per_step']), 'wait', round(d['stats']['wait_s'],3))"
done
rm -f $REC
