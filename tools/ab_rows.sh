# rows staged at the narrowest width (this tree) vs the last commit's 4-byte rows (fscl_amd/_build_phead,
# _build_pheadreh): the permutation parity tests, the C4 job at one GPU alternating, rank 0 of an 8-GPU rehearsal
# alternating, and the scatter kernel's time under rocprofv3.  bash tools/ab_rows.sh [rounds]
set -o pipefail
ROUNDS=${1:-2}
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/ab_rows
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pipelined or throughput or lockstep or full_genomes or sigint or ranks or permut or windowed or two_devices" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
for r in $(seq $ROUNDS); do
  for v in head new; do
    L="FSCL_AMD_AB=1"; [ $v = head ] && L="FSCL_AMD_LIBDIR=$R/fscl_amd/_build_phead"
    env $L timeout -k 10 600 python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c4_${v}_$r.json 2> $OUT/c4_${v}_$r.err || exit 1
    echo "c4 $v $r: $(python3 -c "import json;d=json.load(open('$OUT/c4_${v}_$r.json'));s=d['stats'];print(round(d['ms_per_step']), 'ms/job', d['parity']['jobs_identical'], 'of', d['parity']['jobs_checked'], 'identical; spec_wait', round(s['spec_wait_s'],3))")"
  done
done
REC=/tmp/fscl_sim_rows.bin
FSCL_AMD_LIBDIR=$R/fscl_amd/_build_rehearsal FSCL_AMD_SIM=record:$REC timeout -k 10 600 python3 -u $R/bench.py --config C4 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w1.json 2> $OUT/w1.err || exit 1
for r in $(seq $ROUNDS); do
  for v in head new; do
    L=$R/fscl_amd/_build_rehearsal; [ $v = head ] && L=$R/fscl_amd/_build_pheadreh
    FSCL_AMD_LIBDIR=$L FSCL_AMD_SIM=replay:$REC:8:0 timeout -k 10 600 python3 -u $R/bench.py --config C4 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/w8_${v}_$r.json 2> $OUT/w8_${v}_$r.err || exit 1
    echo "w8 $v $r: $(python3 -c "import json;d=json.load(open('$OUT/w8_${v}_$r.json'));s=d['stats'];print(round(d['ms_per_step']), 'ms/job wait', round(s['wait_s'],3), 'spec_wait', round(s['spec_wait_s'],3), 'host_perm', round(s['host_perm_s'],3))")"
  done
done
rm -f $REC
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/prof.json 2> $OUT/prof.err || exit 1
grep -h scatter $(find $OUT/prof -name "*kernel_stats.csv") | cut -c1-220
