# the working tree's build against fscl_amd/_build_phead (the last commit's build): parity subset on the working tree,
# then interleaved A/B at C4 and C2 (-p 20)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=gpurun_out/ab_head
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "golden or C4_part or C2 or C3 or pipelined or full_genomes_match_oracle_fixture or two_devices" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
timeout -k 10 900 bash tools/gpu_ab2.sh ${AB_ROUNDS:-2} "c4head:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_phead" "c4new:FSCL_AMD_AB=1" > $OUT/ab_c4.log 2>&1 || exit 1
BENCH_ARGS="--config C2" timeout -k 10 600 bash tools/gpu_ab2.sh ${AB_ROUNDS:-2} "c2head:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_phead" "c2new:FSCL_AMD_AB=1" > $OUT/ab_c2.log 2>&1 || exit 1
cat $OUT/ab_c4.log $OUT/ab_c2.log
