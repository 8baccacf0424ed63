# workgroup-shape variants of the same source vs the default build: parity subset on the first variant, then
# interleaved A/B at C4 and C2 (-p 20).  Variants are fscl_amd/_build_<name> (python -m fscl_amd.build variants)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=gpurun_out/ab_shapes
mkdir -p $OUT
V1=$1; shift
FSCL_AMD_LIBDIR=$R/fscl_amd/_build_$V1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "golden or C4_part or C2 or pipelined or full_genomes_match_oracle_fixture" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
specs4=("c4base:FSCL_AMD_AB=1"); specs2=("c2base:FSCL_AMD_AB=1")
for v in $V1 "$@"; do specs4+=("c4$v:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_$v"); specs2+=("c2$v:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_$v"); done
timeout -k 10 900 bash tools/gpu_ab2.sh 2 "${specs4[@]}" > $OUT/ab_c4.log 2>&1 || exit 1
BENCH_ARGS="--config C2" timeout -k 10 600 bash tools/gpu_ab2.sh 2 "${specs2[@]}" > $OUT/ab_c2.log 2>&1 || exit 1
cat $OUT/ab_c4.log $OUT/ab_c2.log
