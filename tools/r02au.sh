# launch look-ahead (the next trial launched with its most likely permutation while the current
# trial's blocking batch runs): GPU suite (on with 2 contexts / 2 ranks), the permutation tests
# again with it forced on at one GPU, 8-GPU rehearsal with and without, one-GPU C4 with and without
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02au
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 || exit 1
FSCL_AMD_SPEC_LAUNCH=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "golden or oracle or pipelined or full_genomes or sigint or back_to_back" > $OUT/gputest_la1.log 2>&1 || exit 1
FSCL_AMD_SPEC_LAUNCH=1 timeout -k 10 300 bash tools/scale_sim.sh C4 r02au_la1 8 > $OUT/sim_la1.log 2>&1 || exit 1
FSCL_AMD_SPEC_LAUNCH=0 timeout -k 10 300 bash tools/scale_sim.sh C4 r02au_la0 8 > $OUT/sim_la0.log 2>&1 || exit 1
FSCL_AMD_SPEC_LAUNCH=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/c4_la1.json 2>$OUT/c4_la1.err || exit 1
FSCL_AMD_SPEC_LAUNCH=0 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/c4_la0.json 2>$OUT/c4_la0.err || exit 1
