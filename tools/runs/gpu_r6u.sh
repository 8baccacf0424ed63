# round 6: site-major slices far-first (_build_far) against near-first (default): golden + full-size
# parity on the variant, then the C4 job, C5 one chromosome (split kernel) and the C5 2-chr scan
set -o pipefail
mkdir -p gpurun_out/r6u
FSCL_AMD_LIBDIR=$PWD/fscl_amd/_build_far timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "golden or fixture or full" --timeout 300 --timeout-method thread > gpurun_out/r6u/gt_far.log 2>&1 || { tail -30 gpurun_out/r6u/gt_far.log; exit 1; }
tail -1 gpurun_out/r6u/gt_far.log
B=fscl_amd/_build
AB_LIMIT=300 bash tools/ab.sh u_c4 2 "--config C4 --steps 2 --warmup 1" near=$B far=fscl_amd/_build_far || exit 1
AB_LIMIT=300 bash tools/ab.sh u_c5chr 1 "--config C5 --chromosomes 1 --steps 1 --warmup 0" near=$B far=fscl_amd/_build_far || exit 1
