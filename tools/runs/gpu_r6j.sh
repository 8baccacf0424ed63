# round 6: site-major segment dealing (default build) against walk-major (_build_wm), band mode in a kernel
# of its own; GPU suite first
set -o pipefail
mkdir -p gpurun_out/r6j
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6j/gputest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6j/gputest.log; exit 1; }
tail -1 gpurun_out/r6j/gputest.log
B=fscl_amd/_build
AB_LIMIT=300 bash tools/ab.sh j_c4 2 "--config C4 --steps 2 --warmup 1" site=$B wm=fscl_amd/_build_wm anc=fscl_amd/_build_anc || exit 1
AB_LIMIT=300 bash tools/ab.sh j_c4s 1 "--config C4 --n-permute 0 --steps 3 --warmup 1" site=$B wm=fscl_amd/_build_wm band=$B,FSCLG_BAND_TH=16 || exit 1
AB_LIMIT=300 bash tools/ab.sh j_c5x2 1 "--config C5 --chromosomes 2 --n-permute 0 --steps 2 --warmup 1" site=$B,FSCLG_BAND_TH=-1 wm=fscl_amd/_build_wm,FSCLG_BAND_TH=-1 band=$B || exit 1
