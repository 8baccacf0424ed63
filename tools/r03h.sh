# A/B: log distances pipelined through LDS by DMA (pdma) vs the interleaved-site build (new); parity subset on pdma first
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03h
FSCL_AMD_LIBDIR=$R/fscl_amd/_build_pdma timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "golden or C4_part or C2 or pipelined or full_genomes_match_oracle_fixture" > gpurun_out/r03h/parity.log 2>&1 || { tail -30 gpurun_out/r03h/parity.log; exit 1; }
tail -2 gpurun_out/r03h/parity.log
timeout -k 10 900 bash tools/gpu_ab2.sh 2 "c4new:FSCL_AMD_AB=1" "c4dma:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_pdma" > gpurun_out/r03h/ab_c4.log 2>&1 || exit 1
BENCH_ARGS="--config C2" timeout -k 10 600 bash tools/gpu_ab2.sh 2 "c2new:FSCL_AMD_AB=1" "c2dma:FSCL_AMD_LIBDIR=$R/fscl_amd/_build_pdma" > gpurun_out/r03h/ab_c2.log 2>&1 || exit 1
cat gpurun_out/r03h/ab_c4.log gpurun_out/r03h/ab_c2.log
