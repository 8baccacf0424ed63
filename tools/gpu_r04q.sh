set -o pipefail
mkdir -p gpurun_out/r04q
# the GPU suite on the submit path without hash maps, then r04p's host profile again
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04q/pytest.log 2>&1 || { tail -30 gpurun_out/r04q/pytest.log; exit 1; }
tail -3 gpurun_out/r04q/pytest.log
bash tools/gpu_r04p.sh && cp -r gpurun_out/r04p/. gpurun_out/r04q/
# slot use of the C5 permutation trials (per-cell trace; analysed on the box, the trace stays there)
FSCLG_CELL_TRACE=/tmp/c5_cells.bin timeout -k 10 600 python3 -u bench.py --config C5 --n-permute 1000 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04q/c5_trace.json 2> gpurun_out/r04q/c5_trace.err || exit 1
python3 tools/slot_use.py /tmp/c5_cells.bin 512 1.0 > gpurun_out/r04q/slot_use.txt && python3 tools/slot_use.py /tmp/c5_cells.bin 512 0.45 >> gpurun_out/r04q/slot_use.txt && cat gpurun_out/r04q/slot_use.txt
