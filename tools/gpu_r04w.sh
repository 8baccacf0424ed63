set -o pipefail
mkdir -p gpurun_out/r04w
# where the one-GPU C4 job's 5.4 s go: per-trial trace, then the per-cell slot-use trace
FSCL_AMD_TRIAL_TRACE=$PWD/gpurun_out/r04w/trials_c4.txt timeout -k 10 300 python3 -u bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r04w/c4.json 2> gpurun_out/r04w/c4.err || { tail -5 gpurun_out/r04w/c4.err; exit 1; }
FSCLG_CELL_TRACE=/tmp/c4_cells.bin timeout -k 10 300 python3 -u bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04w/c4_trace.json 2> gpurun_out/r04w/c4_trace.err || { tail -5 gpurun_out/r04w/c4_trace.err; exit 1; }
python3 tools/slot_use.py /tmp/c4_cells.bin 512 1.0 > gpurun_out/r04w/slot_use.txt && python3 tools/slot_use.py /tmp/c4_cells.bin 512 0.5 >> gpurun_out/r04w/slot_use.txt && cat gpurun_out/r04w/slot_use.txt
