set -o pipefail
mkdir -p gpurun_out
nproc > gpurun_out/r02b_cpu.txt; python3 -c "import os;print(len(os.sched_getaffinity(0)), os.cpu_count())" >> gpurun_out/r02b_cpu.txt
cat /sys/fs/cgroup/cpu.max >> gpurun_out/r02b_cpu.txt 2>&1 || true
grep -m1 "model name" /proc/cpuinfo >> gpurun_out/r02b_cpu.txt
(cd /tmp && timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r02b_counters.txt 2>&1) || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02b_gputest.log 2>&1 && \
timeout -k 10 300 bash tools/scale_sim.sh C4 r02b 2 4 8 > gpurun_out/r02b_sim.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/r02b_bench_c4.json 2> gpurun_out/r02b_bench_c4.err
