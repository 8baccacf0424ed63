# round 2, first GPU call of the re-created session: full GPU suite (with the full-size
# C4/C5 fixtures), the default bench (C4), then rocprofv3 trace + PMC passes on C4 -p 100.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/r02i_counters.txt 2>&1) || true
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r02i_gputest.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r02i_bench_c4.json 2> gpurun_out/r02i_bench_c4.err && \
timeout -k 10 1300 bash tools/profile.sh r02i_c4_p100 --config C4 --n-permute 100 --warmup 1 --steps 1 --no-cpu-baseline > gpurun_out/r02i_prof.log 2>&1
