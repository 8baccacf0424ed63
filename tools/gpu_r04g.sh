set -o pipefail
# C5's whole genome (22 chromosomes, L2 overflow per XCD) at 200 permutations: rocprofv3 trace + PMC passes,
# reduced on the box (the term rate and L2/HBM traffic of the dense phase; the full job's tail is the
# one-chromosome profile's regime)
REDUCE=1 PROF_LIMIT=500 bash tools/profile.sh r04g_c5 --config C5 --n-permute 200 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04g_profile.log 2>&1 || { tail -20 gpurun_out/r04g_profile.log; exit 1; }
cp gpurun_out/prof_r04g_c5/partial_all_summary.json profiles/r04g_c5_p200_summary.json
cp gpurun_out/prof_r04g_c5/partial_all_kernel_stats.csv profiles/r04g_c5_p200_kernel_stats.csv
python3 -c "import json;d=json.load(open('profiles/r04g_c5_p200_summary.json'));print({k: d[k] for k in d if k in ('trace','trace_union','hbm_bytes_per_launch','pmc_per_launch')})" | cut -c1-1500
