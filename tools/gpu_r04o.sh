set -o pipefail
mkdir -p gpurun_out/r04o
FSCL_AMD_TRIAL_TRACE=$PWD/gpurun_out/r04o/trials_c5.txt timeout -k 10 600 python3 -u bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04o/c5.json 2> gpurun_out/r04o/c5.err || exit 1
python3 - <<'PY'
import numpy as np
d = np.loadtxt('gpurun_out/r04o/trials_c5.txt')
names = ['trial','act','A','B','bulkwait','perm','null+up+build','submit','blockwait','flush','m','draws']
for lo, hi in ((0, 25), (25, 200), (200, 1000), (1000, 3000), (3000, 10001)):
    t = d[(d[:,0] >= lo) & (d[:,0] < hi)]
    if len(t): print(lo, hi, 'act', round(t[:,1].mean()), 'A', round(t[:,2].mean()), 'B', round(t[:,3].mean()), {names[k]: round(t[:,k].mean()) for k in range(4, 10)}, 'sum', round(t[:,4:10].sum(1).mean()), 'total s', round(t[:,4:10].sum() / 1e6, 1))
PY
