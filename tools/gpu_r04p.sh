set -o pipefail
mkdir -p gpurun_out/r04p
# where the host's submit time goes on the C5 genome (22 chromosomes) at 1 000 permutations
FSCLG_HOST_PROFILE=1 FSCL_AMD_TRIAL_TRACE=$PWD/gpurun_out/r04p/trials.txt timeout -k 10 600 python3 -u bench.py --config C5 --n-permute 1000 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04p/c5.json 2> gpurun_out/r04p/c5.err || exit 1
grep "host profile" gpurun_out/r04p/c5.err
python3 - <<'PY'
import numpy as np
d = np.loadtxt('gpurun_out/r04p/trials.txt')
names = ['trial','act','A','B','bulkwait','perm','null+up+build','submit','blockwait','flush','m','draws']
for lo, hi in ((0, 25), (25, 200), (200, 1001)):
    t = d[(d[:,0] >= lo) & (d[:,0] < hi)]
    if len(t): print(lo, hi, 'act', round(t[:,1].mean()), 'A', round(t[:,2].mean()), 'B', round(t[:,3].mean()), {names[k]: round(t[:,k].mean()) for k in range(4, 10)}, 'total s', round(t[:,4:10].sum() / 1e6, 1), 'submit s', round(t[:,7].sum() / 1e6, 2))
PY
