set -o pipefail
mkdir -p gpurun_out/r04c
# does a rank's main thread burn a CPU while it waits for the GPU?  (FSCL_AMD_SPEC=0: no worker threads)
FSCL_AMD_SPEC=0 timeout -k 10 150 python3 -c "
import resource, subprocess, sys, time
t = time.time()
r = subprocess.run([sys.executable, 'bench.py', '--config', 'C4', '--steps', '1', '--warmup', '0', '--no-cpu-baseline', '--n-permute', '200'], stdout=open('gpurun_out/r04c/cpuwait0.json', 'w'), stderr=open('gpurun_out/r04c/cpuwait0.err', 'w'))
u = resource.getrusage(resource.RUSAGE_CHILDREN)
print('time_wall_user_sys', round(time.time() - t, 2), u.ru_utime, u.ru_stime)
sys.exit(r.returncode)" || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r04c/cpuwait0.json'));print('job s', d['ms_per_step']/1e3, 'setup s', d['setup_s'])"
BURN=spin VARIANTS="single replicated leader leader_norefine" ROUNDS=2 bash tools/rehearse_ranks.sh C4 r04c 8 || exit 1
BURN=yield VARIANTS="leader leader_all" ROUNDS=1 bash tools/rehearse_ranks.sh C4 r04cy 8 || exit 1
tail -2 gpurun_out/r04c/tests_hot.log
