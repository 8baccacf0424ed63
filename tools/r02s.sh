# (1) split probes, (2) terms in full-window walks (C2, C4), (3) C4 -p 100 throughput of this build
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02s
mkdir -p $OUT
bash $R/tools/r02r.sh || exit 1
for cfg in C2 C4; do
  FSCL_AMD_LIBDIR=$R/fscl_amd/_build_fuse timeout -k 10 300 python3 bench.py --config $cfg --n-permute 20 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/fuse_$cfg.json || exit 1
done
timeout -k 10 300 python3 bench.py --config C4 --n-permute 100 --warmup 1 --steps 2 --no-cpu-baseline > $OUT/c4_p100.json
