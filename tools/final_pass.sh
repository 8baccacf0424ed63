# end-of-round measurement on one GPU: the GPU suite, smoke, the C4 job's profile (trace + PMC passes, reduced on
# the box and copied into profiles/ there so that the bench lines after it cite it), then the bench lines.
# bash tools/final_pass.sh <tag>
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/final_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 || { tail -40 $OUT/gputest.log; exit 1; }
tail -1 $OUT/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
echo "smoke ok"
REDUCE=1 bash tools/profile.sh ${TAG}_c4_p1000 --config C4 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/profile.log 2>&1 || { tail -20 $OUT/profile.log; exit 1; }
cp $R/gpurun_out/prof_${TAG}_c4_p1000/partial_all_summary.json $R/profiles/${TAG}_c4_p1000_summary.json
cp $R/gpurun_out/prof_${TAG}_c4_p1000/partial_all_kernel_stats.csv $R/profiles/${TAG}_c4_p1000_kernel_stats.csv
cd $R
timeout -k 10 600 python -u bench.py > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err; exit 1; }
cat $OUT/bench_c4.json
timeout -k 10 300 python -u bench.py --config C2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
timeout -k 10 300 python -u bench.py --config C3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -20 $OUT/bench_c3.err; exit 1; }
# the driver's SCALE command shape (one rank per GPU under torch.distributed.run), rehearsed with two ranks on
# this one GPU (gloo for torch's own barrier and max-over-ranks; the library's shared-memory exchange)
FSCL_AMD_DEVICE=0 FSCL_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --config C2 --steps 1 --warmup 0 --no-cpu-baseline \
  > $OUT/bench_c2_torchrun2.json 2> $OUT/bench_c2_torchrun2.err || { tail -20 $OUT/bench_c2_torchrun2.err; exit 1; }
cat $OUT/bench_c2_torchrun2.json
# rank 0 of a 2/4/8-GPU C4 job rehearsed on this GPU (needs the rehearsal build: python -m fscl_amd.build --rehearsal)
bash tools/rehearse.sh C4 $TAG "2 4 8" || exit 1
echo done
