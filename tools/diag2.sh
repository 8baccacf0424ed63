# L2 locality probe (development aid): per-cell rates with 2 vs 22 chromosomes, and TCC hit/miss.
set -e
O=gpurun_out/diag2; mkdir -p $O; rm -f $O/*.bin
R=${GRAFT_REPO_ROOT:-$PWD}
B="python -u $R/bench.py --config C4 --n-permute 20 --steps 1 --warmup 0 --no-cpu-baseline"
FSCL_AMD_LIBDIR=fscl_amd/_build_phase FSCLG_CELL_TRACE=$O/c2chr.bin timeout -k 10 300 $B --chromosomes 2 > $O/c2chr.json 2>/dev/null
python tools/cell_trace.py $O/c2chr.bin > $O/c2chr.txt
FSCL_AMD_LIBDIR=fscl_amd/_build_phase FSCLG_CELL_TRACE=$O/c6chr.bin timeout -k 10 300 $B --chromosomes 6 > $O/c6chr.json 2>/dev/null
python tools/cell_trace.py $O/c6chr.bin > $O/c6chr.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/$O/pmc_c4 -o run -- $B > $R/$O/pmc_c4.json 2>/dev/null
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/$O/pmc_c2 -o run -- python -u $R/bench.py --config C2 --n-permute 20 --steps 1 --warmup 0 --no-cpu-baseline > $R/$O/pmc_c2.json 2>/dev/null
echo done
