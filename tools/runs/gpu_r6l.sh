# round 6: segment length with site-major dealing (4096 default, 2048, 8192) on the C4 job; the split
# combine's batched loads on C5 one chromosome (default against FSCLG_COMBINE_BATCH=0); PMC of site-major
# against walk-major dealing (C4 initial scan)
set -o pipefail
B=fscl_amd/_build
AB_LIMIT=300 bash tools/ab.sh l_c4 2 "--config C4 --steps 2 --warmup 1" s4k=$B s2k=fscl_amd/_build_s2k s8k=fscl_amd/_build_s8k || exit 1
AB_LIMIT=300 bash tools/ab.sh l_c5chr 1 "--config C5 --chromosomes 1 --steps 1 --warmup 0" site=$B cmb0=fscl_amd/_build_cmb0 || exit 1
A="--config C4 --n-permute 0 --steps 1 --warmup 0 --no-cpu-baseline"
FSCL_AMD_LIBDIR=$PWD/fscl_amd/_build PMC_GROUPS=$PWD/tools/pmc_site_groups.txt bash tools/pmc.sh c4_site $A || exit 1
FSCL_AMD_LIBDIR=$PWD/fscl_amd/_build_wm PMC_GROUPS=$PWD/tools/pmc_site_groups.txt bash tools/pmc.sh c4_wm $A || exit 1
python3 tools/pmc_sum.py gpurun_out/pmc_c4_site gpurun_out/pmc_c4_wm > gpurun_out/pmc_site_c4.json || exit 1
rm -rf gpurun_out/pmc_c4_site/p*/ gpurun_out/pmc_c4_wm/p*/
