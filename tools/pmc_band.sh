# PMC passes (tools/pmc_groups.txt) of the C4 initial scan, walk-window path against band mode (round 6)
set -o pipefail
for v in old band; do
  E="FSCLG_BAND_TH=16"; [ $v = old ] && E="FSCLG_BAND_TH=-1"
  env $E PMC_GROUPS=$PWD/tools/pmc_band_groups.txt bash tools/pmc.sh band_$v --config C4 --n-permute 0 --steps 1 --warmup 0 --no-cpu-baseline || exit 1
done
echo ok
