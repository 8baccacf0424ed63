# round 6: PMC of band mode against the walk-window path (TA/TD/TCC/LDS/SQ passes), initial scans of C4 and
# of C5's first two chromosomes; then the C5 two-chromosome initial scan A/B by time
set -o pipefail
for cfg in c4 c5; do
  A="--config C4 --n-permute 0 --steps 1 --warmup 0 --no-cpu-baseline"
  [ $cfg = c5 ] && A="--config C5 --chromosomes 2 --n-permute 0 --steps 1 --warmup 0 --no-cpu-baseline"
  for v in old band; do
    E="FSCLG_BAND_TH=16"; [ $v = old ] && E="FSCLG_BAND_TH=-1"
    env $E PMC_GROUPS=$PWD/tools/pmc_band_groups.txt bash tools/pmc.sh ${cfg}_$v $A || exit 1
  done
  python3 tools/pmc_sum.py gpurun_out/pmc_${cfg}_old gpurun_out/pmc_${cfg}_band > gpurun_out/pmc_band_${cfg}.json || exit 1
  rm -rf gpurun_out/pmc_${cfg}_*/p*/
done
B=fscl_amd/_build
AB_LIMIT=300 bash tools/ab.sh i_c5x2 2 "--config C5 --chromosomes 2 --n-permute 0 --steps 2 --warmup 1" old=$B,FSCLG_BAND_TH=-1 band=$B,FSCLG_BAND_TH=16 || exit 1
AB_LIMIT=300 bash tools/ab.sh i_c4s 2 "--config C4 --n-permute 0 --steps 3 --warmup 1" old=$B,FSCLG_BAND_TH=-1 band=$B,FSCLG_BAND_TH=16 || exit 1
