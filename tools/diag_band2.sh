# band mode A/B (round 6): the walk-window path (BAND_TH=-1) against band mode, initial scans of C4, C5 (2
# chromosomes) and C3, then the full C2 job's parity
set -o pipefail
B=fscl_amd/_build
bash tools/ab.sh b3c4 1 "--config C4 --n-permute 0 --steps 2 --warmup 1" old=$B,FSCLG_BAND_TH=-1 band=$B,FSCLG_BAND_TH=16 || exit 1
bash tools/ab.sh b3c5 1 "--config C5 --chromosomes 2 --n-permute 0 --steps 2 --warmup 1" old=$B,FSCLG_BAND_TH=-1 band=$B,FSCLG_BAND_TH=16 || exit 1
bash tools/ab.sh b3c3 1 "--config C3 --n-permute 0 --steps 3 --warmup 1" old=$B,FSCLG_BAND_TH=-1 band=$B,FSCLG_BAND_TH=16 || exit 1
bash tools/ab.sh b3c2 1 "--config C2 --steps 1 --warmup 1" band=$B,FSCLG_BAND_TH=16 || exit 1
