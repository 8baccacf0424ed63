# round 6: the LDS window groups' tolerance under site-major dealing (2 default, 4, 9): C4 job, C5 2-chr scan
set -o pipefail
B=fscl_amd/_build
AB_LIMIT=300 bash tools/ab.sh t_c4 2 "--config C4 --steps 2 --warmup 1" gt2=$B gt4=fscl_amd/_build_gt4 gt9=fscl_amd/_build_gt9 || exit 1
AB_LIMIT=300 bash tools/ab.sh t_c5x2 1 "--config C5 --chromosomes 2 --n-permute 0 --steps 2 --warmup 1" gt2=$B gt4=fscl_amd/_build_gt4 gt9=fscl_amd/_build_gt9 || exit 1
