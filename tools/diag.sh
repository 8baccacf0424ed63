# Diagnostic builds on one config (development aid, run on the GPU box):
#   bash tools/diag.sh <config> <n_permute>
# phase timing + per-cell trace (fscl_amd/_build_phase), trip path mix (fscl_amd/_build_paths),
# then the plain build; each a bench.py run of one step.
set -e
C=$1; P=$2
O=gpurun_out/diag_$C
mkdir -p $O
rm -f $O/ctrace.bin
B="timeout -k 10 300 python -u bench.py --config $C --n-permute $P --steps 1 --warmup 0 --no-cpu-baseline"
FSCL_AMD_LIBDIR=fscl_amd/_build_phase FSCLG_CELL_TRACE=$O/ctrace.bin $B > $O/phase.json 2> $O/phase.err
python tools/cell_trace.py $O/ctrace.bin > $O/phase_summary.txt
FSCL_AMD_LIBDIR=fscl_amd/_build_paths $B > $O/paths.json 2> $O/paths.err
$B > $O/plain.json 2> $O/plain.err
echo done
