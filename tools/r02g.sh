export FSCL_AMD_LIBDIR=$GRAFT_REPO_ROOT/fscl_amd/_build_phase
for cfg in "1 0" "8 0" "8 1"; do set -- $cfg
  if [ $2 = 1 ]; then export FSCLG_NO_WINDOW=1; else unset FSCLG_NO_WINDOW; fi
  rm -f /tmp/ct.bin
  FSCLG_CELL_TRACE=/tmp/ct.bin FSCL_AMD_SPLIT=$1 timeout -k 10 120 python3 tools/split_probe.py 8 2>/dev/null | tail -1
  python3 tools/cell_trace.py /tmp/ct.bin | tail -4
done
