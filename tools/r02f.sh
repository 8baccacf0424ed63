for n in 8 40; do for sp in 1 8; do for w in 0 1; do
  if [ $w = 1 ]; then export FSCLG_NO_WINDOW=1; else unset FSCLG_NO_WINDOW; fi
  echo "nowin=$w $(FSCL_AMD_SPLIT=$sp timeout -k 10 120 python3 tools/split_probe.py $n 2>/dev/null | tail -1)"; done; done; done
