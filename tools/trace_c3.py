"""Development aid: run a small C3-like scan with the trace build (FSCL_AMD_LIBDIR=fscl_amd/_build_trace)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import fscl_amd
from fscl_amd import synth
synth.write_config("/tmp/c3s.snp", "C3", seed=3, scale=0.05)
fscl_amd.set_device(0)
fscl_amd.run("/tmp/c3s.snp", "/tmp/c3s.out", asc_depth=20, asc_min_freq=2)
print(fscl_amd.get_stats())
