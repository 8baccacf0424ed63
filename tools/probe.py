"""Tiny end-to-end probe of the GPU path (development aid)."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import fscl_amd  # noqa: E402
from fscl_amd import synth  # noqa: E402

n_snps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
out = Path(sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/probe")
out.mkdir(parents=True, exist_ok=True)
synth.write_snp_file(str(out / "p.snp"), synth.generate(n_chr=1, chr_len=n_snps * 1000, snps_per_chr=n_snps, n=10,
                                                        seed=5))
t = time.time()
scan = fscl_amd.run(out / "p.snp", out / "p.txt", verbosity=3)
print("run", time.time() - t, "s", fscl_amd.get_stats(), flush=True)
print((out / "p.txt").read_text()[:500])
