"""Latency of one launch of few cells, split vs not (development probe, GPU box):
    python tools/split_probe.py <n_cells>"""
import os, sys, tempfile, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fscl_amd
from fscl_amd import synth
n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
d = tempfile.mkdtemp()
snp = os.path.join(d, "p.snp")
synth.write_snp_file(snp, synth.generate(n_chr=1, chr_len=45_454_545, snps_per_chr=45_455, n=200, seed=4, sweeps_per_chr=2))
fscl_amd.init_log_table()
fscl_amd.get_lib().configure_logmsg(1)
scan = fscl_amd.load_snp_input(snp)
fsp = fscl_amd.background_fsp(scan)
tab = fscl_amd.compute_sweep_model_tables(scan, fsp)
fscl_amd.compute_snp_null_model(scan, fsp)
G = 45_454_545 // n
for rep in range(4):
    fscl_amd.reset_stats()
    t0 = time.perf_counter()
    fscl_amd.scan_chromosome(scan, tab, large_grid_sp=G)
    dt = time.perf_counter() - t0
    st = fscl_amd.get_stats()
    print(f"split={os.environ.get('FSCL_AMD_SPLIT', '8')} cells={scan.contents.n_scan_pts} wall {dt*1e3:.2f} ms "
          f"kernel {st['kernel_ms']:.2f} ms launches {st['n_launches']} terms {st['n_terms']}", flush=True)
