"""Per-call cost of the drop-in search_maxalpha (development probe, GPU box)."""
import ctypes as C, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import fscl_amd
from util import GOLD, manifest, read_dump
case = "g2_p30"
c = manifest()["cases"][case]
scan = fscl_amd.load_snp_input(GOLD / c["input"])
fsp = fscl_amd.background_fsp(scan)
tab = fscl_amd.compute_sweep_model_tables(scan, fsp)
fscl_amd.compute_snp_null_model(scan, fsp)
rows = read_dump(GOLD / f"{case}.dump")
L = fscl_amd.get_lib()
print("sites", scan.contents.n_snps, "points", len(rows), "window", rows[0][8] - rows[0][7] + 1)
def call(row):
    pt = fscl_amd.ScanPtT()
    pt.chr, pt.sweep_pos = row[0], row[1]
    pt.null_logl = row[5]
    pt.nearest_snp, pt.window_start, pt.window_end = row[6], row[7], row[8]
    pt.n_snps = row[8] - row[7] + 1
    pt.sm_logl, pt.lalpha = -1.7976931348623157e308, 4.0
    L.search_maxalpha(C.byref(pt), scan.contents.snps, tab)
for r in rows: call(r)
for rep in range(3):
    fscl_amd.reset_stats()
    t0 = time.perf_counter()
    for _ in range(20): call(rows[5])
    t1 = time.perf_counter()
    st = fscl_amd.get_stats()
    print(f"  kernel {st['kernel_ms'] / 20 * 1e3:.0f} us/call over {st['n_launches']} launches")
    for r in rows: call(r)
    t2 = time.perf_counter()
    print(f"same point x20: {(t1-t0)/20*1e6:.0f} us/call; all {len(rows)} points: {(t2-t1)/len(rows)*1e6:.0f} us/call")
