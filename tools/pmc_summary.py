"""Sum rocprofv3 --pmc counters of the dominant kernel: python tools/pmc_summary.py gpurun_out/pmc_<tag>"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "search_maxpos"
tot = collections.defaultdict(float)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(tot):
    print(f"{k:34s} {tot[k]:.4g}")
g = tot.get("GRBM_GUI_ACTIVE", 0) / 8  # per-XCD cycles
if g:
    for k in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TCP_PENDING_STALL_CYCLES_sum"):
        if k in tot:
            print(f"{k} per CU / cycles = {tot[k] / 256 / g:.3f}")
if "SQ_LDS_IDX_ACTIVE" in tot and g:
    print(f"LDS active per CU / cycles = {tot['SQ_LDS_IDX_ACTIVE'] / 256 / g:.3f}")
if "TCP_TOTAL_CACHE_ACCESSES_sum" in tot and "SQ_INSTS_VMEM_RD" in tot:
    print(f"TCP accesses per vmem instr = {tot['TCP_TOTAL_CACHE_ACCESSES_sum'] / tot['SQ_INSTS_VMEM_RD']:.2f}")
