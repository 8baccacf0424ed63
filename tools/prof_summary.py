"""Summarize a tools/profile.sh run into profiles/<tag>_*.  Usage:
    python tools/prof_summary.py gpurun_out/prof_<tag> profiles/<tag>
Writes <tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats) and
<tag>_summary.json (per-launch PMC averages of search_maxpos_kernel, HBM bytes
with the gfx950 FETCH_SIZE x2 correction of MI355X_MICROARCH.md §HBM)."""
import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

src, dst = Path(sys.argv[1]), sys.argv[2]
Path(dst).parent.mkdir(parents=True, exist_ok=True)
if (src / "trace" / "run_kernel_stats.csv").exists():
    shutil.copy(src / "trace" / "run_kernel_stats.csv", f"{dst}_kernel_stats.csv")
out = {"kernel": "search_maxpos_kernel"}
# every search_maxpos launch, one workgroup per cell or split (the hot path's two instantiations; bench.py's
# HIP events count both alike)
rows = [r for r in (csv.DictReader(open(src / "trace" / "run_kernel_stats.csv"))
                    if (src / "trace" / "run_kernel_stats.csv").exists() else []) if "search_maxpos" in r["Name"]]
if rows:
    calls = sum(int(r["Calls"]) for r in rows)
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out["trace"] = {"calls": calls, "avg_ms": tot / calls / 1e6,
                    "min_ms": min(float(r["MinNs"]) for r in rows) / 1e6,
                    "max_ms": max(float(r["MaxNs"]) for r in rows) / 1e6,
                    "share_pct": sum(float(r["Percentage"]) for r in rows),
                    "by_kernel": {("search_maxpos_split_kernel" if "split" in r["Name"] else "search_maxpos_kernel"):
                                  int(r["Calls"]) for r in rows}}
# launches of different batch streams overlap: the GPU time they occupy is the union of
# their intervals (bench.py divides by the same union, measured with HIP events)
kt = src / "trace" / "run_kernel_trace.csv"
if kt.exists():
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(kt))
                if "search_maxpos" in r["Kernel_Name"])
    busy, a, b = 0, None, None
    for s0, e0 in iv:
        if b is None or s0 > b:
            if b is not None:
                busy += b - a
            a, b = s0, e0
        else:
            b = max(b, e0)
    if b is not None:
        busy += b - a
    out["trace_union"] = {"calls": len(iv), "busy_ms": busy / 1e6,
                          "busy_ms_per_launch": busy / 1e6 / max(1, len(iv)),
                          "sum_ms": sum(e0 - s0 for s0, e0 in iv) / 1e6}
pmc, pmc_ms, tot = {}, {}, defaultdict(float)
for grp in ("fetch", "write", "sq", "f64", "mem", "tcc"):
    f = src / grp / "run_counter_collection.csv"
    if not f.exists():
        continue
    agg, n, dur = defaultdict(float), defaultdict(int), {}
    for r in csv.DictReader(open(f)):
        if "search_maxpos" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k in agg:
        pmc[k] = agg[k] / n[k]
    if dur:  # counter passes serialize the dispatches: each one's own duration, no overlap
        pmc_ms[grp] = sum(dur.values()) / len(dur) / 1e6
out["pmc_per_launch"] = pmc
out["pmc_dispatch_ms"] = pmc_ms
if "FETCH_SIZE" in pmc:
    fetch = pmc["FETCH_SIZE"] * 1024 * 2  # KB; x2: gfx950 FETCH_SIZE counts half of wide coalesced reads
    write = pmc.get("WRITE_SIZE", 0.0) * 1024
    out["hbm_bytes_per_launch"] = fetch + write
    out["hbm_bytes_note"] = "(FETCH_SIZE*2 + WRITE_SIZE) * 1024, MI355X_MICROARCH.md §HBM correction"
# the memory path over the whole job (the mem / tcc passes): TA / TD busy cycles (summed over the CUs) and
# L1 / L2 requests per SNP term, the L2 hit rate, and the HBM fetch bytes per term (the same job's terms)
terms = None
for name in ("bench_mem.json", "bench_tcc.json", "bench_fetch.json"):
    p = src / name
    if p.exists() and p.read_text().strip():
        terms = json.loads(p.read_text().strip().splitlines()[-1])["stats"]["n_terms"]
        break
if terms and any(k in tot for k in ("TA_TA_BUSY_sum", "TCC_HIT_sum")):
    mp = {"n_terms": terms, "per_term": {k: tot[k] / terms for k in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum",
                                                                      "TCP_TOTAL_CACHE_ACCESSES_sum",
                                                                      "TCP_TCC_READ_REQ_sum") if k in tot}}
    if "TCC_HIT_sum" in tot and "TCC_MISS_sum" in tot:
        mp["tcc_hit_rate"] = tot["TCC_HIT_sum"] / max(1.0, tot["TCC_HIT_sum"] + tot["TCC_MISS_sum"])
    if "FETCH_SIZE" in tot:
        mp["hbm_fetch_bytes_per_term"] = tot["FETCH_SIZE"] * 1024 * 2 / terms
    mp["note"] = ("counter totals over the job's search_maxpos dispatches / the job's SNP terms; TA/TD busy summed "
                  "over the CUs (texture-path cycles per term on its CU)")
    out["memory_path"] = mp
for name in ("bench_trace.json", "bench_fetch.json"):
    p = src / name
    if p.exists() and p.read_text().strip():
        b = json.loads(p.read_text().strip().splitlines()[-1])
        out.setdefault("bench", {})[name] = {"avg_launch_ms_hip_events": b["roofline"]["avg_launch_ms"],
                                             "busy_ms_per_launch_hip_events":
                                                 b["roofline"].get("busy_ms", 0.0) / max(1, b["roofline"]["launches"]),
                                             "alg_bytes_per_launch": b["roofline"]["alg_bytes_per_launch"],
                                             "value": b["value"], "ms_per_step": b["ms_per_step"]}
json.dump(out, open(f"{dst}_summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
