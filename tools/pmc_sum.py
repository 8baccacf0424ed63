"""Totals of tools/pmc.sh passes over a job's search_maxpos dispatches, and per SNP term.
    python tools/pmc_sum.py gpurun_out/pmc_<tag> [...]   -> one JSON object per directory
per_term = counter total over the job / the job's SNP terms (the pass's own bench line, stats.n_terms);
TA/TD busy counters are summed over the CUs, so per_term is texture-path cycles per term on its CU."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

res = {}
for d in map(Path, sys.argv[1:]):
    tot, disp, n_terms = defaultdict(float), set(), {}
    for f in sorted(d.glob("p*/run_counter_collection.csv")):
        i = f.parent.name
        for r in csv.DictReader(open(f)):
            if "search_maxpos" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add((i, r["Dispatch_Id"]))
        b = d / f"bench_{i}.json"
        if b.exists() and b.read_text().strip():
            n_terms[i] = json.loads(b.read_text().strip().splitlines()[-1])["stats"]["n_terms"]
    nt = max(n_terms.values()) if n_terms else 0
    out = {"totals_over_job": dict(tot), "n_terms": nt, "dispatches_per_pass": len(disp) / max(1, len(n_terms))}
    if nt:
        out["per_term"] = {k: v / nt for k, v in tot.items() if not k.startswith("GRBM")}
    h, m = tot.get("TCC_HIT_sum"), tot.get("TCC_MISS_sum")
    if h is not None and m is not None and h + m > 0:
        out["tcc_hit_rate"] = h / (h + m)
    if tot.get("SQ_WAVE_CYCLES"):
        out["wait_any_frac"] = tot.get("SQ_WAIT_ANY", 0.0) / tot["SQ_WAVE_CYCLES"]
    res[d.name] = out
print(json.dumps(res, indent=1))
