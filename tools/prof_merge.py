"""Merge partial profile summaries (tools/profile.sh REDUCE=1, one per call) into one:
    python tools/prof_merge.py profiles/<tag> partial1_summary.json partial2_summary.json ...
Keys of later files add to or replace those of earlier ones (pmc_per_launch and pmc_dispatch_ms merge)."""
import json
import sys

out = {}
for f in sys.argv[2:]:
    d = json.load(open(f))
    for k, v in d.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            for k2, v2 in v.items():  # one level deeper too (memory_path.per_term of separate passes)
                if isinstance(v2, dict) and isinstance(out[k].get(k2), dict):
                    out[k][k2].update(v2)
                else:
                    out[k][k2] = v2
        else:
            out[k] = v
pmc = out.get("pmc_per_launch", {})
if "FETCH_SIZE" in pmc:
    out["hbm_bytes_per_launch"] = pmc["FETCH_SIZE"] * 1024 * 2 + pmc.get("WRITE_SIZE", 0.0) * 1024
    out["hbm_bytes_note"] = "(FETCH_SIZE*2 + WRITE_SIZE) * 1024, MI355X_MICROARCH.md §HBM correction"
mp = out.get("memory_path")
if mp and "FETCH_SIZE" in pmc and out.get("trace", {}).get("calls") and mp.get("n_terms"):
    # the passes ran the same deterministic job: FETCH per launch x the trace's launches over its terms
    mp["hbm_fetch_bytes_per_term"] = pmc["FETCH_SIZE"] * 1024 * 2 * out["trace"]["calls"] / mp["n_terms"]
json.dump(out, open(f"{sys.argv[1]}_summary.json", "w"), indent=1)
print(json.dumps(out, indent=1)[:2000])
