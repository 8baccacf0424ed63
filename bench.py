#!/usr/bin/env python3
"""bench.py -- fscl CLR sweep scan + block-permutation test on MI355X.

One step = one whole job of the hot path on resident inputs: the initial scan
(search_maxpos on every grid cell) plus the permutation test (N+1 trials with
pruning), i.e. scan_chromosome + scan_permute of the reference
(scan-chromosome.c:228-652).  Input parsing, background spectrum, spline
tables and the null model are set up once before the timed region.

Workload (default, BASELINE.json configs[3], "C4" -- the north star's target
configuration, which fits one GPU): 22 synthetic chromosomes of 45.45 Mb, 1.0M
SNPs, n = 200, 10,010 grid cells of 100 kb, 1,000 permutations.  --gpus N
strong-scales the SAME job over N GPUs (parity mode: bit-identical to one GPU):
  * `python bench.py --gpus N` (no launcher): this one process drives GPUs 0..N-1
    (fscl_amd_set_devices, the CLI's --n-gpus): the host logic -- rand stream,
    permutation (with its speculative worker threads), pruning -- runs once, and
    every batch of cells is split into N cost-balanced contiguous shares.  Fewer
    than N visible GPUs is an error (exit 2).
  * under torch.distributed.run with N ranks (the driver's SCALE launch): one
    process per GPU; every rank runs the host logic and evaluates its share of
    every batch, one shared-memory all-gather per batch (fscl_amd_set_ranks_shm)
    completes the results on every rank.  --gpus must equal WORLD_SIZE.
Every timed job's final scan points (every field, floats as hex) are hashed and
compared with the oracle's digest of the same job (tests/golden/fullsize.json,
made by tests/golden/make_fullsize.py) where one exists: parity over the whole
job, the initial scan and all permutation trials with their pruning.
--config C2 gives BASELINE configs[1].

value = (grid points + sum of permute_n) / wall seconds (max over ranks).
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import tempfile
import time
import uuid
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "grid-points × permutations / sec; max |ΔCLR| vs reference"
UNIT = "grid-points×permutations/s"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
FP64_PEAK_TFS = 78.6       # MI355X FP64 vector (spec)
N_SIMD = 256 * 4           # 256 CUs x 4 SIMD-32 (MI355X_MICROARCH.md)
BYTES_PER_UNIT = 8         # 8 B per SNP-term and per window-null element


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C4")
    ap.add_argument("--n-permute", type=int, default=None)
    ap.add_argument("--seed", type=int, default=None,
                    help="synthetic genome seed (default 55 for C5 -- the seed of its oracle fixtures -- else 1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU baseline threads (default: every CPU this process may run on)")
    ap.add_argument("--cpu-sample", type=int, default=None, help="CPU baseline: cells in the sample")
    ap.add_argument("--cpu-full-job", action="store_true",
                    help="CPU baseline: also run the WHOLE job through oracle/_ref/ref_harness (the reference's "
                         "compiled hot path under the restated scan loop) and report it beside the sample's "
                         "extrapolation (the anchor of the extrapolation model; minutes at C2)")
    ap.add_argument("--exchange", choices=("shm", "torch"), default="shm",
                    help="multi-process exchange: the library's shared-memory all-gather, or a torch.distributed "
                         "all-reduce callback")
    ap.add_argument("--permute-mode", choices=("parity", "throughput"), default="parity",
                    help="throughput: counter-based random numbers, trials independent (labelled non-parity)")
    ap.add_argument("--contexts", type=int, default=1,
                    help="rehearsal only: this process drives N device contexts on its one GPU (the batch and "
                         "trial split of an N-GPU job, recorded with FSCL_AMD_SIM=record)")
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--chromosomes", type=int, default=None,
                    help="chromosomes (default: the config's; development aid)")
    ap.add_argument("--profile-summary", default=None,
                    help="rocprofv3 summary (tools/prof_summary.py) for roofline.traffic and the issue roofline; "
                         "default: the newest profiles/r*_<config>_*summary.json")
    return ap.parse_args()


def cpu_info() -> dict:
    """The host's CPU model and core counts (CPU-baseline context)."""
    model, phys = None, set()
    try:
        cur = {}
        for line in open("/proc/cpuinfo"):
            if ":" in line:
                k, v = (x.strip() for x in line.split(":", 1))
                if k == "model name" and model is None:
                    model = v
                cur[k] = v
            elif cur:
                phys.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
        if cur:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    quota = None
    try:  # cgroup v2 CPU bandwidth limit of this process (the GPU box's share of the node)
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0))
    return {"cpu_model": model or platform.processor(), "node_logical_cpus": os.cpu_count(),
            "node_physical_cores": len(phys) or None, "affinity_cpus": aff, "cgroup_cpus": quota,
            "usable_cpus": min(aff, quota) if quota else aff}


def profile_summary(args) -> tuple[dict | None, str | None]:
    def tag_order(q: Path):  # rNN then the revision letters: r02z < r02aa < r02ab
        tag = q.name.split("_")[0]
        return (tag[:3], len(tag), tag)
    # a profile of this workload: rNN<rev>_<config>[chr<N>]_...summary.json (chr<N>: a --chromosomes job)
    key = args.config.lower() + (f"chr{args.chromosomes}" if args.chromosomes else "")
    cands = [Path(args.profile_summary)] if args.profile_summary else sorted(
        (ROOT / "profiles").glob(f"r*_{key}_*summary.json"), key=tag_order)
    for q in reversed(cands):
        try:
            d = json.loads(q.read_text())
        except (OSError, ValueError):
            continue
        if d.get("hbm_bytes_per_launch"):
            return d, str(q.relative_to(ROOT) if q.is_absolute() else q)
    return None, None


def issue_roofline(prof: dict) -> dict | None:
    """VALU issue rate of the dominant kernel from the committed rocprofv3 PMC passes alone:
    wave-instructions per launch (SQ_INSTS_VALU; FP64 ones from the SQ_INSTS_VALU_*_F64
    counters where collected) weighted by their issue cost on a SIMD-32 (MI355X_MICROARCH.md:
    a wave64 VALU op 2 cycles, FP64 4), over the SIMD-cycles the launch occupied (the union of
    the overlapping launches x 1024 SIMDs x the clock GRBM_GUI_ACTIVE / 8 / dispatch time)."""
    pmc = prof.get("pmc_per_launch", {})
    tu, tr = prof.get("trace_union"), prof.get("trace")
    if not (pmc.get("SQ_INSTS_VALU") and tu and tr):
        return None
    valu = pmc["SQ_INSTS_VALU"]
    f64 = sum(v for k, v in pmc.items() if k.startswith("SQ_INSTS_VALU_") and k.endswith("_F64"))
    f64_src = "SQ_INSTS_VALU_*_F64 counters" if f64 else None
    if not f64:  # static share of FP64 VALU in the term loop when not collected
        f64 = valu * prof.get("fp64_valu_share", 0.5)
        f64_src = f"static FP64 share {prof.get('fp64_valu_share', 0.5)} of VALU (DESIGN.md §4.6)"
    # effective clock (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE / 8 XCDs / dispatch time) over the
    # counter pass's own dispatches, which rocprofv3 serializes (the trace's overlap excluded)
    d_ms = prof.get("pmc_dispatch_ms", {}).get("sq")
    clk = pmc["GRBM_GUI_ACTIVE"] / 8 / (d_ms * 1e-3) if pmc.get("GRBM_GUI_ACTIVE") and d_ms else 2.4e9
    cycles_used = 2 * (valu - f64) + 4 * f64
    cycles_avail = N_SIMD * clk * tu["busy_ms_per_launch"] * 1e-3
    out = {"bound": "valu-issue", "achieved": cycles_used / (tu["busy_ms_per_launch"] * 1e-3) / 1e12,
           "peak": N_SIMD * clk / 1e12, "unit": "T SIMD-cycles/s", "frac": cycles_used / cycles_avail,
           "valu_insts_per_launch": valu, "fp64_valu_per_launch": f64, "fp64_source": f64_src,
           "clock_ghz": clk / 1e9}
    if pmc.get("SQ_INSTS_LDS"):
        out["lds_insts_per_launch"] = pmc["SQ_INSTS_LDS"]
    if pmc.get("SQ_WAIT_ANY") and pmc.get("SQ_WAVE_CYCLES"):
        out["wait_any_frac"] = pmc["SQ_WAIT_ANY"] / pmc["SQ_WAVE_CYCLES"]
    return out


def full_job_fixture(snp: Path, opts: list[str]) -> tuple[str | None, dict | None]:
    """The oracle fixture of exactly this job (same input bytes, same options), if one exists."""
    import hashlib
    fx_path = ROOT / "tests" / "golden" / "fullsize.json"
    if not fx_path.exists():
        return None, None
    h = hashlib.sha256(snp.read_bytes()).hexdigest()
    for name, fx in json.loads(fx_path.read_text()).items():
        if fx["input_sha256"] == h and sorted(fx["options"]) == sorted(opts):
            return name, fx
    return None, None


def points_digest(pts) -> tuple[str, list[str]]:
    """SHA-256 of the canonical point dump (tests/golden/make_fullsize.py: every field of every
    point in the oracle's dump order, floats as C99 hex) and the canonical rows."""
    import hashlib
    fields = ("chr", "sweep_pos", "clr", "lalpha", "sm_logl", "null_logl", "nearest_snp", "window_start",
              "window_end", "permute_p", "permute_n", "permute_finished")
    h = hashlib.sha256()
    rows = []
    for p in pts:
        row = "\t".join(x.hex() if isinstance(x, float) else str(x) for x in (p[k].item() for k in fields))
        rows.append(row)
        h.update(row.encode())
        h.update(b"\n")
    return h.hexdigest(), rows


def heartbeat(period: float = 30.0) -> None:
    """A line on stderr every `period` seconds (long jobs, e.g. C5, print nothing else for minutes)."""
    import threading
    t0 = time.time()

    def run():
        while True:
            time.sleep(period)
            print(f"bench.py: running, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


def main() -> int:
    args = parse()
    heartbeat()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    import fscl_amd
    from fscl_amd import synth

    # --gpus N: N ranks under a launcher, else N devices driven by this process
    if world > 1 and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} under a launcher with WORLD_SIZE={world}", file=sys.stderr)
        return 2
    n_local = args.gpus if world == 1 else 1
    if n_local > 1:
        vis = fscl_amd.device_count()
        if vis < n_local:
            print(f"bench.py: --gpus {n_local} but {vis} GPU(s) visible", file=sys.stderr)
            return 2

    # FSCL_AMD_DEVICE / FSCL_BENCH_BACKEND=gloo: rehearse several ranks on one GPU (tests only)
    device = int(os.environ.get("FSCL_AMD_DEVICE", local))
    backend = os.environ.get("FSCL_BENCH_BACKEND", "nccl")
    if world > 1:
        torch.cuda.set_device(device)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
            dev = torch.device("cuda", device)
        else:
            dist.init_process_group(backend)
            dev = torch.device("cpu")
        if args.exchange == "shm":
            name = [f"/fscl_amd_{uuid.uuid4().hex}" if rank == 0 else None]
            dist.broadcast_object_list(name, src=0)
            fscl_amd.set_ranks_shm(rank, world, name[0])
        else:
            def allreduce(arr: np.ndarray) -> None:
                t = torch.from_numpy(arr).to(dev)
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
                arr[:] = t.cpu().numpy()

            fscl_amd.set_ranks(rank, world, allreduce)
    if args.contexts > 1:
        fscl_amd.set_devices([device] * args.contexts)
    elif n_local > 1:
        fscl_amd.set_devices(list(range(n_local)))
    else:
        fscl_amd.set_device(device)
    n_gpus = world * n_local

    if args.seed is None:
        args.seed = 55 if args.config == "C5" else 1
    cfg = dict(synth.CONFIGS[args.config])
    if args.chromosomes:
        cfg["n_chr"] = args.chromosomes
    n_permute = cfg["n_permute"] if args.n_permute is None else args.n_permute
    wd = Path(args.workdir or tempfile.mkdtemp(prefix="fscl_bench_"))
    wd.mkdir(parents=True, exist_ok=True)
    snp = wd / f"{args.config}_r{rank}.snp"
    synth.write_snp_file(str(snp), synth.generate(seed=args.seed, sweeps_per_chr=2, **cfg))

    # ---- untimed setup (input and tables reported separately)
    t0 = time.time()
    fscl_amd.get_lib().configure_logmsg(1)
    fscl_amd.init_log_table()
    scan = fscl_amd.load_snp_input(snp)
    fsp = fscl_amd.background_fsp(scan)
    tab = fscl_amd.compute_sweep_model_tables(scan, fsp, cfg.get("asc_depth", 0), cfg.get("asc_min_freq", 1))
    fscl_amd.compute_snp_null_model(scan, fsp)
    setup_s = time.time() - t0

    def barrier():
        if world > 1:
            dist.barrier()
        for d in range(n_local):
            torch.cuda.synchronize(d if n_local > 1 else None)

    job_opts = ([f"--n-permute={n_permute}"] if n_permute > 0 else []) + (
        [f"--asc-depth={cfg['asc_depth']}", f"--asc-minimum-freq={cfg.get('asc_min_freq', 1)}"]
        if cfg.get("asc_depth", 0) else [])
    fx_name, fx = full_job_fixture(snp, job_opts) if rank == 0 and args.permute_mode == "parity" else (None, None)
    # else the oracle's digest of this genome's initial scan alone, where one exists (C5: its 50k-cell
    # initial scan takes the oracle minutes, too long to run live beside the bench)
    sfx_name, sfx = full_job_fixture(snp, []) if rank == 0 and fx is None and job_opts else (None, None)

    fscl_amd.set_permute_mode(args.permute_mode)

    def job():
        fscl_amd.srand()  # every step is the same job (a fresh process's rand stream, fscl.c:135)
        fscl_amd.scan_chromosome(scan, tab)
        n_gp = scan.contents.n_scan_pts
        if n_permute > 0:
            fscl_amd.scan_permute(scan, tab, n_permute)
        pts = fscl_amd.points(scan)
        return n_gp, int(pts["permute_n"].sum()), pts

    for _ in range(args.warmup):
        job()
    fscl_amd.reset_stats()
    barrier()
    t0 = time.perf_counter()
    units, gp, n_perm_units = 0, 0, 0
    timed_pts = []
    for _ in range(args.steps):
        n_gp, n_perm, pts = job()
        units += n_gp + n_perm
        gp, n_perm_units = n_gp, n_perm
        if fx is not None:
            timed_pts.append(pts.copy())  # checked after the timed region
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    st = fscl_amd.get_stats()

    out = bench_line(args, cfg, st, units, elapsed, n_gpus, world, n_local, n_permute, gp, setup_s)

    # ---- parity of every timed job, whole job: initial scan + all permutation trials, their
    # hits, prune draws and saved null CLRs, against the oracle's digest of the same job
    if fx is not None:
        digs = [points_digest(p) for p in timed_pts]
        ok = [d == fx["dump_sha256"] for d, _ in digs]
        bad_rows = 0
        if not all(ok):  # locate: the fixture's sampled rows
            k = fx["sample_every"]
            rows = next(r for (d, r), o in zip(digs, ok) if not o)
            bad_rows = sum(rows[i * k] != want for i, want in enumerate(fx["sample"]))
        out["parity"] = {"scope": "full job", "fixture": f"tests/golden/fullsize.json[{fx_name}]",
                         "what": "SHA-256 of every field of every final scan point (CLR, lalpha, sm_logl, null_logl "
                                 "as hex; positions, windows; permute_p, permute_n, permute_finished) of each timed "
                                 "job against the oracle's run of the same job (oracle/oracle.c, pinned by the "
                                 "reference's own compiled code)",
                         "jobs_checked": len(ok), "jobs_identical": sum(ok), "points": fx["n_points"],
                         "sum_permute_n": fx["sum_permute_n"], "sampled_rows_differing": bad_rows,
                         "negj_per_job": st["negj"] / args.steps}
        out["max_abs_dclr"] = 0.0 if all(ok) else None
        if not all(ok):
            print(f"bench.py: PARITY FAILURE: {len(ok) - sum(ok)} of {len(ok)} timed jobs differ from {fx_name}",
                  file=sys.stderr)
    elif sfx is not None:
        fscl_amd.srand()
        fscl_amd.scan_chromosome(scan, tab)
        dig, rows = points_digest(fscl_amd.points(scan))
        k = sfx["sample_every"]
        ok = dig == sfx["dump_sha256"]
        out["parity"] = {"scope": "initial scan", "fixture": f"tests/golden/fullsize.json[{sfx_name}]",
                         "what": "SHA-256 of every field of every point of the GPU's initial scan of this genome "
                                 "against the oracle's (no fixture of the whole permutation job exists at this size)",
                         "points": sfx["n_points"], "identical": ok,
                         "sampled_rows_differing": 0 if ok else sum(rows[i * k] != w for i, w in enumerate(sfx["sample"]))}
        # not the line's max |dCLR|: the permutation trials of this job are not covered by the check
        out["parity"]["max_abs_dclr_initial_scan"] = 0.0 if ok else None
        out["max_abs_dclr"] = None
        out["max_abs_dclr_note"] = "initial scan only (parity.scope): no oracle fixture of the whole job"
    elif rank == 0:
        out["parity"] = {"scope": "initial scan" if world == 1 and n_local == 1 and not args.no_cpu_baseline else
                         "none in this run", "note": "no oracle fixture of this exact job (tests/golden/fullsize.json)"}

    # ---- CPU baseline (rank 0, one GPU): the reference's own compiled hot path
    # (oracle/_ref/ref_harness: sm-search.c / sm-spline.c / background / asc-bias / input
    # compiled from its sources, under oracle.c's restated scan loop -- scan-chromosome.c
    # needs GSL headers absent here), timed on this host's cores on a bounded sample of the
    # same job: evenly spread scan cells, one block permutation, and those cells'
    # permutation-trial cells; the whole job's CPU time is extrapolated from the per-cell
    # times and the job's own counts.  Then the GPU's initial scan is checked against the
    # reference code's on a spread sample of cells... and against the oracle on all cells.
    # Test infrastructure: timed and compared here, never called by the product.
    if rank == 0 and n_gpus == 1 and not args.no_cpu_baseline:
        info = cpu_info()
        out["cpu_baseline"], scan_dclr, out["position_mismatches"] = cpu_baseline(
            args, cfg, snp, wd, info, fscl_amd, scan, tab, gp, n_perm_units, st["trials"] // max(1, args.steps),
            units / args.steps, elapsed / args.steps, live_parity=fx is None and sfx is None)
        if fx is None and sfx is None:
            out["max_abs_dclr"] = scan_dclr
    if rank == 0:
        live = (out.get("cpu_baseline") or {}).get("node_linear", {}).get("job_s")
        out["north_star_ratio"] = north_star_ratio(args, n_permute, elapsed / args.steps, n_gpus, live)
        if out.get("cpu_baseline"):
            out["cpu_baseline"]["north_star_ratio"] = (out["north_star_ratio"] or {}).get("value")
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    fscl_amd.shutdown()
    if out.get("parity", {}).get("scope") == "full job" and out["parity"]["jobs_identical"] != out["parity"]["jobs_checked"]:
        return 1
    return 0


def bench_line(args, cfg: dict, st: dict, units: float, elapsed: float, n_gpus: int, world: int, n_local: int,
               n_permute: int, gp: int, setup_s: float) -> dict:
    """The JSON line (every key but parity / cpu_baseline) from the library's stats of the timed jobs
    (fscl_amd.get_stats()) and the committed profile of the workload; tests/test_host.py drives it
    from recorded stats on the CPU."""
    # ---- the dominant kernel (search_maxpos_kernel), from HIP events on the streams it is
    # launched on.  Consecutive trials overlap on the GPU (several batch streams), so rates
    # divide by the union of the launches' intervals (busy_ms: overlap counted once);
    # avg_launch_ms is the per-dispatch mean that rocprofv3's kernel stats report.
    busy_s = st["busy_ms"] / 1e3
    launches = max(1, st["n_launches"])
    alg_bytes = BYTES_PER_UNIT * (st["n_terms"] + st["n_null"])
    avg_launch_s = st["kernel_ms"] / launches / 1e3
    # the contract's figure: algorithmic bytes per launch over the average launch duration; launches
    # of consecutive trials overlap, so the device's own rate (overlap counted once) is reported beside it
    alg_gbs = alg_bytes / launches / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    alg_gbs_union = alg_bytes / busy_s / 1e9 if busy_s > 0 else 0.0
    prof, prof_src = profile_summary(args)
    traffic = prof.get("hbm_bytes_per_launch") if prof else None
    issue = issue_roofline(prof) if prof else None
    # FETCH_SIZE sanity: bytes per launch over the counter pass's own (serialized) dispatch time must
    # stay under the memory system's rates; C5's search dispatches report values that imply PB/s
    # (a counter artefact), and those are not used
    traffic_note = None
    if traffic and prof.get("pmc_dispatch_ms", {}).get("fetch"):
        implied = traffic / (prof["pmc_dispatch_ms"]["fetch"] * 1e-3) / 1e9
        if implied > 2 * HBM_PEAK_GBS:
            traffic_note = (f"FETCH_SIZE of this profile implies {implied / 1e3:.0f} TB/s over the dispatches' own "
                            f"duration, above any memory rate: a counter artefact, not used")
            traffic = None
    mem = None
    mem_path = ROOT / "profiles" / "r03b_pmc_mem_c4_c2.json"
    if prof and prof.get("memory_path", {}).get("per_term"):  # the same profile's mem / tcc passes
        m = prof["memory_path"]
        mem = {"source": prof_src, **{k: round(v, 3) for k, v in m["per_term"].items()},
               "tcc_hit_rate": m.get("tcc_hit_rate"), "hbm_fetch_bytes_per_term": m.get("hbm_fetch_bytes_per_term")}
    elif mem_path.exists() and args.config.lower() in ("c4", "c2") and not args.chromosomes:
        m = json.loads(mem_path.read_text())[args.config.lower()]
        t = m["totals_over_job"]
        mem = {"source": str(mem_path.relative_to(ROOT)), **{k: round(v, 3) for k, v in m["per_term"].items()},
               "tcc_hit_rate": t["TCC_HIT_sum"] / max(1.0, t["TCC_HIT_sum"] + t["TCC_MISS_sum"])}
    # SURVEY 8(d)'s roofline: algorithmic bytes (8 B per SNP term and per window-null element) per launch
    # over the average launch duration (live HIP events on the batches' own streams), against HBM peak.
    # the measured limiter leads: the kernel is bound by the latency of its
    # dependent L2/LDS gathers, not by HBM -- the contract's HBM-roofline figures follow it, labelled as what
    # they are (algorithmic bytes against the HBM peak; 8 B/term is served from LDS/L2, so frac_union can pass 1)
    limiter = {"kind": "latency" if issue else "unmeasured",
               "valu_issue_frac": issue["frac"] if issue else None,
               "wait_any_frac": issue.get("wait_any_frac") if issue else None,
               "ta_busy_cycles_per_term": mem.get("TA_TA_BUSY_sum") if mem else None,
               "td_busy_cycles_per_term": mem.get("TD_TD_BUSY_sum") if mem else None,
               "hbm_traffic_frac_of_peak": None,  # filled below from the measured traffic
               "source": prof_src,
               "what": "VALU issue cycles over the launches' SIMD-cycles (SQ_INSTS_VALU), waves waiting on memory "
                       "(SQ_WAIT_ANY / SQ_WAVE_CYCLES), texture-path busy cycles per SNP term (TA/TD, whole-job PMC "
                       "pass), from the committed rocprofv3 profile of this workload: issue and HBM both well below "
                       "peak, waves parked on dependent gathers -- latency-bound"}
    roof = {"limiter": limiter, "bound": "hbm",
            "bound_meaning": "the contract's roofline form for this no-MFMA path: SURVEY 8(d) algorithmic bytes "
                             "(8 B per SNP term and per window-null element) against the 8 TB/s HBM peak.  Those "
                             "bytes are served from LDS and L2, not HBM (traffic_over_alg), so frac is a work rate "
                             "in byte units, and frac_union can exceed 1; the binding ceiling is the limiter above",
            "achieved": alg_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": alg_gbs / HBM_PEAK_GBS,
            "achieved_union": alg_gbs_union, "frac_union": alg_gbs_union / HBM_PEAK_GBS,
            "traffic": traffic, "traffic_note": traffic_note, "source": prof_src, "kernel": "search_maxpos_kernel",
            "alg_bytes_per_launch": alg_bytes / launches,
            "traffic_over_alg": (traffic / (alg_bytes / launches)) if traffic and alg_bytes else None,
            "hbm_frac": (traffic * launches / busy_s / 1e9 / HBM_PEAK_GBS) if traffic and busy_s > 0 else None,
            "avg_launch_ms": st["kernel_ms"] / launches, "launches": st["n_launches"], "busy_ms": st["busy_ms"],
            "busy_ms_per_launch": st["busy_ms"] / launches,
            "rocprof_avg_launch_ms": prof.get("trace", {}).get("avg_ms") if prof else None,
            "rocprof_busy_ms_per_launch": prof.get("trace_union", {}).get("busy_ms_per_launch") if prof else None,
            "terms_per_s": st["n_terms"] / busy_s if busy_s > 0 else 0.0,
            # what actually limits it: not HBM (real traffic is a few % of the algorithmic
            # bytes: sites, tables and coefficient windows stay in L2/LDS) and not issue (VALU issue below
            # half its peak): latency of the dependent L2 gathers per trip, waves parked on memory
            "issue": issue, "memory_path": mem,
            "alg_bytes_served_from": "LDS and L2 (measured HBM traffic: traffic / traffic_over_alg)",
            "note": "achieved/frac: SURVEY 8(d) algorithmic bytes per launch over the average launch duration "
                    "(HIP events; rocprof_avg_launch_ms is the same from the committed trace); *_union: over the "
                    "union of the launches' intervals instead (consecutive trials' launches overlap: the device's "
                    "rate); limiter from the "
                    "committed rocprofv3 PMC of this workload (source): VALU issue (issue.frac), waves waiting on "
                    "memory (issue.wait_any_frac), texture-path cycles per term (memory_path); traffic = measured "
                    "HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE)"}

    limiter["hbm_traffic_frac_of_peak"] = roof["hbm_frac"]
    return {
        "metric": METRIC,
        "value": units / elapsed,
        "unit": UNIT,
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded neutral-spectrum SNPs with planted sweeps, fscl_amd/synth.py)",
        "config": {"workload": f"{args.config}: {cfg['n_chr']} x ({cfg['snps_per_chr']} SNPs, "
                               f"{cfg['chr_len'] // 10**6} Mb, n={cfg['n']}) chromosome(s), G=100kb, "
                               f"{n_permute} permutations, "
                               + ("parity mode" if args.permute_mode == "parity" else
                                  "THROUGHPUT MODE (counter-based random numbers: non-parity, not the metric's mode)")
                               + f", one job split over {n_gpus} GPU(s)",
                   "grid_points": gp, "n_permute": n_permute, "snps": cfg["snps_per_chr"] * cfg["n_chr"],
                   "units_per_step": units / args.steps,
                   "multi_gpu": (f"{world} processes, one GPU each, shared-memory all-gather per batch "
                                 f"(exchange: {args.exchange})" if world > 1 else
                                 f"one process driving {n_local} GPUs" if n_local > 1 else None),
                   # work shared between cells, identical results: a units/s comparison
                   # with the reference, which recomputes them, should read these
                   "dup_cells_per_step": st["n_dup_cells"] / args.steps,
                   "endpoint_evals_saved_per_step": st["n_ep_saved"] / args.steps,
                   "negj_per_step": st["negj"] / args.steps},
        "roofline": roof,
        "cpu_baseline": None,
        "max_abs_dclr": None,
        "setup_s": setup_s,
        "stats": {k: st[k] for k in ("n_terms", "n_null", "n_walks", "n_unsafe", "n_slow", "n_ties", "trials",
                                     "host_perm_s", "scan_s", "permute_s", "gp_evals",
                                     "cache_iv0", "cache_n_iv", "cache_n_rows", "cache_cover", "window_ms",
                                     "host_null_s", "host_upload_s", "search_s", "prune_s", "n_dup_cells",
                                     "n_ep_saved", "wait_s", "n_crit", "n_drain", "spec_threads", "spec_posted",
                                     "spec_hits", "spec_cands", "spec_wait_s", "spec_done", "spec_gen_s",
                                     "spec_claimed", "n_merged", "perm_leader", "plan_mode", "plan_fallback",
                                     "spec_rank", "n_split_retry", "prestaged", "prestage_hits")},
    }



NODE_LINEAR_TABLE = ROOT / "profiles" / "cpu_node_linear.json"
NORTH_STAR_TARGET = 100.0  # BASELINE.json north_star: >= 100x the reference CPU's wall clock (C4 job, 8 GPUs)


def north_star_ratio(args, n_permute: int, gpu_job_s: float, n_gpus: int, live_node_s: float | None = None):
    """Where this line stands against the north star's >= 100x bar: the node-linear CPU job seconds of this
    workload (the reference's compiled hot path over all the node's physical cores, perfectly scaled) over
    this run's seconds per job.  The CPU figure is this run's own (cpu_baseline.node_linear) when it timed
    the CPU, else the committed one of the same workload (profiles/cpu_node_linear.json); None without."""
    src = "this run's cpu_baseline.node_linear"
    node_s = live_node_s
    if node_s is None:
        key = f"{args.config}/chr{args.chromosomes or 'all'}/p{n_permute}/{args.permute_mode}"
        try:
            ent = json.loads(NODE_LINEAR_TABLE.read_text())["workloads"].get(key)
        except (OSError, ValueError, KeyError):
            ent = None
        if not ent:
            return None
        node_s, src = float(ent["job_s"]), f"{NODE_LINEAR_TABLE.relative_to(ROOT)}[{key}] <- {ent['source']}"
    ratio = node_s / gpu_job_s if gpu_job_s > 0 else None
    return {"value": ratio, "n_gpus": n_gpus, "target": NORTH_STAR_TARGET,
            "meets_target": bool(ratio is not None and ratio >= NORTH_STAR_TARGET),
            "node_linear_job_s": node_s, "gpu_job_s": gpu_job_s, "source": src,
            "what": "node-linear CPU seconds per job (reference code, one thread per cell, over the node's "
                    "physical cores, plus the serial permutations) / this run's seconds per job"}


def _harness(snp, cfg, threads, n_cells):
    harness = ROOT / "oracle" / "_ref" / "ref_harness"
    opts = [f"--n-threads={threads}"]
    if cfg.get("asc_depth", 0):
        opts += [f"--asc-depth={cfg['asc_depth']}", f"--asc-minimum-freq={cfg.get('asc_min_freq', 1)}"]
    r = subprocess.run([str(harness), "sample", str(snp), str(n_cells), *opts], capture_output=True, text=True)
    kv = dict(w.split("=", 1) for w in r.stderr.split() if "=" in w and w.split("=", 1)[0] in
              ("sample_cells", "threads", "cell_s", "perm_gen_s", "perm_cells", "perm_cell_s"))
    if r.returncode != 0 or "cell_s" not in kv:
        raise RuntimeError(f"ref_harness sample failed ({r.returncode}): {r.stderr[-400:]}")
    return {k: float(v) for k, v in kv.items()}


def _harness_full(snp, cfg, threads, n_permute, wd):
    """The whole job through the reference's compiled hot path: ref_harness scan (initial scan, then every
    permutation trial: the active points on `threads` threads, the block permutation serial between trials,
    as scan-chromosome.c:412-546 does), wall-clocked."""
    harness = ROOT / "oracle" / "_ref" / "ref_harness"
    opts = [f"--n-threads={threads}", f"--n-permute={n_permute}"]
    if cfg.get("asc_depth", 0):
        opts += [f"--asc-depth={cfg['asc_depth']}", f"--asc-minimum-freq={cfg.get('asc_min_freq', 1)}"]
    t0 = time.perf_counter()
    r = subprocess.run([str(harness), "scan", str(snp), str(Path(wd) / "cpu_full.out"), str(Path(wd) / "cpu_full.dump"),
                        *opts], capture_output=True, text=True)
    wall = time.perf_counter() - t0
    kv = dict(w.split("=", 1) for w in r.stderr.split() if "=" in w)
    if r.returncode not in (0, 3) or "scan_s" not in kv:  # 3: the job hit the reference's negative-j read (Q9)
        raise RuntimeError(f"ref_harness scan failed ({r.returncode}): {r.stderr[-400:]}")
    return {"job_s": wall, "scan_s": float(kv["scan_s"]), "threads": threads, "negj": int(kv.get("negj", 0)),
            "setup_note": "job_s includes the harness's setup (input, background, tables: about a second at C2)"}


def cpu_anchor() -> dict | None:
    """The extrapolation model's measured anchor: the newest committed bench line with a `full_job`
    (profiles/r*_cpu_anchor_*.json, a `--cpu-full-job` run on the GPU box)."""
    cands = sorted((ROOT / "profiles").glob("r*_cpu_anchor_*.json"))
    for q in reversed(cands):
        try:
            d = json.loads(q.read_text().strip().splitlines()[-1])
            fj = d["cpu_baseline"]["full_job"]
        except (OSError, ValueError, KeyError, TypeError, IndexError):
            continue
        return {"source": str(q.relative_to(ROOT)), "workload": d["config"]["workload"],
                "threads": fj["threads"], "measured_job_s": fj["job_s"], "extrapolated_job_s": fj["extrapolated_job_s"],
                "measured_over_extrapolated": fj["measured_over_extrapolated"],
                "note": "the same box's whole job through the reference's compiled hot path, against the sample "
                        "extrapolation this line uses: the model's error at that workload"}
    return None


def cpu_baseline(args, cfg, snp, wd, info, fscl_amd, scan, tab, gp, perm_units, trials, units, gpu_job_s,
                 live_parity=True):
    """Returns (cpu_baseline dict, max |dCLR|, position mismatches); live_parity=False: the parity block
    came from a committed oracle fixture instead of a live oracle run."""
    sys.path.insert(0, str(ROOT / "oracle"))
    from oracle import OracleScan  # noqa: E402
    threads = args.cpu_threads or info["usable_cpus"]  # every CPU this process may use (cgroup quota included)
    n_t = args.cpu_sample or max(64, min(gp, 24 * threads))
    n_1 = max(8, min(gp, 64))
    smp = _harness(snp, cfg, threads, n_t)
    one = _harness(snp, cfg, 1, n_1)
    # per-cell CPU seconds with `threads` threads (wall / cells) and with one; the job's CPU
    # time: its initial-scan cells, its permutation-trial cells, and one serial block
    # permutation per trial (scan-chromosome.c:441-456 runs it on one thread)
    c_scan, c_perm = smp["cell_s"] / smp["sample_cells"], smp["perm_cell_s"] / smp["perm_cells"]
    job_s = gp * c_scan + perm_units * c_perm + trials * smp["perm_gen_s"]
    c1_scan, c1_perm = one["cell_s"] / one["sample_cells"], one["perm_cell_s"] / one["perm_cells"]
    job1_s = gp * c1_scan + perm_units * c1_perm + trials * one["perm_gen_s"]
    phys = info["node_physical_cores"] or info["node_logical_cpus"]
    node_s = (gp * c1_scan + perm_units * c1_perm) / phys + trials * one["perm_gen_s"]  # perfect scaling
    bl = {"value": units / job_s, "unit": UNIT, "cores": threads, "kind": "reference",
          "sample": f"{smp['sample_cells']:.0f} evenly spread grid cells of the same genome, one block permutation "
                    f"and those cells' permutation-trial cells, through the reference's own compiled "
                    f"search_maxalpha (oracle/_ref) on {threads} threads; job time extrapolated: {gp} scan cells x "
                    f"{c_scan * 1e3:.2f} ms + {perm_units} trial cells x {c_perm * 1e3:.2f} ms + {trials} serial "
                    f"permutations x {smp['perm_gen_s'] * 1e3:.2f} ms = {job_s:.1f} s",
          "extrapolated": True, "job_s": job_s,
          "scan_phase_s": gp * c_scan,
          "kind_detail": "reference code for every cell's search_maxalpha / sm_likelihood / spline / tables "
                         "(oracle/_ref, compiled from /root/reference sources); the scan loop, the bisection and "
                         "the serial block permutation are the oracle's restatement (scan-chromosome.c needs GSL "
                         "headers absent in this image)",
          "perm_sample": {"trial_cells": perm_units, "trial_cell_ms": c_perm * 1e3, "trials": trials,
                          "serial_permutation_ms": smp["perm_gen_s"] * 1e3,
                          "serial_permutation_kind": "restated: oracle/ref_harness.c times orc_block_permute, the "
                                                     "oracle's restatement of snp_block_permute (scan-chromosome.c:"
                                                     "336-389) on the same 32-B records; SURVEY §6 measured the "
                                                     "reference's own at about 9.5 ms per trial at C4 geometry, so "
                                                     "this leg favours the CPU",
                          "perm_phase_s": perm_units * c_perm + trials * smp["perm_gen_s"], "extrapolated": True},
          "threads_1": {"value": units / job1_s, "job_s": job1_s, "sample_cells": one["sample_cells"]},
          "node_linear": {"value": units / node_s, "job_s": node_s, "cores": phys,
                          "note": "one-thread per-cell time / the node's physical cores (perfect scaling, "
                                  "an upper bound for the CPU) + the serial permutations"},
          **info, "gpu_over_cpu": job_s / gpu_job_s, "gpu_over_node_linear": node_s / gpu_job_s}
    if args.cpu_full_job:
        full = _harness_full(snp, cfg, threads, args.n_permute if args.n_permute is not None else cfg["n_permute"], wd)
        bl["full_job"] = {**full, "extrapolated_job_s": job_s, "measured_over_extrapolated": full["job_s"] / job_s,
                          "units": units, "value": units / full["job_s"],
                          "what": "the whole job (initial scan + every permutation trial with its pruning) through "
                                  "oracle/_ref/ref_harness scan on the same threads: the measured point the "
                                  "sample's extrapolation is checked against"}
    anchor = cpu_anchor()
    if anchor:
        bl["anchor"] = anchor
    if not live_parity:
        bl["parity"] = "see the line's parity block (committed oracle fixture)"
        return bl, None, None
    # parity of the GPU's initial scan with the oracle on every cell (same run, same host)
    fscl_amd.srand()
    fscl_amd.scan_chromosome(scan, tab)
    gpu = fscl_amd.points(scan)
    orc = OracleScan(snp, threads=threads, asc_depth=cfg.get("asc_depth", 0), asc_min_freq=cfg.get("asc_min_freq", 1))
    orc.scan()
    ref = orc.points()
    assert len(ref) == len(gpu)
    d = rel = 0.0
    m = ma = mw = bits = 0
    for r, g in zip(ref, gpu):
        c, gc = r[2], float(g["clr"])
        d = max(d, abs(c - gc))
        if c != 0.0:
            rel = max(rel, abs(c - gc) / abs(c))
        m += (r[0], r[1]) != (int(g["chr"]), int(g["sweep_pos"]))
        ma += r[3].hex() != float(g["lalpha"]).hex()
        mw += (r[6], r[7], r[8]) != (int(g["nearest_snp"]), int(g["window_start"]), int(g["window_end"]))
        bits += all(x.hex() == float(g[k]).hex() for x, k in zip(r[2:6], ("clr", "lalpha", "sm_logl", "null_logl")))
    bl["parity"] = {"what": "initial scan, every grid point, against oracle/oracle.c (bit-exact restatement pinned "
                            "by the reference's own compiled code, tests/test_oracle.py)",
                    "points": len(ref), "max_abs_dclr": d, "max_rel_dclr": rel, "position_mismatches": m,
                    "lalpha_mismatches": ma, "window_mismatches": mw,
                    "bit_identical_points": bits}
    return bl, d, m


if __name__ == "__main__":
    sys.exit(main())
