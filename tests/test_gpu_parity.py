"""GPU parity: the HIP path (through the C-ABI) against the golden fixtures
(reference-generated) and against the oracle, bit for bit: every scan point's
position, window, lalpha, sm_logl, CLR, and the permutation counts (which pin
the pruning and the rand() stream)."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

from util import (CLI, GOLD, ROOT, assert_rows_equal, manifest, points_rows, read_dump, run_oracle,
                  usable_cpus)
import fscl_amd
from fscl_amd import synth

pytestmark = pytest.mark.gpu


def _kw(options):
    kw = {}
    for a in options:
        k, _, v = a.lstrip("-").partition("=")
        if k == "n-permute":
            kw["n_permute"] = int(v)
        elif k == "asc-depth":
            kw["asc_depth"] = int(v)
        elif k == "asc-minimum-freq":
            kw["asc_min_freq"] = int(v)
        elif k == "ascbias-background-only":
            kw["ascbias_background_only"] = True
        elif k == "include-invariant":
            kw["include_invariant"] = True
        elif k == "force-neutral-spectrum":
            kw["force_neutral"] = True
        elif k == "coarse-grid-spacing":
            kw["large_grid_sp"] = int(v)
        elif k == "permute-nbp":
            kw["permute_nbp"] = float(v)
        elif k == "eval-range":
            kw["eval_range"] = int(v)
        elif k == "sweep-width":
            kw["scan_width_mb"] = float(v)
        else:
            raise ValueError(a)
    return kw


def test_device_present():
    assert fscl_amd.device_count() >= 1


@pytest.mark.parametrize("case", sorted(manifest()["cases"]))
def test_gpu_matches_golden(built, tmp, case):
    c = manifest()["cases"][case]
    scan = fscl_amd.run(GOLD / c["input"], tmp / "o.txt", **_kw(c["options"]))
    assert_rows_equal(points_rows(fscl_amd.points(scan)), read_dump(GOLD / f"{case}.dump"), case)
    assert (tmp / "o.txt").read_text() == (GOLD / f"{case}.out").read_text()


@pytest.mark.parametrize("th,minp,nb", [("0", "1", "8"), ("16", "8", "8"), ("0", "2", "2"), ("0", "1", "0")])
def test_band_mode_matches_golden(built, tmp, monkeypatch, th, minp, nb):
    """The band-mode term loop (the phase's walks evaluated interval band by band
    from LDS windows, pieces cut lazily at |d| thresholds) forced on for every golden case (by
    default it runs where the LDS window is at most 6 intervals: C5): every window staged with no
    merging (the most pieces and lazy cuts), the default merging, two bands, and no bands at all;
    every case's dump and output are the golden ones."""
    monkeypatch.setenv("FSCLG_BAND_TH", th)
    monkeypatch.setenv("FSCLG_BAND_MINP", minp)
    monkeypatch.setenv("FSCLG_BAND_NB", nb)
    for case in sorted(manifest()["cases"]):
        c = manifest()["cases"][case]
        scan = fscl_amd.run(GOLD / c["input"], tmp / "o.txt", **_kw(c["options"]))
        assert_rows_equal(points_rows(fscl_amd.points(scan)), read_dump(GOLD / f"{case}.dump"), case)
        assert (tmp / "o.txt").read_text() == (GOLD / f"{case}.out").read_text(), case


def test_band_mode_full_size_c4_matches_oracle_fixture(built, tmp, monkeypatch):
    """Band mode forced on C4's whole 1.0M-SNP genome (45 Mb chromosomes, n = 200, 3 trials), whose
    default is the walk-window path: the fixture's digest."""
    monkeypatch.setenv("FSCLG_BAND_TH", "16")
    sys.path.insert(0, str(GOLD))
    from make_fullsize import canonical_dump, sha256_file
    fx = _fullsize()["C4_full_p2"]
    snp = tmp / "c4.snp"
    synth.write_snp_file(str(snp), synth.generate(**fx["gen"]))
    scan = fscl_amd.run(snp, tmp / "g.txt", **_kw(fx["options"]))
    assert canonical_dump(points_rows(fscl_amd.points(scan))) == fx["dump_sha256"]
    assert sha256_file(tmp / "g.txt") == fx["out_sha256"]


@pytest.mark.parametrize("lookahead", ["0", "2"])
def test_bisection_lookahead_fallbacks(built, tmp, lookahead):
    """The two-level bisection with the look-ahead off (one level per alpha
    search) and with every prediction wrong on purpose (each look-ahead point dropped, the
    next round evaluates the other half): the golden outputs either way."""
    for case in ("g1_p25", "g1_asc"):
        c = manifest()["cases"][case]
        r = subprocess.run([str(CLI), "-f", str(GOLD / c["input"]), "-o", str(tmp / "o.txt"), *c["options"]],
                           capture_output=True, text=True, timeout=600, env=dict(os.environ, FSCLG_LOOKAHEAD=lookahead))
        assert r.returncode == 0, r.stderr
        assert (tmp / "o.txt").read_text() == (GOLD / f"{case}.out").read_text(), case


@pytest.mark.parametrize("spec", ["1", "2"])
def test_speculative_refine_fallbacks(built, tmp, spec):
    """Split cells can evaluate the refine walks of a guessed coarse winner beside the coarse walks
    (off by default since round 4, §11.3, so every other test runs without).  On,
    and evaluated but every guess taken as missed (each point then takes the second phase): the golden outputs either
    way, and the oracle's on a multi-chromosome permutation job."""
    env = dict(os.environ, FSCLG_SPEC_REFINE=spec)
    for case in ("g1_p25", "g1_asc", "g3_p10"):
        c = manifest()["cases"][case]
        r = subprocess.run([str(CLI), "-f", str(GOLD / c["input"]), "-o", str(tmp / "o.txt"), *c["options"]],
                           capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0, r.stderr
        assert (tmp / "o.txt").read_text() == (GOLD / f"{case}.out").read_text(), case
    snp = tmp / "m.snp"
    synth.write_snp_file(str(snp), synth.generate(n_chr=3, chr_len=3_000_000, snps_per_chr=3000, n=30, seed=71,
                                                  sweeps_per_chr=1))
    opts = ["--n-permute=40"]
    run_oracle(snp, tmp / "r.txt", opts)
    r = subprocess.run([str(CLI), "-f", str(snp), "-o", str(tmp / "g.txt"), *opts], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    assert (tmp / "g.txt").read_text() == (tmp / "r.txt").read_text()


@pytest.mark.parametrize("case", ["g1_p25", "g2_grid50k", "g3_scan"])
def test_cli_matches_golden(built, tmp, case):
    c = manifest()["cases"][case]
    r = subprocess.run([str(CLI), "-f", str(GOLD / c["input"]), "-o", str(tmp / "o.txt"), *c["options"]],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert (tmp / "o.txt").read_text() == (GOLD / f"{case}.out").read_text()


@pytest.mark.parametrize("name,gen,opts", [
    ("c1_like", dict(n_chr=1, chr_len=20_000_000, snps_per_chr=10_000, n=50, seed=31, sweeps_per_chr=2), []),
    ("multi_depth_asc", dict(n_chr=3, chr_len=6_000_000, snps_per_chr=6000, n=40, folded=0.3, seed=32,
                             sweeps_per_chr=1, missing=0.25, max_missing=3, duplicates=0.005),
     ["--asc-depth=10", "--asc-minimum-freq=2", "--n-permute=12"]),
    ("dense", dict(n_chr=2, chr_len=400_000, snps_per_chr=8000, n=20, seed=33, duplicates=0.05),
     ["--coarse-grid-spacing=25000", "--n-permute=6"]),
])
def test_gpu_matches_oracle(built, tmp, name, gen, opts):
    snp = tmp / f"{name}.snp"
    synth.write_snp_file(str(snp), synth.generate(**gen))
    run_oracle(snp, tmp / "o.txt", opts, tmp / "o.dump")
    scan = fscl_amd.run(snp, tmp / "g.txt", **_kw(opts))
    assert_rows_equal(points_rows(fscl_amd.points(scan)), read_dump(tmp / "o.dump"), name)
    assert (tmp / "g.txt").read_text() == (tmp / "o.txt").read_text()
    st = fscl_amd.get_stats()
    assert st["n_terms"] > 0


@pytest.mark.parametrize("name,er,parts,opts", [
    # every chromosome longer than the window 2*er+1: per-window null sums on the device
    ("long", 300, [dict(n_chr=2, chr_len=4_000_000, snps_per_chr=4000, n=30, seed=51, sweeps_per_chr=1)],
     ["--coarse-grid-spacing=40000", "--n-permute=4"]),
    # a mix: chromosomes shorter than, equal to and longer than the window, two depths
    ("mixed", 700, [dict(n_chr=1, chr_len=900_000, snps_per_chr=900, n=24, seed=52, chr_names=["a"]),
                    dict(n_chr=1, chr_len=1_500_000, snps_per_chr=1401, n=24, seed=53, chr_names=["b"]),
                    dict(n_chr=1, chr_len=9_000_000, snps_per_chr=7000, n=24, seed=54, chr_names=["c"],
                         sweeps_per_chr=2, missing=0.2, max_missing=2)],
     ["--coarse-grid-spacing=30000", "--n-permute=3"]),
])
def test_windowed_null_sums_match_oracle(built, tmp, name, er, parts, opts):
    """Chromosomes above 2*eval_range+1 SNPs: each point's null_logl is its own window's
    sequential sum (scan-chromosome.c:92-94), recomputed on the device for every trial."""
    snp = tmp / f"{name}.snp"
    chrs = []
    for p in parts:
        chrs += synth.generate(**p)
    synth.write_snp_file(str(snp), chrs)
    run_oracle(snp, tmp / "o.txt", [*opts, f"--eval-range={er}"], tmp / "o.dump")
    fscl_amd.reset_stats()
    scan = fscl_amd.run(snp, tmp / "g.txt", eval_range=er, **_kw(opts))
    assert_rows_equal(points_rows(fscl_amd.points(scan)), read_dump(tmp / "o.dump"), name)
    assert (tmp / "g.txt").read_text() == (tmp / "o.txt").read_text()
    assert fscl_amd.get_stats()["window_ms"] > 0


def test_shared_cells_and_endpoints_match_oracle(built, tmp):
    """First SNP half a grid step in: neighbouring scan points often share one G-aligned
    permutation cell (scan-chromosome.c:481-486), and every scan cell shares its endpoints
    with its neighbours; both are evaluated once on the device (fsclg_search_maxpos)."""
    chrs = []
    for name, off, seed in (("a", 1_250_000, 61), ("b", 3_030_000, 62)):
        (nm, pos, k, nn, fold), = synth.generate(n_chr=1, chr_len=6_000_000, snps_per_chr=5000, n=30, seed=seed,
                                                  sweeps_per_chr=1, chr_names=[name])
        chrs.append((nm, pos + off, k, nn, fold))
    snp = tmp / "shared.snp"
    synth.write_snp_file(str(snp), chrs)
    opts = ["--coarse-grid-spacing=50000", "--n-permute=6"]
    run_oracle(snp, tmp / "o.txt", opts, tmp / "o.dump")
    scan = fscl_amd.run(snp, tmp / "g.txt", **_kw(opts))
    assert_rows_equal(points_rows(fscl_amd.points(scan)), read_dump(tmp / "o.dump"), "shared")
    assert (tmp / "g.txt").read_text() == (tmp / "o.txt").read_text()


def test_tiny_chromosomes_match_oracle(built, tmp):
    """Chromosomes of 1, 2, 3, 64, 65 and 130 SNPs among larger ones: the edges of the
    wave-parallel searches (search_snppos over n = 1.., walk bounds over empty and
    one-site sides) and windows that are the whole chromosome."""
    chrs = []
    for i, (k, length) in enumerate(((1, 50_000), (2, 90_000), (3, 150_000), (64, 700_000), (65, 900_000),
                                     (130, 1_300_000), (3000, 3_000_000))):
        chrs += synth.generate(n_chr=1, chr_len=length, snps_per_chr=k, n=16, seed=70 + i, chr_names=[f"t{i}"],
                               sweeps_per_chr=1 if k >= 64 else 0)
    snp = tmp / "tiny.snp"
    synth.write_snp_file(str(snp), chrs)
    opts = ["--coarse-grid-spacing=20000", "--n-permute=5"]
    run_oracle(snp, tmp / "o.txt", opts, tmp / "o.dump")
    scan = fscl_amd.run(snp, tmp / "g.txt", **_kw(opts))
    assert_rows_equal(points_rows(fscl_amd.points(scan)), read_dump(tmp / "o.dump"), "tiny")
    assert (tmp / "g.txt").read_text() == (tmp / "o.txt").read_text()


@pytest.mark.parametrize("name,blocks,hap,seg,length,grid", [
    ("blocks", 4, 20, 600, 2_000_000, 50_000),
    # BASELINE configs[0] as specified: one ms-simulated 10k-site block, n=50, a 20 Mb segment,
    # the default 100 kb grid (200 grid points), no permutations
    ("C1", 1, 50, 10_000, 20_000_000, 100_000),
])
def test_ms_input_matches_oracle_on_converted_file(built, tmp, name, blocks, hap, seg, length, grid):
    """The ms path (ms-input.c:93-151, semantics defined in DESIGN.md §6: the reference's is
    non-functional) against the oracle on the same sites written as an SNP file."""
    ms = tmp / "x.ms"
    synth.write_ms_file(str(ms), n_blocks=blocks, n_hap=hap, n_seg=seg, seed=41)
    scan = fscl_amd.load_ms_input(ms, length)
    s = scan.contents
    depth = s.sample_depths[0]
    assert s.n_chromosomes == blocks and s.n_snps > 0.95 * blocks * seg
    with open(tmp / "x.snp", "w") as f:  # the same sites as an SNP file
        for i in range(s.n_snps):
            p = s.snps[i]
            f.write(f"{s.chr_limits[p.chr].name.decode()} {p.pos} {p.obs_freq} {depth} {p.folded}\n")
    r = subprocess.run([str(CLI), "-m", str(ms), f"--ms-segment-length={length}", "-o", str(tmp / "g.txt"),
                        "-G", str(grid)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    run_oracle(tmp / "x.snp", tmp / "o.txt", [f"--coarse-grid-spacing={grid}"])
    out = (tmp / "g.txt").read_text()
    assert out == (tmp / "o.txt").read_text()
    if name == "C1":
        assert len(out.splitlines()) == 200


def test_ms_block_loop_matches_whole_file(built, tmp):
    """fscl.c's ms loop (fscl.c:281-313) through the C-ABI: tables from ms_background's
    spectrum, then compute_snp_null_model / scan_chromosome / scan_output per ms_next_block
    scan_t.  The blocks' outputs, concatenated, are the whole-file scan's output, which
    test_ms_input_matches_oracle_on_converted_file pins to the oracle."""
    ms = tmp / "x.ms"
    synth.write_ms_file(str(ms), n_blocks=3, n_hap=20, n_seg=500, seed=43)
    r = subprocess.run([str(CLI), "-m", str(ms), "--ms-segment-length=2000000", "-o", str(tmp / "g.txt"),
                        "-G", "50000"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    L = fscl_amd.get_lib()
    bg = L.ms_background(str(ms).encode(), 2_000_000, 0, 0, 0)
    fsp = fscl_amd.background_fsp(bg)
    tab = fscl_amd.compute_sweep_model_tables(bg, fsp)
    out = []
    for b, s in enumerate(fscl_amd.ms_blocks(ms, 2_000_000)):
        assert s.contents.n_snps > 0
        fscl_amd.compute_snp_null_model(s, fsp)
        fscl_amd.scan_chromosome(s, tab, large_grid_sp=50000)
        L.scan_output(str(tmp / f"b{b}.txt").encode(), s, 0, 0, None)
        out.append((tmp / f"b{b}.txt").read_text())
    assert len(out) == 3
    assert "".join(out) == (tmp / "g.txt").read_text()


def test_search_maxalpha_dropin(built):
    """search_maxalpha() on caller-initialised points (the reference's own scan loop calls it per
    point, scan-chromosome.c:126-135) equals the golden points, every one of them.  Its tables
    and sites stay resident between calls, and each call spreads its point over up to 8
    workgroups: a call costs one alpha search's latency on the GPU (about 85 us), not a
    re-upload; bounded here at 1 ms per call.  The per-point loop stays slower than one
    scan_chromosome (2.4x on the box), which runs every cell's bisection at once."""
    import ctypes as C
    import time
    case = "g2_p30"
    c = manifest()["cases"][case]
    scan = fscl_amd.load_snp_input(GOLD / c["input"])
    fsp = fscl_amd.background_fsp(scan)
    tab = fscl_amd.compute_sweep_model_tables(scan, fsp)
    fscl_amd.compute_snp_null_model(scan, fsp)
    rows = read_dump(GOLD / f"{case}.dump")
    L = fscl_amd.get_lib()

    def per_point():
        for row in rows:
            pt = fscl_amd.ScanPtT()
            pt.chr, pt.sweep_pos = row[0], row[1]
            pt.null_logl = row[5]
            pt.nearest_snp, pt.window_start, pt.window_end = row[6], row[7], row[8]
            pt.n_snps = row[8] - row[7] + 1
            pt.sm_logl, pt.lalpha = -1.7976931348623157e308, 4.0
            L.search_maxalpha(C.byref(pt), scan.contents.snps, tab)
            assert (pt.lalpha.hex(), pt.sm_logl.hex(), pt.clr.hex()) == (row[3].hex(), row[4].hex(), row[2].hex())

    per_point()  # first call: tables and sites go up once
    fscl_amd.scan_chromosome(scan, tab)
    t0 = time.perf_counter()
    per_point()
    t_pts = time.perf_counter() - t0
    t0 = time.perf_counter()
    fscl_amd.scan_chromosome(scan, tab)
    t_scan = time.perf_counter() - t0
    print(f"search_maxalpha x {len(rows)}: {t_pts * 1e3:.1f} ms; scan_chromosome: {t_scan * 1e3:.1f} ms")
    assert t_pts < 1e-3 * len(rows)


@pytest.mark.parametrize("exchange", ["callback", "shm", "shm_replicated", "shm_copy"])
def test_two_ranks_on_one_gpu_match_one_rank(built, tmp, exchange):
    """Parity mode with 2 processes (both on GPU 0): the exchange through a Python gloo
    callback, or the library's own shared-memory all-gather.  With the shared-memory exchange
    rank 0 builds every trial's permutation once into the node's shared pool and rank 1's device
    reads it (FSCL_AMD_PERM_LEADER=0, "shm_replicated": each rank builds its own;
    "shm_copy": the pool's rows copied into each rank's own pinned staging, the fallback)."""
    c = manifest()["cases"]["g1_p25"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29500 + os.getpid() % 1000), WORLD_SIZE="2",
               FSCL_AMD_DEVICE="0", HSA_ENABLE_IPC_MODE_LEGACY="0", FSCL_AMD_RANK_TIMEOUT="120")
    if exchange.startswith("shm"):
        env["FSCL_MR_SHM"] = f"/fscl_amd_mr_{os.getpid()}"
    if exchange == "shm_replicated":
        env["FSCL_AMD_PERM_LEADER"] = "0"
    if exchange == "shm_copy":  # the fallback when the pool cannot be page-locked: rows copied to own staging
        env["FSCL_AMD_POOL_COPY"] = "1"
    procs = []
    for r in range(2):
        e = dict(env, RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(ROOT / "tests" / "mr_worker.py"), str(GOLD / c["input"]),
                                       str(tmp / f"o{r}.txt"), *c["options"]], env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    errs = []
    for p in procs:
        out, err = p.communicate(timeout=600)
        assert p.returncode == 0, err
        errs.append(err)
    assert (tmp / "o0.txt").read_text() == (GOLD / "g1_p25.out").read_text()
    assert not (tmp / "o1.txt").exists()  # one writer
    if exchange == "shm":  # the leader's permutations: rank 1 builds none (no speculation threads),
        assert "spec_threads 0" in errs[1], errs[1][-400:]
        # and both ranks' devices read the shared pool directly (page-locked, no copy)
        assert not any("could not be page-locked" in e or "permutation pool" in e for e in errs), errs


def _windowed_genome(tmp, seed=93):
    """two 8 000-SNP chromosomes: with --eval-range=300 every window is a proper one (no chromosome's
    whole null sum is read), so the trials run in plan mode"""
    snp = tmp / "plan.snp"
    synth.write_snp_file(str(snp), synth.generate(n_chr=2, chr_len=8_000_000, snps_per_chr=8000, n=60, seed=seed,
                                                  sweeps_per_chr=2))
    return snp, ["--coarse-grid-spacing=100000", "--n-permute=60", "--eval-range=300"]


@pytest.mark.parametrize("variant", ["plan", "plan_no_prestage", "rows", "fallback"])
def test_block_plan_on_the_device_matches_oracle(built, tmp, monkeypatch, variant):
    """Each trial's block permutation as a plan the device applies (fsclg_slot_set_rows_plan,
    DESIGN.md §5.4): the default where no whole-chromosome null sum is read, with the likeliest
    next candidate applied to a spare slot ahead (pre-staging, swapped in when taken), or without
    (FSCL_AMD_PRESTAGE=0); FSCL_AMD_PLAN=0 the rows built on the host; FSCL_AMD_PLAN_ECAP=1 plan
    buffers too small for any plan, so every trial falls back to host rows.  60 permutations with
    pruning: bit-identical to the oracle."""
    snp, opts = _windowed_genome(tmp)
    if variant == "rows":
        monkeypatch.setenv("FSCL_AMD_PLAN", "0")
    if variant == "fallback":
        monkeypatch.setenv("FSCL_AMD_PLAN_ECAP", "1")
    if variant == "plan_no_prestage":
        monkeypatch.setenv("FSCL_AMD_PRESTAGE", "0")
    run_oracle(snp, tmp / "o.txt", opts, tmp / "o.dump")
    fscl_amd.reset_stats()
    scan = fscl_amd.run(snp, tmp / "g.txt", **_kw(opts))
    st = fscl_amd.get_stats()
    pts = fscl_amd.points(scan)
    assert (pts["permute_n"] < 61).any()  # points were pruned: prune draws between plans
    assert_rows_equal(points_rows(pts), read_dump(tmp / "o.dump"), f"plan {variant}")
    assert (tmp / "g.txt").read_text() == (tmp / "o.txt").read_text()
    assert st["plan_mode"] == (variant != "rows")
    assert (st["plan_fallback"] > 0) == (variant == "fallback")
    if variant == "plan":  # spare slots were prepared and some were taken
        assert st["prestage_hits"] > 0 and st["prestaged"] >= st["prestage_hits"], st
    if variant in ("plan_no_prestage", "rows"):
        assert st["prestaged"] == 0


@pytest.mark.parametrize("variant", ["pool", "pool_copy", "pool_fallback"])
def test_two_ranks_plan_mode_match_oracle(built, tmp, variant):
    """Plan mode with one process per GPU (two ranks on GPU 0, shared-memory exchange): the node
    leader publishes each trial's plan in the shared pool and both ranks' devices apply it
    ("pool_copy": the plan copied into each rank's own pinned staging; "pool_fallback": no plan fits,
    the leader publishes a marker and every rank builds the rows from its own rand() stream)."""
    snp, opts = _windowed_genome(tmp, seed=94)
    run_oracle(snp, tmp / "o.txt", opts, tmp / "o.dump")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29700 + os.getpid() % 1000), WORLD_SIZE="2",
               FSCL_AMD_DEVICE="0", HSA_ENABLE_IPC_MODE_LEGACY="0", FSCL_AMD_RANK_TIMEOUT="120",
               FSCL_MR_SHM=f"/fscl_amd_mrp_{os.getpid()}")
    if variant == "pool_copy":
        env["FSCL_AMD_POOL_COPY"] = "1"
    if variant == "pool_fallback":
        env["FSCL_AMD_PLAN_ECAP"] = "1"
    procs = [subprocess.Popen([sys.executable, str(ROOT / "tests" / "mr_worker.py"), str(snp), str(tmp / f"o{r}.txt"),
                               *opts], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for r in range(2)]
    errs = []
    for p in procs:
        _, err = p.communicate(timeout=600)
        assert p.returncode == 0, err
        errs.append(err)
    assert (tmp / "o0.txt").read_text() == (tmp / "o.txt").read_text()
    for e in errs:
        assert "plan_mode 1" in e and "perm_leader 1" in e, e[-400:]
        assert ("plan_fallback 0" in e) == (variant != "pool_fallback"), e[-400:]


def test_block_extension_table_follows_the_genome(built, tmp):
    """Two genomes of the same size one after the other in one process (the per-site extension
    table of the block permutation, perm.c, is keyed by the sites' content, not by where they
    happen to be allocated): both permutation tests bit-identical to the oracle."""
    for seed in (71, 72):
        snp = tmp / f"ext{seed}.snp"
        synth.write_snp_file(str(snp), synth.generate(n_chr=2, chr_len=8_000_000, snps_per_chr=8000, n=30, seed=seed,
                                                      sweeps_per_chr=2))
        opts = ["--coarse-grid-spacing=40000", "--n-permute=30"]
        run_oracle(snp, tmp / f"o{seed}.txt", opts, tmp / f"o{seed}.dump")
        scan = fscl_amd.run(snp, tmp / f"g{seed}.txt", **_kw(opts))
        assert_rows_equal(points_rows(fscl_amd.points(scan)), read_dump(tmp / f"o{seed}.dump"), f"genome {seed}")


def test_pipelined_trials_match_lockstep_and_oracle(built, tmp, monkeypatch):
    """Two trials in flight (scan_permute's default): the rand-stream critical points
    (permute_p >= 19) run ahead of the rest of their trial, the next trial's permutation is
    built and launched before the rest has finished.  Enough trials that points cross the
    critical threshold, draw rand() and are pruned: identical to the lockstep order
    (FSCL_AMD_LOCKSTEP=1) and to the oracle, bit for bit."""
    snp = tmp / "pipe.snp"
    synth.write_snp_file(str(snp), synth.generate(n_chr=2, chr_len=8_000_000, snps_per_chr=8000, n=30, seed=81,
                                                  sweeps_per_chr=2))
    opts = ["--coarse-grid-spacing=40000", "--n-permute=70"]
    run_oracle(snp, tmp / "o.txt", opts, tmp / "o.dump")
    fscl_amd.reset_stats()
    scan = fscl_amd.run(snp, tmp / "g.txt", **_kw(opts))
    st = fscl_amd.get_stats()
    pts = fscl_amd.points(scan)
    assert st["n_crit"] > 0 and (pts["permute_n"] < 71).any()  # critical batches ran, points were pruned
    assert_rows_equal(points_rows(pts), read_dump(tmp / "o.dump"), "pipelined")
    assert (tmp / "g.txt").read_text() == (tmp / "o.txt").read_text()
    monkeypatch.setenv("FSCL_AMD_LOCKSTEP", "1")
    scan = fscl_amd.run(snp, tmp / "l.txt", **_kw(opts))
    assert (tmp / "l.txt").read_text() == (tmp / "o.txt").read_text()
    monkeypatch.delenv("FSCL_AMD_LOCKSTEP")
    # other pipeline shapes: more row slots than the blocking margin (a bulk batch waited only
    # when its slot comes round, S trials later; a point that may draw first drains them), bulk
    # batches split over several workgroups per cell, and both with a margin of 2
    for env in ({"FSCL_AMD_SLOTS": "8"}, {"FSCL_AMD_BULK_SPLIT": "4"}, {"FSCL_AMD_BULK_SPLIT": "1"},
                {"FSCL_AMD_DEPTH": "2", "FSCL_AMD_SLOTS": "8", "FSCL_AMD_BULK_SPLIT": "8"}):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        scan = fscl_amd.run(snp, tmp / "s.txt", **_kw(opts))
        assert_rows_equal(points_rows(fscl_amd.points(scan)), read_dump(tmp / "o.dump"), f"pipelined {env}")
        assert (tmp / "s.txt").read_text() == (tmp / "o.txt").read_text(), env
        for k in env:
            monkeypatch.delenv(k)


def test_c2_scale_scan_and_short_permutation(built, tmp):
    """BASELINE config 2 (100k SNPs, n=100, 200 Mb) at full size: the whole
    initial scan and 3 permutation trials, bit-exact against the oracle."""
    snp = tmp / "c2.snp"
    synth.write_config(str(snp), "C2", seed=1)
    opts = ["--n-permute=2"]
    run_oracle(snp, tmp / "o.txt", opts, tmp / "o.dump")
    scan = fscl_amd.run(snp, tmp / "g.txt", **_kw(opts))
    pts = fscl_amd.points(scan)
    assert len(pts) == 2000
    assert_rows_equal(points_rows(pts), read_dump(tmp / "o.dump"), "C2")
    assert (tmp / "g.txt").read_text() == (tmp / "o.txt").read_text()


@pytest.mark.parametrize("name,gen,opts", [
    # BASELINE config 3 at full size: ascertainment K=2 of M=20 (on ascertained sites), 30 % folded
    ("C3", dict(n_chr=1, chr_len=200_000_000, snps_per_chr=100_000, n=100, folded=0.3, seed=3, sweeps_per_chr=2,
                asc_depth=20, asc_min_freq=2),
     ["--asc-depth=20", "--asc-minimum-freq=2", "--n-permute=2"]),
    # one chromosome of BASELINE config 5 (227k SNPs, n=400): every point's window is a
    # proper 2*81920+1-SNP window of the chromosome (per-window null sums on the device)
    ("C5_chr", dict(n_chr=1, chr_len=227_272_727, snps_per_chr=227_273, n=400, seed=5, sweeps_per_chr=2),
     ["--n-permute=1"]),
    # BASELINE config 4's genome shape at a quarter of the chromosomes (n=200, 45 Mb each)
    ("C4_part", dict(n_chr=6, chr_len=45_454_545, snps_per_chr=45_455, n=200, seed=4, sweeps_per_chr=2),
     ["--n-permute=2"]),
])
def test_full_size_configs_match_oracle(built, tmp, name, gen, opts):
    """Full-size BASELINE workloads beside C2: initial scan plus a short permutation test,
    bit-exact against the oracle (positions, windows, lalpha, sm_logl, CLR, counts)."""
    snp = tmp / f"{name}.snp"
    synth.write_snp_file(str(snp), synth.generate(**gen))
    run_oracle(snp, tmp / "o.txt", opts, tmp / "o.dump")
    fscl_amd.reset_stats()
    scan = fscl_amd.run(snp, tmp / "g.txt", **_kw(opts))
    assert_rows_equal(points_rows(fscl_amd.points(scan)), read_dump(tmp / "o.dump"), name)
    assert (tmp / "g.txt").read_text() == (tmp / "o.txt").read_text()
    if name == "C5_chr":
        assert fscl_amd.get_stats()["window_ms"] > 0


@pytest.mark.parametrize("mode,er", [("0", 300), ("1", 300), ("2", 300), ("2", 3000)])
def test_window_sum_kernels_match_oracle(built, tmp, monkeypatch, mode, er):
    """The window null sums (scan-chromosome.c:92-94) by each kernel for every trial:
    FSCLG_WINDOW_CHUNK=0 the sequential chains for every window start, 1 those for the dense
    trials and the exact chunked sums for the pruned tail's few windows, 2 (the
    default) the chunked sums for every window start.  Windows of 2*300+1 sites (a few chunks
    each: mostly the general step) and 2*3000+1 (~94 chunks: wave-uniform groups) on 2
    chromosomes, with permutations: bit-identical to the oracle."""
    monkeypatch.setenv("FSCLG_WINDOW_CHUNK", mode)
    snp = tmp / "win.snp"
    synth.write_snp_file(str(snp), synth.generate(n_chr=2, chr_len=8_000_000, snps_per_chr=8000, n=60, seed=93,
                                                  sweeps_per_chr=1))
    opts = ["--coarse-grid-spacing=100000", "--n-permute=25", f"--eval-range={er}"]
    run_oracle(snp, tmp / "o.txt", opts, tmp / "o.dump")
    kw = _kw([o for o in opts if not o.startswith("--eval-range=")])
    kw["eval_range"] = er
    fscl_amd.reset_stats()
    scan = fscl_amd.run(snp, tmp / "g.txt", **kw)
    assert_rows_equal(points_rows(fscl_amd.points(scan)), read_dump(tmp / "o.dump"), f"windows mode {mode} er {er}")
    assert fscl_amd.get_stats()["window_ms"] > 0


def test_mixed_window_and_whole_chromosome_sums_match_oracle(built, tmp):
    """One chromosome longer than the window (8000 SNPs, 2*300+1-site windows: device window
    sums) and one shorter (400 SNPs: the window is the whole chromosome, whose null sum the host
    computes per trial -- only for such chromosomes, scan-chromosome.c:75-94), with
    permutations: bit-identical to the oracle."""
    snp = tmp / "mixed.snp"
    chroms = synth.generate(n_chr=1, chr_len=8_000_000, snps_per_chr=8000, n=60, seed=95, sweeps_per_chr=1,
                            chr_names=["chrA"])
    chroms += synth.generate(n_chr=1, chr_len=400_000, snps_per_chr=400, n=60, seed=96, sweeps_per_chr=1,
                             chr_names=["chrB"])
    synth.write_snp_file(str(snp), chroms)
    opts = ["--coarse-grid-spacing=100000", "--n-permute=25", "--eval-range=300"]
    run_oracle(snp, tmp / "o.txt", opts, tmp / "o.dump")
    kw = _kw([o for o in opts if not o.startswith("--eval-range=")])
    kw["eval_range"] = 300
    scan = fscl_amd.run(snp, tmp / "g.txt", **kw)
    assert_rows_equal(points_rows(fscl_amd.points(scan)), read_dump(tmp / "o.dump"), "mixed windows")
    assert (tmp / "g.txt").read_text() == (tmp / "o.txt").read_text()


def _fullsize():
    import json
    return json.loads((GOLD / "fullsize.json").read_text())


@pytest.mark.parametrize("name", sorted(_fullsize()))
def test_full_genomes_match_oracle_fixture(built, tmp, name):
    """Full-size BASELINE genomes whose oracle run is too slow for the box
    (tests/golden/make_fullsize.py ran it here and stored digests):
      C4_full_p2  configs[3]'s whole 22-chromosome 1.0M-SNP genome, n=200, 3 trials;
      C5_full     configs[4]'s whole 5.0M-SNP genome, n=400, initial scan;
      C5_chr_p200 one C5 chromosome at 200 permutations: the early-prune regime
                  (points cross permute_p >= 20 and draw, scan-chromosome.c:488-498).
    Bit-exact: SHA-256 of every field of every point (floats as hex) and of the output."""
    sys.path.insert(0, str(GOLD))
    from make_fullsize import canonical_dump, canonical_row, sha256_file
    fx = _fullsize()[name]
    snp = tmp / f"{name}.snp"
    synth.write_snp_file(str(snp), synth.generate(**fx["gen"]))
    assert sha256_file(snp) == fx["input_sha256"], "synthetic input differs from the fixture's"
    fscl_amd.reset_stats()
    scan = fscl_amd.run(snp, tmp / "g.txt", **_kw(fx["options"]))
    rows = points_rows(fscl_amd.points(scan))
    assert len(rows) == fx["n_points"]
    assert sum(r[10] for r in rows) == fx["sum_permute_n"]
    if canonical_dump(rows) != fx["dump_sha256"]:
        k = fx["sample_every"]
        for i, want in enumerate(fx["sample"]):
            assert canonical_row(rows[i * k]) == want, f"{name}: point {i * k}"
        pytest.fail(f"{name}: dump digest differs (the sampled rows agree)")
    assert sha256_file(tmp / "g.txt") == fx["out_sha256"]
    if name.startswith("C5"):
        assert fscl_amd.get_stats()["window_ms"] > 0
    if name == "C3_bench_p100":  # a real workload: ascertained sites give CLRs, points outlive trial 20
        clr = np.array([r[2] for r in rows])
        assert (clr != 0.0).mean() >= 0.95, (clr != 0.0).mean()
        assert max(r[10] for r in rows) > 21


@pytest.fixture
def two_contexts():
    """This process drives GPU 0 through two device contexts (fscl_amd_set_devices)."""
    fscl_amd.set_devices([0, 0])
    yield
    fscl_amd.set_device(0)


@pytest.mark.parametrize("name,gen,opts", [
    ("multi_chr", dict(n_chr=3, chr_len=6_000_000, snps_per_chr=6000, n=30, seed=91, sweeps_per_chr=1),
     ["--coarse-grid-spacing=40000", "--n-permute=40"]),
    ("windowed", dict(n_chr=2, chr_len=4_000_000, snps_per_chr=4000, n=30, seed=92, sweeps_per_chr=1),
     ["--coarse-grid-spacing=40000", "--n-permute=6", "--eval-range=300"]),
])
def test_two_devices_in_one_process_match_oracle(built, tmp, two_contexts, name, gen, opts):
    """Single-process multi-GPU (the CLI's --n-gpus): every batch split into two cost-balanced
    shares on two contexts, one host permutation and pruning: bit-identical to the oracle."""
    snp = tmp / f"{name}.snp"
    synth.write_snp_file(str(snp), synth.generate(**gen))
    er = [o for o in opts if o.startswith("--eval-range=")]
    kw = _kw([o for o in opts if not o.startswith("--eval-range=")])
    if er:
        kw["eval_range"] = int(er[0].split("=")[1])
    run_oracle(snp, tmp / "o.txt", opts, tmp / "o.dump")
    fscl_amd.reset_stats()
    scan = fscl_amd.run(snp, tmp / "g.txt", **kw)
    assert fscl_amd.get_lib().fscl_amd_n_devices() == 2
    assert_rows_equal(points_rows(fscl_amd.points(scan)), read_dump(tmp / "o.dump"), name)
    assert (tmp / "g.txt").read_text() == (tmp / "o.txt").read_text()
    assert fscl_amd.get_stats()["n_devices"] == 2


def test_cli_one_process_per_gpu(built, tmp):
    """The CLI under a one-process-per-GPU launcher (RANK / WORLD_SIZE in the environment):
    two ranks on GPU 0 exchange through shared memory; rank 0 writes the golden output."""
    c = manifest()["cases"]["g1_p25"]
    env = dict(os.environ, WORLD_SIZE="2", FSCL_AMD_DEVICE="0", FSCL_AMD_SHM_NAME=f"cli_{os.getpid()}",
               FSCL_AMD_RANK_TIMEOUT="120")
    procs = [subprocess.Popen([str(CLI), "-f", str(GOLD / c["input"]), "-o", str(tmp / "o.txt"), *c["options"]],
                              env=dict(env, RANK=str(r), LOCAL_RANK="0"), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    for p in procs:
        out, err = p.communicate(timeout=600)
        assert p.returncode == 0, err
    assert (tmp / "o.txt").read_text() == (GOLD / "g1_p25.out").read_text()


def test_cli_ranks_meet_without_a_segment_name(built, tmp):
    """No FSCL_AMD_SHM_NAME, each rank started through its own wrapper shell (different parent
    processes, as with a per-rank script under torchrun --no-python or srun): the default segment
    name comes from the launcher's variables (MASTER_ADDR / MASTER_PORT here), so the ranks
    still meet, and rank 0 writes the golden output."""
    import shlex
    c = manifest()["cases"]["g1_p25"]
    env = {k: v for k, v in os.environ.items() if k not in ("FSCL_AMD_SHM_NAME", "TORCHELASTIC_RUN_ID")}
    env.update(WORLD_SIZE="2", FSCL_AMD_DEVICE="0", FSCL_AMD_RANK_TIMEOUT="120", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(31000 + os.getpid() % 2000))
    cmd = " ".join(shlex.quote(str(a)) for a in [CLI, "-f", GOLD / c["input"], "-o", tmp / "o.txt", *c["options"]])
    procs = [subprocess.Popen(["bash", "-c", f"{cmd}; exit $?"], env=dict(env, RANK=str(r), LOCAL_RANK="0"),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    for p in procs:
        out, err = p.communicate(timeout=600)
        assert p.returncode == 0, err
    assert (tmp / "o.txt").read_text() == (GOLD / "g1_p25.out").read_text()


def test_cli_n_gpus(built, tmp):
    """fscl --n-gpus=1 and the CLI's default (every visible GPU) reproduce the golden output."""
    c = manifest()["cases"]["g1_p25"]
    env = {k: v for k, v in os.environ.items() if k != "FSCL_AMD_DEVICE"}
    r = subprocess.run([str(CLI), "-f", str(GOLD / c["input"]), "-o", str(tmp / "o.txt"), "--n-gpus=1",
                        *c["options"]], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    assert (tmp / "o.txt").read_text() == (GOLD / "g1_p25.out").read_text()
    r = subprocess.run([str(CLI), "-f", str(GOLD / c["input"]), "-o", str(tmp / "a.txt"), *c["options"]],
                       capture_output=True, text=True, timeout=600, env=env)  # default: every visible GPU
    assert r.returncode == 0, r.stderr
    assert (tmp / "a.txt").read_text() == (GOLD / "g1_p25.out").read_text()


def test_back_to_back_scan_permute_continue_the_stream(built, tmp):
    """The rand() stream is seeded once per process (fscl.c:135) and continues across
    scan_permute calls: two calls in a row equal the oracle driven the same way (counts
    accumulate, scan-chromosome.c:488-498)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    from oracle import OracleScan
    snp = tmp / "b2b.snp"
    synth.write_snp_file(str(snp), synth.generate(n_chr=2, chr_len=5_000_000, snps_per_chr=5000, n=30, seed=95,
                                                  sweeps_per_chr=1))
    orc = OracleScan(snp, threads=usable_cpus(), large_grid_sp=50000)
    orc.reseed()
    orc.scan()
    orc.permute(8)
    orc.permute(12)
    want = orc.points()
    fscl_amd.init_log_table()
    fscl_amd.srand()
    scan = fscl_amd.load_snp_input(snp)
    fsp = fscl_amd.background_fsp(scan)
    tab = fscl_amd.compute_sweep_model_tables(scan, fsp)
    fscl_amd.compute_snp_null_model(scan, fsp)
    fscl_amd.scan_chromosome(scan, tab, large_grid_sp=50000)
    fscl_amd.scan_permute(scan, tab, 8, large_grid_sp=50000)
    fscl_amd.scan_permute(scan, tab, 12, large_grid_sp=50000)
    got = fscl_amd.points(scan)
    assert [tuple(r) for r in got[["chr", "sweep_pos", "permute_p", "permute_n", "permute_finished"]].tolist()] == \
        [(p[0], p[1], p[10], p[9], p[11]) for p in want]
    assert [c.hex() for c in got["clr"]] == [p[2].hex() for p in want]


def test_sigint_dumps_table_and_null_distribution(built, tmp):
    """SIGINT during the permutation test (scan-chromosome.c:557-569): the CLI writes the
    current table and <output>-nulldist (:753-796) and keeps going; an interrupt within the
    window after the start of the permutations or after a dump aborts (exit 255).  The window
    is the reference's 10 s, shortened here to 300 ms (FSCL_AMD_SIGINT_WINDOW_MS) so that the
    dump lands after some hundreds of trials.  The dump shows every trial up to the one it
    follows, so it equals the oracle's final table and null distribution for that many
    permutations."""
    import re
    import signal
    import threading
    import time
    snp = tmp / "sig.snp"
    # strong planted sweeps: some points are never pruned, so the run outlasts the test
    synth.write_snp_file(str(snp), synth.generate(n_chr=2, chr_len=6_000_000, snps_per_chr=6000, n=30, seed=97,
                                                  sweeps_per_chr=2))
    out = tmp / "g.txt"
    env = {k: v for k, v in os.environ.items() if k != "FSCL_AMD_DEVICE"}
    env["FSCL_AMD_SIGINT_WINDOW_MS"] = "300"  # the dump takes a few ms
    proc = subprocess.Popen([str(CLI), "-f", str(snp), "-o", str(out), "--coarse-grid-spacing=60000",
                             "--n-permute=1000000", "--n-gpus=1"], stderr=subprocess.PIPE, env=env)
    seen = [-1]

    def reader():  # progress lines: "\rScanning snp block permutations... <trial> (...)"
        buf = b""
        while True:
            ch = proc.stderr.read(256)
            if not ch:
                return
            buf = (buf + ch)[-4096:]
            for m in re.finditer(rb"permutations\.\.\.\s+(\d+) \(", buf):
                seen[0] = max(seen[0], int(m.group(1)))

    th = threading.Thread(target=reader, daemon=True)
    th.start()
    try:
        t0 = time.time()
        while seen[0] < 0:
            assert proc.poll() is None, "the CLI ended before the permutations"
            assert time.time() - t0 < 300, "no permutation progress"
            time.sleep(0.005)
        t1 = time.time()
        while seen[0] < 60 or time.time() - t1 < 0.6:  # past the window after the start
            assert proc.poll() is None, "the CLI ended before the interrupt"
            time.sleep(0.005)
        at = seen[0]
        proc.send_signal(signal.SIGINT)
        t2 = time.time()
        nd = tmp / "g.txt-nulldist"
        n_pts = None
        while True:  # the dump ends with a complete null-distribution file; then the window restarts
            assert proc.poll() is None, f"the CLI ended after the first interrupt (trial {at}, seen {seen[0]})"
            assert time.time() - t2 < 60, "no dump"
            if nd.exists() and out.exists():
                if n_pts is None:
                    n_pts = len(out.read_text().splitlines()) or None
                txt = nd.read_text()
                if n_pts and txt.endswith("\n") and txt.count("\n") == n_pts + 1:
                    break
            time.sleep(0.0005)
        proc.send_signal(signal.SIGINT)
        t3 = time.time()
        rc = proc.wait(timeout=60)
        assert rc == 255, (f"exit {rc}: first interrupt at trial {at} ({t1 - t0:.2f} s to the first trial, "
                           f"{t2 - t1:.2f} s more), second {t3 - t2:.3f} s later at trial {seen[0]}")
    finally:
        if proc.poll() is None:
            proc.kill()
            proc.wait()
    th.join(timeout=10)
    rows = [line.split("\t") for line in out.read_text().splitlines()]
    n_trials = max(int(r[5]) for r in rows)  # unfinished points counted every trial 0..T
    assert n_trials > 60
    run_oracle(snp, tmp / "o.txt", ["--coarse-grid-spacing=60000", f"--n-permute={n_trials - 1}", "--nulldist"])
    assert out.read_text() == (tmp / "o.txt").read_text()
    assert (tmp / "g.txt-nulldist").read_text() == (tmp / "o.txt-nulldist").read_text()


def test_sigint_with_two_ranks_dumps_collectively(built, tmp):
    """One process per GPU (both ranks on GPU 0 here), SIGINT delivered to rank 1 alone -- the
    rank that writes nothing.  The dump decision is collective (each rank's flag rides on one
    exchange per trial, every rank acts on the OR: ADVICE r02), so both ranks drain their bulk
    batches at the same trial, keep exchanging the same batches, and rank 0 writes the table and
    <output>-nulldist; they equal the oracle's for that many permutations.  A second interrupt
    to both ranks within the window ends both (exit 255)."""
    import re
    import signal
    import threading
    import time
    snp = tmp / "sig2.snp"
    synth.write_snp_file(str(snp), synth.generate(n_chr=2, chr_len=6_000_000, snps_per_chr=6000, n=30, seed=97,
                                                  sweeps_per_chr=2))
    out = tmp / "g.txt"
    env = dict(os.environ, FSCL_AMD_SIGINT_WINDOW_MS="300", WORLD_SIZE="2", FSCL_AMD_DEVICE="0",
               FSCL_AMD_SHM_NAME=f"sig2_{os.getpid()}", FSCL_AMD_RANK_TIMEOUT="60", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([str(CLI), "-f", str(snp), "-o", str(out), "--coarse-grid-spacing=60000",
                               "--n-permute=1000000"], stderr=subprocess.PIPE, env=dict(env, RANK=str(r)))
             for r in range(2)]
    seen = [-1, -1]

    def reader(r):
        buf = b""
        while True:
            ch = procs[r].stderr.read(256)
            if not ch:
                return
            buf = (buf + ch)[-4096:]
            for m in re.finditer(rb"permutations\.\.\.\s+(\d+) \(", buf):
                seen[r] = max(seen[r], int(m.group(1)))

    ths = [threading.Thread(target=reader, args=(r,), daemon=True) for r in range(2)]
    for th in ths:
        th.start()
    try:
        t0 = time.time()
        while min(seen) < 0:
            assert all(p.poll() is None for p in procs), "a rank ended before the permutations"
            assert time.time() - t0 < 300, "no permutation progress"
            time.sleep(0.005)
        t1 = time.time()
        while min(seen) < 60 or time.time() - t1 < 0.6:
            assert all(p.poll() is None for p in procs), "a rank ended before the interrupt"
            time.sleep(0.005)
        at = seen[1]
        procs[1].send_signal(signal.SIGINT)  # the non-writing rank only
        t2 = time.time()
        nd = tmp / "g.txt-nulldist"
        n_pts = None
        while True:
            assert all(p.poll() is None for p in procs), f"a rank ended after the interrupt (trial {at})"
            assert time.time() - t2 < 60, "no dump from rank 0"
            if nd.exists() and out.exists():
                if n_pts is None:
                    n_pts = len(out.read_text().splitlines()) or None
                txt = nd.read_text()
                if n_pts and txt.endswith("\n") and txt.count("\n") == n_pts + 1:
                    break
            time.sleep(0.0005)
        for p in procs:
            p.send_signal(signal.SIGINT)
        rcs = [p.wait(timeout=60) for p in procs]
        assert rcs == [255, 255], rcs
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for th in ths:
        th.join(timeout=10)
    rows = [line.split("\t") for line in out.read_text().splitlines()]
    n_trials = max(int(r[5]) for r in rows)
    assert n_trials > 60
    run_oracle(snp, tmp / "o.txt", ["--coarse-grid-spacing=60000", f"--n-permute={n_trials - 1}", "--nulldist"])
    assert out.read_text() == (tmp / "o.txt").read_text()
    assert (tmp / "g.txt-nulldist").read_text() == (tmp / "o.txt-nulldist").read_text()


def test_split_timeout_reruns_unsplit(built, tmp, monkeypatch):
    """A split launch whose members were not co-resident (PF_SPLIT_TIMEOUT) is re-run with one
    workgroup per cell instead of failing the job; forced here for the first 3
    split launches (FSCLG_FORCE_SPLIT_RETRY): same results as the oracle, retries counted."""
    c = manifest()["cases"]["g1_p25"]
    monkeypatch.setenv("FSCLG_FORCE_SPLIT_RETRY", "3")
    fscl_amd.reset_stats()
    fscl_amd.run(GOLD / c["input"], tmp / "g.txt", **_kw(c["options"]))
    assert fscl_amd.get_stats()["n_split_retry"] == 3
    assert (tmp / "g.txt").read_text() == (GOLD / "g1_p25.out").read_text()


def test_split_retry_of_a_bulk_batch(built, tmp, monkeypatch):
    """The bulk batches (batch >= 2) are split too when they are few cells (FSCL_AMD_BULK_SPLIT,
    DESIGN.md §5.2), and they may run beside a blocking launch that holds the rest of the device
    (ADVICE r05): their retry path, forced for the first 3 split bulk launches only (bulk batches kept
    apart, FSCL_AMD_NO_MERGE)
    (FSCLG_FORCE_SPLIT_RETRY_MINBATCH=2), gives the golden output."""
    c = manifest()["cases"]["g1_p25"]
    monkeypatch.setenv("FSCL_AMD_BULK_SPLIT", "4")
    monkeypatch.setenv("FSCL_AMD_NO_MERGE", "1")  # small bulk batches would otherwise join the blocking one
    monkeypatch.setenv("FSCLG_FORCE_SPLIT_RETRY", "3")
    monkeypatch.setenv("FSCLG_FORCE_SPLIT_RETRY_MINBATCH", "2")
    fscl_amd.reset_stats()
    fscl_amd.run(GOLD / c["input"], tmp / "g.txt", **_kw(c["options"]))
    assert fscl_amd.get_stats()["n_split_retry"] == 3
    assert (tmp / "g.txt").read_text() == (GOLD / "g1_p25.out").read_text()


def test_split_member_late_past_the_wait_is_flagged(built, tmp, monkeypatch):
    """A real timeout, not a forced one: member 0 of cell 0 of every split launch
    sleeps 30 ms before its first arrival (FSCLG_TEST_SPLIT_DELAY_US) while the others wait only
    3 ms (FSCLG_SPLIT_WAIT_US).  The others time out, go on with partial sums and publish the
    timeout in the cell's arrival word; member 0, whose own wait is then satisfied at once by
    their arrivals, must still flag its point, so the launch is re-run unsplit: the output is
    the golden one and the re-runs are counted."""
    c = manifest()["cases"]["g1_p25"]
    monkeypatch.setenv("FSCLG_TEST_SPLIT_DELAY_US", "30000")
    monkeypatch.setenv("FSCLG_SPLIT_WAIT_US", "3000")
    fscl_amd.reset_stats()
    fscl_amd.run(GOLD / c["input"], tmp / "g.txt", **_kw(c["options"]))
    assert fscl_amd.get_stats()["n_split_retry"] >= 1
    assert (tmp / "g.txt").read_text() == (GOLD / "g1_p25.out").read_text()


def test_dropin_search_maxalpha_from_threads(built):
    """The reference calls search_maxalpha from its --n-threads workers (scan-chromosome.c:258,
    514, 531): concurrent calls into the drop-in (serialised inside) each get their
    own point's golden result, with the golden case's points and a second genome's interleaved
    (the drop-in's resident window and tables change between calls)."""
    import ctypes as C
    from concurrent.futures import ThreadPoolExecutor
    L = fscl_amd.get_lib()
    jobs = []
    for case in ("g2_p30", "g1_p25"):
        c = manifest()["cases"][case]
        scan = fscl_amd.load_snp_input(GOLD / c["input"])
        fsp = fscl_amd.background_fsp(scan)
        tab = fscl_amd.compute_sweep_model_tables(scan, fsp)
        fscl_amd.compute_snp_null_model(scan, fsp)
        for row in read_dump(GOLD / f"{case}.dump")[:40]:
            jobs.append((scan, tab, row))
    keep = [j[:2] for j in jobs]  # the scans and tables stay alive while the threads run

    def call(job):
        scan, tab, row = job
        pt = fscl_amd.ScanPtT()
        pt.chr, pt.sweep_pos = row[0], row[1]
        pt.null_logl = row[5]
        pt.nearest_snp, pt.window_start, pt.window_end = row[6], row[7], row[8]
        pt.n_snps = row[8] - row[7] + 1
        pt.sm_logl, pt.lalpha = -1.7976931348623157e308, 4.0
        L.search_maxalpha(C.byref(pt), scan.contents.snps, tab)
        return (pt.lalpha.hex(), pt.sm_logl.hex(), pt.clr.hex()), (row[3].hex(), row[4].hex(), row[2].hex())

    order = [jobs[k // 2] if k % 2 == 0 else jobs[len(jobs) // 2 + k // 2] for k in range(len(jobs))]
    with ThreadPoolExecutor(8) as ex:
        for got, want in ex.map(call, order * 2):
            assert got == want
    assert keep


# ---------------------------------------------------------------- throughput mode
TP_SEED = 0x5EED1234


@pytest.fixture(scope="module")
def tp_case(tmp_path_factory):
    """Enough trials that points reach permute_p >= 20 and are pruned in throughput mode; the
    oracle's serial restatement of the mode (--throughput-seed) is the reference result."""
    d = tmp_path_factory.mktemp("tp")
    snp = d / "tp.snp"
    synth.write_snp_file(str(snp), synth.generate(n_chr=3, chr_len=5_000_000, snps_per_chr=5000, n=30, seed=97,
                                                  sweeps_per_chr=1))
    opts = ["--coarse-grid-spacing=40000", "--n-permute=60"]
    run_oracle(snp, d / "o.txt", [*opts, f"--throughput-seed={TP_SEED}"], d / "o.dump")
    return snp, opts, read_dump(d / "o.dump"), (d / "o.txt").read_text()


@pytest.mark.parametrize("depth", ["8", "3", "1"])
def test_throughput_mode_matches_oracle(built, tmp, tp_case, monkeypatch, depth):
    """Throughput mode (include/fscl_amd.h fscl_amd_set_permute_mode):
    counter-based random numbers, trials independent.  Its results are a function of the seed
    alone -- the same with 8, 3 or 1 rounds in flight -- and equal the oracle's restatement of
    the mode bit for bit, with pruning exercised."""
    snp, opts, want, want_out = tp_case
    monkeypatch.setenv("FSCL_AMD_DEPTH", depth)
    fscl_amd.reset_stats()
    scan = fscl_amd.run(snp, tmp / "g.txt", permute_mode="throughput", permute_seed=TP_SEED, **_kw(opts))
    pts = fscl_amd.points(scan)
    assert (pts["permute_n"] < 61).any() and (pts["permute_n"] == 61).any()  # pruned and surviving points
    assert_rows_equal(points_rows(pts), want, f"throughput depth {depth}")
    assert (tmp / "g.txt").read_text() == want_out
    fscl_amd.set_permute_mode("parity")


def test_throughput_mode_two_devices_and_cli(built, tmp, tp_case):
    """Throughput mode shards whole trials over devices (two contexts on GPU 0 here) and over
    ranks; the CLI's --permute-mode=throughput --permute-seed gives the same output."""
    snp, opts, want, want_out = tp_case
    fscl_amd.set_devices([0, 0])
    try:
        scan = fscl_amd.run(snp, tmp / "g.txt", permute_mode="throughput", permute_seed=TP_SEED, **_kw(opts))
        assert fscl_amd.get_lib().fscl_amd_n_devices() == 2
        assert_rows_equal(points_rows(fscl_amd.points(scan)), want, "throughput, two devices")
    finally:
        fscl_amd.set_device(0)
        fscl_amd.set_permute_mode("parity")
    r = subprocess.run([str(CLI), "-f", str(snp), "-o", str(tmp / "c.txt"), "--permute-mode=throughput",
                        f"--permute-seed={TP_SEED}", *opts], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert (tmp / "c.txt").read_text() == want_out


def test_throughput_mode_windowed_matches_oracle(built, tmp):
    """Throughput mode on chromosomes longer than the window (eval_range 300): every trial's
    window null sums come from its own slot (fsclg_slot_windows per round and device)."""
    snp = tmp / "tpw.snp"
    synth.write_snp_file(str(snp), synth.generate(n_chr=2, chr_len=4_000_000, snps_per_chr=4000, n=30, seed=98,
                                                  sweeps_per_chr=1))
    opts = ["--coarse-grid-spacing=40000", "--n-permute=45"]
    run_oracle(snp, tmp / "o.txt", [*opts, "--eval-range=300", f"--throughput-seed={TP_SEED}"], tmp / "o.dump")
    fscl_amd.reset_stats()
    try:
        scan = fscl_amd.run(snp, tmp / "g.txt", permute_mode="throughput", permute_seed=TP_SEED, eval_range=300,
                            **_kw(opts))
    finally:
        fscl_amd.set_permute_mode("parity")
    assert_rows_equal(points_rows(fscl_amd.points(scan)), read_dump(tmp / "o.dump"), "throughput windowed")
    assert (tmp / "g.txt").read_text() == (tmp / "o.txt").read_text()
    assert fscl_amd.get_stats()["window_ms"] > 0


def test_throughput_mode_two_ranks(built, tmp, tp_case):
    """Two processes on GPU 0, shared-memory exchange: each rank runs every other trial."""
    snp, opts, want, want_out = tp_case
    env = dict(os.environ, WORLD_SIZE="2", FSCL_AMD_DEVICE="0", HSA_ENABLE_IPC_MODE_LEGACY="0",
               FSCL_AMD_RANK_TIMEOUT="120", FSCL_MR_SHM=f"/fscl_amd_tp_{os.getpid()}",
               FSCL_AMD_PERMUTE=f"throughput:{TP_SEED}", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(29600 + os.getpid() % 1000))
    procs = [subprocess.Popen([sys.executable, str(ROOT / "tests" / "mr_worker.py"), str(snp), str(tmp / f"o{r}.txt"),
                               *opts], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for r in range(2)]
    for p in procs:
        out, err = p.communicate(timeout=600)
        assert p.returncode == 0, err
    assert (tmp / "o0.txt").read_text() == want_out


def test_bench_under_torchrun_is_the_drivers_scale_shape(built, tmp):
    """The driver's SCALE command, at two ranks: `python -m torch.distributed.run --nproc-per-node 2
    bench.py --gpus 2`, one process per rank.  Both ranks sit on GPU 0 here (FSCL_AMD_DEVICE=0) and
    torch's own collectives (the segment-name broadcast, the elapsed-time max) run on gloo
    (FSCL_BENCH_BACKEND); on the driver's 8-GPU node the same path inits nccl with device_id.  C2 at
    its full size: rc 0, exactly one JSON line (rank 0's), n_gpus 2, and the timed job identical to
    the oracle's digest of the whole C2 job."""
    import json
    env = dict(os.environ, FSCL_BENCH_BACKEND="gloo", FSCL_AMD_DEVICE="0", HSA_ENABLE_IPC_MODE_LEGACY="0",
               FSCL_AMD_RANK_TIMEOUT="300")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
           f"--master-port={29900 + os.getpid() % 1000}", str(ROOT / "bench.py"), "--gpus", "2", "--config", "C2",
           "--steps", "1", "--warmup", "0", "--workdir", str(tmp)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 1 and d["value"] > 0
    assert d["config"]["multi_gpu"].startswith("2 processes"), d["config"]
    p = d["parity"]
    assert p["scope"] == "full job" and "C2_bench_p100" in p["fixture"], p
    assert p["jobs_checked"] == 1 and p["jobs_identical"] == p["jobs_checked"], p
    assert d["north_star_ratio"]["n_gpus"] == 2 and d["north_star_ratio"]["value"] > 0
