"""Host side of the product (no GPU needed): input, background spectra,
asc-bias, spline tables, alpha grid, null model, partitioning, exports.
Bit-exact against the reference's own compiled code (golden digests)."""
from __future__ import annotations

import ctypes as C
import hashlib
import math
import re
import subprocess

import numpy as np
import pytest

from util import CLI, GOLD, ROOT, manifest
import fscl_amd
from fscl_amd import synth


def _opts(options):
    o = dict(asc_depth=0, asc_min=1, bg_only=0, inv=0)
    for a in options:
        if a.startswith("--asc-depth="):
            o["asc_depth"] = int(a.split("=")[1])
        elif a.startswith("--asc-minimum-freq="):
            o["asc_min"] = int(a.split("=")[1])
        elif a == "--ascbias-background-only":
            o["bg_only"] = 1
        elif a == "--include-invariant":
            o["inv"] = 1
    return o


def _tables(snp, options):
    o = _opts(options)
    s = fscl_amd.load_snp_input(snp, o["inv"], 5)
    fsp = fscl_amd.background_fsp(s, False, None, o["inv"])
    tab = fscl_amd.compute_sweep_model_tables(s, fsp, o["asc_depth"], o["asc_min"], o["bg_only"], o["inv"])
    return s, fsp, tab


@pytest.mark.parametrize("case", sorted(manifest()["tables"]))
def test_tables_bit_exact_vs_reference(built, case):
    t = manifest()["tables"][case]
    s, fsp, tab = _tables(GOLD / t["input"], t["options"])
    assert s.contents.n_depths == len(t["depths"])
    for d, want in enumerate(t["depths"]):
        n = want["n"]
        assert s.contents.sample_depths[d] == n
        got_fsp = [fsp[d][k].hex() for k in range(n + 1)]
        assert got_fsp == want["fsp"], f"depth {n}: background spectrum differs"
        tb = tab[d]
        blocks = []
        for r in range(n + 1 + n // 2 + 1):
            sp = tb.spline_func[r] if r <= n else tb.fspline_func[r - n - 1]
            m = sp.contents.n
            assert m == t["spline_pts"]
            blocks.append(np.ctypeslib.as_array(sp.contents.coef[0], shape=(4 * m,)).tobytes())
        for r, b in enumerate(blocks):
            assert hashlib.sha256(b).hexdigest() == want["row_sha256"][r], f"depth {n} row {r}"
        assert hashlib.sha256(b"".join(blocks)).hexdigest() == want["coef_sha256"]


def test_spline_interpolate_matches_formula(built):
    s, fsp, tab = _tables(GOLD / "g2.snp", [])
    sp = tab[0].spline_func[3]
    L = fscl_amd.get_lib()
    step = 24.0 / 201.0
    for x in np.linspace(-20, 4, 97):
        i = min(max(int((x - (-20.0)) / step), 0), 199)
        c = sp.contents.coef[i]
        want = x * (c[0] * x * x + c[1] * x + c[2]) + c[3]
        assert L.spline_interpolate(sp, float(x)).hex() == want.hex()


def test_alpha_grid_is_the_reference_loop(built):
    """sm-search.c:276-295 evaluated in Python (same IEEE double operations)."""
    L = fscl_amd.get_lib()
    coarse = (C.c_double * 16)()
    refine = (C.c_double * (17 * 16))()
    nref = (C.c_int32 * 17)()
    nc = L.fh_alpha_grid(coarse, 16, refine, nref)
    step = (4.0 - -20.0) / 10.0
    want, la = [], -20.0
    while la <= 4.0:
        want.append(la)
        la += step
    assert nc == len(want) == 11 and [coarse[i] for i in range(nc)] == want
    assert want[-1] == 4.0
    for c in range(nc + 1):
        best = want[c] if c < nc else 4.0
        le, re_ = max(best - step, -20.0), min(best + step, 4.0)
        s2 = (re_ - le) / 15.0
        r, la = [], le + s2
        while la < re_:
            r.append(la)
            la += s2
        assert [refine[c * 16 + k] for k in range(nref[c])] == r
        assert nref[c] in (14, 15)


def test_null_model_and_input(built):
    s, fsp, _ = _tables(GOLD / "g1.snp", [])
    fscl_amd.compute_snp_null_model(s, fsp)
    sc = s.contents
    # input: sorted by (chromosome index, position), chromosomes in first-appearance order
    rows = [ln.split() for ln in (GOLD / "g1.snp").read_text().splitlines()]
    names = list(dict.fromkeys(r[0] for r in rows))
    assert [sc.chr_limits[c].name.decode() for c in range(sc.n_chromosomes)] == names
    assert sc.n_snps == len(rows)
    prev = (-1, -1)
    for i in range(sc.n_snps):
        p = sc.snps[i]
        assert (p.chr, p.pos) >= prev
        prev = (p.chr, p.pos)
        n = sc.sample_depths[p.depth_p]
        if p.folded:
            assert p.obs_freq <= n - p.obs_freq
        f = fsp[p.depth_p]
        want = math.log(f[p.obs_freq] + f[n - p.obs_freq]) if p.folded and p.obs_freq != n - p.obs_freq \
            else math.log(f[p.obs_freq])
        assert p.null_logl.hex() == want.hex()
    for c in range(sc.n_chromosomes):
        lim = sc.chr_limits[c]
        assert sc.snps[lim.start_index].pos == lim.start_pos
        assert sc.snps[lim.start_index + lim.n_snps - 1].pos == lim.bp_length


def test_input_filters(built, tmp):
    f = tmp / "x.snp"
    f.write_text("# comment\nchromosome\n\nc1 100 3 10 0\nc1 50 0 10 0\nc1 60 10 10 0\nc1 70 2 4 0\n"
                 "c2 5 8 10 1\nbad line\nc1 40 7 10 1\n")
    s = fscl_amd.load_snp_input(f, False, 5).contents
    got = [(s.snps[i].chr, s.snps[i].pos, s.snps[i].obs_freq, s.snps[i].folded) for i in range(s.n_snps)]
    # invariant (0 / n) and depth < 5 dropped; folded counts become minor counts; sorted per chromosome
    assert got == [(0, 40, 3, 1), (0, 100, 3, 0), (1, 5, 2, 1)]
    s2 = fscl_amd.load_snp_input(f, True, 5).contents
    assert s2.n_snps == 5


def test_ms_reader_semantics(built, tmp):
    ms = tmp / "x.ms"
    synth.write_ms_file(str(ms), n_blocks=3, n_hap=12, n_seg=40, seed=5)
    s = fscl_amd.load_ms_input(ms, 1_000_000, folded=False).contents
    s_f = fscl_amd.load_ms_input(ms, 1_000_000, folded=True).contents
    # Python restatement of the defined semantics
    blocks, cur = [], None
    lines = ms.read_text().splitlines()
    i = 0
    while i < len(lines):
        if lines[i].startswith("//"):
            seg = int(lines[i + 1].split()[1])
            pos = [float(x) for x in lines[i + 2].split()[1:]]
            hap = lines[i + 3:i + 3 + 12]
            blocks.append((pos, hap))
            i += 3 + 12
        else:
            i += 1
    want = []
    for b, (pos, hap) in enumerate(blocks):
        for j, x in enumerate(pos):
            d = sum(h[j] == "1" for h in hap)
            if 0 < d < 12:
                want.append((b, int(x * 1_000_000), d))
    want.sort(key=lambda t: (t[0], t[1]))
    got = [(s.snps[k].chr, s.snps[k].pos, s.snps[k].obs_freq) for k in range(s.n_snps)]
    assert got == want
    assert [s.chr_limits[c].name.decode() for c in range(s.n_chromosomes)] == ["1", "2", "3"]
    assert all(s_f.snps[k].folded == 1 and s_f.snps[k].obs_freq == min(want[k][2], 12 - want[k][2])
               for k in range(s_f.n_snps))


def test_ms_block_interface(built, tmp):
    """ms_background / ms_openfile / ms_next_block (fscl.h:118-123) as fscl.c:281-313 drives
    them: the background is every block, then one single-chromosome scan_t per block (a block
    without polymorphic sites gives n_snps 0), then NULL."""
    ms = tmp / "x.ms"
    synth.write_ms_file(str(ms), n_blocks=3, n_hap=12, n_seg=40, seed=5)
    with open(ms, "a") as f:  # a fourth block whose sites are all monomorphic in the sample
        f.write("\n//\nsegsites: 2\npositions: 0.25 0.5\n" + "11\n" * 12)
    L = fscl_amd.get_lib()
    whole = fscl_amd.load_ms_input(ms, 1_000_000).contents
    bg = L.ms_background(str(ms).encode(), 1_000_000, 0, 0, 0).contents
    snps = lambda s: [(s.snps[k].chr, s.snps[k].pos, s.snps[k].obs_freq, s.snps[k].folded,
                       s.sample_depths[s.snps[k].depth_p]) for k in range(s.n_snps)]
    assert snps(bg) == snps(whole) and bg.n_chromosomes == whole.n_chromosomes
    blocks = list(fscl_amd.ms_blocks(ms, 1_000_000))
    assert len(blocks) == 4
    for b, sp in enumerate(blocks):
        s = sp.contents
        assert s.n_chromosomes == 1 and s.chr_limits[0].name.decode() == str(b + 1)
        want = [(0, *w[1:]) for w in snps(whole) if w[0] == b]
        assert snps(s) == want
        if want:
            cl = s.chr_limits[0]
            assert (cl.start_index, cl.n_snps, cl.start_pos) == (0, len(want), want[0][1])
    assert blocks[3].contents.n_snps == 0
    # reopening restarts at the first block; folded and a sub-sample are passed through
    f1 = next(fscl_amd.ms_blocks(ms, 1_000_000, folded=True, sample_first=2, sample_size=8)).contents
    w1 = fscl_amd.load_ms_input(ms, 1_000_000, folded=True, sample_first=2, sample_size=8).contents
    assert snps(f1) == [w for w in snps(w1) if w[0] == 0]


def test_partition_is_contiguous_and_balanced(built):
    rng = np.random.default_rng(0)
    for n, world in [(10, 3), (1, 4), (0, 2), (257, 8), (40, 1)]:
        cost = rng.integers(1, 100, size=n).astype(float)
        spans = [fscl_amd.partition(cost, r, world) for r in range(world)]
        covered = [i for lo, hi in spans for i in range(lo, hi)]
        assert covered == list(range(n))
        if n >= world * 8:
            shares = [cost[lo:hi].sum() for lo, hi in spans]
            assert max(shares) <= cost.sum() / world + cost.max()


def test_library_exports_every_declared_symbol(built):
    lib = fscl_amd.get_lib()
    declared = set()
    for h in (ROOT / "include").glob("*.h"):
        txt = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        for m in re.finditer(r"^\s*(?!typedef)(?:[\w]+\s+\**)+\**(\w+)\s*\(", txt, flags=re.M):
            if m.group(1) not in ("if", "while", "return"):
                declared.add(m.group(1))
    assert set(fscl_amd.EXPORTS) <= declared | {"fscl_amd_partition"}
    for name in sorted(declared):
        assert hasattr(lib, name), f"{name} declared in include/ but not exported"


def test_cli_fails_loudly_without_gpu(built, tmp):
    if fscl_amd.device_count() > 0:
        pytest.skip("a GPU is present")
    r = subprocess.run([str(CLI), "-f", str(GOLD / "g1.snp"), "-o", str(tmp / "o")], capture_output=True, text=True)
    assert r.returncode != 0
    assert "GPU" in r.stderr


def test_cli_validation_matches_reference(built, tmp):
    for args in (["-o", str(tmp / "o")], ["-f", str(GOLD / "g1.snp")], ["-f", "x", "-m", "y", "-o", "z"],
                 ["-f", str(GOLD / "g1.snp"), "-o", str(tmp / "o"), "-d", "1"],
                 ["-f", str(GOLD / "g1.snp"), "-o", str(tmp / "o"), "-g", "333"]):
        r = subprocess.run([str(CLI), *args], capture_output=True, text=True)
        assert r.returncode == 255, args


def test_output_bs_and_no_scan(built, tmp):
    bs = tmp / "bs.txt"
    r = subprocess.run([str(CLI), "-f", str(GOLD / "g1.snp"), "-o", str(tmp / "o"), f"--output-bs={bs}", "--no-scan"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    t = manifest()["tables"]["g1"]
    lines = bs.read_text().splitlines()
    assert len(lines) == len(t["depths"])
    for line, d in zip(lines, t["depths"]):
        f = line.split("\t")
        assert int(f[0]) == d["n"]
        assert [float(x) for x in f[1:]] == pytest.approx([float.fromhex(h) for h in d["fsp"]], abs=5e-7)
    # -b reads back what --output-bs wrote
    r = subprocess.run([str(CLI), "-f", str(GOLD / "g1.snp"), "-o", str(tmp / "o"), "-b", str(bs), "--no-scan",
                        f"--output-bs={tmp / 'bs2.txt'}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert (tmp / "bs2.txt").read_text() == bs.read_text()


@pytest.mark.parametrize("n_iv", [200, 257, 500])
def test_interval_thresholds_reproduce_the_division(built, n_iv):
    """The kernel picks spline intervals by multiply + exact thresholds instead of
    sm-spline.c:52's division; the thresholds must reproduce the division exactly."""
    L = fscl_amd.get_lib()
    step = 24.0 / (n_iv + 1.0)
    thr = (C.c_double * (n_iv + 1))()
    assert L.fsclg_interval_thresholds(step, n_iv, thr) == 0
    T = np.array(thr[:])
    rng = np.random.default_rng(n_iv)
    xs = np.concatenate([rng.uniform(-20.0, 4.0, 200_000), T[1:n_iv], np.nextafter(T[1:n_iv], -np.inf),
                         np.nextafter(T[1:n_iv], np.inf), [-20.0, 4.0]])
    ref = np.clip(((xs - -20.0) / step).astype(np.int64), 0, n_iv - 1)
    iv = np.clip(((xs - -20.0) * (1.0 / step)).astype(np.int64), 0, n_iv - 1)
    up = (iv + 1 < n_iv) & (xs >= T[np.minimum(iv + 1, n_iv)])
    down = ~up & (iv > 0) & (xs < T[iv])
    got = iv + up - down
    assert np.array_equal(got, ref)


def _chunked_window_sum(v, W, a, emin, ne, C=64):
    """Python restatement of window_chunk_kernel / chunk_table_kernel (fsclg.hip): the exact
    chunked form of acc = 0.0; acc += v[i] for i = a .. a + W - 1."""
    import math

    def table(c, e):
        vals = v[c * C:(c + 1) * C]
        if len(vals) < C or any(not (x <= 0.0) or x == -math.inf for x in vals):
            return None
        u = math.ldexp(1.0, e - 52)
        out = []
        for p in (0, 1):
            d, par = 0, p
            for x in vals:
                q = x / u
                F = math.floor(q)
                if q - F == 0.5:
                    d += F + ((par + F) & 1)
                    par = 0
                else:
                    R = round(q)
                    d += R
                    par = (par + R) & 1
            out.append(d)
        return out

    s, i, end = 0.0, a, a + W
    while i < end:  # head
        if i % C == 0 and s <= -math.ldexp(1.0, emin):
            break
        s = s + v[i]
        i += 1
    while i + C <= end:  # chunks
        e = math.frexp(-s)[1] - 1 if s < 0.0 else None
        t = table(i // C, e) if e is not None and emin <= e < emin + ne else None
        if t is not None:
            u = math.ldexp(1.0, e - 52)
            m = int(s / u)
            mn = m + t[m & 1]
            if mn > -(1 << 53):
                s, i = mn * u, i + C
                continue
        for j in range(C):
            s = s + v[i + j]
        i += C
    while i < end:
        s = s + v[i]
        i += 1
    return s


def _tree_window_sum(v, W, a, emin, ne, C=64, lmax=11):
    """Python restatement of the block steps of window_chunk_kernel (fsclg.hip):
    the chunk maps m -> m + D[m & 1] of chunk_table_kernel composed over aligned blocks of 2^L
    chunks (chunk_tree_kernel), and the running sum advanced by the largest aligned block that
    keeps it in its binade, halving the block on a crossing; the rest as the chunked form."""
    import math

    def table(c, e):
        vals = v[c * C:(c + 1) * C]
        if len(vals) < C or any(not (x <= 0.0) or x == -math.inf for x in vals):
            return None
        u = math.ldexp(1.0, e - 52)
        out = []
        for p in (0, 1):
            d, par = 0, p
            for x in vals:
                q = x / u
                F = math.floor(q)
                if q - F == 0.5:
                    d += F + ((par + F) & 1)
                    par = 0
                else:
                    R = round(q)
                    d += R
                    par = (par + R) & 1
            out.append(d)
        return out

    def compose(f1, f2):  # f2 after f1: the block map for either entry parity
        if f1 is None or f2 is None:
            return None
        return [f1[p] + f2[(p + f1[p]) & 1] for p in (0, 1)]

    memo = {}

    def block(L, b, e):  # the map of chunks [b 2^L, (b + 1) 2^L) in binade e
        key = (L, b, e)
        if key not in memo:
            memo[key] = table(b, e) if L == 0 else compose(block(L - 1, 2 * b, e), block(L - 1, 2 * b + 1, e))
        return memo[key]

    s, i, end = 0.0, a, a + W
    while i < end:  # head
        if i % C == 0 and s <= -math.ldexp(1.0, emin):
            break
        s = s + v[i]
        i += 1
    L = lmax
    while i + C <= end:  # whole chunks: aligned blocks
        e = math.frexp(-s)[1] - 1 if s < 0.0 else None
        c = i // C
        if e is not None and emin <= e < emin + ne:
            Lc = min(L, lmax, ((c & -c).bit_length() - 1) if c else lmax, ((end - i) // C).bit_length() - 1)
            t = block(Lc, c >> Lc, e)
            u = math.ldexp(1.0, e - 52)
            m = int(s / u)
            if t is not None and m + t[m & 1] > -(1 << 53):
                s, i, L = (m + t[m & 1]) * u, i + (C << Lc), lmax
                continue
            if Lc > 0:
                L = Lc - 1
                continue
        for j in range(C):  # the general step: chunk c site by site
            s = s + v[i + j]
        i += C
        L = lmax
    while i < end:
        s = s + v[i]
        i += 1
    return s


def test_block_window_sums_are_the_sequential_sums():
    """The block steps of the window sums restated in Python: composing the
    chunk maps over aligned blocks (their increment depends on the running sum only through its
    parity, so they compose) and stepping by the largest block that stays in the binade gives
    the sequential sum bit for bit, at every window offset, with ties, zeros, a positive value
    and windows long enough for blocks of up to 2^5 chunks."""
    import math
    import random
    rng = random.Random(13)
    classes = [-rng.randint(1, 4000) / 64.0 if k % 3 == 0 else -rng.uniform(0.5, 60.0) for k in range(300)]
    classes[5], classes[6] = 0.0, 3.5
    v = [classes[rng.randrange(len(classes))] for _ in range(9000)]
    v[4321] = 2.0  # a positive value: its chunk's blocks are invalid, that chunk site by site
    mx = max(abs(x) for x in v)
    W = 4100
    emin = math.frexp(64 * mx)[1]
    ne = math.frexp(W * mx)[1] - emin + 1
    for a in list(range(0, 70, 3)) + list(range(70, len(v) - W + 1, 97)):
        seq = 0.0
        for i in range(a, a + W):
            seq = seq + v[i]
        assert _tree_window_sum(v, W, a, emin, ne, lmax=5).hex() == seq.hex(), a


def test_chunked_window_sums_are_the_sequential_sums():
    """The chunked window null sums (fsclg.hip window_chunk_kernel) restated in
    Python: bit-identical to the sequential sum for windows at every offset, over null values
    with short mantissas (ties at many binades), zeros and a positive value (its chunks fall back
    to site-by-site adds)."""
    import math
    import random
    rng = random.Random(11)
    classes = [-rng.randint(1, 4000) / 64.0 if k % 3 == 0 else -rng.uniform(0.5, 60.0) for k in range(300)]
    classes[5], classes[6] = 0.0, 3.5
    v = [classes[rng.randrange(len(classes))] for _ in range(5000)]
    mx = max(abs(x) for x in v)
    W = 1800
    emin = math.frexp(64 * mx)[1]
    ne = math.frexp(W * mx)[1] - emin + 1
    for a in list(range(0, 64)) + list(range(64, len(v) - W + 1, 53)):
        seq = 0.0
        for i in range(a, a + W):
            seq = seq + v[i]
        assert _chunked_window_sum(v, W, a, emin, ne).hex() == seq.hex(), a


def test_c3_input_is_ascertained_and_its_fixture_is_not_degenerate():
    """BASELINE configs[2] (K=2 of M=20 ascertainment correction) runs on ascertained sites
    (synth.ascertained: the reference's double-hit panel rule, ascbias-segments.c:88-101):
    100 000 sites, none with fewer than 2 copies of either allele -- on unascertained sites
    every C3 CLR was 0.0.  The oracle's run of bench.py's C3 job
    (tests/golden/fullsize.json[C3_bench_p100]) has non-zero CLRs and points that outlive
    trial 20 (the prune tail), in its sampled rows and its permutation count."""
    import json
    cfg = dict(synth.CONFIGS["C3"])
    (name, pos, k, nn, fold), = synth.generate(seed=1, sweeps_per_chr=2, **cfg)
    assert len(pos) == cfg["snps_per_chr"] and (np.diff(pos) > 0).all()
    assert np.minimum(k, nn - k).min() >= cfg["asc_min_freq"]
    # the filter itself: a site is kept iff both alleles appear >= K times in the M-panel
    rng = np.random.default_rng(0)
    kk = np.arange(1, 100)
    keep = np.array([synth.ascertained(rng, np.full(4000, x), 100, 20, 2).mean() for x in kk])
    assert keep[0] == 0.0 and keep[-1] == 0.0 and keep[49] > 0.99
    fx = json.loads((GOLD / "fullsize.json").read_text())["C3_bench_p100"]
    assert fx["gen"].get("asc_depth") == 20 and fx["gen"].get("asc_min_freq") == 2
    rows = [r.split("\t") for r in fx["sample"]]
    assert all(float.fromhex(r[2]) != 0.0 for r in rows)
    assert fx["sum_permute_n"] > 21 * fx["n_points"]
    assert max(int(r[10]) for r in rows) > 21


def test_cell_order_dedup_and_search(tmp_path):
    """The submit path's ordering of cells (fscl_amd/csrc/device/cell_order.h: identical cells and
    shared endpoints found by ordered comparison, the windows' bucketed site index), built
    here with g++ and checked against std::map / std::lower_bound restatements over 4 000 cell
    lists: the host's ascending order, two ascending runs, shuffled, with duplicates, nested
    cells and negative positions."""
    exe = tmp_path / "cell_order_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", str(ROOT / "tests" / "cpp" / "cell_order_check.cpp"),
                    "-o", str(exe)], check=True, timeout=120)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr


ORC_SNP = np.dtype([("chr", "<i4"), ("pos", "<i4"), ("null_logl", "<f8"), ("obs_freq", "<i4"), ("depth_p", "<i4"),
                    ("folded", "<i4"), ("pad", "<i4")])
ORC_STATS = C.c_longlong * 6  # orc_stats_t: ..., negj last


def _plan_geometry(n_chr, per_chr, chr_len, seed):
    rng = np.random.default_rng(seed)
    pos = np.concatenate([np.sort(rng.choice(chr_len, per_chr, replace=False)).astype(np.int32) + 1
                          for _ in range(n_chr)])
    chr_start = (np.arange(n_chr) * per_chr).astype(np.int32)
    return pos, chr_start, np.full(n_chr, per_chr, np.int32)


@pytest.mark.parametrize("geom", [
    # (chromosomes, SNPs each, bp, trials, nbp, width Mb): C5's chromosome over 1 000 trials; the whole C5
    # genome; short chromosomes where blocks run past the end (Q9) and overlap themselves
    (1, 227_273, 227_000_000, 1000, 0.1, 1.0),
    (22, 227_273, 227_000_000, 4, 0.1, 1.0),
    (3, 2_000, 2_000_000, 400, 0.1, 1.0),
    (2, 500, 100_000, 400, 0.01, 0.05),
])
def test_block_plan_is_the_sequential_block_permutation(built, geom):
    """perm.c's plan (blocks drawn from the rand() stream, leveled, grouped; applied as the device
    applies it, fh_plan_apply_u32) against the oracle's orc_block_permute (scan-chromosome.c:336-389,
    Q9 repaired the same way): the same rows, the same rand() state after, the same negative-j count,
    trial after trial of one stream"""
    n_chr, per, L, trials, nbp, width = geom
    pos, cs, cn = _plan_geometry(n_chr, per, L, seed=n_chr * 7 + per)
    n = len(pos)
    lib = fscl_amd.get_lib()
    lib.fscl_amd_plan_permute_test.restype = C.c_int
    lib.fscl_amd_plan_permute_test.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_double,
                                               C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.fh_srand.argtypes = [C.c_void_p, C.c_uint]
    orc = C.CDLL(str(ROOT / "oracle" / "_build" / "liboracle.so"))
    orc.orc_block_permute.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_double, C.c_double, C.c_void_p,
                                      C.c_void_p]
    orc.orc_srand.argtypes = [C.c_void_p, C.c_uint]
    snps = np.zeros(n, ORC_SNP)
    snps["chr"] = np.repeat(np.arange(n_chr), per)
    snps["pos"] = pos
    snps["obs_freq"] = np.arange(n)
    p = np.zeros_like(snps)
    g_prod, g_orc = (C.c_int32 * 33)(), (C.c_int32 * 33)()
    lib.fh_srand(g_prod, 0xFD821A6)
    orc.orc_srand(g_orc, 0xFD821A6)
    st = ORC_STATS()
    out = (C.c_longlong * 4)()
    negj = rot = 0
    for t in range(trials):
        rows = np.arange(n, dtype=np.uint32)
        assert lib.fscl_amd_plan_permute_test(n, pos.ctypes.data, cs.ctypes.data, cn.ctypes.data, n_chr, nbp, width,
                                              g_prod, rows.ctypes.data, out) == 0
        orc.orc_block_permute(p.ctypes.data, snps.ctypes.data, n, nbp, width, g_orc, st)
        assert np.array_equal(rows, p["obs_freq"].astype(np.uint32)), f"trial {t}: rows differ"
        assert list(g_prod) == list(g_orc), f"trial {t}: rand() state differs"
        negj += out[0]
        rot += out[3]
        assert negj == st[5]
    if n < 10_000:  # the edge cases this geometry is there for
        assert negj > 0 and rot > 0, (negj, rot)


def test_bench_line_assembly_from_recorded_stats(built, monkeypatch):
    """bench.py's JSON line (roofline with the committed profile, the stats block, cpu_baseline with
    its anchor) assembled on the CPU from a recorded stats dict: a missing stats field or a key error
    in the line's assembly fails here, not after minutes of GPU time."""
    import argparse
    import json as _json
    import bench
    rec = _json.loads((ROOT / "profiles" / "r04z_bench_c4.json").read_text().strip().splitlines()[-1])
    st = fscl_amd.Stats().as_dict()
    st.update({k: v for k, v in rec["stats"].items() if k in st})
    st.update(kernel_ms=11617.0, n_launches=4002, busy_ms=5349.0, n_dup_cells=1, n_ep_saved=2, negj=26)
    args = argparse.Namespace(config="C4", chromosomes=None, profile_summary=None, steps=2, warmup=1,
                              permute_mode="parity", exchange="shm", cpu_threads=None, cpu_sample=None,
                              cpu_full_job=False, n_permute=None)
    cfg = dict(synth.CONFIGS["C4"])
    line = bench.bench_line(args, cfg, st, 2.2e6, 10.0, 1, 1, 1, 1000, 10010, 3.0)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "stats"):
        assert k in line, k
    roof = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "limiter", "source"):
        assert k in roof, k
    assert roof["source"] and roof["traffic"] and 0 < roof["frac"] < 2
    assert line["stats"]["perm_leader"] == 0 and "plan_mode" in line["stats"]
    canned = {"sample_cells": 384.0, "threads": 16.0, "cell_s": 2.0, "perm_gen_s": 0.003, "perm_cells": 384.0,
              "perm_cell_s": 2.1}
    monkeypatch.setattr(bench, "_harness", lambda snp, cfg, threads, n: dict(canned))
    info = bench.cpu_info()
    bl, d, m = bench.cpu_baseline(args, cfg, None, None, info, fscl_amd, None, None, 10010, 1_170_000, 1001, 1.18e6,
                                  5.4, live_parity=False)
    for k in ("value", "unit", "cores", "kind", "sample", "threads_1", "node_linear", "anchor"):
        assert k in bl, k
    assert bl["anchor"]["source"].startswith("profiles/") and 0.5 < bl["anchor"]["measured_over_extrapolated"] < 2
    line["cpu_baseline"] = bl
    # the north-star ratio: live from this run's node-linear CPU figure, or the committed one of the workload
    ns = bench.north_star_ratio(args, 1000, 5.4, 1, bl["node_linear"]["job_s"])
    assert ns["value"] == bl["node_linear"]["job_s"] / 5.4 and ns["n_gpus"] == 1 and ns["target"] == 100.0
    ns8 = bench.north_star_ratio(args, 1000, 1.0, 8)
    tab = _json.loads((ROOT / "profiles" / "cpu_node_linear.json").read_text())["workloads"]["C4/chrall/p1000/parity"]
    assert ns8["value"] == tab["job_s"] and ns8["n_gpus"] == 8 and (ROOT / tab["source"]).exists()
    assert ns8["meets_target"] == (tab["job_s"] >= 100.0)
    assert bench.north_star_ratio(argparse.Namespace(**{**vars(args), "config": "C1"}), 0, 1.0, 1) is None
    line["north_star_ratio"] = ns
    _json.dumps(line)
