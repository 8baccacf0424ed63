"""ctypes view of oracle/_build/liboracle.so (TEST INFRASTRUCTURE ONLY).

Used by tests/ and by bench.py's cpu_baseline leg, never by the product.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

LIB = Path(__file__).resolve().parent / "_build" / "liboracle.so"


class OrcOpts(C.Structure):
    _fields_ = [("spline_pts", C.c_int), ("include_invariant", C.c_int), ("minimum_depth", C.c_int),
                ("force_neutral", C.c_int), ("asc_depth", C.c_int), ("asc_min_freq", C.c_int),
                ("ascbias_background_only", C.c_int), ("n_permute", C.c_int), ("permute_nbp", C.c_double),
                ("scan_width_mb", C.c_double), ("large_grid_sp", C.c_int), ("eval_range", C.c_int),
                ("bp_resl", C.c_int), ("max_only", C.c_int), ("n_threads", C.c_int)]


class OrcStats(C.Structure):
    _fields_ = [(k, C.c_longlong) for k in ("n_terms", "n_null", "n_walks", "n_maxalpha", "n_gp", "negj")]


class OrcPt(C.Structure):
    _fields_ = [("chr", C.c_int), ("nearest_snp", C.c_int), ("sweep_pos", C.c_int), ("n_snps", C.c_int),
                ("window_start", C.c_int), ("window_end", C.c_int), ("lalpha", C.c_double),
                ("null_logl", C.c_double), ("sm_logl", C.c_double), ("clr", C.c_double),
                ("permute_n", C.c_int), ("permute_p", C.c_int), ("permute_finished", C.c_int),
                ("scan_running", C.c_int), ("permute_clr", C.c_void_p)]


class OrcScan(C.Structure):
    _fields_ = [("n_snps", C.c_int), ("snps", C.c_void_p), ("n_depths", C.c_int), ("sample_depths", C.c_void_p),
                ("n_pts", C.c_int), ("pts", C.POINTER(OrcPt)), ("chr", C.c_void_p), ("n_chr", C.c_int)]


def load() -> C.CDLL:
    L = C.CDLL(str(LIB))
    P = C.POINTER
    L.orc_default_opts.argtypes = [P(OrcOpts)]
    L.orc_init_log_table.argtypes = []
    L.orc_load_snp_input.restype = P(OrcScan)
    L.orc_load_snp_input.argtypes = [C.c_char_p, C.c_int, C.c_int]
    L.orc_background_fsp.restype = C.c_void_p
    L.orc_background_fsp.argtypes = [P(OrcScan), C.c_int, C.c_int]
    L.orc_compute_tables.restype = C.c_void_p
    L.orc_compute_tables.argtypes = [P(OrcScan), C.c_void_p, P(OrcOpts)]
    L.orc_null_model.argtypes = [P(OrcScan), C.c_void_p]
    L.orc_scan_chromosome.argtypes = [P(OrcScan), C.c_void_p, P(OrcOpts), P(OrcStats)]
    L.orc_scan_permute.argtypes = [P(OrcScan), C.c_void_p, P(OrcOpts), P(OrcStats)]
    L.orc_reseed.argtypes = [C.c_uint]
    return L


class OracleScan:
    """Set up an SNP file in the oracle (input, background, tables, null model)."""

    def __init__(self, snp_file, threads: int = 1, **opts):
        self.L = load()
        self.o = OrcOpts()
        self.L.orc_default_opts(C.byref(self.o))
        for k, v in opts.items():
            setattr(self.o, k, v)
        self.o.n_threads = threads
        self.L.orc_init_log_table()
        self.s = self.L.orc_load_snp_input(str(snp_file).encode(), self.o.include_invariant, self.o.minimum_depth)
        self.fsp = self.L.orc_background_fsp(self.s, self.o.force_neutral, self.o.include_invariant)
        self.tab = self.L.orc_compute_tables(self.s, self.fsp, C.byref(self.o))
        self.L.orc_null_model(self.s, self.fsp)
        self.stats = OrcStats()

    def scan(self) -> None:
        self.L.orc_scan_chromosome(self.s, self.tab, C.byref(self.o), C.byref(self.stats))

    def reseed(self, seed: int = 0xFD821A6) -> None:
        """Restart the oracle's process-wide permutation stream (srand, fscl.c:135)."""
        self.L.orc_reseed(seed)

    def permute(self, n_permute: int) -> None:
        """One scan_permute call (the stream continues from the previous call)."""
        self.o.n_permute = n_permute
        self.L.orc_scan_permute(self.s, self.tab, C.byref(self.o), C.byref(self.stats))

    def points(self) -> list[tuple]:
        """(chr, sweep_pos, clr, lalpha, sm_logl, null_logl, nearest, ws, we, permute_n, permute_p, finished)"""
        s = self.s.contents
        out = []
        for i in range(s.n_pts):
            q = s.pts[i]
            out.append((q.chr, q.sweep_pos, q.clr, q.lalpha, q.sm_logl, q.null_logl, q.nearest_snp, q.window_start,
                        q.window_end, q.permute_n, q.permute_p, q.permute_finished))
        return out

    def clr(self) -> list[tuple[int, int, float]]:
        s = self.s.contents
        return [(s.pts[i].chr, s.pts[i].sweep_pos, s.pts[i].clr) for i in range(s.n_pts)]
