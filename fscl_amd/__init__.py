"""fscl_amd -- MI355X-native drop-in for slowkoni/fscl's CLR sweep scan and
block-permutation test.

The product is the C-ABI library ``fscl_amd/_build/libfscl_amd.so`` (host C +
gfx950 HIP kernels, see include/fscl_amd.h and include/fsclg.h) and the
``fscl_amd/_build/fscl`` command line.  This module is the Python mirror of the
reference's entry points (fscl.h:86-128) over ctypes: same names, same argument
meaning, same fatal-error behaviour (the library prints and exits, as
logmsg(MSG_FATAL) does in the reference).

There is no CPU fallback: importing works without a GPU (so the library's
exports can be inspected), but every scan entry point needs the HIP device and
fails loudly without it.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

__all__ = [
    "lib", "LIB_PATH", "CLI_PATH", "SnpT", "ScanPtT", "ScanT", "ChrLimitsT", "SplineT", "SmPtableT", "Stats",
    "load_snp_input", "load_ms_input", "background_fsp", "compute_sweep_model_tables", "compute_snp_null_model",
    "init_log_table", "scan_chromosome", "scan_permute", "scan_output", "output_background_fs", "points",
    "get_stats", "reset_stats", "set_device", "set_devices", "set_ranks", "set_ranks_shm", "srand", "shutdown", "run",
    "device_count", "set_dump_output",
]

ROOT = Path(__file__).resolve().parent
LIB_PATH = (Path(os.environ["FSCL_AMD_LIBDIR"]) if os.environ.get("FSCL_AMD_LIBDIR") else
            ROOT / ("_build_trace" if os.environ.get("FSCL_AMD_TRACE") else "_build")) / "libfscl_amd.so"
CLI_PATH = ROOT / "_build" / "fscl"


class SnpT(C.Structure):  # fscl.h:7-14
    _fields_ = [("chr", C.c_int), ("pos", C.c_int), ("null_logl", C.c_double), ("obs_freq", C.c_int),
                ("depth_p", C.c_int), ("folded", C.c_int)]


class ChrLimitsT(C.Structure):  # fscl.h:26-33
    _fields_ = [("chr", C.c_int), ("name", C.c_char_p), ("start_index", C.c_int), ("n_snps", C.c_int),
                ("start_pos", C.c_int), ("bp_length", C.c_int)]


class ScanPtT(C.Structure):  # fscl.h:35-51
    _fields_ = [("chr", C.c_int), ("nearest_snp", C.c_int), ("sweep_pos", C.c_int), ("n_snps", C.c_int),
                ("window_start", C.c_int), ("window_end", C.c_int), ("lalpha", C.c_double),
                ("null_logl", C.c_double), ("sm_logl", C.c_double), ("clr", C.c_double),
                ("permute_n", C.c_int), ("permute_p", C.c_int), ("permute_finished", C.c_int),
                ("scan_running", C.c_int), ("permute_clr", C.POINTER(C.c_float))]


class ScanT(C.Structure):  # fscl.h:53-62
    _fields_ = [("n_snps", C.c_int), ("snps", C.POINTER(SnpT)), ("n_depths", C.c_int),
                ("sample_depths", C.POINTER(C.c_int)), ("n_scan_pts", C.c_int),
                ("scan_pts", C.POINTER(ScanPtT)), ("chr_limits", C.POINTER(ChrLimitsT)),
                ("n_chromosomes", C.c_int)]


class SplineT(C.Structure):  # fscl.h:64-68
    _fields_ = [("n", C.c_int), ("knot_points", C.POINTER(C.c_double)),
                ("coef", C.POINTER(C.POINTER(C.c_double)))]


class SmPtableT(C.Structure):  # fscl.h:70-76
    _fields_ = [("spline_func", C.POINTER(C.POINTER(SplineT))), ("fspline_func", C.POINTER(C.POINTER(SplineT))),
                ("sample_size", C.c_int), ("pbk", C.POINTER(C.POINTER(C.c_double))),
                ("fsp", C.POINTER(C.c_double))]


class Stats(C.Structure):  # fscl_amd_stats_t
    _fields_ = [("scan_s", C.c_double), ("permute_s", C.c_double), ("host_perm_s", C.c_double),
                ("kernel_ms", C.c_double), ("gp_evals", C.c_ulonglong), ("n_terms", C.c_ulonglong),
                ("n_null", C.c_ulonglong), ("n_walks", C.c_ulonglong), ("n_maxalpha", C.c_ulonglong),
                ("n_unsafe", C.c_ulonglong), ("n_slow", C.c_ulonglong), ("n_ties", C.c_ulonglong),
                ("n_launches", C.c_ulonglong), ("negj", C.c_ulonglong), ("trials", C.c_int),
                ("cache_iv0", C.c_int), ("cache_n_iv", C.c_int), ("cache_n_rows", C.c_int),
                ("cache_cover", C.c_double), ("window_ms", C.c_double), ("host_null_s", C.c_double),
                ("host_upload_s", C.c_double), ("search_s", C.c_double), ("prune_s", C.c_double),
                ("n_dup_cells", C.c_ulonglong), ("n_ep_saved", C.c_ulonglong), ("busy_ms", C.c_double),
                ("wait_s", C.c_double), ("n_crit", C.c_ulonglong), ("n_drain", C.c_ulonglong),
                ("n_devices", C.c_int), ("spec_threads", C.c_int), ("spec_posted", C.c_ulonglong),
                ("spec_hits", C.c_ulonglong), ("spec_cands", C.c_ulonglong), ("spec_wait_s", C.c_double),
                ("spec_done", C.c_ulonglong), ("spec_gen_s", C.c_double),
                ("n_split_retry", C.c_ulonglong), ("spec_claimed", C.c_ulonglong), ("n_merged", C.c_ulonglong),
                ("perm_leader", C.c_int), ("plan_mode", C.c_int), ("plan_fallback", C.c_ulonglong),
                ("spec_rank", C.c_ulonglong * 8), ("prestaged", C.c_ulonglong), ("prestage_hits", C.c_ulonglong)]

    def as_dict(self) -> dict:
        return {k: (list(v) if isinstance(v, C.Array) else v) for k, v in ((k, getattr(self, k)) for k, _ in self._fields_)}


EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_longlong), C.c_int, C.c_void_p)

# exported symbols of include/fscl_amd.h and include/fsclg.h (checked by tests)
EXPORTS = [
    "load_snp_input", "background_fsp", "output_background_fs", "lchoose", "compute_sweep_model_tables",
    "spline_interpolate", "init_log_table", "search_maxalpha", "compute_snp_null_model", "scan_chromosome",
    "scan_permute", "scan_output", "ascbias_adjust_background", "ascbias_adjust_expect", "configure_logmsg",
    "logmsg", "cr_logmsg", "fscl_amd_load_ms_input", "fscl_amd_set_device", "fscl_amd_set_ranks",
    "fscl_amd_get_stats", "fscl_amd_reset_stats", "fscl_amd_shutdown", "fscl_amd_partition",
    "fscl_amd_set_devices", "fscl_amd_n_devices", "fscl_amd_set_ranks_shm", "fscl_amd_srand",
    "fscl_amd_set_dump_output", "fsclg_host_alloc", "fsclg_host_free", "fsclg_slot_wait",
    "fsclg_slot_set_rows_host", "fsclg_slot_set_rows_packed",
    "fsclg_open", "fsclg_close", "fsclg_last_error", "fsclg_device_count", "fsclg_upload_tables",
    "fsclg_upload_snps", "fsclg_set_rows", "fsclg_set_chr_null", "fsclg_set_alpha_grid", "fsclg_search_maxpos",
    "fsclg_search_points", "fsclg_get_stats", "fsclg_reset_stats", "fsclg_interval_thresholds",
    "fsclg_row_buffer", "fsclg_slot_row_buffer", "fsclg_slot_set_rows", "fsclg_search_submit", "fsclg_search_wait",
    "fsclg_slot_windows", "ms_openfile", "ms_background", "ms_next_block",
    "fscl_amd_set_permute_mode",
]


def _load() -> C.CDLL:
    if not LIB_PATH.exists():
        raise ImportError(f"fscl_amd native library missing at {LIB_PATH}; run `python -m fscl_amd.build`")
    L = C.CDLL(str(LIB_PATH))
    P = C.POINTER
    sigs = {
        "load_snp_input": (P(ScanT), [C.c_char_p, C.c_int, C.c_int]),
        "fscl_amd_load_ms_input": (P(ScanT), [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int]),
        "ms_openfile": (None, [C.c_char_p]),
        "fscl_amd_set_permute_mode": (C.c_int, [C.c_int, C.c_ulonglong]),
        "ms_background": (P(ScanT), [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int]),
        "ms_next_block": (P(ScanT), [C.c_int, C.c_int, C.c_int, C.c_int]),
        "background_fsp": (P(P(C.c_double)), [P(ScanT), C.c_int, C.c_char_p, C.c_int]),
        "output_background_fs": (None, [C.c_char_p, P(ScanT), P(P(C.c_double))]),
        "lchoose": (C.c_double, [C.c_int, C.c_int]),
        "compute_sweep_model_tables": (P(SmPtableT), [P(ScanT), P(P(C.c_double)), C.c_int, C.c_int, C.c_int,
                                                      C.c_int]),
        "spline_interpolate": (C.c_double, [P(SplineT), C.c_double]),
        "init_log_table": (None, []),
        "search_maxalpha": (None, [P(ScanPtT), P(SnpT), P(SmPtableT)]),
        "compute_snp_null_model": (None, [P(ScanT), P(P(C.c_double))]),
        "scan_chromosome": (None, [P(ScanT), P(SmPtableT), C.c_int, C.c_int, C.c_int, C.c_int]),
        "scan_permute": (None, [P(ScanT), P(SmPtableT), C.c_int, C.c_double, C.c_double, C.c_int, C.c_int, C.c_int,
                                C.c_int, C.c_double]),
        "scan_output": (None, [C.c_char_p, P(ScanT), C.c_int, C.c_int, C.c_char_p]),
        "ascbias_adjust_background": (P(C.c_double), [P(C.c_double), C.c_int, C.c_int, C.c_int]),
        "ascbias_adjust_expect": (None, [P(C.c_double), C.c_int, C.c_int, C.c_int]),
        "configure_logmsg": (None, [C.c_int]),
        "fscl_amd_set_device": (C.c_int, [C.c_int]),
        "fscl_amd_set_devices": (C.c_int, [P(C.c_int), C.c_int]),
        "fscl_amd_n_devices": (C.c_int, []),
        "fscl_amd_set_ranks_shm": (C.c_int, [C.c_int, C.c_int, C.c_char_p]),
        "fscl_amd_srand": (None, [C.c_uint]),
        "fscl_amd_set_dump_output": (None, [C.c_char_p, C.c_char_p]),
        "fscl_amd_set_ranks": (C.c_int, [C.c_int, C.c_int, EXCHANGE_FN, C.c_void_p]),
        "fscl_amd_get_stats": (None, [P(Stats)]),
        "fscl_amd_partition": (None, [P(C.c_double), C.c_int, C.c_int, C.c_int, P(C.c_int), P(C.c_int)]),
        "fh_srand": (None, [C.c_void_p, C.c_uint]),
        "fh_rand": (C.c_int, [C.c_void_p]),
        "fscl_amd_reset_stats": (None, []),
        "fscl_amd_shutdown": (None, []),
        "fsclg_device_count": (C.c_int, []),
        "fsclg_last_error": (C.c_char_p, []),
        "fsclg_interval_thresholds": (C.c_int, [C.c_double, C.c_int, P(C.c_double)]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


_lib = None
_keep = []  # ctypes callbacks and buffers that must outlive their C users


def get_lib() -> C.CDLL:
    """The loaded native library (loaded on first use, so `python -m fscl_amd.build` works without it)."""
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def __getattr__(name):  # PEP 562: fscl_amd.lib
    if name == "lib":
        return get_lib()
    raise AttributeError(name)


def _b(s):
    return None if s is None else os.fsencode(str(s))


def device_count() -> int:
    return int(get_lib().fsclg_device_count())


def init_log_table() -> None:
    get_lib().init_log_table()


def load_snp_input(path, include_invariant: bool = False, minimum_depth: int = 5):
    return get_lib().load_snp_input(_b(path), int(include_invariant), max(5, int(minimum_depth)))


def load_ms_input(path, segment_length: int, folded: bool = False, sample_first: int = 0, sample_size: int = 0):
    return get_lib().fscl_amd_load_ms_input(_b(path), int(segment_length), int(folded), int(sample_first),
                                      int(sample_size))


def ms_blocks(path, segment_length: int, folded: bool = False, sample_first: int = 0, sample_size: int = 0):
    """The reference's block loop (fscl.c:296-313): ms_openfile, then one
    scan_t per ms_next_block until it returns NULL."""
    L = get_lib()
    L.ms_openfile(_b(path))
    while True:
        s = L.ms_next_block(int(segment_length), int(folded), int(sample_first), int(sample_size))
        if not s:
            return
        yield s


PERMUTE_MODES = {"parity": 0, "throughput": 1}


def set_permute_mode(mode: str = "parity", seed: int = 0xFD821A6) -> None:
    """scan_permute's mode (include/fscl_amd.h): "parity" (the reference's rand() stream) or
    "throughput" (counter-based random numbers from `seed`, labelled non-parity)."""
    if get_lib().fscl_amd_set_permute_mode(PERMUTE_MODES[mode], int(seed)) != 0:
        raise ValueError(mode)


def background_fsp(scan, force_neutral: bool = False, bs_file=None, include_invariant: bool = False):
    return get_lib().background_fsp(scan, int(force_neutral), _b(bs_file), int(include_invariant))


def output_background_fs(path, scan, fsp) -> None:
    get_lib().output_background_fs(_b(path), scan, fsp)


def compute_sweep_model_tables(scan, fsp, asc_depth: int = 0, asc_min_freq: int = 1,
                               ascbias_background_only: bool = False, include_invariant: bool = False):
    return get_lib().compute_sweep_model_tables(scan, fsp, int(asc_depth), int(asc_min_freq),
                                          int(ascbias_background_only), int(include_invariant))


def compute_snp_null_model(scan, fsp) -> None:
    get_lib().compute_snp_null_model(scan, fsp)


def scan_chromosome(scan, tables, eval_range: int = 81920, bp_resl: int = 128, large_grid_sp: int = 100000,
                    n_threads: int = 1) -> None:
    get_lib().scan_chromosome(scan, tables, eval_range, bp_resl, large_grid_sp, n_threads)


def scan_permute(scan, tables, n_permute: int, permute_nbp: float = 0.1, alpha_factor: float = 1.0,
                 n_threads: int = 1, eval_range: int = 81920, bp_resl: int = 128, large_grid_sp: int = 100000,
                 scan_width_mb: float = 1.0) -> None:
    get_lib().scan_permute(scan, tables, int(n_permute), float(permute_nbp), float(alpha_factor), int(n_threads),
                     int(eval_range), int(bp_resl), int(large_grid_sp), float(scan_width_mb))


def scan_output(path, scan, max_only: bool = False, n_permute: int = 0, label=None) -> None:
    get_lib().scan_output(_b(path), scan, int(max_only), int(n_permute), _b(label))


POINT_DTYPE = np.dtype([("chr", "i4"), ("sweep_pos", "i4"), ("clr", "f8"), ("lalpha", "f8"), ("sm_logl", "f8"),
                        ("null_logl", "f8"), ("nearest_snp", "i4"), ("window_start", "i4"), ("window_end", "i4"),
                        ("n_snps", "i4"), ("permute_p", "i4"), ("permute_n", "i4"), ("permute_finished", "i4")])


def points(scan) -> np.ndarray:
    """The scan points of a scan_t as a numpy structured array."""
    s = scan.contents
    out = np.zeros(s.n_scan_pts, dtype=POINT_DTYPE)
    for i in range(s.n_scan_pts):
        p = s.scan_pts[i]
        out[i] = (p.chr, p.sweep_pos, p.clr, p.lalpha, p.sm_logl, p.null_logl, p.nearest_snp, p.window_start,
                  p.window_end, p.n_snps, p.permute_p, p.permute_n, p.permute_finished)
    return out


def get_stats() -> dict:
    st = Stats()
    get_lib().fscl_amd_get_stats(C.byref(st))
    return st.as_dict()


def reset_stats() -> None:
    get_lib().fscl_amd_reset_stats()


def set_device(device: int) -> None:
    get_lib().fscl_amd_set_device(int(device))


def set_devices(devices=None, n: int | None = None) -> None:
    """This process drives several GPUs: ``devices`` (a list of ids) or the first ``n``;
    ``n=0`` (or nothing given): every visible GPU."""
    if devices is not None:
        arr = (C.c_int * len(devices))(*[int(d) for d in devices])
        r = get_lib().fscl_amd_set_devices(arr, len(devices))
    else:
        r = get_lib().fscl_amd_set_devices(None, int(n or 0))
    if r != 0:
        raise ValueError("bad device list")


def srand(seed: int = 0xFD821A6) -> None:
    """Restart the process-wide permutation rand() stream (srand, fscl.c:135)."""
    get_lib().fscl_amd_srand(int(seed))


_dump_names = []


def set_dump_output(path=None, label=None) -> None:
    """What a SIGINT during scan_permute writes (the reference reads fscl.c's globals)."""
    b = (_b(path), _b(label))
    _dump_names.append(b)  # the C side keeps the pointers
    get_lib().fscl_amd_set_dump_output(*b)


def set_ranks_shm(rank: int, world: int, name: str) -> None:
    """Multi-process parity mode with the library's own shared-memory exchange (one node)."""
    if get_lib().fscl_amd_set_ranks_shm(int(rank), int(world), name.encode()) != 0:
        raise RuntimeError(f"fscl_amd_set_ranks_shm({rank}, {world}, {name!r}) failed")


def set_ranks(rank: int, world: int, allreduce_sum_int64=None) -> None:
    """Multi-process parity mode.  ``allreduce_sum_int64(np.ndarray[int64]) -> None``
    must sum the array in place across ranks (torch.distributed over RCCL in
    bench.py, gloo in the CPU tests)."""
    if world == 1:
        cb = EXCHANGE_FN()
    else:
        def _cb(buf, n, _ctx):
            try:
                arr = np.ctypeslib.as_array(buf, shape=(n,))
                allreduce_sum_int64(arr)
                return 0
            except Exception as e:  # noqa: BLE001 -- a failed exchange must not unwind through C
                import sys
                print(f"fscl_amd exchange failed: {e!r}", file=sys.stderr)
                return 1
        cb = EXCHANGE_FN(_cb)
    _keep.append(cb)
    if get_lib().fscl_amd_set_ranks(int(rank), int(world), cb, None) != 0:
        raise ValueError("bad rank/world")


def partition(cost, rank: int, world: int) -> tuple[int, int]:
    c = np.ascontiguousarray(cost, dtype=np.float64)
    lo, hi = C.c_int(), C.c_int()
    get_lib().fscl_amd_partition(c.ctypes.data_as(C.POINTER(C.c_double)), len(c), rank, world, C.byref(lo), C.byref(hi))
    return lo.value, hi.value


def shutdown() -> None:
    get_lib().fscl_amd_shutdown()


def run(snp_file=None, output=None, *, ms_file=None, ms_segment_length=0, ms_folded=False, n_permute=0,
        permute_nbp=0.1, asc_depth=0, asc_min_freq=1, ascbias_background_only=False, include_invariant=False,
        force_neutral=False, minimum_depth=5, large_grid_sp=100000, scan_width_mb=1.0, max_only=False,
        label=None, eval_range=81920, bp_resl=128, verbosity=1, permute_mode="parity", permute_seed=0xFD821A6):
    """The fscl main() pipeline (fscl.c:316-337) in-process; returns the scan_t
    pointer (points(scan) reads the results).  permute_mode "throughput": the
    counter-based permutation test (set_permute_mode)."""
    get_lib().configure_logmsg(int(verbosity))
    set_permute_mode(permute_mode, permute_seed)
    init_log_table()
    srand()  # init_options (fscl.c:135): a fresh process's stream
    set_dump_output(output, label)
    scan = (load_ms_input(ms_file, ms_segment_length, ms_folded) if ms_file else
            load_snp_input(snp_file, include_invariant, minimum_depth))
    fsp = background_fsp(scan, force_neutral, None, include_invariant)
    tab = compute_sweep_model_tables(scan, fsp, asc_depth, asc_min_freq, ascbias_background_only,
                                     include_invariant)
    compute_snp_null_model(scan, fsp)
    scan_chromosome(scan, tab, eval_range, bp_resl, large_grid_sp)
    if n_permute > 0:
        scan_permute(scan, tab, n_permute, permute_nbp, 1.0, 1, eval_range, bp_resl, large_grid_sp, scan_width_mb)
    if output is not None:
        scan_output(output, scan, max_only, n_permute, label)
    return scan
