#!/usr/bin/env python3
"""Latency of the rank exchange (ranks.c fh_shm_allgather_flags) with W processes on this
host's CPUs: the cost the 8-GPU rehearsal (FSCL_AMD_SIM replay, which takes the other ranks'
shares from a recording) does not pay.  Each rank makes N exchanges of a tail-sized batch
(n cells of 64 B, its contiguous share), with a little uneven host work between exchanges
as in the trial loop.  Prints one JSON line: microseconds per exchange (median, p90) as seen
by rank 0, and the exchanges a C4 job makes per trial.

    python tools/shm_latency.py [W] [N] [n]
"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess
import sys
import time
import uuid
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def worker(rank: int, world: int, name: str, N: int, n: int) -> None:
    sys.path.insert(0, str(ROOT))
    import numpy as np
    import fscl_amd
    L = fscl_amd.get_lib()
    L.fh_shm_open.restype = C.c_void_p
    L.fh_shm_open.argtypes = [C.c_int, C.c_int, C.c_char_p, C.c_size_t]
    L.fh_shm_allgather_flags.restype = C.c_int
    L.fh_shm_allgather_flags.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                         C.POINTER(C.c_uint)]
    m = L.fh_shm_open(rank, world, name.encode(), 1 << 20)
    assert m
    buf = np.zeros((n, 8), dtype=np.int64)
    lo, hi = n * rank // world, n * (rank + 1) // world
    rng = np.random.default_rng(rank)
    ts = []
    f = C.c_uint(0)
    for i in range(N):
        t_end = time.perf_counter() + rng.random() * 20e-6  # uneven host work before the exchange
        while time.perf_counter() < t_end:
            pass
        t0 = time.perf_counter()
        assert L.fh_shm_allgather_flags(m, buf.ctypes.data, 64, n, lo, hi, C.byref(f)) == 0
        ts.append(time.perf_counter() - t0)
    if rank == 0:
        ts = sorted(ts[N // 10:])
        print(json.dumps({"world": world, "exchanges": N, "cells": n, "cpus": len(os.sched_getaffinity(0)),
                          "median_us": ts[len(ts) // 2] * 1e6, "p90_us": ts[int(len(ts) * 0.9)] * 1e6,
                          "note": "time in fh_shm_allgather_flags on rank 0 (arrival to last rank's arrival "
                                  "+ copy); a parity-mode trial makes 2 (blocking batch with the SIGINT flag, "
                                  "bulk batch)"}), flush=True)


def main() -> int:
    if len(sys.argv) > 1 and sys.argv[1] == "--worker":
        worker(*map(int, sys.argv[2:4]), sys.argv[4], *map(int, sys.argv[5:7]))
        return 0
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 344
    name = f"/fscl_lat_{uuid.uuid4().hex[:12]}"
    procs = [subprocess.Popen([sys.executable, __file__, "--worker", str(r), str(W), name, str(N), str(n)])
             for r in range(W)]
    return max(p.wait() for p in procs)


if __name__ == "__main__":
    sys.exit(main())
