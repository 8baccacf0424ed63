"""The rank exchange protocol on CPU (gloo, world_size 2): the int64 sum of
slots that are non-zero on exactly one rank reproduces every 64-bit pattern,
including -0.0, infinities and NaN payloads."""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent

WORKER = r"""
import os, sys
import numpy as np
import torch, torch.distributed as dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
vals = np.array([0.0, -0.0, 1.5, -2.75, np.inf, -np.inf, 1e-310, 3.0e300], dtype=np.float64)
bits = vals.view(np.int64).copy()
nan_bits = np.array([0x7FF8000000000001, 0x7FF0000000000ABC], dtype=np.int64)
allv = np.concatenate([bits, nan_bits])
n = len(allv)
buf = np.zeros(n, dtype=np.int64)
lo, hi = (0, n // 2) if rank == 0 else (n // 2, n)
buf[lo:hi] = allv[lo:hi]
t = torch.from_numpy(buf)
dist.all_reduce(t, op=dist.ReduceOp.SUM)
assert np.array_equal(buf, allv), (rank, buf, allv)
# the library's own partition must give the same split on every rank
sys.path.insert(0, os.environ["REPO"])
import fscl_amd
cost = np.arange(1, 101, dtype=np.float64)
spans = [fscl_amd.partition(cost, r, world) for r in range(world)]
assert spans[0][0] == 0 and spans[-1][1] == 100 and spans[0][1] == spans[1][0]
dist.destroy_process_group()
print("ok", rank)
"""


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_int64_sum_exchange_preserves_bit_patterns(built, tmp_path):
    script = tmp_path / "w.py"
    script.write_text(WORKER)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), WORLD_SIZE="2", REPO=str(ROOT))
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    for p in procs:
        out, err = p.communicate(timeout=300)
        assert p.returncode == 0, err
        assert "ok" in out.split(), out
