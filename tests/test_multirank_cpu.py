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


SHM_WORKER = r"""
import ctypes as C, os, sys
import numpy as np
sys.path.insert(0, os.environ["REPO"])
import fscl_amd
L = fscl_amd.get_lib()
L.fh_shm_open.restype = C.c_void_p
L.fh_shm_open.argtypes = [C.c_int, C.c_int, C.c_char_p, C.c_size_t]
L.fh_shm_allgather.restype = C.c_int
L.fh_shm_allgather.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int]
L.fh_shm_close.argtypes = [C.c_void_p]
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
m = L.fh_shm_open(rank, world, os.environ["SHM_NAME"].encode(), 1 << 20)
assert m, "attach"
rng = np.random.default_rng(7)
for it in range(200):  # many exchanges of varying sizes: both areas, every ordering
    n = int(rng.integers(0, 300))
    full = rng.integers(-2**62, 2**62, size=(n, 8), dtype=np.int64)  # 64-B items (fsclg_point_t)
    cost = rng.random(n) + 0.01
    lo, hi = fscl_amd.partition(cost, rank, world)
    buf = np.zeros_like(full)
    buf[lo:hi] = full[lo:hi]
    assert L.fh_shm_allgather(m, buf.ctypes.data, 64, n, lo, hi) == 0
    assert np.array_equal(buf, full), (rank, it)
L.fh_shm_close(m)
assert not os.path.exists("/dev/shm" + os.environ["SHM_NAME"])  # unlinked once all attached
print("ok", rank)
"""


@pytest.mark.parametrize("world", [2, 3])
def test_shared_memory_allgather(built, tmp_path, world):
    """The library's own multi-process exchange (ranks.c): every rank writes its cost-balanced
    contiguous share of a batch's 64-B results and reads the whole batch, 200 times over."""
    script = tmp_path / "s.py"
    script.write_text(SHM_WORKER)
    env = dict(os.environ, WORLD_SIZE=str(world), REPO=str(ROOT), SHM_NAME=f"/fscl_amd_test_{os.getpid()}_{world}",
               FSCL_AMD_RANK_TIMEOUT="60")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(world)]
    for p in procs:
        out, err = p.communicate(timeout=300)
        assert p.returncode == 0, err
        assert "ok" in out.split(), out


def test_stale_segment_of_a_dead_launch_is_replaced(built, tmp_path):
    """A launch whose rank 0 died before every rank attached leaves its segment (rank 0 unlinks the
    name only once all have attached).  The CLI's default name repeats across launches of one
    launcher, so the next launch's rank 0 removes a segment whose creator is gone, and
    its other ranks skip it: the ranks meet."""
    import signal
    import time
    script = tmp_path / "s.py"
    script.write_text(SHM_WORKER)
    name = f"/fscl_amd_test_stale_{os.getpid()}"
    env = dict(os.environ, WORLD_SIZE="2", REPO=str(ROOT), SHM_NAME=name, FSCL_AMD_RANK_TIMEOUT="60")
    dead = subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK="0"), stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True)  # waits for a rank 1 that never comes
    t0 = time.time()
    while not os.path.exists("/dev/shm" + name) and time.time() - t0 < 60:
        time.sleep(0.05)
    time.sleep(0.5)
    dead.send_signal(signal.SIGKILL)
    dead.communicate(timeout=60)
    assert os.path.exists("/dev/shm" + name)  # the stale segment
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in (1, 0)]  # rank 1 first: it must skip it
    try:
        for p in procs:
            out, err = p.communicate(timeout=300)
            assert p.returncode == 0, err
            assert "ok" in out.split(), out
    finally:
        if os.path.exists("/dev/shm" + name):
            os.unlink("/dev/shm" + name)


def test_segment_of_another_pid_namespace_counts_as_live(built):
    """A creator pid means something only in the creator's pid namespace: a segment whose
    header names a pid that is dead HERE but another namespace is a live job in another container
    sharing /dev/shm.  Rank 0 must not unlink it (it fails with 'already exists' instead)."""
    import ctypes as C
    import struct
    import fscl_amd
    L = fscl_amd.get_lib()
    L.fh_shm_open.restype = C.c_void_p
    L.fh_shm_open.argtypes = [C.c_int, C.c_int, C.c_char_p, C.c_size_t]
    name = f"/fscl_amd_test_ns_{os.getpid()}"
    dead_pid = subprocess.run([sys.executable, "-c", "import os; print(os.getpid())"], capture_output=True,
                              text=True).stdout.strip()
    ns = os.stat("/proc/self/ns/pid").st_ino
    # arrive u64, attached u32, magic u32, world u32, creator u32, cap u64, creator_ns u64 (ranks.c shm_hdr_t)
    hdr = struct.pack("<QIIIIQQ", 0, 0, 0x6673636C, 2, int(dead_pid), 1 << 20, ns + 1)
    path = "/dev/shm" + name
    try:
        with open(path, "wb") as f:
            f.write(hdr + b"\0" * (4096 * 4 - len(hdr)))
        assert L.fh_shm_open(0, 2, name.encode(), 1 << 20) is None
        assert os.path.exists(path)  # left alone
        # the same header in OUR namespace: the creator is provably gone, the segment is replaced
        with open(path, "r+b") as f:
            f.write(struct.pack("<QIIIIQQ", 0, 0, 0x6673636C, 2, int(dead_pid), 1 << 20, ns))
        env = dict(os.environ, WORLD_SIZE="2", REPO=str(ROOT), SHM_NAME=name, FSCL_AMD_RANK_TIMEOUT="60")
        import tempfile
        with tempfile.TemporaryDirectory() as td:
            script = Path(td) / "s.py"
            script.write_text(SHM_WORKER)
            procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r)),
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in (1, 0)]
            for p in procs:
                out, err = p.communicate(timeout=300)
                assert p.returncode == 0, err
    finally:
        if os.path.exists(path):
            os.unlink(path)


def test_device_shares_are_contiguous_and_cover(built):
    """world * n_dev shares (rank r's local device l takes share r * n_dev + l): consecutive,
    disjoint, covering, and each rank's devices form one contiguous range."""
    import fscl_amd
    rng = np.random.default_rng(3)
    for n in (0, 1, 7, 100, 5000):
        cost = rng.random(n) * 10 + 0.1
        for world, n_dev in ((1, 2), (2, 2), (2, 4), (4, 2), (1, 8)):
            T = world * n_dev
            spans = [fscl_amd.partition(cost, g, T) for g in range(T)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for a, b in zip(spans, spans[1:]):
                assert a[1] == b[0] and a[0] <= a[1]
            tot = cost.sum()
            for lo, hi in spans:  # no share far above its part of the cost
                assert cost[lo:hi].sum() <= tot / T + (cost.max() if n else 0) + 1e-9


SHM_CHECK_WORKER = r"""
import ctypes as C, os, sys
import numpy as np
sys.path.insert(0, os.environ["REPO"])
import fscl_amd
L = fscl_amd.get_lib()
L.fh_shm_open.restype = C.c_void_p
L.fh_shm_open.argtypes = [C.c_int, C.c_int, C.c_char_p, C.c_size_t]
L.fh_shm_allgather_flags.restype = C.c_int
L.fh_shm_allgather_flags.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                     C.POINTER(C.c_uint)]
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
m = L.fh_shm_open(rank, world, os.environ["SHM_NAME"].encode(), 1 << 20)
assert m, "attach"
buf = np.zeros(16, dtype=np.int64)
for it in range(50):  # the OR of every rank's flag word, the same on every rank
    f = C.c_uint((1 << rank) if it % (rank + 2) == 0 else 0)
    assert L.fh_shm_allgather_flags(m, buf.ctypes.data, 8, 16, 0, 0, C.byref(f)) == 0
    want = sum(1 << r for r in range(world) if it % (r + 2) == 0)
    assert f.value == want, (rank, it, f.value, want)
# control flow diverges: rank 1 exchanges a batch of a different size -> every rank fails
n = 16 if rank != 1 else 12
f = C.c_uint(0)
r = L.fh_shm_allgather_flags(m, buf.ctypes.data, 8, n, 0, 0, C.byref(f))
assert r != 0, "size mismatch not detected"
print("ok", rank)
"""


def test_shared_memory_exchange_flags_and_divergence(built, tmp_path):
    """ranks.c: every exchange carries a flag word (the OR over ranks: the collective SIGINT
    dump decision) and a (sequence, size) check -- ranks that exchange different batches
    fail instead of mixing results."""
    script = tmp_path / "c.py"
    script.write_text(SHM_CHECK_WORKER)
    env = dict(os.environ, WORLD_SIZE="3", REPO=str(ROOT), SHM_NAME=f"/fscl_amd_testc_{os.getpid()}",
               FSCL_AMD_RANK_TIMEOUT="60")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(3)]
    for p in procs:
        out, err = p.communicate(timeout=300)
        assert p.returncode == 0, err
        assert "ok" in out.split(), out
        assert "rank exchange mismatch" in err


POOL_WORKER = r"""
import ctypes as C, os, sys, time
import numpy as np
sys.path.insert(0, os.environ["REPO"])
import fscl_amd
L = fscl_amd.get_lib()
L.fh_shm_open.restype = C.c_void_p
L.fh_shm_open.argtypes = [C.c_int, C.c_int, C.c_char_p, C.c_size_t]
L.fh_pool_open.restype = C.c_void_p
L.fh_pool_open.argtypes = [C.c_void_p, C.c_size_t]
L.fh_pool_data.restype = C.c_void_p
L.fh_pool_data.argtypes = [C.c_void_p]
L.fh_pool_bytes.restype = C.c_size_t
L.fh_pool_bytes.argtypes = [C.c_void_p]
Rand = C.c_int32 * 33  # fh_rand_t: r[31], f, b
L.fh_srand.argtypes = [C.c_void_p, C.c_uint]
L.fh_pool_publish.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, C.c_ulonglong]
L.fh_pool_take.argtypes = [C.c_void_p, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t), C.c_void_p,
                           C.POINTER(C.c_ulonglong)]
L.fh_pool_release.argtypes = [C.c_void_p]
L.fh_pool_wait_released.argtypes = [C.c_void_p]
L.fh_pool_close.argtypes = [C.c_void_p]
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
m = L.fh_shm_open(rank, world, os.environ["SHM_NAME"].encode(), 1 << 16)
assert m, "attach"
NB, BUF, K, T = 6, 4096, 4, 300
p = L.fh_pool_open(m, NB * BUF if rank == 0 else 0)
assert p and L.fh_pool_bytes(p) >= NB * BUF
base = L.fh_pool_data(p)
owner = [-1] * NB          # leader: the slot whose trial reads each buffer
slot_buf = [None] * K
rng = np.random.default_rng(rank)
for t in range(T):
    slot = t % K
    if t >= K:             # the slot's previous trial: this rank is done reading it
        L.fh_pool_release(p)
        if rank == 0:
            assert L.fh_pool_wait_released(p) == 0
            for b in range(NB):
                if owner[b] == slot:
                    owner[b] = -1
    if rank == 0:          # build trial t's "permutation" into a free buffer and publish it
        b = owner.index(-1)
        owner[b] = slot
        arr = np.frombuffer((C.c_char * BUF).from_address(base + b * BUF), dtype=np.uint8)
        arr[:] = t % 251
        g = Rand()
        L.fh_srand(g, t + 1)
        assert L.fh_pool_publish(p, b * BUF, b * BUF + 8, g, t) == 0
        slot_buf[slot] = b * BUF
    else:
        ro, no, nj = C.c_size_t(), C.c_size_t(), C.c_ulonglong()
        g = Rand()
        assert L.fh_pool_take(p, C.byref(ro), C.byref(no), g, C.byref(nj)) == 0
        want = Rand()
        L.fh_srand(want, t + 1)
        assert bytes(g) == bytes(want) and nj.value == t and no.value == ro.value + 8
        slot_buf[slot] = ro.value
    if rng.random() < 0.2:
        time.sleep(0.001)  # ranks out of step
    # every rank "reads" its slots still in flight: none was overwritten
    for back in range(min(K, t + 1)):
        tr = t - back
        arr = np.frombuffer((C.c_char * BUF).from_address(base + slot_buf[tr % K]), dtype=np.uint8)
        assert (arr[16:] == tr % 251).all(), (rank, t, tr)
for k in range(K):
    L.fh_pool_release(p)
if rank == 0:
    assert L.fh_pool_wait_released(p) == 0
L.fh_pool_close(p)
print("ok", rank)
"""


@pytest.mark.parametrize("world", [2, 3])
def test_permutation_pool_protocol(built, tmp_path, world):
    """ranks.c's node-leader pool: rank 0 writes 300 trials' buffers into a
    shared segment and publishes each with a rand() state; the other ranks take them in order
    (state and count intact) and release their row slots.  A buffer is reused only after every
    rank released the slot that read it: every rank checks, every trial, that the K trials it
    still has in flight keep their contents while the ranks drift out of step."""
    script = tmp_path / "p.py"
    script.write_text(POOL_WORKER)
    env = dict(os.environ, WORLD_SIZE=str(world), REPO=str(ROOT), SHM_NAME=f"/fscl_amd_testp_{os.getpid()}_{world}",
               FSCL_AMD_RANK_TIMEOUT="60")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(world)]
    for p in procs:
        out, err = p.communicate(timeout=300)
        assert p.returncode == 0, err
        assert "ok" in out.split(), out
    assert not list(Path("/dev/shm").glob(f"fscl_amd_testp_{os.getpid()}_{world}*"))
