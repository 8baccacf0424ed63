"""Test helpers: run the oracle (CPU restatement) and read scan-point dumps."""
from __future__ import annotations

import json
import os
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
GOLD = ROOT / "tests" / "golden"
ORACLE = ROOT / "oracle" / "_build" / "fscl_oracle"
HARNESS = ROOT / "oracle" / "_ref" / "ref_harness"
CLI = ROOT / "fscl_amd" / "_build" / "fscl"

DUMP_FIELDS = ("chr", "sweep_pos", "clr", "lalpha", "sm_logl", "null_logl", "nearest_snp", "window_start",
               "window_end", "permute_p", "permute_n", "permute_finished")


def manifest() -> dict:
    return json.loads((GOLD / "manifest.json").read_text())


def read_dump(path) -> list[tuple]:
    """oracle/harness dump: ints and hex floats (C %a) per point."""
    rows = []
    for line in Path(path).read_text().splitlines():
        f = line.split("\t")
        rows.append((int(f[0]), int(f[1]), float.fromhex(f[2]), float.fromhex(f[3]), float.fromhex(f[4]),
                     float.fromhex(f[5]), int(f[6]), int(f[7]), int(f[8]), int(f[9]), int(f[10]), int(f[11])))
    return rows


def points_rows(pts) -> list[tuple]:
    """numpy POINT_DTYPE array -> the dump's tuple layout."""
    return [tuple(p[k].item() for k in DUMP_FIELDS) for p in pts]


def usable_cpus() -> int:
    """CPUs this process may run on: the affinity mask, capped by the cgroup v2 CPU quota
    (a GPU box's share of its node)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return n


def run_oracle(snp, out, opts, dump=None, threads: int | None = None) -> subprocess.CompletedProcess:
    """The oracle CLI; threads default to every CPU this process may use."""
    cmd = [str(ORACLE), "-f", str(snp), "-o", str(out), f"--n-threads={threads or usable_cpus()}", *opts]
    if dump:
        cmd.append(f"--dump-points={dump}")
    return subprocess.run(cmd, capture_output=True, text=True, check=True)


def same_bits(a: float, b: float) -> bool:
    return a.hex() == b.hex() or (a != a and b != b)


def assert_rows_equal(got: list[tuple], want: list[tuple], what: str = "") -> None:
    assert len(got) == len(want), f"{what}: {len(got)} points vs {len(want)}"
    for i, (g, w) in enumerate(zip(got, want)):
        for k, (x, y) in enumerate(zip(g, w)):
            ok = same_bits(x, y) if isinstance(x, float) else x == y
            assert ok, f"{what}: point {i} field {DUMP_FIELDS[k]}: {x!r} != {y!r} (row {g} vs {w})"
