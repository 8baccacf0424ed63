"""The oracle (CPU restatement) against the reference's own compiled code.

Golden fixtures under tests/golden/ were produced by oracle/_ref/ref_harness,
which runs the reference's load_snp_input / background_fsp /
compute_sweep_model_tables / search_maxalpha compiled from /root/reference
(tests/golden/make_golden.py).  Where /root/reference is present the harness is
also run live on fresh seeded inputs.
"""
from __future__ import annotations

import ctypes as C
import subprocess

import pytest

from util import GOLD, HARNESS, ORACLE, ROOT, assert_rows_equal, manifest, read_dump, run_oracle
from fscl_amd import synth


@pytest.mark.parametrize("case", sorted(manifest()["cases"]))
def test_oracle_matches_golden(built, tmp, case):
    c = manifest()["cases"][case]
    out, dump = tmp / "o.txt", tmp / "o.dump"
    run_oracle(GOLD / c["input"], out, c["options"], dump)
    assert out.read_text() == (GOLD / f"{case}.out").read_text()
    assert_rows_equal(read_dump(dump), read_dump(GOLD / f"{case}.dump"), case)


def test_oracle_threads_do_not_change_results(built, tmp):
    c = manifest()["cases"]["g1_p25"]
    run_oracle(GOLD / c["input"], tmp / "a", c["options"], tmp / "a.dump", threads=1)
    run_oracle(GOLD / c["input"], tmp / "b", c["options"], tmp / "b.dump", threads=4)
    assert (tmp / "a").read_bytes() == (tmp / "b").read_bytes()
    assert (tmp / "a.dump").read_bytes() == (tmp / "b.dump").read_bytes()


def test_throughput_mode_restatement(built, tmp):
    """The oracle's restatement of the product's throughput mode (--throughput-seed): thread
    count does not change it, another seed does, and its permutation counts follow the
    reference's procedure (N+1 trials for surviving points; a pruned point stopped at a hit
    with permute_p >= 20)."""
    c = manifest()["cases"]["g1_p25"]
    snp = GOLD / c["input"]
    opts = ["--n-permute=60"]
    run_oracle(snp, tmp / "a", [*opts, "--throughput-seed=7"], tmp / "a.dump", threads=1)
    run_oracle(snp, tmp / "b", [*opts, "--throughput-seed=7"], tmp / "b.dump", threads=4)
    run_oracle(snp, tmp / "c", [*opts, "--throughput-seed=8"], tmp / "c.dump", threads=4)
    assert (tmp / "a.dump").read_bytes() == (tmp / "b.dump").read_bytes()
    assert (tmp / "a.dump").read_bytes() != (tmp / "c.dump").read_bytes()
    rows = read_dump(tmp / "a.dump")
    for r in rows:
        p, n, fin = r[9], r[10], r[11]
        assert (n == 61 and not fin) or (fin and p >= 20 and n < 61) or (fin and n == 61)
    assert any(r[11] for r in rows)


def _glibc_stream(seed: int, n: int) -> list[int]:
    libc = C.CDLL("libc.so.6")
    libc.srand(seed)
    return [libc.rand() for _ in range(n)]


def test_rand_restatements_match_glibc(built):
    """oracle.c's and the product's glibc TYPE_3 streams vs libc's rand()."""
    want = _glibc_stream(0xFD821A6, 5000)
    orc = C.CDLL(str(ROOT / "oracle" / "_build" / "liboracle.so"))
    st = C.create_string_buffer(256)
    orc.orc_srand(st, C.c_uint(0xFD821A6))
    assert [orc.orc_rand(st) for _ in range(5000)] == want
    import fscl_amd
    L = fscl_amd.get_lib()
    st2 = C.create_string_buffer(256)
    L.fh_srand(st2, 0xFD821A6)
    assert [L.fh_rand(st2) for _ in range(5000)] == want
    for seed in (0, 1, 12345, 2**31 + 7):
        L.fh_srand(st2, seed)
        assert [L.fh_rand(st2) for _ in range(300)] == _glibc_stream(seed, 300)


@pytest.mark.skipif(not HARNESS.exists(), reason="needs /root/reference (oracle/_ref)")
@pytest.mark.parametrize("seed,opts", [
    (7, ["--n-permute=12"]),
    (8, ["--asc-depth=6", "--asc-minimum-freq=1", "--n-permute=8"]),
    (9, ["--coarse-grid-spacing=30000"]),
])
def test_oracle_matches_live_reference(built, tmp, seed, opts):
    snp = tmp / "x.snp"
    synth.write_snp_file(str(snp), synth.generate(n_chr=2, chr_len=900_000, snps_per_chr=900, n=14, folded=0.3,
                                                  seed=seed, sweeps_per_chr=1, missing=0.15, max_missing=3))
    r = subprocess.run([str(HARNESS), "scan", str(snp), str(tmp / "r.out"), str(tmp / "r.dump"), *opts],
                       capture_output=True, text=True)
    if r.returncode == 3:
        pytest.skip("a trial hit the reference's negative-j bug; not comparable")
    assert r.returncode == 0, r.stderr
    run_oracle(snp, tmp / "o.out", opts, tmp / "o.dump")
    assert (tmp / "o.out").read_text() == (tmp / "r.out").read_text()
    assert_rows_equal(read_dump(tmp / "o.dump"), read_dump(tmp / "r.dump"), f"seed {seed}")


@pytest.mark.skipif(not HARNESS.exists(), reason="needs /root/reference (oracle/_ref)")
def test_reference_harness_threads_do_not_change_results(built, tmp):
    """bench.py times the reference's own search_maxalpha on OpenMP threads (its
    cpu_baseline leg): the threaded harness gives the single-threaded results."""
    c = manifest()["cases"]["g1_p25"]
    outs = []
    for th in (1, 4):
        r = subprocess.run([str(HARNESS), "scan", str(GOLD / c["input"]), str(tmp / f"h{th}.out"),
                            str(tmp / f"h{th}.dump"), f"--n-threads={th}"], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        assert "scan_s=" in r.stderr
        outs.append(((tmp / f"h{th}.out").read_bytes(), (tmp / f"h{th}.dump").read_bytes()))
    assert outs[0] == outs[1]


def test_oracle_cli_rejects_bad_options(built, tmp):
    r = subprocess.run([str(ORACLE), "-o", str(tmp / "x")], capture_output=True, text=True)
    assert r.returncode != 0
    r = subprocess.run([str(ORACLE), "-f", str(GOLD / "g1.snp"), "-o", str(tmp / "x"), "--splines=100"],
                       capture_output=True, text=True)
    assert r.returncode != 0
