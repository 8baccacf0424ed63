#!/usr/bin/env python3
"""Expected results of the full-size BASELINE workloads that are too slow to run
the oracle live on the GPU box (test infrastructure).

For each case: regenerate the seeded synthetic input (fscl_amd/synth.py), run the
oracle (oracle/_build/fscl_oracle, the CPU restatement pinned by the golden
fixtures of make_golden.py) and store, in fullsize.json,
  * the SHA-256 of the input file (the box regenerates it and checks the digest),
  * the SHA-256 of the canonical scan-point dump (every field of every point, floats as
    C99 hex: canonical_dump() below) and of the output file,
  * every 97th dump row for diagnostics.

    python tests/golden/make_fullsize.py [case ...] [--threads N]

Cases (SURVEY §8(d) / BASELINE.json):
  C4_full_p2  22 x 45k SNPs (1.0M), n=200, --n-permute=2         (configs[3] genome)
  C5_full     22 x 227k SNPs (5.0M), n=400, initial scan          (configs[4] genome)
  C5_chr_p200 one C5 chromosome, --n-permute=200 (early prune)    (configs[4] regime)
  C4_bench_p1000  bench.py's default job exactly (seed 1), --n-permute=1000 (configs[3], the metric's job)
  C5_full_p25 the C5 genome (seed 55), --n-permute=25 (windowed null sums per trial, first prunes)
  C2_bench_p100, C3_bench_p100  bench.py --config C2 / C3 exactly (seed 1, 100 permutations)
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from fscl_amd import synth  # noqa: E402
from util import ORACLE, read_dump  # noqa: E402

CASES = {
    "C4_full_p2": dict(gen=dict(n_chr=22, chr_len=45_454_545, snps_per_chr=45_455, n=200, seed=44, sweeps_per_chr=2),
                       opts=["--n-permute=2"]),
    "C5_full": dict(gen=dict(n_chr=22, chr_len=227_272_727, snps_per_chr=227_273, n=400, seed=55, sweeps_per_chr=2),
                    opts=[]),
    "C5_chr_p200": dict(gen=dict(n_chr=1, chr_len=227_272_727, snps_per_chr=227_273, n=400, seed=57,
                                 sweeps_per_chr=2), opts=["--n-permute=200"]),
    # bench.py's own default job, exactly (seed 1, synth.CONFIGS["C4"], 1000 permutations): bench.py
    # checks every timed job's final points against this digest (parity scope "full job")
    "C4_bench_p1000": dict(gen=dict(n_chr=22, chr_len=45_454_545, snps_per_chr=45_455, n=200, folded=0.0, seed=1,
                                    sweeps_per_chr=2), opts=["--n-permute=1000"]),
    # the whole C5 genome with permutations: per-trial windowed null sums on every chromosome and
    # the first prune draws (permute_p reaches 20 only after 20 trials)
    "C5_full_p25": dict(gen=dict(n_chr=22, chr_len=227_272_727, snps_per_chr=227_273, n=400, folded=0.0, seed=55,
                                 sweeps_per_chr=2), opts=["--n-permute=25"]),
    # bench.py --config C2 / C3, exactly (seed 1, 100 permutations; C3 with its ascertainment
    # options, on ascertained sites -- synth.ascertained(), the reference's double-hit panel rule
    # ascbias-segments.c:88-101): their bench lines check every timed job against these digests too
    "C2_bench_p100": dict(gen=dict(n_chr=1, chr_len=200_000_000, snps_per_chr=100_000, n=100, folded=0.0, seed=1,
                                   sweeps_per_chr=2), opts=["--n-permute=100"]),
    "C3_bench_p100": dict(gen=dict(n_chr=1, chr_len=200_000_000, snps_per_chr=100_000, n=100, folded=0.3, seed=1,
                                   sweeps_per_chr=2, asc_depth=20, asc_min_freq=2),
                          opts=["--n-permute=100", "--asc-depth=20", "--asc-minimum-freq=2"]),
    # configs[4]'s permutation regime at its real depth: one whole C5 chromosome (chromosome 1 of
    # the seed-55 genome, i.e. bench.py --config C5 --chromosomes 1 --seed 55) with 10 000
    # permutations -- the early-prune tail: survivors running thousands of trials, per-trial
    # windowed null sums on few cells (scan-chromosome.c:412-546, prune :488-498, windows :92-94)
    "C5_chr_p10000": dict(gen=dict(n_chr=1, chr_len=227_272_727, snps_per_chr=227_273, n=400, folded=0.0, seed=55,
                                   sweeps_per_chr=2), opts=["--n-permute=10000"]),
}


def sha256_file(p: Path) -> str:
    h = hashlib.sha256()
    with open(p, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()


def canonical_row(r: tuple) -> str:
    return "\t".join(x.hex() if isinstance(x, float) else str(x) for x in r)


def canonical_dump(rows: list[tuple]) -> str:
    h = hashlib.sha256()
    for r in rows:
        h.update(canonical_row(r).encode())
        h.update(b"\n")
    return h.hexdigest()


def main(argv: list[str]) -> int:
    threads = os.cpu_count() or 1
    names = []
    it = iter(argv)
    for a in it:
        if a == "--threads":
            threads = int(next(it))
        else:
            names.append(a)
    names = names or list(CASES)
    fx_path = HERE / "fullsize.json"
    for name in names:
        c = CASES[name]
        with tempfile.TemporaryDirectory() as d:
            d = Path(d)
            snp = d / f"{name}.snp"
            synth.write_snp_file(str(snp), synth.generate(**c["gen"]))
            t0 = time.time()
            subprocess.run([str(ORACLE), "-f", str(snp), "-o", str(d / "o.txt"), f"--n-threads={threads}",
                            *c["opts"], f"--dump-points={d / 'o.dump'}"], check=True, capture_output=True)
            dt = time.time() - t0
            rows = read_dump(d / "o.dump")
            # re-read at write time: cases run concurrently (hours apart) must not drop each other's entries
            fx = json.loads(fx_path.read_text()) if fx_path.exists() else {}
            fx[name] = dict(gen=c["gen"], options=c["opts"], input_sha256=sha256_file(snp),
                            dump_sha256=canonical_dump(rows), out_sha256=sha256_file(d / "o.txt"),
                            n_points=len(rows), sum_permute_n=sum(r[10] for r in rows),
                            sample_every=97, sample=[canonical_row(r) for r in rows[::97]],
                            oracle_s=round(dt, 1), oracle_threads=threads)
        print(f"{name}: {len(rows)} points, oracle {dt:.1f} s on {threads} threads", flush=True)
        fx_path.write_text(json.dumps(fx, indent=1) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
