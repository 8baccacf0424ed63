"""Seeded synthetic inputs for fscl's SNP-frequency format (and ms format).

SURVEY §8(d): positions uniform without replacement on [1, L] per chromosome,
derived-allele counts drawn from the neutral spectrum (P(k) ∝ 1/k on
[1, n-1]), one sample depth, an optional fraction of folded sites, and
optionally planted sweeps that push nearby sites toward extreme frequencies
(the idea of the reference's sm-sample.c:164-212, with a much simpler
perturbation) so that some grid points survive permutation pruning.

Line format (snp-input.c:55): ``chr pos derived_count sample_size folded``.
"""
from __future__ import annotations

import numpy as np

# BASELINE.json configs (C1..C5); "lines" is what the generator writes.
CONFIGS = {
    "C1": dict(n_chr=1, chr_len=20_000_000, snps_per_chr=10_000, n=50, folded=0.0, n_permute=0),
    "C2": dict(n_chr=1, chr_len=200_000_000, snps_per_chr=100_000, n=100, folded=0.0, n_permute=100),
    "C3": dict(n_chr=1, chr_len=200_000_000, snps_per_chr=100_000, n=100, folded=0.3, n_permute=100,
               asc_depth=20, asc_min_freq=2),
    "C4": dict(n_chr=22, chr_len=45_454_545, snps_per_chr=45_455, n=200, folded=0.0, n_permute=1000),
    "C5": dict(n_chr=22, chr_len=227_272_727, snps_per_chr=227_273, n=400, folded=0.0, n_permute=10000),
}


def _positions(rng: np.random.Generator, length: int, count: int) -> np.ndarray:
    if count > length:
        raise ValueError("more SNPs than base pairs")
    pos = np.unique(rng.integers(1, length + 1, size=count + count // 8 + 16))
    while pos.size < count:
        pos = np.unique(np.concatenate([pos, rng.integers(1, length + 1, size=count)]))
    pos = rng.choice(pos, size=count, replace=False)
    pos.sort()
    return pos.astype(np.int64)


def _neutral_counts(rng: np.random.Generator, n: int, count: int) -> np.ndarray:
    k = np.arange(1, n, dtype=np.float64)
    p = 1.0 / k
    p /= p.sum()
    return rng.choice(np.arange(1, n), size=count, p=p)


def ascertained(rng: np.random.Generator, k: np.ndarray, n: int, asc_depth: int, asc_min_freq: int) -> np.ndarray:
    """Which sites an ascertainment panel of ``asc_depth`` of the n haplotypes would discover.

    The reference simulates ascertainment exactly this way (ascbias-segments.c:88-101): the
    first asc_depth haplotypes form the panel, d = derived copies among them, and with
    ``double_hit`` a site is kept iff 1 < d < asc_depth - 1, i.e. both alleles seen at least
    twice.  fscl's correction models the same event with K = --asc-minimum-freq
    (asc-bias.c:12-25: not ascertained iff d < K or asc_depth - d < K).  A random panel of
    haplotypes makes d hypergeometric(k derived, n - k ancestral, asc_depth draws)."""
    d = rng.hypergeometric(k, n - k, asc_depth)
    return (d >= asc_min_freq) & (asc_depth - d >= asc_min_freq)


def _chromosome_ascertained(rng, chr_len, count, n, sweeps_per_chr, sweep_scale, asc_depth, asc_min_freq):
    """One chromosome of ``count`` ascertained sites: a larger pool of sites (neutral spectrum,
    planted sweeps) is drawn, every site goes through the panel filter (ascertained()), and
    ``count`` of the kept sites are taken.  Planted-sweep sites go through the same filter; they
    are set to extreme but ascertainable counts (2..6 copies of one allele) instead of the
    unascertainable singletons of the unascertained configurations."""
    pool = 3 * count + 64
    while True:
        if pool > chr_len:
            raise ValueError("chromosome too short for the ascertained site count")
        pos = _positions(rng, chr_len, pool)
        k = _neutral_counts(rng, n, pool)
        for _ in range(sweeps_per_chr):
            centre = rng.integers(1, chr_len + 1)
            d = np.abs(pos - centre).astype(np.float64)
            hit = rng.random(pool) < np.exp(-d / sweep_scale)
            hi = rng.random(pool) < 0.15
            x = rng.integers(2, 7, size=pool)
            k = np.where(hit, np.where(hi, n - x, x), k)
        keep = np.nonzero(ascertained(rng, k, n, asc_depth, asc_min_freq))[0]
        if keep.size >= count:
            sel = np.sort(rng.choice(keep, size=count, replace=False))
            return pos[sel], k[sel]
        pool *= 2


def generate(n_chr: int, chr_len: int, snps_per_chr: int, n: int, folded: float = 0.0,
             seed: int = 1, sweeps_per_chr: int = 0, sweep_scale: float = 20_000.0,
             chr_names: list[str] | None = None, missing: float = 0.0, max_missing: int = 4,
             duplicates: float = 0.0, asc_depth: int = 0, asc_min_freq: int = 1, **_unused):
    """Return a list of per-chromosome (name, pos, k, n_arr, folded_arr) arrays.

    ``missing``: fraction of sites whose sample size is n - U{1..max_missing}
    (several sample depths, as with missing genotypes); ``duplicates``: fraction
    of sites moved onto the previous site's position (ties in position);
    ``asc_depth`` > 0: only sites an ascertainment panel of that many haplotypes
    discovers with both alleles seen ``asc_min_freq`` times (ascertained(): the data
    that fscl's -d / --asc-minimum-freq correction models), ``snps_per_chr`` of them."""
    rng = np.random.default_rng(seed)
    out = []
    for c in range(n_chr):
        name = chr_names[c] if chr_names else f"chr{c + 1}"
        if asc_depth > 0:
            pos, k = _chromosome_ascertained(rng, chr_len, snps_per_chr, n, sweeps_per_chr, sweep_scale,
                                             asc_depth, asc_min_freq)
        else:
            pos = _positions(rng, chr_len, snps_per_chr)
            k = _neutral_counts(rng, n, snps_per_chr)
            for _ in range(sweeps_per_chr):
                centre = rng.integers(1, chr_len + 1)
                d = np.abs(pos - centre).astype(np.float64)
                hit = rng.random(snps_per_chr) < np.exp(-d / sweep_scale)
                hi = rng.random(snps_per_chr) < 0.15
                k = np.where(hit, np.where(hi, n - 1, 1), k)
        fold = (rng.random(snps_per_chr) < folded).astype(np.int64)
        nn = np.full(snps_per_chr, n, dtype=np.int64)
        if missing > 0:
            m = rng.random(snps_per_chr) < missing
            nn = np.where(m, n - rng.integers(1, max_missing + 1, size=snps_per_chr), nn)
            k = np.minimum(k, nn - 1)
        if duplicates > 0:
            d = np.nonzero(rng.random(snps_per_chr) < duplicates)[0]
            d = d[d > 0]
            pos[d] = pos[d - 1]
        out.append((name, pos, k.astype(np.int64), nn, fold))
    return out


def write_snp_file(path: str, chroms) -> int:
    lines = 0
    with open(path, "w") as f:
        for name, pos, k, nn, fold in chroms:
            block = "\n".join(f"{name} {p} {kk} {m} {fo}" for p, kk, m, fo in zip(pos, k, nn, fold))
            f.write(block)
            f.write("\n")
            lines += len(pos)
    return lines


def write_config(path: str, config: str, seed: int = 1, scale: float = 1.0, sweeps_per_chr: int = 2) -> dict:
    """Write configuration ``config`` (optionally scaled down) and return its parameters."""
    cfg = dict(CONFIGS[config])
    if scale != 1.0:
        cfg["snps_per_chr"] = max(8, int(cfg["snps_per_chr"] * scale))
        cfg["chr_len"] = max(cfg["snps_per_chr"] * 4, int(cfg["chr_len"] * scale))
    write_snp_file(path, generate(seed=seed, sweeps_per_chr=sweeps_per_chr, **cfg))
    return cfg


def write_ms_file(path: str, n_blocks: int, n_hap: int, n_seg: int, seed: int = 1) -> None:
    """Hudson-ms style output: header, then per block ``//``, ``segsites``,
    ``positions`` in (0,1) with 8 decimals, and one 0/1 haplotype per line."""
    rng = np.random.default_rng(seed)
    with open(path, "w") as f:
        f.write(f"ms {n_hap} {n_blocks} -t 100.0\n1 2 3\n")
        for _ in range(n_blocks):
            pos = np.sort(rng.choice(np.arange(1, 10**8), size=n_seg, replace=False)) / 1e8
            freq = _neutral_counts(rng, n_hap, n_seg)
            hap = np.zeros((n_hap, n_seg), dtype=np.uint8)
            for j in range(n_seg):
                hap[rng.choice(n_hap, size=freq[j], replace=False), j] = 1
            f.write("\n//\nsegsites: %d\npositions: %s\n" % (n_seg, " ".join(f"{p:.8f}" for p in pos)))
            for h in range(n_hap):
                f.write("".join("1" if v else "0" for v in hap[h]) + "\n")
