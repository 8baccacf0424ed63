"""Gather-footprint model of the term loop (development aid).

For a C2-like chromosome, sample grid points, walk every coarse alpha plus the
refine grid of the first coarse value, and count per 64-lane wave instruction
the distinct 64-byte chunks touched by the log-table gather and by the
coefficient gathers under different layouts; also the interval histogram
(terms per interval), to size an LDS coefficient cache.
"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fscl_amd import synth  # noqa: E402

LOG_AD_MIN, LOG_AD_MAX = -20.0, 4.0
cfg = dict(synth.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C2"])
n_iv = 200
step = (LOG_AD_MAX - LOG_AD_MIN) / (n_iv + 1.0)
(name, pos, k, nn, fold), = synth.generate(seed=1, sweeps_per_chr=2, **{**cfg, "n_chr": 1})
pos = pos.astype(np.int64)
rows_used = np.unique(k)
rowid = np.searchsorted(rows_used, k)
stride = len(rows_used) + 1
cstep = (LOG_AD_MAX - LOG_AD_MIN) / 10.0
coarse = [LOG_AD_MIN + i * cstep for i in range(11)]
refine = [LOG_AD_MIN + (i + 1) * (cstep / 15.0) for i in range(14)]
las = coarse + refine


def lt_index(ad):
    return np.where(ad > 0xFFFFFF, (ad >> 16) + 131072, np.where(ad > 0xFFFF, (ad >> 8) + 65536, ad))


rng = np.random.default_rng(0)
hist = np.zeros(n_iv, np.int64)
chunks = {"lt": 0, "coef_inter2": 0, "coef_plane2": 0, "pos": 0}
waves = 0
for g in rng.integers(0, pos[-1], size=24):
    near = int(np.clip(np.searchsorted(pos, g), 0, len(pos) - 1))
    for la in las:
        ad = np.abs(pos - g)
        x = np.log(np.maximum(ad, 1)) + la
        ok = x <= LOG_AD_MAX
        # walk = contiguous ok range around near (approximately)
        lo = near
        while lo > 0 and ok[lo - 1]:
            lo -= 1
        hi = near
        while hi < len(pos) - 1 and ok[hi + 1]:
            hi += 1
        idx = np.arange(lo, hi + 1)
        xs = x[idx]
        iv = np.clip(((xs - LOG_AD_MIN) / step).astype(np.int64), 0, n_iv - 1)
        np.add.at(hist, iv, 1)
        r = rowid[idx]
        lt = lt_index(ad[idx])
        for w0 in range(0, len(idx), 64):
            sl = slice(w0, w0 + 64)
            waves += 1
            chunks["lt"] += len(np.unique(lt[sl] * 8 // 64))
            chunks["coef_inter2"] += 2 * len(np.unique((iv[sl] * stride + r[sl]) * 32 // 64))
            chunks["coef_plane2"] += 2 * len(np.unique((iv[sl] * stride + r[sl]) * 16 // 64))
            chunks["pos"] += 1
tot = hist.sum()
print(f"rows used {len(rows_used)}, waves {waves}, terms {tot}")
for kk, v in chunks.items():
    print(f"  {kk:12s} chunks/wave-instr {v / waves:6.1f}")
order = np.argsort(-hist)
cum = np.cumsum(hist[order]) / tot
for K in (10, 16, 21, 32, 43, 64):
    # best contiguous window of K intervals
    c = np.convolve(hist, np.ones(K, np.int64), mode="valid")
    b = int(np.argmax(c))
    print(f"  K={K:3d}: best window [{b},{b + K}) covers {c[b] / tot:.3f}; top-K set covers {cum[K - 1]:.3f}")

# wave-level hit/miss for a given window (argv[2], argv[3])
if len(sys.argv) > 3:
    w0, K = int(sys.argv[2]), int(sys.argv[3])
    anyhit = anymiss = both = wv = 0
    lanes_hit = lanes = 0
    for g in rng.integers(0, pos[-1], size=24):
        near = int(np.clip(np.searchsorted(pos, g), 0, len(pos) - 1))
        for la in las:
            ad = np.abs(pos - g)
            x = np.log(np.maximum(ad, 1)) + la
            ok = x <= LOG_AD_MAX
            lo = near
            while lo > 0 and ok[lo - 1]:
                lo -= 1
            hi = near
            while hi < len(pos) - 1 and ok[hi + 1]:
                hi += 1
            iv = np.clip(((x[lo:hi + 1] - LOG_AD_MIN) / step).astype(np.int64), 0, n_iv - 1)
            hit = (iv >= w0) & (iv < w0 + K)
            for j in range(0, len(iv), 64):
                h = hit[j:j + 64]
                wv += 1
                anyhit += h.any(); anymiss += (~h).any(); both += h.any() and (~h).any()
                lanes_hit += h.sum(); lanes += len(h)
    print(f"window [{w0},{w0 + K}): lane hit {lanes_hit / lanes:.3f}; waves any-hit {anyhit / wv:.3f} "
          f"any-miss {anymiss / wv:.3f} both {both / wv:.3f}")
