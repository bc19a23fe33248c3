"""Synthetic packet batches for the benchmark configurations (BASELINE.json).

* payload bytes: the counter-based splitmix64 stream, generated on the device
  by ``wc_synth_fill`` (8-byte word k = splitmix64 output k for the seed), so
  a host can regenerate identical bytes for checking;
* C4 lengths: Zipf(s = 1) over ranks 1..1409 mapped to 64..1472 B, packed
  with no padding (arbitrary start alignment), offsets = uint64 prefix sum.
"""
from __future__ import annotations

import numpy as np

SEED = 0x5EED
ZIPF_SEED = 0xC0FFEE


def zipf_lengths(n: int, seed: int = ZIPF_SEED, lo: int = 64, hi: int = 1472,
                 s: float = 1.0) -> np.ndarray:
    """n packet lengths, P(lo - 1 + r) ∝ r^-s for rank r in 1..hi-lo+1."""
    ranks = np.arange(1, hi - lo + 2, dtype=np.float64)
    cdf = np.cumsum(ranks ** -s)
    cdf /= cdf[-1]
    u = np.random.default_rng(seed).random(n)
    r = np.searchsorted(cdf, u, side="right")
    return (lo + np.minimum(r, ranks.size - 1)).astype(np.uint16)


def packed_offsets(lengths: np.ndarray, lead: int = 0) -> np.ndarray:
    off = np.empty(lengths.size, dtype=np.uint64)
    off[0:1] = lead
    np.cumsum(lengths[:-1], dtype=np.uint64, out=off[1:])
    if lead:
        off[1:] += np.uint64(lead)
    return off
