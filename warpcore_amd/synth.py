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


def make_rx_ring(buf, n: int, ip_lens, slot: int = 2048, v6_every: int = 3, packed: bool = False):
    """A netmap RX ring of well-formed UDP frames in `buf` (uint8 device
    tensor of >= n * slot bytes, already filled with synthetic bytes): frame i
    in slot i, an Ethernet header (random MACs, EtherType per version,
    eth.h:44-53) and an IPv4 (IHL 5, DF, no fragment offset) or IPv6 UDP
    datagram of ip_lens[i] bytes at +14 (stamp_udp_headers), its IPv4 header
    checksum and UDP checksum computed on the device (wc_cksum_ip_udp_ragged)
    and stored raw, as mk_ip4_hdr / udp_tx do (ip4.c:184-186, udp.c:209-213).
    `packed`: frames back to back instead (frame i right after frame i - 1,
    any alignment; `buf` needs >= sum of the frame lengths).
    Returns (frame offsets uint64, frame lengths uint16) as numpy arrays."""
    import torch

    from . import cksum

    dev = buf.device
    ip_lens = np.asarray(ip_lens, dtype=np.uint16)
    f_len = (ip_lens.astype(np.int64) + 14).astype(np.uint16)
    f_off = (packed_offsets(f_len) if packed
             else (np.arange(n, dtype=np.uint64) * slot).astype(np.uint64))
    d_foff = torch.from_numpy(f_off.astype(np.int64)).to(dev)
    d_ipoff = d_foff + 14
    d_iplen = torch.from_numpy(ip_lens.astype(np.int64)).to(dev)
    stamp_udp_headers(buf, d_ipoff, d_iplen, v6_every=v6_every)
    v6 = (torch.arange(n, device=dev) % v6_every) == 0
    # EtherType (network order) and, for IPv4, DF with a zero fragment
    # offset and a zero header checksum field before it is computed.
    buf[d_foff + 12] = torch.where(v6, 0x86, 0x08).to(torch.uint8)
    buf[d_foff + 13] = torch.where(v6, 0xDD, 0x00).to(torch.uint8)
    o4 = d_ipoff[~v6]
    for at, val in ((6, 0x40), (7, 0), (10, 0), (11, 0)):
        buf[o4 + at] = val
    hdr, pay = cksum.cksum_ip_udp_ragged(buf, d_ipoff.to(torch.int64).view(torch.int64),
                                         d_iplen.to(torch.int16), check=False)
    h = hdr.view(torch.int16).to(torch.int32) & 0xFFFF
    p = pay.view(torch.int16).to(torch.int32) & 0xFFFF
    buf[o4 + 10] = (h[~v6] & 0xFF).to(torch.uint8)
    buf[o4 + 11] = (h[~v6] >> 8).to(torch.uint8)
    ucs = d_ipoff + torch.where(v6, 46, 26)
    buf[ucs] = (p & 0xFF).to(torch.uint8)
    buf[ucs + 1] = (p >> 8).to(torch.uint8)
    return f_off, f_len


def stamp_udp_headers(buf, offs, lens, v6_every: int = 3, chunk: int = 1 << 21) -> None:
    """Turn packet i of a synthetic batch into a well-formed UDP datagram in
    place, on the device: IPv6 (every `v6_every`-th packet) or IPv4 with IHL 5
    (ip4.h:55-66, ip6.h:45-57, udp.h:41-46), next header / protocol 17, IP
    and UDP lengths matching `lens`, UDP checksum 0.  The other header bytes
    (ports, addresses, TTL, ...) stay random.  This is what a netmap TX queue
    or RX ring holds, as opposed to random bytes read as IP headers (random
    version, IHL and next_hdr).  `buf`: uint8 device tensor; `offs` / `lens`:
    packet offsets and lengths (numpy or tensors); every len >= 48."""
    import torch

    dev = buf.device
    n = int(offs.shape[0])
    o_all = torch.as_tensor(np.asarray(offs, dtype=np.int64) if isinstance(offs, np.ndarray)
                            else offs.to(torch.int64), device=dev)
    l_all = torch.as_tensor(np.asarray(lens, dtype=np.int64) if isinstance(lens, np.ndarray)
                            else lens.to(torch.int64) & 0xFFFF, device=dev)
    for s in range(0, n, chunk):
        o = o_all[s:s + chunk]
        ln = l_all[s:s + chunk]
        v6 = (torch.arange(s, s + o.numel(), device=dev) % v6_every) == 0
        for sel, fields in (
            (~v6, lambda L: [(0, 0x45), (2, L >> 8), (3, L), (9, 17),
                             (24, (L - 20) >> 8), (25, L - 20), (26, 0), (27, 0)]),
            (v6, lambda L: [(0, 0x60), (4, (L - 40) >> 8), (5, L - 40), (6, 17),
                            (44, (L - 40) >> 8), (45, L - 40), (46, 0), (47, 0)]),
        ):
            oo, LL = o[sel], ln[sel]
            for at, val in fields(LL):
                v = val if torch.is_tensor(val) else torch.full_like(oo, val)
                buf[oo + at] = (v & 0xFF).to(torch.uint8)
