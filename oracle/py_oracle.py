"""TEST INFRASTRUCTURE ONLY -- independent pure-Python restatement.

Written from the behaviour of /root/reference/lib/src/in_cksum.c, separately
from wc_oracle.c, so the two restatements cross-check each other.  Loops over
bytes: for small cases only.
"""
from __future__ import annotations


def word_sum(b: bytes) -> int:
    """Σ of little-endian 16-bit words, odd last byte as a low byte
    (in_cksum.c:107-120).  Returned as an exact (unbounded) integer."""
    total = 0
    for k in range(0, len(b) - 1, 2):
        total += b[k] | (b[k + 1] << 8)
    if len(b) % 2:
        total += b[-1]
    return total


def reduce16(acc: int) -> int:
    """in_cksum.c:74-80 on a uint32 accumulator."""
    acc &= 0xFFFFFFFF
    while acc >> 16:
        acc = (acc & 0xFFFF) + (acc >> 16)
    return (~acc) & 0xFFFF


def ip_cksum(buf: bytes, length: int | None = None) -> int:
    """in_cksum.c:133-137."""
    length = len(buf) if length is None else length
    return reduce16(word_sum(bytes(buf[:length])))


def payload_sum(buf: bytes, length: int) -> int:
    """in_cksum.c:140-164, accumulator mod 2^32 (the reference's uint32)."""
    b = bytes(buf)
    if b[0] >> 4 == 4:
        hl = (b[0] & 0x0F) * 4
        acc = b[9] << 8
        acc += word_sum(b[12:16]) + word_sum(b[16:20])
        plen = (((b[2] << 8) | b[3]) - hl) & 0xFFFF
        acc += ((plen & 0xFF) << 8) | (plen >> 8)  # network order read natively
    else:
        hl = 40
        acc = b[6] << 24
        acc += word_sum(b[8:24]) + word_sum(b[24:40]) + word_sum(b[4:6])
    if length < hl:
        raise ValueError("len < IP header length (the reference reads ~4 GiB)")
    acc += word_sum(b[hl:length])
    return acc & 0xFFFFFFFF


def payload_cksum(buf: bytes, length: int | None = None) -> int:
    length = len(buf) if length is None else length
    return reduce16(payload_sum(buf, length))


def ip_hdr_cksum(buf: bytes) -> int:
    """What ip4_rx checks / mk_ip4_hdr stores: ip_cksum(ip, ip4_hl(vhl))
    (ip4.c:110-115, 184-186) for IPv4; IPv6 has no header checksum -> 0."""
    b = bytes(buf)
    if b[0] >> 4 != 4:
        return 0
    return ip_cksum(b[: (b[0] & 0x0F) * 4])
