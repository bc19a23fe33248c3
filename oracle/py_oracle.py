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


RX_OK, RX_OK_NO_CKSUM, RX_BAD_IP_CKSUM, RX_BAD_UDP_CKSUM, RX_SHORT, RX_FRAGMENT, \
    RX_BAD_VERSION, RX_NOT_UDP, RX_NOT_IP, RX_TRUNCATED = range(10)
RX_DROPS = {RX_BAD_IP_CKSUM, RX_BAD_UDP_CKSUM, RX_SHORT, RX_FRAGMENT, RX_BAD_VERSION,
            RX_TRUNCATED}


def rx_verdict(frame: bytes, flen: int | None = None) -> int:
    """The checksum / format decision of the reference's RX path for one
    Ethernet frame: eth_rx (eth.c:75-86) -> ip4_rx (ip4.c:95-138) / ip6_rx
    (ip6.c:91-111) -> udp_rx (udp.c:99-139).  Only frame bytes [0, flen) are
    read; whatever the reference would read past them is RX_TRUNCATED."""
    f = bytes(frame)
    flen = len(f) if flen is None else flen
    f = f[:flen]
    if flen < 14:
        return RX_TRUNCATED
    etype = (f[12] << 8) | f[13]
    if etype not in (0x0800, 0x86DD):
        return RX_NOT_IP
    ip = f[14:]
    if not ip:
        return RX_TRUNCATED
    want_v = 4 if etype == 0x0800 else 6
    if ip[0] >> 4 != want_v:
        return RX_BAD_VERSION
    if want_v == 4:
        hl = (ip[0] & 0x0F) * 4
        if len(ip) < max(hl, 20):
            return RX_TRUNCATED
        if ip_cksum(ip[:hl]) != 0:
            return RX_BAD_IP_CKSUM
        off_native = ip[6] | (ip[7] << 8)
        if off_native & 0xFF1F:          # IP4_OFFMASK, network byte order
            return RX_FRAGMENT
        proto = ip[9]
        ip_plen = (((ip[2] << 8) | ip[3]) - hl) & 0xFFFF
    else:
        hl = 40
        if len(ip) < 40:
            return RX_TRUNCATED
        proto = ip[6]
        ip_plen = (ip[4] << 8) | ip[5]
    if proto != 17:
        return RX_NOT_UDP
    if ip_plen < 8:
        return RX_SHORT
    if len(ip) < hl + 8:
        return RX_TRUNCATED
    udp = ip[hl:hl + 8]
    udp_len = min((udp[4] << 8) | udp[5], ip_plen)
    if udp[6] == 0 and udp[7] == 0:
        return RX_OK_NO_CKSUM
    plen = udp_len + hl
    if len(ip) < max(plen, 20):
        return RX_TRUNCATED
    return RX_BAD_UDP_CKSUM if payload_cksum(ip, plen) != 0 else RX_OK


def ip_hdr_cksum(buf: bytes) -> int:
    """What ip4_rx checks / mk_ip4_hdr stores: ip_cksum(ip, ip4_hl(vhl))
    (ip4.c:110-115, 184-186) for IPv4; IPv6 has no header checksum -> 0."""
    b = bytes(buf)
    if b[0] >> 4 != 4:
        return 0
    return ip_cksum(b[: (b[0] & 0x0F) * 4])
