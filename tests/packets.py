"""Packet builders for tests (IPv4 / IPv6 + UDP, reference header layouts
ip4.h:55-66, ip6.h:45-57, udp.h:41-46).

Each builder returns (packet_bytes, len_arg) where len_arg is what the
reference passes to payload_cksum: IP header length + UDP length
(udp.c:134 on RX, udp.c:213 on TX where v->len covers the same bytes).
"""
from __future__ import annotations

import numpy as np


def _u16be(v: int) -> bytes:
    return bytes([(v >> 8) & 0xFF, v & 0xFF])


def ipv4_udp(payload: bytes, rng: np.random.Generator, ihl: int = 5,
             proto: int = 17, tot_len_delta: int = 0) -> tuple[bytes, int]:
    hl = ihl * 4
    udp_len = 8 + len(payload)
    tot = (hl + udp_len + tot_len_delta) & 0xFFFF
    hdr = bytearray(hl)
    hdr[0] = 0x40 | (ihl & 0x0F)
    hdr[1] = int(rng.integers(0, 256))                 # tos
    hdr[2:4] = _u16be(tot)
    hdr[4:6] = rng.integers(0, 256, 2, dtype=np.uint8).tobytes()  # id
    hdr[6:8] = b"\x40\x00"                             # DF
    hdr[8] = int(rng.integers(1, 256))                 # ttl
    hdr[9] = proto
    hdr[12:20] = rng.integers(0, 256, 8, dtype=np.uint8).tobytes()  # src, dst
    if hl > 20:
        hdr[20:hl] = rng.integers(0, 256, hl - 20, dtype=np.uint8).tobytes()
    udp = bytearray(8)
    udp[0:4] = rng.integers(0, 256, 4, dtype=np.uint8).tobytes()    # ports
    udp[4:6] = _u16be(udp_len & 0xFFFF)
    pkt = bytes(hdr) + bytes(udp) + payload
    return pkt, hl + udp_len


def ipv6_udp(payload: bytes, rng: np.random.Generator,
             next_hdr: int = 17) -> tuple[bytes, int]:
    udp_len = 8 + len(payload)
    hdr = bytearray(40)
    hdr[0] = 0x60
    hdr[1:4] = rng.integers(0, 256, 3, dtype=np.uint8).tobytes()
    hdr[4:6] = _u16be(udp_len & 0xFFFF)
    hdr[6] = next_hdr
    hdr[7] = int(rng.integers(1, 256))
    hdr[8:40] = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    udp = bytearray(8)
    udp[0:4] = rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
    udp[4:6] = _u16be(udp_len & 0xFFFF)
    return bytes(hdr) + bytes(udp) + payload, 40 + udp_len


def udp_cksum_offset(pkt: bytes) -> int:
    """Byte offset of udp->cksum inside an IP packet built above."""
    hl = (pkt[0] & 0x0F) * 4 if pkt[0] >> 4 == 4 else 40
    return hl + 6


def insert_checksum(pkt: bytes, cksum: int) -> bytes:
    """Store the native uint16 result raw, as udp.c:213 does."""
    o = udp_cksum_offset(pkt)
    b = bytearray(pkt)
    b[o] = cksum & 0xFF
    b[o + 1] = cksum >> 8
    return bytes(b)


def random_packets(rng: np.random.Generator, count: int, max_payload: int = 1472,
                   v6_share: float = 0.5, wild: bool = False) -> list[tuple[bytes, int]]:
    """Mixed IPv4/IPv6 UDP packets; `wild` adds IPv4 options, odd lengths,
    large next_hdr values (uint32 wrap in in_cksum.c:157) and short IHLs."""
    pkts = []
    for _ in range(count):
        plen = int(rng.integers(0, max_payload + 1))
        payload = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
        if rng.random() < v6_share:
            nh = int(rng.integers(0, 256)) if wild else 17
            pkts.append(ipv6_udp(payload, rng, next_hdr=nh))
        else:
            ihl = int(rng.integers(5, 16)) if wild and rng.random() < 0.5 else 5
            pkts.append(ipv4_udp(payload, rng, ihl=ihl,
                                 tot_len_delta=int(rng.integers(-3, 4)) if wild else 0))
    return pkts


def _u16le_store(b: bytearray, at: int, v: int) -> None:
    b[at] = v & 0xFF
    b[at + 1] = (v >> 8) & 0xFF


def finish_udp(pkt: bytes, zero_udp: bool = False) -> bytes:
    """TX side of the reference on an IP packet built above: the IPv4 header
    checksum over [0, hl) with the field 0 (ip4.c:184-186), then the UDP
    checksum with the field 0 (udp.c:209-213), both stored raw.  A computed
    UDP checksum of 0 is sent as 0, i.e. "no checksum" (udp.c:212)."""
    from oracle import py_oracle  # test infrastructure
    b = bytearray(pkt)
    v4 = b[0] >> 4 == 4
    hl = (b[0] & 0x0F) * 4 if v4 else 40
    if v4:
        b[10:12] = b"\x00\x00"
        _u16le_store(b, 10, py_oracle.ip_cksum(bytes(b[:hl])))
    o = hl + 6
    b[o:o + 2] = b"\x00\x00"
    if not zero_udp:
        ln = hl + ((b[hl + 4] << 8) | b[hl + 5])
        _u16le_store(b, o, py_oracle.payload_cksum(bytes(b), min(ln, len(b))))
    return bytes(b)


def eth_frame(ip_pkt: bytes, rng: np.random.Generator, etype: int = 0x0800) -> bytes:
    """Ethernet II frame around an IP packet (eth.h:44-53): random MACs."""
    return rng.integers(0, 256, 12, dtype=np.uint8).tobytes() + _u16be(etype) + ip_pkt


RX_CASES = ("ok4", "ok6", "ok4opt", "nocksum", "badudp", "badip", "frag", "mf", "short", "icmp4",
            "icmp6", "arp", "badver", "trunc", "ulen_big", "ulen_small", "totlen_wrap",
            "ihl_small", "garbage", "tiny")


def rx_frame(rng: np.random.Generator, case: str, max_payload: int = 1472) -> tuple[bytes, int]:
    """One Ethernet frame of an RX ring exercising `case` of the reference's
    RX checks (ip4.c:95-138, ip6.c:91-111, udp.c:99-139); returns (bytes,
    frame length), the length possibly shorter than the bytes (a truncated
    slot: what lies past it is not part of the frame)."""
    plen = int(rng.integers(0, max_payload + 1))
    payload = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
    v6 = case in ("ok6", "icmp6") or (case in ("nocksum", "badudp", "short", "trunc",
                                               "ulen_big", "ulen_small") and rng.random() < 0.4)
    ihl = int(rng.integers(6, 16)) if case == "ok4opt" else 5
    if case == "arp":
        fr = eth_frame(rng.integers(0, 256, 28, dtype=np.uint8).tobytes(), rng, 0x0806)
        return fr, len(fr)
    if case == "garbage":
        body = bytearray(rng.integers(0, 256, int(rng.integers(1, 200)), dtype=np.uint8).tobytes())
        et = 0x0800 if rng.random() < 0.5 else 0x86DD
        body[0] = ((4 if et == 0x0800 else 6) << 4) | (body[0] & 0x0F)
        if rng.random() < 0.5 and len(body) > 9:
            body[6 if et == 0x86DD else 9] = 17
        fr = eth_frame(bytes(body), rng, et)
        return fr, len(fr)
    if case == "tiny":
        fr = rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()
        if len(fr) >= 14 and rng.random() < 0.7:
            fr = fr[:12] + _u16be(0x0800 if rng.random() < 0.5 else 0x86DD) + fr[14:]
        return fr, len(fr)
    if v6:
        pkt, _ = ipv6_udp(payload, rng, next_hdr=58 if case == "icmp6" else 17)
    else:
        pkt, _ = ipv4_udp(payload, rng, ihl=ihl, proto=1 if case == "icmp4" else 17)
    b = bytearray(pkt)
    hl = 40 if v6 else ihl * 4
    if case == "short":  # IP payload < 8 (udp.c:123-126)
        if v6:
            b[4:6] = _u16be(int(rng.integers(0, 8)))
        else:
            b[2:4] = _u16be(hl + int(rng.integers(0, 8)))
    if case == "ulen_big":  # udp->len > ip_plen: MIN() takes ip_plen (udp.c:128)
        b[hl + 4:hl + 6] = _u16be(int(rng.integers(len(b) - hl + 1, 65536)))
    if case == "ulen_small":  # udp->len < 8 or shorter than the datagram
        b[hl + 4:hl + 6] = _u16be(int(rng.integers(0, max(9, len(b) - hl))))
    if case == "totlen_wrap":  # IPv4 total length < hl: ip_plen wraps (udp.c:104)
        b[2:4] = _u16be(int(rng.integers(0, hl)))
    if case == "frag":
        b[6] = (b[6] & 0xE0) | int(rng.integers(0, 32))
        b[7] = int(rng.integers(1 if b[6] & 0x1F == 0 else 0, 256))
    if case == "mf":  # More Fragments alone is not in IP4_OFFMASK (ip4.h:49)
        b[6], b[7] = 0x20, 0x00
    if case == "ihl_small":  # malformed IHL < 5 with a valid header checksum
        b[0] = 0x40 | int(rng.integers(0, 5))
    pkt = finish_udp(bytes(b), zero_udp=(case == "nocksum"))
    b = bytearray(pkt)
    if case == "badudp":
        k = int(rng.integers(hl, len(b)))
        b[k] ^= 1 << int(rng.integers(0, 8))
    if case == "badip":
        b[int(rng.integers(0, hl))] ^= 1 << int(rng.integers(0, 8))
    if case == "badver":
        b[0] = (int(rng.choice([0, 1, 5, 7, 15] + ([4] if v6 else [6]))) << 4) | (b[0] & 0x0F)
    fr = eth_frame(bytes(b), rng, 0x86DD if v6 else 0x0800)
    flen = len(fr)
    if case == "trunc":
        flen = int(rng.integers(14, len(fr)))
    return fr, flen


def rx_ring(rng: np.random.Generator, count: int, cases=RX_CASES, max_payload: int = 1472):
    """`count` frames cycling through `cases`: list of (bytes, frame length)."""
    return [rx_frame(rng, cases[i % len(cases)], max_payload) for i in range(count)]


def pack(pkts: list[tuple[bytes, int]], align: int = 1, lead: int = 0):
    """Concatenate packets (each start rounded up to `align`, after `lead`
    bytes) -> (buffer, offsets uint64, lens uint16)."""
    offs, lens, parts = [], [], []
    pos = lead
    parts.append(b"\x00" * lead)
    for pkt, ln in pkts:
        pad = (-pos) % align
        parts.append(b"\x00" * pad)
        pos += pad
        offs.append(pos)
        lens.append(ln)
        parts.append(pkt)
        pos += len(pkt)
    parts.append(b"\x00" * 64)
    buf = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    return buf, np.array(offs, dtype=np.uint64), np.array(lens, dtype=np.uint16)
