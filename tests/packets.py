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
