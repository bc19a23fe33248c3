"""Regenerate tests/golden/linux_vectors.npz: checksums computed by the Linux
kernel's own RFC 1071 code, an implementation independent of this project
and of the reference.

The reference (lib/src/in_cksum.c) cannot be built here, and its tests hold
no checksum vectors.  These fixtures pin the oracle and
the GPU kernels to an external implementation on the same bytes:

* ``icmp``  -- ICMP echo replies from the loopback host.  The kernel builds
  each reply (icmp_reply -> csum_partial / csum_fold) over the request's
  payload, so the stored checksum is Linux's ip_cksum over 8 + L bytes, for
  L = 0..130, MTU edges and up to 65507 bytes (odd lengths included).
* ``ip4hdr`` -- IPv4 headers sent through an IP_HDRINCL raw socket with the
  checksum field zero: the kernel fills it (ip_fast_csum over ihl words,
  raw_send_hdrinc) -- ip_cksum(ip, ip4_hl) as ip4.c:186 computes it, for
  IHL 5..15 (NOP/EOL option bytes) and random TOS / id / TTL / fragment /
  addresses.
* ``udp6``  -- UDP over IPv6 sent through a raw socket with IPV6_CHECKSUM:
  the kernel computes the checksum with the IPv6 pseudo-header
  (csum_ipv6_magic) -- payload_cksum of the IPv6 packet (in_cksum.c:155-160)
  for next_hdr 17.  The IPv6 header is rebuilt from what the kernel used
  (::1 -> ::1, payload length, next header 17).
* ``udp4``  -- UDP over IPv4 (IHL 5..8 with NOP options) whose checksum this
  project's pure-Python oracle computed, each ACCEPTED by the kernel's UDP
  receive path (udp4_csum_init / __skb_checksum_complete); a corrupted copy
  of every 10th packet is checked to be dropped with InCsumErrors + 1, so the
  kernel really verified.  Datagrams whose checksum is 0x0000 (= "none sent"
  for UDP over IPv4) are skipped.

Each group is stored as blob / off / len / expect (uint8 / uint64 / uint16 /
uint16): the packet with its checksum field zeroed, and the checksum value
as the native uint16 the reference returns (memory bytes = the field).

Needs root (raw sockets) and a loopback interface; it runs in the build
container only -- the GPU box reads the committed .npz.

    python tests/golden/make_kernel_vectors.py
"""
from __future__ import annotations

import select
import socket
import struct
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))

from oracle import py_oracle  # noqa: E402  (only for the udp4 requests)

SEED = 0x11E7
IPV6_CHECKSUM = 7  # linux/in6.h
PROTO_A, PROTO_B = 253, 254  # RFC 3692 experimental protocol numbers
LO6 = socket.inet_pton(socket.AF_INET6, "::1")


def recv_match(sock, pred, timeout=2.0):
    end = time.time() + timeout
    while True:
        left = end - time.time()
        if left <= 0:
            return None
        r, _, _ = select.select([sock], [], [], left)
        if not r:
            return None
        data = sock.recv(1 << 17)
        if pred(data):
            return data


def lengths(rng, top):
    ls = list(range(0, 131)) + [1471, 1472, 1473, 8999, 9000, 9001, top]
    ls += [int(x) for x in rng.integers(131, 4000, 20)]
    return ls


class Group:
    def __init__(self):
        self.parts, self.offs, self.lens, self.expect = [], [], [], []
        self.pos = 0

    def add(self, pkt: bytes, expect: int):
        self.offs.append(self.pos)
        self.lens.append(len(pkt))
        self.expect.append(expect)
        self.parts.append(pkt)
        self.pos += len(pkt)

    def arrays(self, name):
        return {f"{name}_blob": np.frombuffer(b"".join(self.parts) + b"\0" * 64, np.uint8),
                f"{name}_off": np.array(self.offs, np.uint64),
                f"{name}_len": np.array(self.lens, np.uint16),
                f"{name}_expect": np.array(self.expect, np.uint16)}


def icmp_vectors(rng) -> Group:
    g = Group()
    s = socket.socket(socket.AF_INET, socket.SOCK_RAW, socket.IPPROTO_ICMP)
    for seq, L in enumerate(lengths(rng, 65507)):
        payload = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        head = struct.pack("!BBHHH", 8, 0, 0, 0x5EED, seq)
        req = bytearray(head + payload)
        req[2:4] = struct.pack("<H", py_oracle.ip_cksum(bytes(req), len(req)))
        s.sendto(bytes(req), ("127.0.0.1", 0))

        def is_reply(d):
            hl = (d[0] & 15) * 4
            return d[hl] == 0 and d[hl + 4:hl + 8] == head[4:8] and len(d) - hl == len(req)
        d = recv_match(s, is_reply)
        if d is None:
            raise RuntimeError(f"no echo reply for L={L}")
        hl = (d[0] & 15) * 4
        msg = bytearray(d[hl:])
        k = struct.unpack("<H", msg[2:4])[0]
        msg[2:4] = b"\0\0"
        g.add(bytes(msg), k)
    return g


def ip4hdr_vectors(rng, count=300) -> Group:
    g = Group()
    rx = {p: socket.socket(socket.AF_INET, socket.SOCK_RAW, p) for p in (PROTO_A, PROTO_B)}
    tx = socket.socket(socket.AF_INET, socket.SOCK_RAW, socket.IPPROTO_RAW)
    for i in range(count):
        ihl = 5 + i % 11
        nopt = 4 * (ihl - 5)
        opts = bytes([1] * max(0, nopt - 1 - int(rng.integers(0, 4)))) if nopt else b""
        opts = opts + b"\0" * (nopt - len(opts))  # NOPs then EOL padding
        proto = (PROTO_A, PROTO_B)[i & 1]
        ident = 0x4000 + i
        frag = int(rng.integers(0, 2)) << 14  # DF or not
        src = bytes([127, *rng.integers(0, 256, 2).tolist(), int(rng.integers(1, 255))])
        dst = bytes([127, *rng.integers(0, 256, 2).tolist(), int(rng.integers(1, 255))])
        hdr = struct.pack("!BBHHHBBH4s4s", 0x40 | ihl, int(rng.integers(0, 256)), 0, ident,
                          frag, int(rng.integers(1, 256)), proto, 0, src, dst) + opts
        tx.sendto(hdr + rng.integers(0, 256, int(rng.integers(0, 200)),
                                     dtype=np.uint8).tobytes(), (socket.inet_ntoa(dst), 0))
        d = recv_match(rx[proto], lambda d: d[4:6] == struct.pack("!H", ident))
        if d is None:
            raise RuntimeError(f"no raw copy of header {i}")
        h = bytearray(d[:4 * (d[0] & 15)])
        k = struct.unpack("<H", h[10:12])[0]
        h[10:12] = b"\0\0"
        g.add(bytes(h), k)
    return g


def udp6_vectors(rng) -> Group:
    g = Group()
    tx = socket.socket(socket.AF_INET6, socket.SOCK_RAW, socket.IPPROTO_UDP)
    tx.setsockopt(socket.IPPROTO_IPV6, IPV6_CHECKSUM, 6)
    rx = socket.socket(socket.AF_INET6, socket.SOCK_RAW, socket.IPPROTO_UDP)
    for i, L in enumerate(lengths(rng, 65535 - 48)):  # payload_cksum len is uint16
        payload = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        sport = 20000 + i
        udp = struct.pack("!HHHH", sport, 9, (8 + L) & 0xFFFF, 0) + payload
        tx.sendto(udp, ("::1", 0))
        d = recv_match(rx, lambda d: d[:2] == udp[:2] and len(d) == len(udp))
        if d is None:
            raise RuntimeError(f"no raw6 copy for L={L}")
        k = struct.unpack("<H", d[6:8])[0]
        if k == 0xFFFF:  # the kernel sends a computed 0 as 0xFFFF (RFC 768); skip
            continue
        ip6 = struct.pack("!IHBB16s16s", 0x60000000, 8 + L, 17, 64, LO6, LO6)
        g.add(ip6 + d[:6] + b"\0\0" + d[8:], k)
    return g


def udp_snmp():
    rows = [ln.split() for ln in open("/proc/net/snmp") if ln.startswith("Udp:")]
    return dict(zip(rows[0][1:], map(int, rows[1][1:])))


def udp4_vectors(rng) -> Group:
    g = Group()
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.bind(("127.0.0.1", 0))
    port = rx.getsockname()[1]
    tx = socket.socket(socket.AF_INET, socket.SOCK_RAW, socket.IPPROTO_RAW)
    for i, L in enumerate(lengths(rng, 65535 - 20 - 32 - 8)):
        ihl = 5 + i % 4
        opts = b"\x01" * (4 * (ihl - 5))
        payload = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        ulen = 8 + L
        ip = struct.pack("!BBHHHBBH4s4s", 0x40 | ihl, 0, 4 * ihl + ulen, 0x7000 + i, 0x4000,
                         64, 17, 0, socket.inet_aton("127.0.0.1"),
                         socket.inet_aton("127.0.0.1")) + opts
        pkt = bytearray(ip + struct.pack("!HHHH", 30000 + (i & 0x3FFF), port, ulen, 0) + payload)
        o = 4 * ihl + 6
        c = py_oracle.payload_cksum(bytes(pkt), len(pkt))
        if c == 0:
            continue
        if i % 10 == 0:  # negative control: a wrong checksum must be dropped
            bad = bytearray(pkt)
            bad[o:o + 2] = struct.pack("<H", c ^ 0x0100)
            before = udp_snmp()["InCsumErrors"]
            tx.sendto(bytes(bad), ("127.0.0.1", 0))
            if recv_match(rx, lambda d: d == payload, timeout=0.3) is not None:
                raise RuntimeError("kernel accepted a corrupted UDP checksum")
            if udp_snmp()["InCsumErrors"] != before + 1:
                raise RuntimeError("corrupted datagram not counted as a checksum error")
        pkt[o:o + 2] = struct.pack("<H", c)
        tx.sendto(bytes(pkt), ("127.0.0.1", 0))
        if recv_match(rx, lambda d: d == payload) is None:
            raise RuntimeError(f"kernel rejected datagram {i} (L={L})")
        pkt[o:o + 2] = b"\0\0"
        g.add(bytes(pkt), c)
    return g


def main():
    rng = np.random.default_rng(SEED)
    out = {}
    for name, fn in (("icmp", icmp_vectors), ("ip4hdr", ip4hdr_vectors),
                     ("udp6", udp6_vectors), ("udp4", udp4_vectors)):
        g = fn(rng)
        out.update(g.arrays(name))
        print(f"{name}: {len(g.lens)} vectors, {g.pos} bytes")
    import platform
    out["kernel_release"] = np.frombuffer(platform.release().encode(), np.uint8)
    np.savez_compressed(HERE / "linux_vectors.npz", **out)


if __name__ == "__main__":
    main()
