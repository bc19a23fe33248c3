"""CPU tests of the parity oracle (no GPU): known answers, cross-check of the
two independent restatements, golden regression vectors, RFC 1071 properties
and the synthetic-data generator."""
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import c_oracle, py_oracle
from packets import (RX_CASES, eth_frame, finish_udp, insert_checksum, ipv4_udp, ipv6_udp, pack,
                     random_packets, rx_ring)

GOLDEN = Path(__file__).resolve().parent / "golden"


def kat_cases():
    kat = json.loads((GOLDEN / "kat.json").read_text())
    for case in kat["ip_cksum"]:
        if "hex_repeat" in case:
            b, k = case["hex_repeat"]
            data = bytes.fromhex(b) * k
        else:
            data = bytes.fromhex(case["hex"])
        yield pytest.param(data, int(case["expect"], 16), id=case["name"])


@pytest.mark.parametrize("data,expect", list(kat_cases()))
def test_kat_py_and_c(data, expect):
    assert py_oracle.ip_cksum(data) == expect
    assert c_oracle.ip_cksum(data if data else b"\x00", len(data)) == expect


def test_rfc1071_memory_bytes():
    v = c_oracle.ip_cksum(bytes.fromhex("0001f203f4f5f6f7"))
    assert v.to_bytes(2, "little") == bytes.fromhex("220d")


def test_golden_vectors_ip():
    g = np.load(GOLDEN / "vectors.npz")
    got = c_oracle.cksum_ragged(g["ip_blob"], g["ip_off"], g["ip_len"], kind=0)
    np.testing.assert_array_equal(got, g["ip_expect"])


def test_golden_vectors_payload():
    g = np.load(GOLDEN / "vectors.npz")
    got = c_oracle.cksum_ragged(g["pl_blob"], g["pl_off"], g["pl_len"], kind=1)
    np.testing.assert_array_equal(got, g["pl_expect"])


LINUX_GROUPS = [("icmp", 0), ("ip4hdr", 0), ("udp6", 1), ("udp4", 1)]


@pytest.mark.parametrize("group,kind", LINUX_GROUPS)
def test_linux_kernel_vectors(group, kind):
    """Both restatements reproduce checksums the Linux kernel computed (or,
    for udp4, accepted) on the same bytes -- tests/golden/make_kernel_vectors.py."""
    g = np.load(GOLDEN / "linux_vectors.npz")
    blob, offs, lens = g[group + "_blob"], g[group + "_off"], g[group + "_len"]
    got = c_oracle.cksum_ragged(blob, offs, lens, kind=kind)
    np.testing.assert_array_equal(got, g[group + "_expect"])
    b = blob.tobytes()
    fn = py_oracle.payload_cksum if kind else py_oracle.ip_cksum
    for o, n, e in list(zip(offs.tolist(), lens.tolist(), g[group + "_expect"].tolist()))[:60]:
        assert fn(b[o:o + n], n) == e


def test_c_vs_py_ip_sweep():
    rng = np.random.default_rng(1)
    blob = rng.integers(0, 256, 20000, dtype=np.uint8)
    b = blob.tobytes()
    offs, lens = [], []
    for start in range(16):
        for ln in list(range(0, 70)) + [255, 256, 257, 1471, 1472, 1473, 9000, 9001]:
            offs.append(start)
            lens.append(ln)
    got = c_oracle.cksum_ragged(blob, np.array(offs), np.array(lens), kind=0)
    want = [py_oracle.ip_cksum(b[o:o + n]) for o, n in zip(offs, lens)]
    np.testing.assert_array_equal(got, np.array(want, np.uint16))


def test_c_vs_py_payload_wild():
    rng = np.random.default_rng(2)
    pkts = random_packets(rng, 400, max_payload=600, wild=True)
    buf, offs, lens = pack(pkts, align=1, lead=7)
    b = buf.tobytes()
    got = c_oracle.cksum_ragged(buf, offs, lens, kind=1)
    want = [py_oracle.payload_cksum(b[o:o + max(n, 40)], n) for o, n in zip(offs, lens)]
    np.testing.assert_array_equal(got, np.array(want, np.uint16))


def test_ipv6_next_hdr_wrap_is_reproduced():
    """in_cksum.c:157 adds next_hdr << 24 into a uint32: for next_hdr >= 128
    and a large payload the accumulator wraps mod 2^32 (a one-off deviation
    from a true one's-complement sum that the restatement must keep)."""
    rng = np.random.default_rng(3)
    payload = bytes([0xFF]) * 65000
    pkt, ln = ipv6_udp(payload, rng, next_hdr=255)
    s = py_oracle.payload_sum(pkt, ln)
    exact = (255 << 24) + py_oracle.word_sum(pkt[8:40]) + py_oracle.word_sum(pkt[4:6]) \
        + py_oracle.word_sum(pkt[40:ln])
    assert exact >= 1 << 32           # the wrap really happens here
    assert s == exact & 0xFFFFFFFF
    a = np.frombuffer(pkt, dtype=np.uint8)
    assert c_oracle.payload_cksum(a, ln) == py_oracle.reduce16(s)


@pytest.mark.parametrize("v6", [False, True])
def test_payload_roundtrip_property(v6):
    """TX computes the checksum with udp->cksum = 0 (udp.c:209-213); RX
    re-checksums the packet carrying it and must get 0 (udp.c:132-139)."""
    rng = np.random.default_rng(4)
    for plen in (0, 1, 17, 64, 511, 1472):
        payload = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
        pkt, ln = (ipv6_udp if v6 else ipv4_udp)(payload, rng)
        c = c_oracle.payload_cksum(np.frombuffer(pkt, np.uint8), ln)
        rx = insert_checksum(pkt, c)
        assert c_oracle.payload_cksum(np.frombuffer(rx, np.uint8), ln) == 0


def test_negative_zero():
    # 0xFFFF only for an all-zero sum; a nonzero multiple of 0xFFFF gives 0.
    assert c_oracle.ip_cksum(b"\x00" * 10) == 0xFFFF
    assert c_oracle.ip_cksum(b"\xff\xff" * 3) == 0x0000
    assert c_oracle.ip_cksum(b"\x01\x00\xfe\xff") == 0x0000  # 0x0001 + 0xFFFE


def test_synth_generator_matches_numpy():
    n = 1000
    got = c_oracle.synth(n, 0x5EED)
    k = np.arange((n + 7) // 8, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(0x5EED) + (k + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    want = z.astype("<u8").view(np.uint8)[:n]
    np.testing.assert_array_equal(got, want)


def test_strided_matches_scalar():
    rng = np.random.default_rng(5)
    buf = rng.integers(0, 256, 1472 * 64 + 32, dtype=np.uint8)
    got = c_oracle.cksum_strided(buf, 1472, 1472, 64, threads=4)
    want = [c_oracle.ip_cksum(buf[i * 1472:(i + 1) * 1472]) for i in range(64)]
    np.testing.assert_array_equal(got, np.array(want, np.uint16))


# ---------------------------------------------------------------------------
# RX verdicts: the reference's RX checks (eth.c:75-86, ip4.c:95-138,
# ip6.c:91-111, udp.c:99-139), two independent restatements.

def test_rx_verdict_c_vs_py_every_case():
    rng = np.random.default_rng(11)
    frames = rx_ring(rng, 60 * len(RX_CASES), max_payload=700)
    buf, offs, lens = pack(frames, align=1, lead=3)
    got = c_oracle.rx_verdict_ragged(buf, offs, lens, threads=4)
    b = buf.tobytes()
    want = [py_oracle.rx_verdict(b[o:o + n], n) for o, n in zip(offs.tolist(), lens.tolist())]
    np.testing.assert_array_equal(got, np.array(want, np.uint8))
    # the frame mix reaches every verdict code
    assert set(np.unique(got).tolist()) == set(range(10))


def _v4_frame(rng, payload=b"x" * 100, **kw):
    pkt, _ = ipv4_udp(payload, rng, **kw)
    return eth_frame(finish_udp(pkt), rng)


def test_rx_verdict_reference_details():
    """Decisions where the reference is easy to misread."""
    rng = np.random.default_rng(12)
    v = py_oracle
    f = _v4_frame(rng)
    assert v.rx_verdict(f) == v.RX_OK and c_oracle.rx_verdict(f) == v.RX_OK
    # More Fragments alone is not in IP4_OFFMASK 0xff1f (ip4.h:49): accepted
    b = bytearray(f)
    b[14 + 6] = 0x20
    b[14 + 6:14 + 8] = b"\x20\x00"
    fr = eth_frame(finish_udp(bytes(b[14:])), rng)
    assert v.rx_verdict(fr) == v.RX_OK == c_oracle.rx_verdict(fr)
    # a fragment offset (low 5 bits of byte 6 or byte 7) is dropped (ip4.c:123)
    b = bytearray(f[14:])
    b[7] = 1
    fr = eth_frame(finish_udp(bytes(b)), rng)
    assert v.rx_verdict(fr) == v.RX_FRAGMENT == c_oracle.rx_verdict(fr)
    # a UDP checksum field of 0 skips the payload check (udp.c:132) even if
    # the payload is corrupted afterwards
    pkt, _ = ipv4_udp(b"y" * 50, rng)
    fr = bytearray(eth_frame(finish_udp(pkt, zero_udp=True), rng))
    fr[-1] ^= 0xFF
    assert v.rx_verdict(bytes(fr)) == v.RX_OK_NO_CKSUM == c_oracle.rx_verdict(bytes(fr))
    # IHL 0: ip_cksum(ip, 0) == 0xFFFF != 0 (ip4.c:111)
    b = bytearray(f)
    b[14] = 0x40
    assert v.rx_verdict(bytes(b)) == v.RX_BAD_IP_CKSUM == c_oracle.rx_verdict(bytes(b))
    # the frame ends inside the UDP payload: the reference would read past it
    assert v.rx_verdict(f, len(f) - 1) == v.RX_TRUNCATED == c_oracle.rx_verdict(f, len(f) - 1)
    # udp->len shorter than the datagram: only udp_len + hl is summed
    # (udp.c:128, 134), so bytes after it do not matter
    pkt, _ = ipv4_udp(b"z" * 64, rng)
    b = bytearray(pkt)
    b[20 + 4:20 + 6] = (8 + 10).to_bytes(2, "big")
    fr = bytearray(eth_frame(finish_udp(bytes(b)), rng))
    fr[14 + 20 + 8 + 30] ^= 0x55
    assert v.rx_verdict(bytes(fr)) == v.RX_OK == c_oracle.rx_verdict(bytes(fr))
    # ARP and the rest go to the host (eth.c:75-86)
    arp = bytes(12) + b"\x08\x06" + bytes(28)
    assert v.rx_verdict(arp) == v.RX_NOT_IP == c_oracle.rx_verdict(arp)


def test_oracle_build_is_safe_for_concurrent_ranks(tmp_path):
    """The ranks of a multi-GPU bench start at once; on a host CPU model with
    no oracle build yet, every rank builds it on first use.  Round 6 saw 8
    gloo ranks collide on the same output file (`file too short`, a vanished
    `.tmp`); warpcore_amd/_build.py now serializes the build with a lock and
    gives each process its own temporary file.  Six processes build a fresh
    tag's oracle at once, and every one of them loads it."""
    import os
    import shutil
    import subprocess
    import sys

    root = Path(__file__).resolve().parent.parent
    tag = f"racetest-{os.getpid()}"
    code = ("import ctypes; from warpcore_amd import _build; "
            "p = _build.build_oracle(); ctypes.CDLL(str(p)); print(p)")
    env = dict(os.environ, WC_ORACLE_BUILD_TAG=tag, PYTHONPATH=str(root))
    try:
        procs = [subprocess.Popen([sys.executable, "-c", code], cwd=root, env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
                 for _ in range(6)]
        outs = [p.communicate(timeout=300) for p in procs]
        for p, (out, err) in zip(procs, outs):
            assert p.returncode == 0, err[-2000:]
        assert len({o.strip() for o, _ in outs}) == 1
    finally:
        shutil.rmtree(root / "oracle" / f"build-{tag}", ignore_errors=True)
