"""CPU tests of the parity oracle (no GPU): known answers, cross-check of the
two independent restatements, golden regression vectors, RFC 1071 properties
and the synthetic-data generator."""
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import c_oracle, py_oracle
from packets import insert_checksum, ipv4_udp, ipv6_udp, pack, random_packets

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
