"""The C test programs (tests/c) build against include/ and the shipped
library, and the RX ring loop's frame construction agrees with the oracle
(no GPU: --oracle-only makes no library compute call)."""
import subprocess

import pytest

from cprog import build


@pytest.mark.parametrize("name", ["rx_ring_loop", "host_latency", "dropin_test",
                                  "multi_test", "sock_verify", "tx_queue_loop",
                                  "thread_engines"])
def test_c_program_builds(name, tmp_path):
    assert build(name, tmp_path).exists()


def test_rx_ring_frames_hit_every_decision(tmp_path):
    """Every frame case of rx_ring_loop.c is built to hit one decision of the
    reference's RX order (eth.c:75-86, ip4.c:95-138, ip6.c:91-111,
    udp.c:99-139); the oracle must give the code intended by construction."""
    exe = build("rx_ring_loop", tmp_path)
    r = subprocess.run([str(exe), "1", "64", "--oracle-only"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "oracle-only ok (18 cases" in r.stdout


def test_tx_queue_frames_pass_the_rx_checks(tmp_path):
    """tx_queue_loop.c's TX hook with the oracle in place of the GPU call:
    headers built as mk_ip4_hdr / mk_ip6_hdr / udp_tx do (udp.c:189-220),
    both checksums stored raw, the ring-full retry, and every wire frame
    passes the reference's RX checks (WC_RX_OK, or WC_RX_OK_NO_CKSUM for the
    zero-checksum sockets) -- the construction the GPU run relies on."""
    exe = build("tx_queue_loop", tmp_path)
    r = subprocess.run([str(exe), "1", "--oracle-only"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "oracle-only ok" in r.stdout
