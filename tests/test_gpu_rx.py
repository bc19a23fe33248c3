"""RX verdicts on the GPU (wc_rx_verdict_ragged / wc_rx_verdict_host) against
the oracle's restatement of the reference's RX checks (oracle_rx_verdict:
eth.c:75-86, ip4.c:95-138, ip6.c:91-111, udp.c:99-139) -- every frame, exact
code.

Layouts: a netmap RX ring (one frame per 2048-B slot buffer, slots listed in
a scrambled order as a ring's buf_idx are), frames packed back to back at odd
alignment, and a ring drained into a registered host pool (zero-copy and
pipelined host paths).
"""
import numpy as np
import pytest
import torch

import warpcore_amd as wc
from oracle import c_oracle
from packets import RX_CASES, pack, rx_ring

pytestmark = pytest.mark.gpu


def dev(a: np.ndarray, d) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a)).to(d)


def slot_ring(frames, slot: int = 2048, rng=None, pad: int = 64):
    """Frames in `slot`-byte buffers (netmap_slot buf_idx order scrambled)."""
    n = len(frames)
    idx = np.arange(n) if rng is None else rng.permutation(n)
    buf = np.zeros(n * slot + pad, dtype=np.uint8)
    offs = (idx * slot).astype(np.uint64)
    lens = np.empty(n, dtype=np.uint16)
    for i, (fr, flen) in enumerate(frames):
        o = int(offs[i])
        buf[o:o + len(fr)] = np.frombuffer(fr, np.uint8)
        lens[i] = flen
    return buf, offs, lens


RX_MODES = {"default": {}, "ht": {"WC_RX_ADAPT": "0"},
            "plain": {"WC_RX_HDRT": "0", "WC_RX_SKIP": "0"},
            "skip": {"WC_RX_SKIP": "1"}, "skip_plain": {"WC_RX_SKIP": "1", "WC_RX_HDRT": "0"},
            "early": {"WC_RX_EARLY": "1"},
            "early_plain": {"WC_RX_EARLY": "1", "WC_RX_HDRT": "0"},
            "early_skip": {"WC_RX_EARLY": "1", "WC_RX_SKIP": "1"},
            # ADAPT's two tallying kernels pinned (the decision fixed, ADVICE
            # r05), and a capped grid: each wave walks several tiles, the
            # next tile's slots prefetched
            "adapt_ht": {"WC_RX_FORCE": "1"}, "adapt_early": {"WC_RX_FORCE": "2"},
            "grid4": {"WC_RX_GRID": "4"}, "grid4_early": {"WC_RX_GRID": "4", "WC_RX_EARLY": "1"}}


@pytest.fixture(params=list(RX_MODES))
def rx_mode(request, monkeypatch, gpu):
    """Every kernel mode of wc_rx_verdict_* (the default ADAPT: EARLY or the
    HT stream per tile by the launch's running share of ruled-out frames;
    WC_RX_EARLY: parse before or during the stream; WC_RX_HDRT: header
    chunks loaded transposed; WC_RX_SKIP: ruled-out frames leave the stream)
    must give the same verdicts."""
    for k, v in RX_MODES[request.param].items():
        monkeypatch.setenv(k, v)
    wc.reload_config()
    yield request.param
    for k in RX_MODES[request.param]:
        monkeypatch.delenv(k)
    wc.reload_config()


def check(buf, offs, lens, d):
    want = c_oracle.rx_verdict_ragged(buf, offs, lens)
    t = torch.zeros(buf.size + 64, dtype=torch.uint8, device=d)
    t[:buf.size] = dev(buf, d)
    got, drops = wc.rx_verdict_ragged(t, dev(offs, d), dev(lens, d))
    got = got.cpu().numpy()
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (f"{bad.size} verdicts differ, first {bad[:8]}: "
                           f"got {got[bad[:8]]} want {want[bad[:8]]}")
    assert int(drops.item()) == int(np.isin(want, wc.RX_DROPS).sum())
    return want


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_rx_verdict_netmap_ring(gpu, seed, rx_mode):
    rng = np.random.default_rng(seed)
    frames = rx_ring(rng, 30 * len(RX_CASES))
    buf, offs, lens = slot_ring(frames, rng=rng)
    want = check(buf, offs, lens, gpu)
    assert set(np.unique(want).tolist()) == set(range(10))


@pytest.mark.parametrize("align,lead", [(1, 0), (1, 5), (2, 14), (16, 3)])
def test_rx_verdict_packed(gpu, align, lead, rx_mode):
    """Frames back to back at every alignment (a ring drained into one buffer)."""
    rng = np.random.default_rng(align * 10 + lead)
    frames = rx_ring(rng, 20 * len(RX_CASES))
    buf, offs, lens = pack(frames, align=align, lead=lead)
    check(buf, offs, lens, gpu)


def test_rx_verdict_valid_ring_mtu(gpu, rx_mode):
    """2^16 well-formed MTU frames (IPv4 / IPv6, ~1/7 with IPv4 options) in
    2048-B slots: every verdict OK (or OK_NO_CKSUM for a computed 0), then
    flip a bit in 1000 of them: every one the oracle drops is dropped (IPv6
    flow label / hop limit bits are covered by no checksum, so not all)."""
    rng = np.random.default_rng(7)
    cases = ("ok4", "ok6", "ok4", "ok6", "ok4", "ok6", "ok4opt")
    frames = rx_ring(rng, 1 << 16, cases=cases, max_payload=1400)
    buf, offs, lens = slot_ring(frames)
    want = check(buf, offs, lens, gpu)
    assert np.isin(want, (wc.RX_OK, wc.RX_OK_NO_CKSUM)).all()
    hit = rng.choice(len(frames), 1000, replace=False)
    for i in hit:
        o = int(offs[i])
        k = o + 14 + int(rng.integers(0, int(lens[i]) - 14))
        buf[k] ^= 0x10
    want = check(buf, offs, lens, gpu)
    assert 900 <= int(np.isin(want, wc.RX_DROPS).sum()) <= 1000


def test_rx_verdict_empty_and_tiny(gpu):
    frames = [(b"", 0), (b"\x00" * 13, 13), (b"\x00" * 12 + b"\x08\x00", 14),
              (b"\x00" * 12 + b"\x86\xdd\x60", 15)]
    buf, offs, lens = slot_ring(frames)
    check(buf, offs, lens, gpu)
    got, drops = wc.rx_verdict_ragged(torch.zeros(64, dtype=torch.uint8, device=gpu),
                                      torch.zeros(0, dtype=torch.int64, device=gpu),
                                      torch.zeros(0, dtype=torch.int16, device=gpu))
    assert got.numel() == 0 and int(drops.item()) == 0


def test_rx_verdict_frames_at_buffer_end(gpu, rx_mode):
    """Frames ending on the buffer's last byte, their lengths bounding every
    load (a fault here would take the GPU down, so the bound is tested)."""
    rng = np.random.default_rng(9)
    frames = rx_ring(rng, 3 * len(RX_CASES))
    for fr, flen in frames:
        buf = np.frombuffer(fr[:flen], np.uint8).copy()
        t = dev(buf, gpu) if buf.size else torch.zeros(1, dtype=torch.uint8, device=gpu)
        got, _ = wc.rx_verdict_ragged(t, dev(np.zeros(1, np.uint64), gpu),
                                      dev(np.array([flen], np.uint16), gpu))
        assert int(got.item()) == c_oracle.rx_verdict(fr, flen)


@pytest.mark.parametrize("register", [False, True])
@pytest.mark.parametrize("n", [64, 4096, 200000])
def test_rx_verdict_host(gpu, register, n, rx_mode):
    """The RX ring in host memory (netmap's w->mem): zero-copy for a small
    registered batch, the pipelined copy otherwise."""
    rng = np.random.default_rng(n + register)
    frames = rx_ring(rng, n, max_payload=1200 if n > 4096 else 1472)
    buf, offs, lens = slot_ring(frames, rng=rng)
    want = c_oracle.rx_verdict_ragged(buf, offs, lens)
    if register:
        wc.host_register(buf)
    s0 = wc.server_stats()
    try:
        got, drops = wc.rx_verdict_host(buf, offs, lens)
    finally:
        if register:
            wc.host_unregister(buf)
    s1 = wc.server_stats()
    np.testing.assert_array_equal(got, want)
    assert drops == int(np.isin(want, wc.RX_DROPS).sum())
    # a small registered ring is answered by the resident server, not the
    # launch path it falls back to
    served = 1 if register and n <= 256 else 0
    assert (s1["served"] - s0["served"], s1["fallbacks"] - s0["fallbacks"]) == (served, 0)


def test_c_rx_ring_loop(gpu, tmp_path):
    """INTEGRATION.md section 3's RX hook compiled in C and driven like
    w_nic_rx (backend_netmap.c:379-391): 4 netmap-shaped rings whose pending
    span wraps, one wc_rx_verdict_host per ring, a per-slot branch on
    WC_RX_IS_DROP; every frame's code equals the oracle's and the one it was
    built to get, the drop count equals the slots dropped; zero-copy and
    pageable passes."""
    import subprocess

    from cprog import build
    exe = build("rx_ring_loop", tmp_path)
    r = subprocess.run([str(exe), "4", "1024"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "rx_ring_loop: ok" in r.stdout


def test_c_host_latency_tool(gpu, tmp_path):
    """The C latency tool (tests/c/host_latency.c) runs and its GPU results
    (zero-copy, pipelined, RX verdicts) match the oracle at every batch size."""
    import subprocess

    from cprog import build
    exe = build("host_latency", tmp_path)
    r = subprocess.run([str(exe), "4", "0.01"], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_latency: ok" in r.stdout


def test_c_tx_queue_loop(gpu, tmp_path):
    """INTEGRATION.md section 3's TX hook compiled in C and driven like w_tx
    (backend_netmap.c:348-358): per w_iov_sq, headers built as mk_ip4_hdr /
    mk_ip6_hdr / udp_tx do, ONE wc_cksum_ip_udp_host call, both results
    stored raw (zero-checksum sockets keep udp->cksum 0), the TX-ring-full
    retry without recomputing; every result equals the oracle's and every
    frame on the wire passes the RX checks (wc_rx_verdict_host: WC_RX_OK /
    WC_RX_OK_NO_CKSUM); registered (server, zero-copy, DMA) and pageable."""
    import subprocess

    from cprog import build
    exe = build("tx_queue_loop", tmp_path)
    r = subprocess.run([str(exe), "2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "tx_queue_loop: ok" in r.stdout


def test_c_thread_engines(gpu, tmp_path):
    """Several engines on their own threads call the library at once
    (tests/c/thread_engines.c): host engines over registered and pageable
    buffer regions (server, zero-copy, pipeline; ip / payload / fused / RX
    verdicts), device engines on their own streams (strided / ragged / fused /
    RX), the scalar drop-in, a thread that keeps registering and
    unregistering a region (each stops the server grid), and one that keeps
    pausing the server, synchronising the whole device (bounded: no grid
    left) and resuming it.  Every result equals the oracle's, and the server
    answered with no fallback."""
    import subprocess

    from cprog import build
    exe = build("thread_engines", tmp_path)
    r = subprocess.run([str(exe), "4", "4", "2"], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "thread_engines: ok" in r.stdout
