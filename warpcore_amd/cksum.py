"""Python mirror of warpcore's checksum interface, backed by the gfx950 library.

Names and argument meaning follow the reference
(/root/reference/lib/src/in_cksum.h:32-36):

* :func:`ip_cksum` ``(buf, len)`` -- RFC 1071 checksum of ``len`` bytes
  (in_cksum.c:133-137);
* :func:`payload_cksum` ``(buf, len)`` -- UDP/ICMPv6 checksum with the IPv4 or
  IPv6 pseudo-header, ``buf`` at the IP header and ``len`` = IP header + UDP
  length (in_cksum.c:140-167).

Both return the checksum as the native ``uint16`` the reference returns (its
in-memory bytes are the network-order checksum).  Around them sit the batch
calls the reference's per-packet loops would use at their batch points
(backend_netmap.c:348-358 TX, 379-391 RX) on device-resident ``torch``
buffers.  Every call goes through libwccksum.so; nothing here computes a
checksum on the CPU.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple, Union

import numpy as np
import torch

from . import _lib

KIND_IP = 0
KIND_PAYLOAD = 1
_KINDS = {"ip": KIND_IP, "payload": KIND_PAYLOAD, KIND_IP: KIND_IP,
          KIND_PAYLOAD: KIND_PAYLOAD}


class WcError(RuntimeError):
    """A libwccksum call returned an error code."""

    def __init__(self, func: str, code: int):
        msg = _lib.active().wc_strerror(code).decode()
        super().__init__(f"{func}: {msg} ({code})")
        self.code = code


def _check(func: str, rc: int) -> None:
    if rc != 0:
        raise WcError(func, rc)


def _kind(kind) -> int:
    try:
        return _KINDS[kind]
    except KeyError:
        raise ValueError(f"kind must be 'ip' or 'payload', not {kind!r}") from None


def _stream_ptr(stream, device=None) -> int:
    if stream is None:
        return torch.cuda.current_stream(device).cuda_stream
    if isinstance(stream, torch.cuda.Stream):
        return stream.cuda_stream
    return int(stream)


def _dev_ptr(t: Union[torch.Tensor, int]) -> int:
    if isinstance(t, torch.Tensor):
        if not t.is_cuda:
            raise ValueError("batch buffers must be device (cuda) tensors")
        return t.data_ptr()
    return int(t)


def reload_config() -> None:
    """Re-read the WC_* environment (read once at first init).  The shipped
    library reads only the server's knobs (_lib.INTEGRATOR_KNOBS); while any
    path knob (WC_SHAPE, WC_SEG, WC_RX_EARLY, ...) is set, the calls of this
    module go to the tuning build, which reads them (tools and the tests that
    pin every path against the oracle)."""
    _check("wc_config_reload", _lib.select_for_env().wc_config_reload())


def _span(length: int, kind: int) -> int:
    # payload_cksum reads the IPv4 header fields up to byte 19 whatever len is
    # (in_cksum.c:149-151)
    return max(length, 20) if kind == KIND_PAYLOAD else length


def _check_len(length: int) -> int:
    if not 0 <= int(length) <= 0xFFFF:
        raise ValueError("len is a uint16 in the reference (0..65535)")
    return int(length)


def _same_device(base: torch.Tensor, **others) -> None:
    if not isinstance(base, torch.Tensor) or not base.is_cuda:
        raise ValueError("base must be a device (cuda) tensor")
    for name, t in others.items():
        if t is None:
            continue
        if not isinstance(t, torch.Tensor) or not t.is_cuda:
            raise ValueError(f"{name} must be a device (cuda) tensor")
        if t.device != base.device:
            raise ValueError(f"{name} is on {t.device}, base on {base.device}")


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


def _check_strided(base: torch.Tensor, byte_offset: int, stride: int, length: int, n: int,
                   kind: int) -> None:
    if byte_offset < 0 or stride < 0 or n < 0:
        raise ValueError("byte_offset, stride and n must be >= 0")
    if not base.is_contiguous():
        raise ValueError("base must be contiguous")
    if n and byte_offset + (n - 1) * stride + _span(length, kind) > _nbytes(base):
        raise ValueError(f"batch of {n} x {length} B at stride {stride} (+{byte_offset}) "
                         f"runs past the {_nbytes(base)}-byte buffer")


def _check_ragged(base: torch.Tensor, offsets: torch.Tensor, lengths: torch.Tensor,
                  kind: int, check: bool) -> int:
    _same_device(base, offsets=offsets, lengths=lengths)
    n = _check_ragged_shapes(offsets, lengths)
    if not base.is_contiguous():
        raise ValueError("base must be contiguous")
    if check and n:
        # one device reduction + sync -- pass check=False on a hot loop whose
        # layout was validated once
        _ragged_bounds(_nbytes(base), offsets, lengths, kind)
    return n


def _check_ragged_shapes(offsets: torch.Tensor, lengths: torch.Tensor) -> int:
    n = offsets.numel()
    if (lengths.numel() != n or offsets.element_size() != 8 or lengths.element_size() != 2
            or offsets.is_floating_point() or lengths.is_floating_point()):
        raise ValueError("offsets must be 8-byte and lengths 2-byte integers, same count")
    if not (offsets.is_contiguous() and lengths.is_contiguous()):
        raise ValueError("offsets and lengths must be contiguous")
    return n


def _ragged_bounds(nbytes: int, offsets: torch.Tensor, lengths: torch.Tensor,
                   kind: int) -> None:
    """Every packet (and payload_cksum's 20 header bytes) inside [0, nbytes)."""
    off = offsets.view(torch.int64)
    ln = lengths.view(torch.int16).to(torch.int64) & 0xFFFF
    if kind == KIND_PAYLOAD:
        ln = torch.clamp(ln, min=20)
    if bool((off < 0).any()) or int((off + ln).max()) > nbytes:
        raise ValueError("a packet [off, off + len) runs past the buffer")


class _on_device:
    """Make base's device current for the library call (it resolves its
    device with hipGetDevice)."""

    def __init__(self, device: torch.device):
        self.idx = device.index if device.index is not None else torch.cuda.current_device()
        self.prev = None

    def __enter__(self):
        cur = torch.cuda.current_device()
        if cur != self.idx:
            self.prev = cur
            torch.cuda.set_device(self.idx)
        return self

    def __exit__(self, *exc):
        if self.prev is not None:
            torch.cuda.set_device(self.prev)
        return False


# --------------------------------------------------------------------------
# Scalar drop-ins (reference in_cksum.h:32-36).

def _host_buffer(buf, length: Optional[int]) -> Tuple[ctypes.c_void_p, int, object]:
    arr = np.frombuffer(memoryview(buf).cast("B"), dtype=np.uint8) \
        if not isinstance(buf, np.ndarray) else buf.reshape(-1).view(np.uint8)
    if length is None:
        length = arr.size
    if not 0 <= length <= 0xFFFF:
        raise ValueError("len is a uint16 in the reference (0..65535)")
    keep = np.ascontiguousarray(arr)
    return ctypes.c_void_p(keep.ctypes.data), length, keep


def ip_cksum(buf, length: Optional[int] = None) -> int:
    """GPU-computed ``ip_cksum(buf, len)`` (in_cksum.c:133-137)."""
    p, n, keep = _host_buffer(buf, length)
    if keep.size < n:
        raise ValueError("buffer shorter than len")
    return int(_lib.active().ip_cksum(p, n))


def payload_cksum(buf, length: Optional[int] = None) -> int:
    """GPU-computed ``payload_cksum(buf, len)`` (in_cksum.c:140-167)."""
    p, n, keep = _host_buffer(buf, length)
    if keep.size < max(n, 20):
        raise ValueError("payload_cksum reads at least the 20-byte IPv4 header")
    return int(_lib.active().payload_cksum(p, n))


# --------------------------------------------------------------------------
# Device-resident batches.

def _out_tensor(out: Optional[torch.Tensor], n: int, device) -> torch.Tensor:
    if out is None:
        out = torch.empty(n, dtype=torch.uint16, device=device)
    if out.numel() < n or out.element_size() != 2 or not out.is_contiguous():
        raise ValueError("out must be a contiguous 2-byte tensor of >= n entries")
    if not out.is_cuda or out.device != torch.device(device):
        raise ValueError(f"out must be on {device}")
    return out


def cksum_strided(base: torch.Tensor, stride: int, length: int, n: int,
                  out: Optional[torch.Tensor] = None, kind="ip",
                  stream=None, byte_offset: int = 0) -> torch.Tensor:
    """Checksum packets ``base[byte_offset + i*stride : ... + length]``, i < n."""
    k = _kind(kind)
    _same_device(base)
    _check_strided(base, byte_offset, stride, _check_len(length), n, k)
    out = _out_tensor(out, n, base.device)
    with _on_device(base.device):
        _check("wc_cksum_strided", _lib.active().wc_cksum_strided(
            _dev_ptr(base) + byte_offset, stride, length, n, out.data_ptr(),
            k, _stream_ptr(stream, base.device)))
    return out


def cksum_ragged(base: torch.Tensor, offsets: torch.Tensor, lengths: torch.Tensor,
                 out: Optional[torch.Tensor] = None, kind="ip",
                 stream=None, check: bool = True) -> torch.Tensor:
    """Checksum packets ``base[off[i] : off[i] + len[i]]`` (uint64 / uint16
    arrays).  ``check`` validates every packet against ``base`` (one device
    reduction and a sync); pass False on a loop over an already-checked
    layout."""
    k = _kind(kind)
    n = _check_ragged(base, offsets, lengths, k, check)
    out = _out_tensor(out, n, base.device)
    with _on_device(base.device):
        _check("wc_cksum_ragged", _lib.active().wc_cksum_ragged(
            _dev_ptr(base), _dev_ptr(offsets), _dev_ptr(lengths), n, out.data_ptr(),
            k, _stream_ptr(stream, base.device)))
    return out


def verify_strided(base, stride, length, n, kind="payload", out=None,
                   stream=None, byte_offset: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """RX check (udp.c:132-139): results plus the count of non-zero checksums."""
    k = _kind(kind)
    _same_device(base)
    _check_strided(base, byte_offset, stride, _check_len(length), n, k)
    out = _out_tensor(out, n, base.device)
    bad = torch.zeros(1, dtype=torch.int64, device=base.device)
    with _on_device(base.device):
        _check("wc_verify_strided", _lib.active().wc_verify_strided(
            _dev_ptr(base) + byte_offset, stride, length, n, out.data_ptr(), bad.data_ptr(),
            k, _stream_ptr(stream, base.device)))
    return out, bad


def verify_ragged(base, offsets, lengths, kind="payload", out=None,
                  stream=None, check: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    k = _kind(kind)
    n = _check_ragged(base, offsets, lengths, k, check)
    out = _out_tensor(out, n, base.device)
    bad = torch.zeros(1, dtype=torch.int64, device=base.device)
    with _on_device(base.device):
        _check("wc_verify_ragged", _lib.active().wc_verify_ragged(
            _dev_ptr(base), _dev_ptr(offsets), _dev_ptr(lengths), n, out.data_ptr(),
            bad.data_ptr(), k, _stream_ptr(stream, base.device)))
    return out, bad


def cksum_ip_udp_strided(base: torch.Tensor, stride: int, length: int, n: int,
                         stream=None, byte_offset: int = 0, out_hdr: Optional[torch.Tensor] = None,
                         out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """One pass over IP/UDP packets: (IPv4 header checksums, payload_cksum).
    The header checksum is ip_cksum(ip, ip4_hl) (ip4.c:110-115, 184-186); 0
    for IPv6 packets."""
    _same_device(base)
    _check_strided(base, byte_offset, stride, _check_len(length), n, KIND_PAYLOAD)
    hdr = _out_tensor(out_hdr, n, base.device)
    pay = _out_tensor(out, n, base.device)
    with _on_device(base.device):
        _check("wc_cksum_ip_udp_strided", _lib.active().wc_cksum_ip_udp_strided(
            _dev_ptr(base) + byte_offset, stride, length, n, hdr.data_ptr(), pay.data_ptr(),
            _stream_ptr(stream, base.device)))
    return hdr, pay


def cksum_ip_udp_ragged(base: torch.Tensor, offsets: torch.Tensor, lengths: torch.Tensor,
                        stream=None, check: bool = True, out_hdr: Optional[torch.Tensor] = None,
                        out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    n = _check_ragged(base, offsets, lengths, KIND_PAYLOAD, check)
    hdr = _out_tensor(out_hdr, n, base.device)
    pay = _out_tensor(out, n, base.device)
    with _on_device(base.device):
        _check("wc_cksum_ip_udp_ragged", _lib.active().wc_cksum_ip_udp_ragged(
            _dev_ptr(base), _dev_ptr(offsets), _dev_ptr(lengths), n, hdr.data_ptr(),
            pay.data_ptr(), _stream_ptr(stream, base.device)))
    return hdr, pay


# --------------------------------------------------------------------------
# RX verdicts (the reference's eth_rx -> ip4_rx / ip6_rx -> udp_rx checks).

# enum wc_rx_verdict (include/warpcore_gpu/wc_cksum.h)
RX_OK, RX_OK_NO_CKSUM, RX_BAD_IP_CKSUM, RX_BAD_UDP_CKSUM, RX_SHORT, RX_FRAGMENT, \
    RX_BAD_VERSION, RX_NOT_UDP, RX_NOT_IP, RX_TRUNCATED = range(10)
RX_NAMES = ("ok", "ok_no_cksum", "bad_ip_cksum", "bad_udp_cksum", "short", "fragment",
            "bad_version", "not_udp", "not_ip", "truncated")
RX_DROPS = (RX_BAD_IP_CKSUM, RX_BAD_UDP_CKSUM, RX_SHORT, RX_FRAGMENT, RX_BAD_VERSION,
            RX_TRUNCATED)


def rx_verdict_ragged(base: torch.Tensor, offsets: torch.Tensor, frame_lens: torch.Tensor,
                      out: Optional[torch.Tensor] = None, stream=None,
                      check: bool = True,
                      drops: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """RX verdict of every Ethernet frame ``base[off[i] : off[i] + frame_len[i]]``
    (a netmap RX ring's slot buffers and slot lengths): a uint8 code per frame
    (``RX_*``) and the number of frames the reference's RX path drops.  No
    header is parsed on the host (wc_rx_verdict_ragged).  A given ``drops``
    tensor is accumulated into, not reset."""
    _same_device(base, offsets=offsets, lengths=frame_lens)
    n = _check_ragged_shapes(offsets, frame_lens)
    if not base.is_contiguous():
        raise ValueError("base must be contiguous")
    if check and n:
        _ragged_bounds(_nbytes(base), offsets, frame_lens, KIND_IP)
    if out is None:
        out = torch.empty(n, dtype=torch.uint8, device=base.device)
    if out.numel() < n or out.element_size() != 1 or not out.is_contiguous() \
            or out.device != base.device:
        raise ValueError(f"out must be a contiguous 1-byte tensor of >= n entries on {base.device}")
    if drops is None:
        drops = torch.zeros(1, dtype=torch.int64, device=base.device)
    elif (drops.numel() < 1 or drops.dtype not in (torch.int64, torch.uint64)
          or not drops.is_contiguous() or drops.device != base.device):
        raise ValueError("drops must be a contiguous int64 / uint64 device tensor (accumulated)")
    with _on_device(base.device):
        _check("wc_rx_verdict_ragged", _lib.active().wc_rx_verdict_ragged(
            _dev_ptr(base), _dev_ptr(offsets), _dev_ptr(frame_lens), n, out.data_ptr(),
            drops.data_ptr(), _stream_ptr(stream, base.device)))
    return out, drops


def rx_verdict_host(buf: np.ndarray, offsets: np.ndarray,
                    frame_lens: np.ndarray) -> Tuple[np.ndarray, int]:
    """rx_verdict_ragged over host memory (wc_rx_verdict_host, synchronous):
    (uint8 verdicts, drop count)."""
    buf = np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
    lens_in = np.asarray(frame_lens)
    if lens_in.size and (lens_in.min() < 0 or lens_in.max() > 0xFFFF):
        raise ValueError("frame lengths are uint16 (netmap_slot.len)")
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(lens_in, dtype=np.uint16)
    if off.shape != lens.shape:
        raise ValueError("offsets and frame_lens must have the same shape")
    out = np.empty(off.size, dtype=np.uint8)
    drops = ctypes.c_uint64()
    _check("wc_rx_verdict_host", _lib.active().wc_rx_verdict_host(
        buf.ctypes.data, buf.size, off.ctypes.data, lens.ctypes.data, off.size,
        out.ctypes.data, ctypes.byref(drops)))
    return out, int(drops.value)


# --------------------------------------------------------------------------
# Host-memory batches (end-to-end path).

def cksum_host(buf: np.ndarray, offsets: np.ndarray, lengths: np.ndarray,
               kind="ip") -> np.ndarray:
    """Checksum host-resident packets (synchronous), offsets in any order.

    Small batches in a registered buffer are read in place by one kernel;
    larger ones are streamed over pinned H2D copies (wc_cksum_host)."""
    buf = np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
    lens_in = np.asarray(lengths)
    if lens_in.size and (lens_in.min() < 0 or lens_in.max() > 0xFFFF):
        raise ValueError("len is a uint16 in the reference (0..65535)")
    offs_in = np.asarray(offsets)
    if offs_in.size and offs_in.dtype.kind == "i" and offs_in.min() < 0:
        raise ValueError("negative offset")
    if offs_in.shape != lens_in.shape:
        raise ValueError("offsets and lengths must have the same shape")
    off = np.ascontiguousarray(offs_in, dtype=np.uint64)
    lens = np.ascontiguousarray(lens_in, dtype=np.uint16)
    out = np.empty(off.size, dtype=np.uint16)
    _check("wc_cksum_host", _lib.active().wc_cksum_host(
        buf.ctypes.data, buf.size, off.ctypes.data, lens.ctypes.data, off.size,
        out.ctypes.data, _kind(kind)))
    return out


def _host_batch_args(buf, offsets, lengths):
    buf = np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
    lens_in = np.asarray(lengths)
    if lens_in.size and (lens_in.min() < 0 or lens_in.max() > 0xFFFF):
        raise ValueError("len is a uint16 in the reference (0..65535)")
    offs_in = np.asarray(offsets)
    if offs_in.size and offs_in.dtype.kind == "i" and offs_in.min() < 0:
        raise ValueError("negative offset")
    if offs_in.shape != lens_in.shape:
        raise ValueError("offsets and lengths must have the same shape")
    return (buf, np.ascontiguousarray(offs_in, dtype=np.uint64),
            np.ascontiguousarray(lens_in, dtype=np.uint16))


def cksum_ip_udp_host(buf: np.ndarray, offsets: np.ndarray,
                      lengths: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """The fused TX pair over host-memory IP packets (wc_cksum_ip_udp_host,
    synchronous): (IPv4 header checksums -- 0 for IPv6 --, payload_cksum
    results), what mk_ip4_hdr and udp_tx store (ip4.c:184-186,
    udp.c:209-213)."""
    buf, off, lens = _host_batch_args(buf, offsets, lengths)
    hdr = np.empty(off.size, dtype=np.uint16)
    out = np.empty(off.size, dtype=np.uint16)
    _check("wc_cksum_ip_udp_host", _lib.active().wc_cksum_ip_udp_host(
        buf.ctypes.data, buf.size, off.ctypes.data, lens.ctypes.data, off.size,
        hdr.ctypes.data, out.ctypes.data))
    return hdr, out


def server_pause() -> None:
    """Stop the resident server grid on every device (wc_server_pause); small
    registered batches take the zero-copy launch until server_resume().  A
    device-wide synchronisation then never waits for the grid."""
    _check("wc_server_pause", _lib.active().wc_server_pause())


def server_resume() -> None:
    _check("wc_server_resume", _lib.active().wc_server_resume())


class server_paused:
    """``with server_paused(): ...`` -- server_pause() / server_resume()."""

    def __enter__(self):
        server_pause()
        return self

    def __exit__(self, *exc):
        server_resume()
        return False


def server_stats() -> dict:
    """The resident server's counters (wc_server_stats): batches served,
    fallbacks to the launch path, grid launches -- process totals."""
    v = [ctypes.c_uint64() for _ in range(3)]
    _check("wc_server_stats", _lib.active().wc_server_stats(*[ctypes.byref(x) for x in v]))
    return dict(zip(("served", "fallbacks", "launches"), (x.value for x in v)))


# Buffers page-locked through host_register, by base address: the library
# pins the pages mapped at that address, so the array is kept alive here until
# host_unregister (a buffer garbage-collected while registered could give its
# address to a new one that the old pinned pages do not back).
_registered: dict = {}


def host_register(buf: np.ndarray) -> None:
    """Page-lock `buf` for the zero-copy / direct-DMA host path.  The array
    is held until host_unregister(buf); registering it (or a new array at the
    same address) again re-pins the pages mapped there now."""
    if not isinstance(buf, np.ndarray) or not buf.flags["C_CONTIGUOUS"]:
        raise ValueError("host_register needs a C-contiguous numpy array")
    _check("wc_host_register", _lib.active().wc_host_register(buf.ctypes.data, buf.nbytes))
    _registered[buf.ctypes.data] = buf


def host_unregister(buf: np.ndarray) -> None:
    addr = buf.ctypes.data
    try:
        _check("wc_host_unregister", _lib.active().wc_host_unregister(addr))
    finally:
        _registered.pop(addr, None)


# --------------------------------------------------------------------------
# Synthetic data / introspection.

def synth_fill(buf: torch.Tensor, seed: int, nbytes: Optional[int] = None,
               stream=None) -> torch.Tensor:
    """Fill a device buffer with the counter-based splitmix64 byte stream."""
    _same_device(buf)
    nbytes = _nbytes(buf) if nbytes is None else nbytes
    if not 0 <= nbytes <= _nbytes(buf):
        raise ValueError(f"nbytes {nbytes} outside the {_nbytes(buf)}-byte buffer")
    with _on_device(buf.device):
        _check("wc_synth_fill", _lib.active().wc_synth_fill(
            _dev_ptr(buf), nbytes, seed & 0xFFFFFFFFFFFFFFFF, _stream_ptr(stream, buf.device)))
    return buf


class SclkProbe:
    """The shader clock beside a timed workload (wc_sclk_probe): one wave on
    a stream of its own samples the 100-MHz wall clock and the shader clock
    counter every `every_us`.  start() before the timed launches (after the
    work before them), mhz() after: the median clock over the samples taken.
    The probe ends by itself after the samples asked for -- keep that inside
    a timed region that ends with a device-wide synchronisation."""

    def __init__(self, device, max_samples: int = 200000):
        self.device = torch.device(device)
        self.max = max_samples
        self.buf = torch.zeros(2 * max_samples, dtype=torch.int64, device=self.device)
        self.stream = torch.cuda.Stream(device=self.device)
        self.n = 0

    def start(self, ms: float, every_us: int = 20) -> None:
        self.n = int(min(self.max, max(8, ms * 1e3 / every_us)))
        self.buf.zero_()
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with _on_device(self.device):
            _check("wc_sclk_probe", _lib.active().wc_sclk_probe(
                self.buf.data_ptr(), self.n, every_us * 100, self.stream.cuda_stream))

    def mhz(self) -> float:
        self.stream.synchronize()
        s = self.buf[: 2 * self.n].view(self.n, 2).cpu().double()
        dt = s[1:, 0] - s[:-1, 0]
        dc = s[1:, 1] - s[:-1, 1]
        ok = dt > 0
        if not bool(ok.any()):
            return float("nan")
        return float((dc[ok] / dt[ok] * 100.0).median())


def plan_strided(base_addr: int, stride: int, length: int, n: int, kind="ip") -> dict:
    vals = [ctypes.c_int() for _ in range(4)]
    _check("wc_plan_strided", _lib.active().wc_plan_strided(
        base_addr, stride, length, n, _kind(kind), *[ctypes.byref(v) for v in vals]))
    plan = dict(zip(("group", "chunks_per_lane", "unroll", "grid"), (v.value for v in vals)))
    plan["kernel"] = _lib.active().wc_plan_strided_kernel(base_addr, stride, length, n,
                                                        _kind(kind)).decode()
    return plan


def gpu_init(device: int = -1) -> None:
    _check("wc_gpu_init", _lib.active().wc_gpu_init(device))


def version() -> str:
    return _lib.active().wc_version().decode()


# --------------------------------------------------------------------------
# Multi-GPU from one host thread (the C host's path).

def shard_range(n: int, g: int, ngpus: int) -> Tuple[int, int]:
    """The library's even contiguous split: packets [lo, hi) of n for shard g."""
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    _check("wc_shard_range", _lib.active().wc_shard_range(n, g, ngpus, ctypes.byref(lo),
                                                        ctypes.byref(hi)))
    return lo.value, hi.value


_shard_devices: list = []


def gpu_init_multi(ngpus: int = 0, devices=None) -> int:
    """Set up one shard executor per device (devices[g], or g); returns G."""
    global _shard_devices
    arr = None
    if devices is not None:
        devices = [int(d) for d in devices]
        ngpus = len(devices)
        arr = (ctypes.c_int * ngpus)(*devices)
    _check("wc_gpu_init_multi", _lib.active().wc_gpu_init_multi(ngpus, arr))
    G = int(_lib.active().wc_gpu_multi_count())
    _shard_devices = list(devices) if devices is not None else list(range(G))
    return G


def shard_devices() -> list:
    """Device index of every shard executor (after gpu_init_multi)."""
    G = int(_lib.active().wc_gpu_multi_count())
    if len(_shard_devices) != G:
        raise RuntimeError("shard executors not set up by gpu_init_multi")
    return list(_shard_devices)


def cksum_host_multi(buf: np.ndarray, offsets: np.ndarray, lengths: np.ndarray,
                     kind="ip") -> np.ndarray:
    """cksum_host split evenly over the shard devices (wc_cksum_host_multi)."""
    buf = np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
    lens_in = np.asarray(lengths)
    if lens_in.size and (lens_in.min() < 0 or lens_in.max() > 0xFFFF):
        raise ValueError("len is a uint16 in the reference (0..65535)")
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(lens_in, dtype=np.uint16)
    if off.shape != lens.shape:
        raise ValueError("offsets and lengths must have the same shape")
    out = np.empty(off.size, dtype=np.uint16)
    _check("wc_cksum_host_multi", _lib.active().wc_cksum_host_multi(
        buf.ctypes.data, buf.size, off.ctypes.data, lens.ctypes.data, off.size,
        out.ctypes.data, _kind(kind)))
    return out


def _ptrs(ts) -> ctypes.Array:
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() if isinstance(t, torch.Tensor) else t
                                         for t in ts])


def _per_shard(name: str, items, devs) -> list:
    """The C side reads one entry per shard executor from every array: each
    list must have exactly that many entries, each on its shard's device."""
    items = list(items)
    if len(items) != len(devs):
        raise ValueError(f"{name}: {len(items)} entries for {len(devs)} shard executors")
    for g, (t, d) in enumerate(zip(items, devs)):
        if t is None:
            continue
        if not isinstance(t, torch.Tensor) or not t.is_cuda:
            raise ValueError(f"{name}[{g}] must be a device (cuda) tensor")
        if t.device.index != d:
            raise ValueError(f"{name}[{g}] is on {t.device}, shard {g} runs on cuda:{d}")
    return items


def _shard_streams(streams, devs):
    if streams is None:
        return _ptrs([_stream_ptr(None, torch.device("cuda", d)) for d in devs])
    streams = list(streams)
    if len(streams) != len(devs):
        raise ValueError(f"streams: {len(streams)} entries for {len(devs)} shard executors")
    return _ptrs([_stream_ptr(s, torch.device("cuda", d)) for s, d in zip(streams, devs)])


def cksum_ragged_multi(bases, offsets, lengths, outs, kind="ip", streams=None) -> None:
    """Shard g's device-resident batch (bases[g], offsets[g], lengths[g]) into
    outs[g], each on shard g's device (asynchronous)."""
    k = _kind(kind)
    devs = shard_devices()
    bases = _per_shard("bases", bases, devs)
    offsets = _per_shard("offsets", offsets, devs)
    lengths = _per_shard("lengths", lengths, devs)
    outs = _per_shard("outs", outs, devs)
    for b, o, l, r in zip(bases, offsets, lengths, outs):
        n = _check_ragged(b, o, l, k, True)
        _out_tensor(r, n, b.device)
    ns = (ctypes.c_uint64 * len(devs))(*[o.numel() for o in offsets])
    _check("wc_cksum_ragged_multi", _lib.active().wc_cksum_ragged_multi(
        _ptrs(bases), _ptrs(offsets), _ptrs(lengths), ns, _ptrs(outs), k,
        _shard_streams(streams, devs)))


def gather_results_multi(shard_outs, counts, all_outs, streams=None) -> None:
    """RCCL all-gather of every shard's results into all_outs[g] (packet order)."""
    devs = shard_devices()
    shard_outs = _per_shard("shard_outs", shard_outs, devs)
    all_outs = _per_shard("all_outs", all_outs, devs)
    counts = [int(c) for c in counts]
    if len(counts) != len(devs):
        raise ValueError(f"counts: {len(counts)} entries for {len(devs)} shard executors")
    total = sum(counts)
    for g, (src, c) in enumerate(zip(shard_outs, counts)):
        if c < 0 or src.numel() < c or src.element_size() != 2 or not src.is_contiguous():
            raise ValueError(f"shard_outs[{g}] needs >= {c} contiguous 2-byte entries")
    for g, a in enumerate(all_outs):
        if a.numel() < total or a.element_size() != 2 or not a.is_contiguous():
            raise ValueError("each all_outs tensor needs sum(counts) contiguous 2-byte entries")
    ns = (ctypes.c_uint64 * len(devs))(*counts)
    _check("wc_gather_results_multi", _lib.active().wc_gather_results_multi(
        _ptrs(shard_outs), ns, _ptrs(all_outs), _shard_streams(streams, devs)))
