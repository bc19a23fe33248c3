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
        msg = _lib.load().wc_strerror(code).decode()
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


def _stream_ptr(stream) -> int:
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, torch.cuda.Stream):
        return stream.cuda_stream
    return int(stream)


def _dev_ptr(t: Union[torch.Tensor, int]) -> int:
    if isinstance(t, torch.Tensor):
        if not t.is_cuda:
            raise ValueError("batch buffers must be device (cuda) tensors")
        return t.data_ptr()
    return int(t)


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
    return int(_lib.load().ip_cksum(p, n))


def payload_cksum(buf, length: Optional[int] = None) -> int:
    """GPU-computed ``payload_cksum(buf, len)`` (in_cksum.c:140-167)."""
    p, n, keep = _host_buffer(buf, length)
    if keep.size < max(n, 20):
        raise ValueError("payload_cksum reads at least the 20-byte IPv4 header")
    return int(_lib.load().payload_cksum(p, n))


# --------------------------------------------------------------------------
# Device-resident batches.

def _out_tensor(out: Optional[torch.Tensor], n: int, device) -> torch.Tensor:
    if out is None:
        out = torch.empty(n, dtype=torch.uint16, device=device)
    if out.numel() < n or out.element_size() != 2 or not out.is_contiguous():
        raise ValueError("out must be a contiguous 2-byte tensor of >= n entries")
    return out


def cksum_strided(base: torch.Tensor, stride: int, length: int, n: int,
                  out: Optional[torch.Tensor] = None, kind="ip",
                  stream=None, byte_offset: int = 0) -> torch.Tensor:
    """Checksum packets ``base[byte_offset + i*stride : ... + length]``, i < n."""
    out = _out_tensor(out, n, base.device)
    _check("wc_cksum_strided", _lib.load().wc_cksum_strided(
        _dev_ptr(base) + byte_offset, stride, length, n, out.data_ptr(),
        _kind(kind), _stream_ptr(stream)))
    return out


def cksum_ragged(base: torch.Tensor, offsets: torch.Tensor, lengths: torch.Tensor,
                 out: Optional[torch.Tensor] = None, kind="ip",
                 stream=None) -> torch.Tensor:
    """Checksum packets ``base[off[i] : off[i] + len[i]]`` (uint64 / uint16 arrays)."""
    n = offsets.numel()
    if lengths.numel() != n or offsets.element_size() != 8 or lengths.element_size() != 2:
        raise ValueError("offsets must be 8-byte and lengths 2-byte, same count")
    out = _out_tensor(out, n, base.device)
    _check("wc_cksum_ragged", _lib.load().wc_cksum_ragged(
        _dev_ptr(base), _dev_ptr(offsets), _dev_ptr(lengths), n, out.data_ptr(),
        _kind(kind), _stream_ptr(stream)))
    return out


def verify_strided(base, stride, length, n, kind="payload", out=None,
                   stream=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """RX check (udp.c:132-139): results plus the count of non-zero checksums."""
    out = _out_tensor(out, n, base.device)
    bad = torch.zeros(1, dtype=torch.int64, device=base.device)
    _check("wc_verify_strided", _lib.load().wc_verify_strided(
        _dev_ptr(base), stride, length, n, out.data_ptr(), bad.data_ptr(),
        _kind(kind), _stream_ptr(stream)))
    return out, bad


def verify_ragged(base, offsets, lengths, kind="payload", out=None,
                  stream=None) -> Tuple[torch.Tensor, torch.Tensor]:
    n = offsets.numel()
    out = _out_tensor(out, n, base.device)
    bad = torch.zeros(1, dtype=torch.int64, device=base.device)
    _check("wc_verify_ragged", _lib.load().wc_verify_ragged(
        _dev_ptr(base), _dev_ptr(offsets), _dev_ptr(lengths), n, out.data_ptr(),
        bad.data_ptr(), _kind(kind), _stream_ptr(stream)))
    return out, bad


def cksum_ip_udp_strided(base: torch.Tensor, stride: int, length: int, n: int,
                        stream=None, byte_offset: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """One pass over IP/UDP packets: (IPv4 header checksums, payload_cksum).
    The header checksum is ip_cksum(ip, ip4_hl) (ip4.c:110-115, 184-186); 0
    for IPv6 packets."""
    hdr = _out_tensor(None, n, base.device)
    pay = _out_tensor(None, n, base.device)
    _check("wc_cksum_ip_udp_strided", _lib.load().wc_cksum_ip_udp_strided(
        _dev_ptr(base) + byte_offset, stride, length, n, hdr.data_ptr(), pay.data_ptr(),
        _stream_ptr(stream)))
    return hdr, pay


def cksum_ip_udp_ragged(base: torch.Tensor, offsets: torch.Tensor, lengths: torch.Tensor,
                        stream=None) -> Tuple[torch.Tensor, torch.Tensor]:
    n = offsets.numel()
    hdr = _out_tensor(None, n, base.device)
    pay = _out_tensor(None, n, base.device)
    _check("wc_cksum_ip_udp_ragged", _lib.load().wc_cksum_ip_udp_ragged(
        _dev_ptr(base), _dev_ptr(offsets), _dev_ptr(lengths), n, hdr.data_ptr(),
        pay.data_ptr(), _stream_ptr(stream)))
    return hdr, pay


# --------------------------------------------------------------------------
# Host-memory batches (end-to-end path).

def cksum_host(buf: np.ndarray, offsets: np.ndarray, lengths: np.ndarray,
               kind="ip") -> np.ndarray:
    """Checksum host-resident packets (synchronous), offsets in any order.

    Small batches in a registered buffer are read in place by one kernel;
    larger ones are streamed over pinned H2D copies (wc_cksum_host)."""
    buf = np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(lengths, dtype=np.uint16)
    out = np.empty(off.size, dtype=np.uint16)
    _check("wc_cksum_host", _lib.load().wc_cksum_host(
        buf.ctypes.data, buf.size, off.ctypes.data, lens.ctypes.data, off.size,
        out.ctypes.data, _kind(kind)))
    return out


def host_register(buf: np.ndarray) -> None:
    _check("wc_host_register", _lib.load().wc_host_register(buf.ctypes.data, buf.nbytes))


def host_unregister(buf: np.ndarray) -> None:
    _check("wc_host_unregister", _lib.load().wc_host_unregister(buf.ctypes.data))


# --------------------------------------------------------------------------
# Synthetic data / introspection.

def synth_fill(buf: torch.Tensor, seed: int, nbytes: Optional[int] = None,
               stream=None) -> torch.Tensor:
    """Fill a device buffer with the counter-based splitmix64 byte stream."""
    nbytes = buf.numel() * buf.element_size() if nbytes is None else nbytes
    _check("wc_synth_fill", _lib.load().wc_synth_fill(
        _dev_ptr(buf), nbytes, seed & 0xFFFFFFFFFFFFFFFF, _stream_ptr(stream)))
    return buf


def plan_strided(base_addr: int, stride: int, length: int, n: int, kind="ip") -> dict:
    vals = [ctypes.c_int() for _ in range(4)]
    _check("wc_plan_strided", _lib.load().wc_plan_strided(
        base_addr, stride, length, n, _kind(kind), *[ctypes.byref(v) for v in vals]))
    return dict(zip(("group", "chunks_per_lane", "unroll", "grid"), (v.value for v in vals)))


def gpu_init(device: int = -1) -> None:
    _check("wc_gpu_init", _lib.load().wc_gpu_init(device))


def version() -> str:
    return _lib.load().wc_version().decode()
