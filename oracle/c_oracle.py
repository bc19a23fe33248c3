"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the C restatement (wc_oracle.c).

Used by tests/ as the parity checker at full sizes and by bench.py's
cpu_baseline leg as the timed CPU baseline ("port").  Never imported by the
product package.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_lock = threading.Lock()
_lib = None


def load() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            from warpcore_amd import _build  # build recipe only (no product code)
            path = _build.build_oracle()
            lib = ctypes.CDLL(str(path))
            u16, u32, u64, i, vp = (ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64,
                                    ctypes.c_int, ctypes.c_void_p)
            sig = {
                "oracle_ip_sum": (u32, [vp, u16]),
                "oracle_payload_sum": (u32, [vp, u16]),
                "oracle_fold": (u16, [u32]),
                "oracle_ip_cksum": (u16, [vp, u16]),
                "oracle_payload_cksum": (u16, [vp, u16]),
                "oracle_cksum_strided": (None, [vp, u64, u16, u64, vp, i, i]),
                "oracle_cksum_ragged": (None, [vp, vp, vp, u64, vp, i, i]),
                "oracle_bench_strided": (ctypes.c_double,
                                         [vp, u64, u16, u64, vp, i, i, ctypes.c_double,
                                          ctypes.POINTER(u64)]),
                "oracle_synth_fill": (None, [vp, u64, u64]),
                "oracle_rx_verdict": (i, [vp, u16]),
                "oracle_rx_verdict_ragged": (None, [vp, vp, vp, u64, vp, i]),
            }
            for name, (res, args) in sig.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def default_threads() -> int:
    """Host threads for batch checks (the GPU box's share is 16 cores)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


def _u8(buf) -> np.ndarray:
    a = np.ascontiguousarray(buf)
    return a.reshape(-1).view(np.uint8)


def ip_cksum(buf, length=None) -> int:
    a = _u8(np.frombuffer(bytes(buf), dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf)
    length = a.size if length is None else length
    return int(load().oracle_ip_cksum(a.ctypes.data, length))


def payload_cksum(buf, length=None) -> int:
    a = _u8(np.frombuffer(bytes(buf), dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf)
    length = a.size if length is None else length
    return int(load().oracle_payload_cksum(a.ctypes.data, length))


def cksum_strided(buf: np.ndarray, stride: int, length: int, n: int, kind: int = 0,
                  threads: int | None = None, byte_offset: int = 0) -> np.ndarray:
    a = _u8(buf)
    if n and byte_offset + (n - 1) * stride + (max(length, 20) if kind else length) > a.size:
        raise ValueError("batch exceeds buffer")
    out = np.empty(n, dtype=np.uint16)
    load().oracle_cksum_strided(a.ctypes.data + byte_offset, stride, length, n,
                                out.ctypes.data, kind, threads or default_threads())
    return out


def cksum_ragged(buf: np.ndarray, off: np.ndarray, lens: np.ndarray, kind: int = 0,
                 threads: int | None = None) -> np.ndarray:
    a = _u8(buf)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    out = np.empty(off.size, dtype=np.uint16)
    load().oracle_cksum_ragged(a.ctypes.data, off.ctypes.data, lens.ctypes.data, off.size,
                               out.ctypes.data, kind, threads or default_threads())
    return out


def rx_verdict(frame, flen=None) -> int:
    a = _u8(np.frombuffer(bytes(frame), dtype=np.uint8) if not isinstance(frame, np.ndarray)
            else frame)
    flen = a.size if flen is None else flen
    if flen > a.size:
        raise ValueError("frame shorter than flen")
    return int(load().oracle_rx_verdict(a.ctypes.data, flen))


def rx_verdict_ragged(buf: np.ndarray, off: np.ndarray, flen: np.ndarray,
                      threads: int | None = None) -> np.ndarray:
    """RX verdicts (uint8 codes) of the frames buf[off[i] : off[i] + flen[i]]."""
    a = _u8(buf)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    flen = np.ascontiguousarray(flen, dtype=np.uint16)
    if off.size and int((off + flen).max()) > a.size:
        raise ValueError("a frame runs past the buffer")
    out = np.empty(off.size, dtype=np.uint8)
    load().oracle_rx_verdict_ragged(a.ctypes.data, off.ctypes.data, flen.ctypes.data, off.size,
                                    out.ctypes.data, threads or default_threads())
    return out


def bench_strided(buf: np.ndarray, stride: int, length: int, n: int, kind: int = 0,
                  threads: int = 1, min_seconds: float = 10.0):
    """Time the CPU restatement; returns (bytes_per_second, passes)."""
    a = _u8(buf)
    out = np.empty(n, dtype=np.uint16)
    passes = ctypes.c_uint64()
    bps = load().oracle_bench_strided(a.ctypes.data, stride, length, n, out.ctypes.data,
                                      kind, threads, min_seconds, ctypes.byref(passes))
    return float(bps), int(passes.value)


def synth(nbytes: int, seed: int) -> np.ndarray:
    """Host copy of the counter-based splitmix64 byte stream (wc_synth_fill)."""
    out = np.empty(nbytes, dtype=np.uint8)
    load().oracle_synth_fill(out.ctypes.data, nbytes, seed & 0xFFFFFFFFFFFFFFFF)
    return out
