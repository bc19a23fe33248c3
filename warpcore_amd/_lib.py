"""ctypes binding of libwccksum.so (the C ABI in include/warpcore_gpu/wc_cksum.h).

The library links the HIP runtime by SONAME (libamdhip64.so.7).  torch is
imported first so that, inside a Python process, the library binds to the same
HIP runtime instance torch already loaded (one runtime, one set of streams);
standalone C callers get /opt/rocm's copy.

There is no fallback: if the shared object is missing or fails to load, every
entry point raises.  On a GPU box the library is (re)built in-tree first.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  -- must precede the CDLL load (shared HIP runtime)

from . import _build

_lock = threading.Lock()
_lib = None

# Every symbol the public header declares, with its ctypes signature.
_u16, _u64, _int, _vp = ctypes.c_uint16, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p
SIGNATURES = {
    "ip_cksum": (_u16, [_vp, _u16]),
    "payload_cksum": (_u16, [_vp, _u16]),
    "wc_cksum_strided": (_int, [_vp, _u64, _u16, _u64, _vp, _int, _vp]),
    "wc_cksum_ragged": (_int, [_vp, _vp, _vp, _u64, _vp, _int, _vp]),
    "wc_verify_strided": (_int, [_vp, _u64, _u16, _u64, _vp, _vp, _int, _vp]),
    "wc_verify_ragged": (_int, [_vp, _vp, _vp, _u64, _vp, _vp, _int, _vp]),
    "wc_cksum_ip_udp_strided": (_int, [_vp, _u64, _u16, _u64, _vp, _vp, _vp]),
    "wc_cksum_ip_udp_ragged": (_int, [_vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    "wc_rx_verdict_ragged": (_int, [_vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    "wc_rx_verdict_host": (_int, [_vp, _u64, _vp, _vp, _u64, _vp, _vp]),
    "wc_cksum_host": (_int, [_vp, _u64, _vp, _vp, _u64, _vp, _int]),
    "wc_cksum_ip_udp_host": (_int, [_vp, _u64, _vp, _vp, _u64, _vp, _vp]),
    "wc_server_stats": (_int, [ctypes.POINTER(_u64), ctypes.POINTER(_u64),
                               ctypes.POINTER(_u64)]),
    "wc_host_register": (_int, [_vp, _u64]),
    "wc_host_unregister": (_int, [_vp]),
    "wc_gpu_init": (_int, [_int]),
    "wc_gpu_init_multi": (_int, [_int, _vp]),
    "wc_gpu_multi_count": (_int, []),
    "wc_shard_range": (_int, [_u64, _int, _int, ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    "wc_cksum_host_multi": (_int, [_vp, _u64, _vp, _vp, _u64, _vp, _int]),
    "wc_cksum_strided_multi": (_int, [_vp, _u64, _u16, _vp, _vp, _int, _vp]),
    "wc_cksum_ragged_multi": (_int, [_vp, _vp, _vp, _vp, _vp, _int, _vp]),
    "wc_gather_results_multi": (_int, [_vp, _vp, _vp, _vp]),
    "wc_gpu_fini": (_int, []),
    "wc_config_reload": (_int, []),
    "wc_synth_fill": (_int, [_vp, _u64, _u64, _vp]),
    "wc_sclk_probe": (_int, [_vp, _int, _u64, _vp]),
    "wc_plan_strided": (_int, [_u64, _u64, _u16, _u64, _int,
                               ctypes.POINTER(_int), ctypes.POINTER(_int),
                               ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "wc_plan_strided_kernel": (ctypes.c_char_p, [_u64, _u64, _u16, _u64, _int]),
    "wc_strerror": (ctypes.c_char_p, [_int]),
    "wc_version": (ctypes.c_char_p, []),
}


def load(build_if_missing: bool = True) -> ctypes.CDLL:
    """Load (building in-tree first if absent or stale) libwccksum.so."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        # WC_TUNING=1 (tools/ only): the -DWC_TUNING build, where the
        # experimental WC_VARIANT branches and WC_DIAG_NOLOAD are live.
        tuning = os.environ.get("WC_TUNING") == "1"
        path = _build.lib_path(tuning)
        if os.environ.get("WC_LIB"):  # A/B tuning of two builds (tools/)
            path = _build.Path(os.environ["WC_LIB"])
        elif build_if_missing and os.environ.get("WC_NO_BUILD") != "1":
            _build.build_lib(tuning=tuning)
        if not path.exists():
            raise RuntimeError(
                f"{path} is missing: the gfx950 HIP library must be built "
                "(python -m warpcore_amd._build); there is no CPU fallback")
        lib = ctypes.CDLL(str(path))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib
