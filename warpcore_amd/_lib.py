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
    "wc_server_pause": (_int, []),
    "wc_server_resume": (_int, []),
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


# The shipped library reads only these WC_* variables: the resident server's
# sizing and lifetime and the staging pool.  Every
# other WC_* path knob (kernel shapes, tile paths, RX modes, ...) is read by
# the tuning build alone (-DWC_TUNING, libwccksum_tune.so).
INTEGRATOR_KNOBS = frozenset({"WC_SERVE", "WC_SERVE_IDLE_US", "WC_SERVE_WAVES", "WC_SERVE_MAX",
                              "WC_STAGE_THREADS"})
# WC_* variables of the Python side, the build and the bench: not the library's.
NOT_LIBRARY = frozenset({"WC_NO_BUILD", "WC_TUNING", "WC_LIB", "WC_ALLOW_NO_GPU",
                         "WC_DIST_BACKEND", "WC_DIST_FORCE_PG"})

_tune = None     # the tuning build, once loaded
_active = None   # the build the mirror calls when it is not the primary one


def tuning_knobs(env=None) -> list:
    """The path knobs set in `env` (default os.environ): WC_* variables that
    only the tuning build reads."""
    env = os.environ if env is None else env
    return sorted(k for k, v in env.items() if k.startswith("WC_") and v != "" and
                  k not in INTEGRATOR_KNOBS and k not in NOT_LIBRARY)


def _open(path) -> ctypes.CDLL:
    lib = ctypes.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def is_tuning(lib: ctypes.CDLL) -> bool:
    return b"TUNING" in lib.wc_version()


def load(build_if_missing: bool = True) -> ctypes.CDLL:
    """Load (building in-tree first if absent or stale) libwccksum.so -- the
    primary library of this process."""
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
        _lib = _open(path)
        return _lib


def load_tuning() -> ctypes.CDLL:
    """The tuning build beside the primary library (built first if stale)."""
    global _tune
    primary = load()
    if is_tuning(primary):
        return primary
    with _lock:
        if _tune is None:
            path = _build.lib_path(True)
            if os.environ.get("WC_NO_BUILD") != "1":
                _build.build_lib(tuning=True)
            if not path.exists():
                raise RuntimeError(f"{path} is missing: build it with "
                                   "python -m warpcore_amd._build --tuning")
            _tune = _open(path)
        return _tune


def active() -> ctypes.CDLL:
    """The build every wrapper in warpcore_amd calls: the primary library,
    or the tuning build while select_for_env() found path knobs set."""
    return _active if _active is not None else load()


def select_for_env() -> ctypes.CDLL:
    """Pick the build for the current environment: the tuning build while any
    path knob is set (only it reads them), else the shipped library.  Called
    by warpcore_amd.reload_config()."""
    global _active
    _active = load_tuning() if tuning_knobs() and not is_tuning(load()) else None
    return active()
