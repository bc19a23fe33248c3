"""Build recipes for the native pieces.

* ``libwccksum.so`` -- the product: gfx950 HIP kernels + C ABI
  (``include/warpcore_gpu/wc_cksum.h``), built in-tree with ``hipcc`` so the
  ``.so`` travels with the repo snapshot to the GPU box.
* ``libwccksum_tune.so`` -- the same sources with ``-DWC_TUNING``: the only
  build that reads the WC_* path knobs (kernel shapes, tile paths, RX modes),
  and where the experimental kernel branches (``WC_VARIANT``) and the
  timing-only no-load kernel (``WC_DIAG_NOLOAD``) are live.  ``tools/`` load
  it (``WC_TUNING=1``), and the tests that pin each path against the oracle
  reach it through ``warpcore_amd.reload_config()``; it is never the default.
* ``oracle/libwc_oracle.so`` -- TEST INFRASTRUCTURE (parity checker / CPU
  baseline).  Built per host CPU model (``-march=native``), into
  ``oracle/build-<cpu>/`` so a box with a different host CPU rebuilds it.

Staleness is decided by a hash of the sources and flags stored next to each
library (``<lib>.srchash``), not by file times: a tree copied to another
machine keeps its binary only if it was built from exactly these sources.
"""
from __future__ import annotations

import contextlib
import fcntl
import hashlib
import os
import platform
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "warpcore_amd"
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
LIB = PKG / "libwccksum.so"
LIB_TUNE = PKG / "libwccksum_tune.so"
ORACLE_DIR = ROOT / "oracle"

HIP_SOURCES = [CSRC / "wc_k_strided.hip", CSRC / "wc_k_lean.hip", CSRC / "wc_k_seg.hip",
               CSRC / "wc_k_flat.hip",
               CSRC / "wc_k_rx.hip", CSRC / "wc_k_serve.hip", CSRC / "wc_rccl.cpp",
               CSRC / "wc_k_synth.hip",
               CSRC / "wc_rt_config.cpp", CSRC / "wc_rt_plan.cpp", CSRC / "wc_rt_rx.cpp",
               CSRC / "wc_rt_server.cpp", CSRC / "wc_rt_host.cpp", CSRC / "wc_rt_multi.cpp"]
HIP_DEPS = HIP_SOURCES + [CSRC / "wc_cksum_kernels.h", CSRC / "wc_rccl.h", CSRC / "wc_device.h",
                          CSRC / "wc_rt.h",
                          CSRC / "wc_flat.h", CSRC / "wc_seg.h",
                          INCLUDE / "warpcore_gpu" / "wc_cksum.h"]
ORACLE_SOURCES = [ORACLE_DIR / "wc_oracle.c", ORACLE_DIR / "wc_oracle.h", ORACLE_DIR / "Makefile"]
BASE_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall",
              f"-I{INCLUDE}", f"-I{CSRC}"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    return "hipcc"


def _src_hash(deps, flags) -> str:
    h = hashlib.sha256()
    for d in deps:
        h.update(Path(d).name.encode())
        h.update(Path(d).read_bytes())
    h.update(" ".join(str(f) for f in flags).replace(str(ROOT), "<root>").encode())
    return h.hexdigest()


def _stamp(target: Path) -> Path:
    return target.with_name(target.name + ".srchash")


@contextlib.contextmanager
def _build_lock(target: Path):
    """One builder per target across processes: the ranks of a multi-GPU run
    start at once, and on a host whose CPU model has no oracle build yet every
    rank would otherwise compile it into the same file (seen in round 6: 8
    gloo ranks, `file too short` / a vanished `.tmp`).  The others wait, then
    find it current."""
    target.parent.mkdir(parents=True, exist_ok=True)
    with open(target.parent / f".{target.name}.lock", "w") as lf:
        try:
            fcntl.flock(lf, fcntl.LOCK_EX)
            locked = True
        except OSError:  # a filesystem without flock: per-process temp files still apply
            locked = False
        try:
            yield
        finally:
            if locked:
                fcntl.flock(lf, fcntl.LOCK_UN)


def _stale(target: Path, deps, flags) -> bool:
    st = _stamp(target)
    if not target.exists() or not st.exists():
        return True
    return st.read_text().strip() != _src_hash(deps, flags)


def lib_flags(tuning: bool = False) -> list:
    return BASE_FLAGS + (["-DWC_TUNING"] if tuning else [])


def lib_path(tuning: bool = False) -> Path:
    return LIB_TUNE if tuning else LIB


def lib_is_current(tuning: bool = False) -> bool:
    return not _stale(lib_path(tuning), HIP_DEPS, lib_flags(tuning))


def build_lib(force: bool = False, verbose: bool = False, tuning: bool = False) -> Path:
    """Compile libwccksum.so (or the tuning build) for gfx950 -- cross-compiles
    without a GPU: every translation unit in parallel into a scratch
    directory, then one link."""
    target, flags = lib_path(tuning), lib_flags(tuning)
    if not force and not _stale(target, HIP_DEPS, flags):
        return target
    with _build_lock(target):
        if not force and not _stale(target, HIP_DEPS, flags):
            return target  # another process built it while this one waited
        return _build_lib_locked(target, flags, verbose)


def _build_lib_locked(target: Path, flags, verbose: bool) -> Path:
    digest = _src_hash(HIP_DEPS, flags)
    with tempfile.TemporaryDirectory(prefix="wccksum-") as tmpdir:
        objs, procs = [], []
        for src in HIP_SOURCES:
            obj = Path(tmpdir) / (src.stem + ".o")
            cmd = [_hipcc(), *flags, "-c", str(src), "-o", str(obj)]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            procs.append((cmd, subprocess.Popen(cmd)))
            objs.append(str(obj))
        failed = [cmd for cmd, p in procs if p.wait() != 0]
        if failed:
            raise subprocess.CalledProcessError(1, failed[0])
        tmp = target.with_name(f"{target.name}.{os.getpid()}.tmp")
        cmd = [_hipcc(), "--offload-arch=gfx950", "-fPIC", "-shared", "-o", str(tmp), *objs]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    os.replace(tmp, target)
    _stamp(target).write_text(digest + "\n")
    return target


def _cpu_tag() -> str:
    model = platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name") or line.startswith("flags"):
                    model += line
    except OSError:
        pass
    return hashlib.sha1(model.encode()).hexdigest()[:10]


def oracle_path() -> Path:
    # WC_ORACLE_BUILD_TAG (tests only) names a build directory of its own
    tag = os.environ.get("WC_ORACLE_BUILD_TAG") or _cpu_tag()
    return ORACLE_DIR / f"build-{tag}" / "libwc_oracle.so"


def build_oracle(force: bool = False, verbose: bool = False) -> Path:
    """Compile the CPU restatement (test infrastructure) for this host CPU."""
    out = oracle_path()
    if not force and not _stale(out, ORACLE_SOURCES, ["oracle"]):
        return out
    with _build_lock(out):
        if not force and not _stale(out, ORACLE_SOURCES, ["oracle"]):
            return out  # another process built it while this one waited
        tmp = out.with_name(f"{out.name}.{os.getpid()}.tmp")
        cmd = ["make", "-s", "-C", str(ORACLE_DIR), f"OUT={tmp}", "oracle"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(tmp, out)
        _stamp(out).write_text(_src_hash(ORACLE_SOURCES, ["oracle"]) + "\n")
    return out


def build_all(force: bool = False, verbose: bool = False, tuning: bool = True) -> None:
    """The product library, the tuning build (the tests pin every path knob's
    kernels through it) and the oracle."""
    build_lib(force=force, verbose=verbose)
    if tuning:
        build_lib(force=force, verbose=verbose, tuning=True)
    build_oracle(force=force, verbose=verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, verbose=True, tuning="--no-tuning" not in sys.argv)
