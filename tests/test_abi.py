"""CPU tests of the drop-in boundary: the gfx950 library builds, loads and
exports exactly the C ABI that include/warpcore_gpu/wc_cksum.h declares
(no compute calls -- there is no GPU here)."""
import re
import subprocess
from pathlib import Path

from warpcore_amd import _build, _lib

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "warpcore_gpu" / "wc_cksum.h"


def declared_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*([a-z_0-9]+)\s*\(", text, re.M))


def exported_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", str(path)], check=True,
                         capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_header_declares_reference_entry_points():
    names = declared_functions()
    # in_cksum.h:32-36 -- the two functions the reference's callers bind.
    assert {"ip_cksum", "payload_cksum"} <= names
    assert "wc_cksum_strided" in names and "wc_cksum_ragged" in names


def test_library_builds_and_exports_every_declared_symbol():
    lib = _build.build_lib()
    exported = exported_symbols(lib)
    missing = declared_functions() - exported
    assert not missing, f"declared but not exported: {missing}"


def test_python_binding_covers_header():
    assert declared_functions() == set(_lib.SIGNATURES)


def test_ctypes_load():
    lib = _lib.load()
    assert lib.wc_version().decode().startswith("wccksum")
    assert lib.wc_strerror(-10001).decode() == "invalid argument"


def test_code_object_targets_gfx950_only():
    blob = _build.build_lib().read_bytes()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-[-a-z0-9:+]*gfx[0-9a-z]+", blob))
    assert targets == {b"amdgcn-amd-amdhsa--gfx950"}


def test_production_library_has_no_tuning_paths():
    """WC_VARIANT / WC_DIAG_NOLOAD (result-dropping A/B knobs) exist only in
    the -DWC_TUNING build: the shipped library carries no no-load kernel,
    and its version string says it is not the tuning build."""
    lib = _build.build_lib()
    syms = subprocess.run(["nm", "-DC", str(lib)], check=True, capture_output=True,
                          text=True).stdout
    flat = re.findall(r"wc::k_cksum_flat<(\d+), (\d+), (\w+), (\w+), (\w+), (\d+)>", syms)
    assert flat and not any(noload == "true" for *_, noload, _pk in flat)
    assert "TUNING" not in _lib.load().wc_version().decode()
    text = (ROOT / "warpcore_amd" / "csrc" / "wc_rt_config.cpp").read_text()
    # the env reads of both knobs sit inside #ifdef WC_TUNING
    block = text[text.index("#ifdef WC_TUNING"):text.index("#endif", text.index("#ifdef WC_TUNING"))]
    assert '"WC_VARIANT"' in block and '"WC_DIAG_NOLOAD"' in block
    assert text.count('"WC_VARIANT"') == 1 and text.count('"WC_DIAG_NOLOAD"') == 1


def _env_reads_outside_tuning(text: str) -> set:
    """WC_* names a source reads from the environment outside its
    #ifdef WC_TUNING ... #endif blocks."""
    out = re.sub(r"#ifdef WC_TUNING.*?#endif", "", text, flags=re.S)
    return set(re.findall(r'(?:env_int|env_u64|getenv|parse_shape\(getenv)\("(WC_[A-Z_]+)"', out))


def test_production_library_reads_only_integrator_knobs():
    """The shipped library's paths are a compile-time table: outside the
    tuning build it reads only the server's sizing / lifetime and the
    staging pool's width from the environment."""
    reads = set()
    for src in sorted((ROOT / "warpcore_amd" / "csrc").glob("wc_rt*.cpp")):
        reads |= _env_reads_outside_tuning(src.read_text())
    assert reads == set(_lib.INTEGRATOR_KNOBS), reads


def test_path_knobs_select_the_tuning_build(monkeypatch):
    """warpcore_amd.reload_config() sends the mirror's calls to the tuning
    build while a path knob is set (only it reads them), and back to the
    shipped library once none is."""
    for k in _lib.tuning_knobs():
        monkeypatch.delenv(k)
    assert not _lib.is_tuning(_lib.select_for_env())
    monkeypatch.setenv("WC_SHAPE", "32,4,1")
    monkeypatch.setenv("WC_SERVE_IDLE_US", "5000")  # an integrator knob: not a path knob
    assert _lib.tuning_knobs() == ["WC_SHAPE"]
    assert _lib.is_tuning(_lib.select_for_env())
    monkeypatch.delenv("WC_SHAPE")
    assert not _lib.is_tuning(_lib.select_for_env())
    assert _lib.active() is _lib.load()


def test_build_staleness_is_a_source_hash():
    """A copied tree keeps its binary only if the sources hash the same."""
    _build.build_lib()
    assert _build.lib_is_current()
    stamp = _build._stamp(_build.LIB)
    assert stamp.read_text().strip() == _build._src_hash(_build.HIP_DEPS, _build.lib_flags())


def test_argument_errors_need_no_gpu():
    """The C ABI rejects bad arguments before it touches a device, the way
    the reference's callers see errors: WC_EINVAL for a NULL buffer or result
    pointer and an unknown kind, WC_OK for an empty batch -- none of these
    calls reaches HIP, so they run here without a GPU."""
    lib = _lib.load()
    ok, einval = 0, -10001
    p = 0x100000  # never dereferenced: every call below returns first
    # empty batches
    assert lib.wc_cksum_strided(None, 2048, 64, 0, None, 0, None) == ok
    assert lib.wc_cksum_ragged(None, None, None, 0, None, 1, None) == ok
    assert lib.wc_rx_verdict_ragged(None, None, None, 0, None, None, None) == ok
    # missing result arrays
    assert lib.wc_cksum_strided(p, 2048, 64, 8, None, 0, None) == einval
    assert lib.wc_cksum_ragged(p, p, p, 8, None, 0, None) == einval
    assert lib.wc_verify_strided(p, 2048, 64, 8, p, None, 0, None) == einval
    assert lib.wc_cksum_ip_udp_strided(p, 2048, 64, 8, None, p, None) == einval
    assert lib.wc_cksum_ip_udp_strided(p, 2048, 64, 8, p, None, None) == einval
    # missing packet arrays
    assert lib.wc_cksum_strided(None, 2048, 64, 8, p, 0, None) == einval
    assert lib.wc_cksum_ragged(p, None, p, 8, p, 0, None) == einval
    assert lib.wc_rx_verdict_ragged(p, p, None, 8, p, None, None) == einval
    # unknown kind (WC_CKSUM_IP = 0, WC_CKSUM_PAYLOAD = 1)
    assert lib.wc_cksum_strided(p, 2048, 64, 8, p, 7, None) == einval
    assert lib.wc_cksum_ragged(p, p, p, 8, p, -1, None) == einval
    # the shader-clock probe: nothing to do, or no / misaligned sample array
    assert lib.wc_sclk_probe(None, 0, 2000, None) == ok
    assert lib.wc_sclk_probe(None, 8, 2000, None) == einval
    assert lib.wc_sclk_probe(p + 4, 8, 2000, None) == einval
    assert lib.wc_sclk_probe(p, 8, 0, None) == einval
    assert lib.wc_strerror(einval).decode() == "invalid argument"


def test_host_call_argument_errors_need_no_gpu():
    """The host-memory calls check their batch against the region before
    touching a device: NULL result arrays, packets past the region -- for the
    fused pair also an IPv4 header (hl bytes, options included) that runs past
    it even where len is shorter -- are WC_EINVAL; an empty batch is WC_OK;
    wc_server_stats needs no device either."""
    import ctypes

    import numpy as np
    lib = _lib.load()
    ok, einval = 0, -10001
    buf = np.zeros(100, dtype=np.uint8)
    off = np.array([50], dtype=np.uint64)
    ln = np.array([20], dtype=np.uint16)
    out = np.zeros(1, dtype=np.uint16)
    hdr = np.zeros(1, dtype=np.uint16)
    b, o, n_, r, h = (a.ctypes.data for a in (buf, off, ln, out, hdr))
    assert lib.wc_cksum_ip_udp_host(b, 100, o, n_, 0, None, None) == ok
    assert lib.wc_cksum_ip_udp_host(b, 100, o, n_, 1, None, r) == einval
    assert lib.wc_cksum_ip_udp_host(b, 100, o, n_, 1, h, None) == einval
    assert lib.wc_cksum_host(b, 100, o, n_, 1, None, 0) == einval
    off[0] = 90  # 20 bytes from 90: past the 100-byte region
    assert lib.wc_cksum_host(b, 100, o, n_, 1, r, 0) == einval
    assert lib.wc_cksum_ip_udp_host(b, 100, o, n_, 1, h, r) == einval
    off[0] = 50
    buf[50] = 0x4F  # IPv4, IHL 15: ip_cksum reads 60 bytes, 50 are left
    assert lib.wc_cksum_ip_udp_host(b, 100, o, n_, 1, h, r) == einval
    vals = [ctypes.c_uint64(7) for _ in range(3)]
    assert lib.wc_server_stats(*[ctypes.byref(v) for v in vals]) == ok
    assert lib.wc_server_stats(None, None, None) == ok
