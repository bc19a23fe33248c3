import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
TESTS = Path(__file__).resolve().parent
if str(TESTS) not in sys.path:
    sys.path.insert(0, str(TESTS))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def gpu():
    """The GPU is required: a gpu-marked test never silently skips on a box
    that should have one (set WC_ALLOW_NO_GPU=1 to skip instead)."""
    import torch
    if not torch.cuda.is_available():
        if os.environ.get("WC_ALLOW_NO_GPU") == "1":
            pytest.skip("no GPU")
        raise RuntimeError("gpu-marked test but torch.cuda.is_available() is False")
    import warpcore_amd
    warpcore_amd.gpu_init(0)
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _fresh_wc_config():
    """libwccksum reads its WC_* environment once; a test that monkeypatches
    it calls wc.reload_config() (which also moves the mirror's calls to the
    tuning build while a path knob is set: only that build reads them), and
    every test starts from the (restored) environment of the session, on the
    shipped library."""
    from warpcore_amd import _lib
    if _lib._lib is not None:
        for lib in {id(x): x for x in (_lib._lib, _lib._tune) if x is not None}.values():
            lib.wc_config_reload()
        _lib.select_for_env()
    yield
