"""Build the C test programs under tests/c (gcc, linked against the in-tree
libwccksum.so and the oracle's C restatement) -- shared by the CPU and GPU
tests that run them."""
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def build(name: str, out_dir: Path) -> Path:
    exe = Path(out_dir) / name
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-D__HIP_PLATFORM_AMD__",
                    "-I/opt/rocm/include", f"-I{ROOT / 'include'}", f"-I{ROOT / 'oracle'}",
                    str(ROOT / "tests" / "c" / f"{name}.c"), str(ROOT / "oracle" / "wc_oracle.c"),
                    "-o", str(exe), f"-L{ROOT / 'warpcore_amd'}", "-lwccksum",
                    "-L/opt/rocm/lib", "-lamdhip64", "-lpthread",
                    f"-Wl,-rpath,{ROOT / 'warpcore_amd'}"], check=True)
    return exe
