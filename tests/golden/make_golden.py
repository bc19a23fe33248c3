"""Regenerate tests/golden/vectors.npz (regression vectors).

Expected values come from the independent pure-Python restatement
(oracle/py_oracle.py), NOT from the reference (which cannot be built here --
DESIGN.md section 3).  The file pins the C restatement, the GPU kernels and
future edits to one spec; the reference-derived known answers live in
kat.json.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
sys.path.insert(0, str(HERE.parent))

from oracle import py_oracle  # noqa: E402
from packets import pack, random_packets  # noqa: E402

SEED = 0x601DE7


def ip_cases(rng):
    blob = rng.integers(0, 256, 9100, dtype=np.uint8)
    blob[4000:4200] = 0x00
    blob[5000:5200] = 0xFF
    offs, lens = [], []
    lengths = list(range(0, 131)) + [1471, 1472, 1473, 8999, 9000, 9001]
    for start in range(16):
        for ln in lengths:
            offs.append(start)
            lens.append(ln)
    for base in (4000, 5000):          # all-zero / all-0xFF regions
        for start in range(4):
            for ln in (0, 1, 2, 63, 64, 65, 128, 150):
                offs.append(base + start)
                lens.append(ln)
    for _ in range(200):               # random placements
        ln = int(rng.integers(0, 9000))
        offs.append(int(rng.integers(0, 9100 - ln)))
        lens.append(ln)
    b = blob.tobytes()
    expect = [py_oracle.ip_cksum(b[o:o + ln]) for o, ln in zip(offs, lens)]
    return blob, np.array(offs, np.uint64), np.array(lens, np.uint16), np.array(expect, np.uint16)


def payload_cases(rng):
    pkts = random_packets(rng, 300, max_payload=1472, wild=True)
    buf, offs, lens = pack(pkts, align=1, lead=3)
    b = buf.tobytes()
    expect = [py_oracle.payload_cksum(b[int(o):int(o) + max(int(ln), 40)], int(ln))
              for o, ln in zip(offs, lens)]
    return buf, offs, lens, np.array(expect, np.uint16)


def main():
    rng = np.random.default_rng(SEED)
    ip_blob, ip_off, ip_len, ip_exp = ip_cases(rng)
    pl_blob, pl_off, pl_len, pl_exp = payload_cases(rng)
    np.savez_compressed(HERE / "vectors.npz", ip_blob=ip_blob, ip_off=ip_off, ip_len=ip_len,
                        ip_expect=ip_exp, pl_blob=pl_blob, pl_off=pl_off, pl_len=pl_len,
                        pl_expect=pl_exp)
    print(f"ip cases {ip_off.size}, payload cases {pl_off.size}")


if __name__ == "__main__":
    main()
