"""Synthetic workload helpers (CPU): stamped UDP headers are well-formed."""
import numpy as np
import torch

from oracle import py_oracle
from packets import insert_checksum
from warpcore_amd import synth


def test_stamp_udp_headers_well_formed():
    rng = np.random.default_rng(5)
    lens = rng.integers(48, 1501, 300).astype(np.uint16)
    offs = synth.packed_offsets(lens, lead=3)
    buf = torch.from_numpy(rng.integers(0, 256, int(offs[-1]) + 1600, dtype=np.uint8))
    synth.stamp_udp_headers(buf, offs, lens)
    b = buf.numpy()
    for i, (o, ln) in enumerate(zip(offs.tolist(), lens.tolist())):
        p = bytes(b[o:o + ln])
        if i % 3 == 0:  # IPv6
            assert p[0] == 0x60 and p[6] == 17
            assert int.from_bytes(p[4:6], "big") == ln - 40
            assert int.from_bytes(p[44:46], "big") == ln - 40 and p[46:48] == b"\0\0"
        else:           # IPv4, IHL 5
            assert p[0] == 0x45 and p[9] == 17
            assert int.from_bytes(p[2:4], "big") == ln
            assert int.from_bytes(p[24:26], "big") == ln - 20 and p[26:28] == b"\0\0"
        # the TX checksum stored into udp->cksum makes the RX check 0 (udp.c:132-139)
        assert py_oracle.payload_cksum(insert_checksum(p, py_oracle.payload_cksum(p, ln)), ln) == 0
