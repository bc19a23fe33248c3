"""CPU tests of the Python mirror's argument checks: a wrong count, a short
buffer, a length past uint16 or a host tensor raise ValueError before any
pointer reaches the library (no GPU here, so no compute call is made)."""
import numpy as np
import pytest
import torch

import warpcore_amd as wc
from warpcore_amd import cksum


def test_strided_extent_checked():
    base = torch.empty(1472 * 10, dtype=torch.uint8)
    cksum._check_strided(base, 0, 1472, 1472, 10, wc.KIND_IP)
    with pytest.raises(ValueError, match="runs past"):
        cksum._check_strided(base, 0, 1472, 1472, 11, wc.KIND_IP)
    with pytest.raises(ValueError, match="runs past"):
        cksum._check_strided(base, 1, 1472, 1472, 10, wc.KIND_IP)
    # overlapping stride (stride < len) is allowed while it fits
    cksum._check_strided(base, 0, 16, 1472, 100, wc.KIND_IP)
    # payload_cksum reads the 20-byte IPv4 header whatever len is
    small = torch.empty(19, dtype=torch.uint8)
    cksum._check_strided(small, 0, 0, 4, 1, wc.KIND_IP)
    with pytest.raises(ValueError):
        cksum._check_strided(small, 0, 0, 4, 1, wc.KIND_PAYLOAD)
    with pytest.raises(ValueError):
        cksum._check_strided(base, -1, 1472, 1472, 1, wc.KIND_IP)


def test_ragged_bounds_checked():
    off = torch.tensor([0, 100, 4000], dtype=torch.int64)
    ln = torch.tensor([100, 1472, 96], dtype=torch.int16)
    cksum._ragged_bounds(4096, off, ln, wc.KIND_IP)
    with pytest.raises(ValueError, match="runs past"):
        cksum._ragged_bounds(4095, off, ln, wc.KIND_IP)
    # uint16 lengths above 32767 are read unsigned
    big = torch.from_numpy(np.array([40000], dtype=np.uint16).view(np.int16))
    with pytest.raises(ValueError):
        cksum._ragged_bounds(39999, torch.tensor([0]), big, wc.KIND_IP)
    cksum._ragged_bounds(40000, torch.tensor([0]), big, wc.KIND_IP)
    with pytest.raises(ValueError):
        cksum._ragged_bounds(1 << 20, torch.tensor([-1]), ln[:1], wc.KIND_IP)
    with pytest.raises(ValueError):  # 20 header bytes for payload_cksum
        cksum._ragged_bounds(4010, torch.tensor([3995]), torch.tensor([4], dtype=torch.int16),
                             wc.KIND_PAYLOAD)


def test_length_range():
    for bad in (-1, 65536, 1 << 20):
        with pytest.raises(ValueError):
            cksum._check_len(bad)
    assert cksum._check_len(65535) == 65535


def test_host_tensors_rejected():
    base = torch.zeros(4096, dtype=torch.uint8)
    with pytest.raises(ValueError, match="device"):
        wc.cksum_strided(base, 64, 64, 4)
    with pytest.raises(ValueError, match="device"):
        wc.cksum_ragged(base, torch.zeros(1, dtype=torch.int64), torch.zeros(1, dtype=torch.int16))
    with pytest.raises(ValueError, match="device"):
        wc.synth_fill(base, 1)


def test_ragged_dtypes_checked():
    cases = ((torch.zeros(2, dtype=torch.int32), torch.zeros(2, dtype=torch.int16)),
             (torch.zeros(2, dtype=torch.int64), torch.zeros(3, dtype=torch.int16)),
             (torch.zeros(2, dtype=torch.float64), torch.zeros(2, dtype=torch.int16)),
             (torch.zeros(2, dtype=torch.int64), torch.zeros(2, dtype=torch.float16)),
             (torch.zeros(4, dtype=torch.int64)[::2], torch.zeros(2, dtype=torch.int16)))
    for off, ln in cases:
        with pytest.raises(ValueError):
            cksum._check_ragged_shapes(off, ln)
    assert cksum._check_ragged_shapes(torch.zeros(5, dtype=torch.int64),
                                      torch.zeros(5, dtype=torch.int16)) == 5


def test_host_path_lengths_checked():
    buf = np.zeros(1 << 17, dtype=np.uint8)
    with pytest.raises(ValueError, match="uint16"):
        wc.cksum_host(buf, np.array([0]), np.array([70000]))
    with pytest.raises(ValueError):
        wc.cksum_host(buf, np.array([-5]), np.array([10]))
    with pytest.raises(ValueError):
        wc.cksum_host(buf, np.array([0, 1]), np.array([10]))
