"""Multi-process (gloo, world sizes 2, 4 and 8, CPU) tests of the packet sharding used by
bench.py --gpus N: even contiguous shards, no data-path collective, results
gathered in packet order afterwards.  On CPU the per-rank compute is the
oracle (test infrastructure); on the GPU box it is libwccksum."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from warpcore_amd import dist as wdist
from warpcore_amd import synth


def test_shard_range_even_contiguous():
    for n in (0, 1, 7, 1 << 20, (1 << 28) + 3):
        for w in (1, 2, 3, 4, 8):
            ranges = [wdist.shard_range(n, r, w) for r in range(w)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


def test_shard_range_rejects_bad_rank():
    with pytest.raises(ValueError):
        wdist.shard_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, L, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import c_oracle
        buf = c_oracle.synth(n * L, synth.SEED)

        def compute(lo, hi):
            r = c_oracle.cksum_strided(buf[lo * L: hi * L], L, L, hi - lo, kind=0, threads=1)
            return torch.from_numpy(r.view(np.int16).copy())

        got = wdist.run_sharded(n, compute, gather=True)
        t = wdist.max_over_ranks(float(rank + 1))
        bad = wdist.sum_over_ranks(rank)
        wdist.barrier()
        q.put((rank, got.numpy().view(np.uint16).copy(), t, bad))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1001), (2, 4096), (4, 1001), (8, 1001), (8, 4099)])
def test_gloo_sharded_equals_whole_batch(world, n):
    """World sizes 2, 4 and 8 (the driver's 8-GPU run, rehearsed on gloo):
    uneven shards, the padded all-gather back in packet order, max and sum
    over the ranks."""
    from oracle import c_oracle
    L = 1472
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, L, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = c_oracle.cksum_strided(c_oracle.synth(n * L, synth.SEED), L, L, n, kind=0)
    for rank, got, t, bad in res:
        np.testing.assert_array_equal(got, whole)
        assert t == float(world)            # max over ranks
        assert bad == sum(range(world))     # sum over ranks


def test_library_split_matches_for_1_to_8_gpus():
    """wc_shard_range (the split the C host's *_multi calls use; pure
    arithmetic, no GPU) equals the torch.distributed shard split, G = 1..8,
    including uneven and 64-bit-sized batches."""
    import warpcore_amd as wc
    for n in (0, 1, 7, 1000, 1 << 20, (1 << 28) + 3, (1 << 62) + 5):
        for w in range(1, 9):
            got = [wc.shard_range(n, r, w) for r in range(w)]
            assert got == [wdist.shard_range(n, r, w) for r in range(w)]
            assert got[0][0] == 0 and got[-1][1] == n


def test_library_split_rejects_bad_shard():
    import warpcore_amd as wc
    for g, w in ((2, 2), (-1, 2), (0, 0)):
        with pytest.raises(wc.WcError):
            wc.shard_range(10, g, w)


def test_ragged_shards_cover_batch_in_order():
    """Ragged shards (offsets/lengths split by packet count) rebased per
    shard reproduce the whole batch in packet order."""
    lens = synth.zipf_lengths(10007, seed=3)
    offs = synth.packed_offsets(lens, lead=5)
    for w in range(1, 9):
        seen = []
        for r in range(w):
            o, l, first = wdist.shard_ragged(offs, lens, r, w)
            assert first == wdist.shard_range(offs.size, r, w)[0]
            seen.append((o, l))
        np.testing.assert_array_equal(np.concatenate([o for o, _ in seen]), offs)
        np.testing.assert_array_equal(np.concatenate([l for _, l in seen]), lens)
