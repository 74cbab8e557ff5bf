"""Multi-GPU sharding host logic, including a world_size-2
gloo run of the same orchestration bench.py uses: per-rank digests gathered
over torch.distributed and combined into the global digest."""
import json
import os
import socket

import numpy as np
import pytest

from consus_amd import shard

GOLD = os.path.join(os.path.dirname(__file__), "golden", "digests.json")


def test_balanced_ranges_cover_and_balance():
    rng = np.random.default_rng(0)
    lens = rng.integers(1, 65536, 10000)
    for world in (1, 2, 3, 8):
        rs = shard.balanced_ranges(lens, world)
        assert rs[0][0] == 0 and rs[-1][1] == len(lens)
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        sums = [int(lens[lo:hi].sum()) for lo, hi in rs]
        assert max(sums) - min(sums) <= 2 * 65536


def test_balanced_ranges_fewer_records_than_ranks():
    rs = shard.balanced_ranges(np.array([5, 7]), 4)
    assert rs[-1][1] == 2 and sum(hi - lo for lo, hi in rs) == 2


def test_combine_block_digests_equals_global():
    g = json.load(open(GOLD))["fixed_4096_seed0xc0de_per_1048576"]
    blocks = g["block_digests"]
    assert shard.combine_digests(blocks, [1 << 20] * 16) == g["global_16M_digest"]
    assert shard.combine_digests(blocks[:8], [1 << 20] * 8) == g["global_8M_digest"]
    pairs = [shard.combine_digests(blocks[2 * k:2 * k + 2], [1 << 20] * 2) for k in range(8)]
    assert pairs == g["global_2M_blocks_digests"]


def _worker(rank, world, port, result_path):
    import torch
    import torch.distributed as dist
    from oracle.oracle import Oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orc = Oracle()
    rng = np.random.default_rng(42)
    lens = rng.integers(0, 20000, 3000).astype(np.uint32)
    offs = np.zeros(lens.size, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    data = orc.fill(int(lens.sum()), 0x5EED, 0)
    lo, hi = shard.balanced_ranges(lens, world)[rank]
    crcs = orc.batch(data, offs[lo:hi], lens[lo:hi])
    d = orc.digest(crcs)[0] if hi > lo else 0
    got = [None] * world
    dist.all_gather_object(got, (d, hi - lo))
    if rank == 0:
        glob = shard.combine_digests([x[0] for x in got], [x[1] for x in got])
        full = orc.digest(orc.batch(data, offs, lens))[0]
        with open(result_path, "w") as f:
            json.dump({"combined": glob, "full": full}, f)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_digest_gather(tmp_path):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tmp_path / "r.json"
    mp.spawn(_worker, args=(2, port, str(out)), nprocs=2, join=True)
    r = json.load(open(out))
    assert r["combined"] == r["full"]


def test_record_slices_cover():
    for n in (0, 1, 4095, 4096 * 8 - 1, 4096 * 8, 10**7 + 3):
        for world in (1, 2, 3, 8):
            sl = shard.record_slices(n, world)
            assert len(sl) == world and sl[0][0] == 0
            assert all(a[0] + a[1] == b[0] for a, b in zip(sl, sl[1:]))
            assert sl[-1][0] + sl[-1][1] == n
            assert all(s % 4096 == 0 for s, _ in sl)


def test_fold_slice_crcs_matches_whole_record(oracle):
    """One record split over 1..8 ranks: the fold of the per-slice CRCs
    equals crc32c(init, record) from the oracle, empty slices included."""
    rng = np.random.default_rng(7)
    for n in (0, 100, 4096 * 3 + 5, 200000):
        buf = rng.integers(0, 256, n, dtype=np.uint8)
        for world in (1, 2, 3, 8):
            for init in (0, int(rng.integers(0, 2**32))):
                sl = shard.record_slices(n, world, align=4096)
                crcs = [oracle.crc32c(0, buf[s:s + L]) for s, L in sl]
                assert shard.fold_slice_crcs(crcs, [L for _, L in sl], init) == \
                    oracle.crc32c(init, buf)


def _split_worker(rank, world, port, result_path):
    import torch.distributed as dist
    from oracle.oracle import Oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orc = Oracle()
    n = 3 * 4096 * 5 + 777
    data = orc.fill(n, 0xC0DE, 0)
    s, L = shard.record_slices(n, world)[rank]
    got = shard.gather_fold(orc.crc32c(0, data[s:s + L]), L, init=0x1234ABCD)
    if rank == 0:
        with open(result_path, "w") as f:
            json.dump({"folded": got, "whole": orc.crc32c(0x1234ABCD, data)}, f)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_split_record(tmp_path):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tmp_path / "split.json"
    mp.spawn(_split_worker, args=(2, port, str(out)), nprocs=2, join=True)
    r = json.load(open(out))
    assert r["folded"] == r["whole"]
