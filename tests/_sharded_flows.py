"""One rank of the N > 1 flows with the ENGINE on every rank
(not the oracle): driven by tests/test_gpu_multi.py as 2 processes sharing
the one GPU of the test box, gloo as the control plane (RCCL needs one GPU
per rank; the driver's 8-GPU run covers it).  The same flows as bench.py's
multi-rank paths, at the sizes bench.py runs them per rank:

  fixed   each rank hashes its own 2M x 4 KiB shard of the configs[1]/[3]
          stream (record offset rank * 2M), generated in HBM;
  zipf    configs[2]'s record stream continued to world x 1M records, split
          by bytes (shard.balanced_ranges), each rank generating exactly its
          records' bytes;
  single  one world x 4 GiB record, rank r holding slice r
          (shard.record_slices), folded from the gathered (crc, length) pairs.

Rank 0 checks every flow against the reference's golden digests and prints
one JSON line.  Environment: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT.
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import consus_amd as E
    from consus_amd import shard
    from consus_amd import workload as W
    E.init(0)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    gold = json.load(open(os.path.join(REPO, "tests", "golden", "digests.json")))
    res = {}

    # fixed: 2M x 4 KiB per rank
    R, L, blk = 2 << 20, 4096, 1 << 20
    data = E.DeviceBuffer(R * L)
    out = E.DeviceBuffer(R * 4)
    data.fill_splitmix64(0xC0DE, byte_offset=rank * R * L)
    E.device_batch_fixed(data, L, L, R, out)
    dig = E.crc32c_device(out, R * 4)
    data.free()
    out.free()
    got = [None] * world
    dist.all_gather_object(got, dig)
    if rank == 0:
        bd = gold["fixed_4096_seed0xc0de_per_1048576"]["block_digests"]
        k = R // blk
        want = [shard.combine_digests(bd[i * k:(i + 1) * k], [blk] * k) for i in range(world)]
        res["fixed"] = got == want

    # zipf: the stream continued to world x 1M records, split by bytes
    n = world << 20
    lengths = E.zipf_lengths(W.ZIPF_SEED, n)
    offsets = np.zeros(n, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    lo, hi = shard.balanced_ranges(lengths, world)[rank]
    assert (lo, hi) == E.balanced_ranges(lengths, world)[rank]  # engine's own split rule
    cnt = hi - lo
    a = int(offsets[lo]) & ~7
    nbytes = int(offsets[hi - 1]) + int(lengths[hi - 1]) - a
    total = int(lengths[lo:hi].sum(dtype=np.uint64))
    data = E.DeviceBuffer(nbytes + 16)
    data.fill_splitmix64(W.DATA_SEED, byte_offset=a, nbytes=(nbytes + 7) & ~7)
    d_off, d_len, out = E.DeviceBuffer(cnt * 8), E.DeviceBuffer(cnt * 4), E.DeviceBuffer(cnt * 4)
    d_off.upload(offsets[lo:hi] - np.uint64(a))
    d_len.upload(lengths[lo:hi])
    E.device_batch(data, d_off, d_len, cnt, out, total_bytes=total)
    dig = E.crc32c_device(out, cnt * 4)
    for b in (data, d_off, d_len, out):
        b.free()
    got = [None] * world
    dist.all_gather_object(got, (dig, cnt))
    if rank == 0:
        bd = gold["zipf_seed0x5eed_data0xda7a5eed_blocks"]["block_digests"]
        want = shard.combine_digests(bd[:world], [1 << 20] * world)
        res["zipf"] = shard.combine_digests([g[0] for g in got], [g[1] for g in got]) == want
        res["zipf_records_per_rank"] = [g[1] for g in got]

    # single: one world x 4 GiB record split into byte slices
    size = world << 32
    start, length = shard.record_slices(size, world)[rank]
    data = E.DeviceBuffer(length)
    data.fill_splitmix64(0xC0DE, byte_offset=start)
    crc = E.crc32c_device(data, length)
    data.free()
    whole = shard.gather_fold(crc, length)
    if rank == 0:
        res["single"] = whole == gold["single_record_seed0xc0de"]["crc"][str(size)]

    st = E.stats()
    got = [None] * world
    dist.all_gather_object(got, st["fallback_calls"])
    if rank == 0:
        res["fallback_calls"] = got
        print("RESULT " + json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
