"""The N > 1 bench line proves its ranks (VERDICT r2 Next 6), checked on CPU.

bench.multi_rank_fields adds every rank's identity, the count of distinct
GPUs and the RCCL communicator's rank count, and turns a failed gather or
ranks sharing a GPU into exit code 4.  The committed two-rank rehearsal line
(profiles/r03_bench_n2_rehearsal_one_gpu.json, two ranks on the one GPU of a
gpurun box) must carry the same keys.
"""
import json
import os

import pytest

import bench

HERE = os.path.dirname(os.path.abspath(__file__))


def ranks_on(pcis):
    return [{"rank": i, "device": i, "pci_bus_id": p, "launch_ms": 0.65 + 0.01 * i}
            for i, p in enumerate(pcis)]


def gather_ok(world):
    return {"collective": "rccl all-gather of u32 CRC vectors", "bytes_per_rank": 8 << 20,
            "ms_median": 1.2, "verified": True, "rccl_ranks": world,
            "rccl_devices": list(range(world))}


@pytest.mark.parametrize("world", [2, 4, 8])
def test_distinct_gpus_and_verified_gather_pass(world):
    rec = {"roofline": {}}
    pcis = [f"0000:{0x11 + 0x20 * i:02x}:00.0" for i in range(world)]
    assert bench.multi_rank_fields(rec, ranks_on(pcis), gather_ok(world), world, False) == 0
    assert rec["distinct_gpus"] == world and rec["rccl_ranks"] == world
    assert [r["rank"] for r in rec["ranks"]] == list(range(world))
    for r in rec["ranks"]:
        assert set(r) == {"rank", "device", "pci_bus_id", "launch_ms"}
    json.dumps(rec)  # the line stays JSON


def test_ranks_sharing_a_gpu_fail_outside_a_rehearsal():
    rec = {}
    same = ranks_on(["0000:5d:00.0"] * 2)
    assert bench.multi_rank_fields(rec, same, gather_ok(2), 2, False) == 4
    assert rec["distinct_gpus"] == 1
    rec = {}
    assert bench.multi_rank_fields(rec, same, None, 2, True) == 0  # --share-device rehearsal


def test_failed_or_short_gather_fails():
    pcis = ["0000:11:00.0", "0000:31:00.0"]
    rec = {}
    err = {"collective": "rccl all-gather", "error": "timed out after 120 s"}
    assert bench.multi_rank_fields(rec, ranks_on(pcis), err, 2, False) == 4
    assert rec["gather"]["error"]
    short = dict(gather_ok(2), rccl_ranks=1)
    assert bench.multi_rank_fields({}, ranks_on(pcis), short, 2, False) == 4


def test_committed_rehearsal_line_has_the_keys():
    path = os.path.join(HERE, "..", "profiles", "r03_bench_n2_rehearsal_one_gpu.json")
    lines = [json.loads(x) for x in open(path) if x.strip().startswith("{")]
    assert lines
    rec = lines[-1]
    assert rec["n_gpus"] == 2 and len(rec["ranks"]) == 2
    for k in ("ranks", "distinct_gpus", "gather", "rccl_ranks"):
        assert k in rec, k
    for r in rec["ranks"]:
        assert set(r) >= {"rank", "device", "pci_bus_id", "launch_ms"}
