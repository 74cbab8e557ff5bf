"""One rank of bench.py's N > 1 flow on the CPU (tests/test_bench_multirank.py).

Run under torch.distributed.run with the gloo backend.  Before bench.main()
imports the engine, `consus_amd` is replaced in sys.modules by a CPU
stand-in whose records are hashed by the oracle (test infrastructure) and
whose RCCL calls (comm_*) are carried by gloo: the collective is the only
thing stubbed, everything around it -- the uid broadcast, the warm-up and
timed gathers, rank 0's per-block digest check, the ranks' identities,
multi_rank_fields and the exit codes -- is bench.py's own code.

STUB_MODE selects the collective's behaviour:
  ok      all-gather over gloo, every rank on its own PCI bus id
  error   the all-gather raises (an RCCL error)
  short   the communicator reports one rank (a short gather)
  shared  every rank reports the same PCI bus id (two ranks on one GPU)
  hang    rank 1 never enters the all-gather (a hung collective)
"""
import os
import sys
import time
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

from oracle.oracle import Oracle  # noqa: E402  (the checker computes the stub's CRCs)

MODE = os.environ.get("STUB_MODE", "ok")
RANK = int(os.environ.get("RANK", "0"))
_orc = Oracle()
_comm = {}
_t = [0.0]


class DeviceBuffer:
    def __init__(self, nbytes: int):
        self.nbytes = nbytes
        self.a = np.zeros(nbytes, dtype=np.uint8)

    def fill_splitmix64(self, seed: int, byte_offset: int = 0, nbytes=None, dst_offset: int = 0):
        n = self.nbytes if nbytes is None else nbytes
        self.a[dst_offset:dst_offset + n] = _orc.fill(n, seed, byte_offset)

    def download(self, dtype=np.uint8, count=None, offset: int = 0):
        v = self.a[offset:].view(dtype)
        return v[:count].copy() if count is not None else v.copy()

    def upload(self, arr, offset: int = 0):
        b = np.ascontiguousarray(arr).view(np.uint8)
        self.a[offset:offset + b.size] = b


def device_batch_fixed(data, stride, length, count, out, inits=None, asynchronous=False):
    out.a[:count * 4] = _orc.fixed(data.a, stride, length, count).view(np.uint8)


def crc32c_device(buf, nbytes=None, init_crc: int = 0, offset: int = 0):
    n = buf.nbytes - offset if nbytes is None else nbytes
    return _orc.crc32c(init_crc, buf.a[offset:offset + n])


def timer_start():
    _t[0] = time.perf_counter()


def timer_stop():
    return (time.perf_counter() - _t[0]) * 1e3


def device_pci_bus_id(device: int) -> str:
    return "0000:5d:00.0" if MODE == "shared" else f"0000:{0x11 + 0x20 * RANK:02x}:00.0"


def comm_unique_id() -> bytes:
    return b"gloo-stub-unique-id"


def comm_init(unique_id: bytes, nranks: int, rank: int) -> None:
    _comm.update(nranks=nranks, rank=rank)


def comm_info() -> dict:
    return {"nranks": 1 if MODE == "short" else _comm["nranks"], "rank": _comm["rank"],
            "device": _comm["rank"]}


def comm_allgather_u32(send, count, recv):
    import torch
    import torch.distributed as dist
    if MODE == "error":
        raise RuntimeError("ncclAllGather: unhandled system error (stub)")
    if MODE == "hang" and RANK == 1:
        time.sleep(3600)
    mine = torch.from_numpy(send.a[:count * 4].view(np.int32).copy())
    parts = [torch.empty_like(mine) for _ in range(_comm["nranks"])]
    dist.all_gather(parts, mine)
    for i, p in enumerate(parts):
        recv.a[i * count * 4:(i + 1) * count * 4] = p.numpy().view(np.uint8)


def comm_destroy() -> None:
    _comm.clear()


stub = types.ModuleType("consus_amd")
for _name, _obj in list(globals().items()):
    if _name in ("DeviceBuffer", "device_batch_fixed", "crc32c_device", "timer_start", "timer_stop",
                 "device_pci_bus_id", "comm_unique_id", "comm_init", "comm_info",
                 "comm_allgather_u32", "comm_destroy"):
        setattr(stub, _name, _obj)
stub.init = lambda device=0: None
stub.sync = lambda: None
sys.modules["consus_amd"] = stub

import bench  # noqa: E402

if __name__ == "__main__":
    sys.argv = ["bench.py"] + sys.argv[1:]
    bench.main()
