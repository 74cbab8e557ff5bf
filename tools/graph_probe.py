"""hipGraph replay vs eager launches for the variable-length device path (dev tool).

The device batch (plan: count, scan, scatter, long items; chunks; finalize,
long finalize = 7 kernels) is captured once from the engine's stream with
hipStreamBeginCapture and replayed with hipGraphLaunch; both are timed with
HIP events over back-to-back calls.  Results are checked against the eager
launch's CRCs.   python tools/graph_probe.py
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import consus_amd as E  # noqa: E402

E.init(0)
L = E.lib()
hip = C.CDLL("libamdhip64.so")
s = C.c_void_p(L.mi_crc32c_stream())


def chk(r, what):
    if r != 0:
        raise RuntimeError(f"{what}: hip error {r}")


def events_ms(fn, n):
    e0, e1 = C.c_void_p(), C.c_void_p()
    chk(hip.hipEventCreate(C.byref(e0)), "event")
    chk(hip.hipEventCreate(C.byref(e1)), "event")
    chk(hip.hipEventRecord(e0, s), "record")
    for _ in range(n):
        fn()
    chk(hip.hipEventRecord(e1, s), "record")
    chk(hip.hipEventSynchronize(e1), "sync")
    ms = C.c_float()
    chk(hip.hipEventElapsedTime(C.byref(ms), e0, e1), "elapsed")
    return ms.value / n


rng = np.random.default_rng(5)
print("records  mean_len  eager_us  graph_us  (per call, back-to-back, events)")
for count in (256, 2048, 16384, 131072):
    lens = np.minimum(rng.zipf(1.3, count) * 64, 65536).astype(np.uint32)
    offs = np.zeros(count, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(lens.sum(dtype=np.uint64))
    data = E.DeviceBuffer(total + 64)
    data.fill_splitmix64(0x5EED)
    d_off, d_len = E.DeviceBuffer(count * 8), E.DeviceBuffer(count * 4)
    out_e, out_g = E.DeviceBuffer(count * 4), E.DeviceBuffer(count * 4)
    d_off.upload(offs)
    d_len.upload(lens)

    def eager(out=out_e):
        E.device_batch(data, d_off, d_len, count, out, total_bytes=total, asynchronous=True)
    for _ in range(3):
        eager()          # workspaces reserved before capture (no hipMalloc inside it)
    E.sync()
    graph, exe = C.c_void_p(), C.c_void_p()
    chk(hip.hipStreamBeginCapture(s, 0), "begin capture")  # hipStreamCaptureModeGlobal
    eager(out_g)
    chk(hip.hipStreamEndCapture(s, C.byref(graph)), "end capture")
    chk(hip.hipGraphInstantiate(C.byref(exe), graph, None, None, 0), "instantiate")

    def replay():
        chk(hip.hipGraphLaunch(exe, s), "graph launch")
    replay()
    E.sync()
    assert np.array_equal(out_g.download(np.uint32, count), out_e.download(np.uint32, count))
    reps = 200 if count <= 16384 else 50
    te = min(events_ms(eager, reps) for _ in range(3))
    tg = min(events_ms(replay, reps) for _ in range(3))
    print(f"{count:7d}  {total / count:8.0f}  {te * 1e3:8.1f}  {tg * 1e3:8.1f}", flush=True)
    hip.hipGraphExecDestroy(exe)
    hip.hipGraphDestroy(graph)
    for b in (data, d_off, d_len, out_e, out_g):
        b.free()
