"""Sustained vs isolated launch rate of the fixed 4 KiB kernel and of the
pure-read team probe (dev tool): python tools/sustain.py

Under rocprofv3 the first launches after an idle gap ran ~6 % faster than
back-to-back ones; this separates the kernel's own cost from a sustained-load
(clock / power) effect.
"""
import ctypes as C
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import consus_amd as E  # noqa: E402

so = os.path.join(HERE, "libprobe.so")
if not os.path.exists(so):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                    "-o", so, os.path.join(HERE, "probe.hip")], check=True)
E.init(0)
P = C.CDLL(so)
P.probe_run.restype = C.c_float
P.probe_run.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_void_p]
count, L = 1 << 20, 4096
nbytes = count * L
data = E.DeviceBuffer(nbytes)
out = E.DeviceBuffer(count * 4)
sink = E.DeviceBuffer(4096 * 4)
data.fill_splitmix64(0xC0DE)


def kernel_block(n):
    E.timer_start()
    for _ in range(n):
        E.device_batch_fixed(data, L, L, count, out, asynchronous=True)
    return E.timer_stop() / n


def rate(ms):
    return f"{ms:.4f} ms {nbytes / ms / 1e6:7.1f} GB/s"


for _ in range(3):
    kernel_block(1)
print("kernel, blocks of 10 back-to-back:", flush=True)
for i in range(8):
    print(f"  block {i}: {rate(kernel_block(10))}", flush=True)
print("kernel, isolated launches (2 ms idle before each):", flush=True)
iso = []
for i in range(10):
    time.sleep(0.002)
    iso.append(kernel_block(1))
print("  " + "  ".join(f"{t:.4f}" for t in iso), flush=True)
print("kernel, isolated launches (50 ms idle before each):", flush=True)
iso = []
for i in range(6):
    time.sleep(0.05)
    iso.append(kernel_block(1))
print("  " + "  ".join(f"{t:.4f}" for t in iso), flush=True)
print("probe team nt, blocks of 10 back-to-back:", flush=True)
for i in range(4):
    ms = P.probe_run(4, C.c_void_p(data.ptr), nbytes, 256, 10, C.c_void_p(sink.ptr))
    print(f"  block {i}: {rate(ms)}", flush=True)
print("probe team nt, single launches after 50 ms idle:", flush=True)
iso = []
for i in range(6):
    time.sleep(0.05)
    iso.append(P.probe_run(4, C.c_void_p(data.ptr), nbytes, 256, 1, C.c_void_p(sink.ptr)))
print("  " + "  ".join(f"{t:.4f}" for t in iso), flush=True)
print("kernel, 60 back-to-back then blocks of 10:", flush=True)
kernel_block(60)
for i in range(3):
    print(f"  block {i}: {rate(kernel_block(10))}", flush=True)
