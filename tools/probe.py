"""HBM read-ceiling calibration (dev tool): python tools/probe.py [GiB]."""
import ctypes as C
import os
import subprocess
import sys

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
gib = float(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1][0].isdigit() else 4.0
nbytes = int(gib * (1 << 30))
buf = E.DeviceBuffer(nbytes)
buf.fill_splitmix64(0xC0DE)
sink = E.DeviceBuffer(4096 * 4)
names = {0: "stream plain U8", 1: "stream nt U8", 2: "stream plain U16", 3: "team plain",
         4: "team nt", 5: "team nt skew16", 6: "team nt skew64", 7: "team nt skew80",
         8: "team4 nt", 9: "team8 nt", 10: "team16 nt", 11: "team2 nt",
         20: "asm none", 21: "asm nt", 22: "asm sc1", 23: "asm sc0 sc1", 24: "asm sc1 nt",
         25: "asm sc0 sc1 nt", 26: "asm sc0 nt", 27: "asm sc0",
         30: "pipe D=1", 31: "pipe D=2", 32: "pipe D=3", 33: "pipe D=2 XCD-contig"}
if "--pipe" in sys.argv:
    plan = [(w, (256,)) for w in (30, 31, 32, 4)] * 3
elif "--xcd" in sys.argv:
    plan = [(w, (256,)) for w in (31, 33)] * 4
elif "--policy" in sys.argv:
    plan = [(w, (256,)) for w in (20, 21, 22, 23, 24, 25, 26, 27, 4)] * 2
else:
    plan = None
for which, grids in plan or ((0, (2048, 4096, 8192)), (1, (2048, 4096, 8192)), (2, (2048, 4096)),
                     (3, (256,)), (4, (256,)), (5, (256,)), (6, (256,)), (7, (256,)),
                     (8, (256,)), (9, (256,)), (10, (256,)), (11, (256,)), (4, (256,))):
    for g in grids:
        ms = P.probe_run(which, C.c_void_p(buf.ptr), nbytes, g, 10, C.c_void_p(sink.ptr))
        print(f"{names[which]:18s} grid {g:5d}: {ms:.4f} ms  {nbytes / ms / 1e6:8.1f} GB/s "
              f"({100 * nbytes / ms / 1e6 / 8000:.1f}% of 8 TB/s)", flush=True)
