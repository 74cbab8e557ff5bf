"""Build ablation variants of the engine (MI_CRC_ABLATE modes) and time the
fixed 4 KiB kernel of each in one process (dev tool).  python tools/ablate.py"""
import ctypes as C
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
MODES = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,1,2,4,6".split(","))]
SRC = os.path.join(ROOT, "consus_amd", "csrc")


def build(mode):
    out = os.path.join(HERE, f"libablate_{mode}.so")
    if not os.path.exists(out):
        objs = []
        for f in ("crc32c_kernels.hip", "engine.hip", "workload.cc"):
            o = os.path.join("/tmp", f"abl_{mode}_{f}.o")
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                            "-fPIC", f"-DMI_CRC_ABLATE={mode}", "-I", os.path.join(ROOT, "include"),
                            "-c", "-o", o, os.path.join(SRC, f)], check=True)
            objs.append(o)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o", out,
                        *objs, "-lrccl"], check=True)
    return out


if __name__ == "__main__":
    import consus_amd
    libs = {}
    for m in MODES:
        L = C.CDLL(build(m))
        for name, (res, args) in consus_amd._SIGS.items():  # every call fully typed
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        libs[m] = L
    if "--build-only" in sys.argv:
        sys.exit(0)
    L0 = libs[MODES[0]]
    count, R = 1 << 20, 4096
    for L in libs.values():
        assert L.mi_crc32c_init(0) == 0
    p = C.c_void_p()
    assert L0.mi_dev_malloc(C.byref(p), count * R) == 0
    o = C.c_void_p()
    assert L0.mi_dev_malloc(C.byref(o), count * 4) == 0
    assert L0.mi_fill_splitmix64(p, count * R, 0xC0DE, 0) == 0
    for rnd in range(3):
        for m, L in libs.items():
            for _ in range(3):
                assert L.mi_crc32c_batch_fixed(p, R, R, None, count, o, 1) == 0
            L.mi_timer_start()
            for _ in range(10):
                L.mi_crc32c_batch_fixed(p, R, R, None, count, o, 3)
            ms = C.c_float()
            L.mi_timer_stop(C.byref(ms))
            t = ms.value / 10
            print(f"round {rnd} mode {m}: {t:.4f} ms  {count * R / t / 1e6:.1f} GB/s", flush=True)
