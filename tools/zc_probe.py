"""What the HIP runtime reports for mapped host memory (dev tool): pointer
attributes and hipMemGetAddressRange for a hipHostMalloc buffer (the engine's
PinnedBuffer) and for a hipHostRegister'ed part of an anonymous mapping."""
import ctypes as C
import mmap
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import consus_amd as E  # noqa: E402


class Attr(C.Structure):
    _fields_ = [("type", C.c_int), ("device", C.c_int), ("devicePointer", C.c_void_p),
                ("hostPointer", C.c_void_p), ("isManaged", C.c_int), ("allocationFlags", C.c_uint)]


hip = C.CDLL("libamdhip64.so")
E.init(0)


def show(tag, p):
    a = Attr()
    st = hip.hipPointerGetAttributes(C.byref(a), C.c_void_p(p))
    base, size = C.c_void_p(), C.c_size_t()
    st2 = hip.hipMemGetAddressRange(C.byref(base), C.byref(size), C.c_void_p(a.devicePointer or 0))
    st3 = hip.hipMemGetAddressRange(C.byref(base), C.byref(size), C.c_void_p(p))
    print(f"{tag:28s} p={p:#x} st={st} type={a.type} dev={a.device} devptr={a.devicePointer or 0:#x} "
          f"hostptr={a.hostPointer or 0:#x} flags={a.allocationFlags:#x} | range(devptr) st={st2} "
          f"| range(p) st={st3} base={base.value or 0:#x} size={size.value}")
    hip.hipGetLastError()


pb = E.PinnedBuffer(1 << 20)
p0 = pb.array.ctypes.data
for off in (0, 4096, (1 << 20) - 1):
    show(f"hipHostMalloc +{off}", p0 + off)
mm = mmap.mmap(-1, 2 << 20)
buf = np.frombuffer(mm, dtype=np.uint8)
addr = buf.ctypes.data
print("register", hip.hipHostRegister(C.c_void_p(addr), C.c_size_t(1 << 20), C.c_uint(3)))
for off in (0, 4096, (1 << 20) - 1, 1 << 20, (2 << 20) - 1):
    show(f"registered +{off}", addr + off)
print("unregister", hip.hipHostUnregister(C.c_void_p(addr)))
