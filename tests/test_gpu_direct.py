"""GPU parity of the direct kernel's two forms.

Host batches of records <= 16 KiB take one launch of crc32c_direct_kernel:
with the 152 KiB LDS table image (1024-thread workgroups) or, for batches of
at most kLiteMaxBytes, the LDS-free form (256-thread workgroups, lane-table
row update).  MI_CRC32C_DIRECT_LITE=0/1 forces either form; records already
in mapped pinned memory (a durable-log flush) are read in place and the
host waits on the kernel's completion word (MI_CRC32C_DONE_WORD=0: a stream
sync instead).  Every case bit-exact against the oracle.
"""
import numpy as np
import pytest

from tests.test_gpu_parity import make_frames

pytestmark = pytest.mark.gpu

FORMS = pytest.mark.parametrize("lite", ["0", "1"], ids=["lds", "lite"])


def _sweep():
    rng = np.random.default_rng(91)
    starts = list(range(0, 128, 3)) + [4096 - d for d in (1, 2, 15, 16, 17, 127, 128, 129)]
    lens = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 33, 63, 64, 127, 128, 129, 255, 256, 257,
            1023, 1024, 1025, 2047, 2048, 2049, 4095, 4096, 4097, 8191, 8192, 16383, 16384]
    offsets, lengths = [], []
    for i, s in enumerate(starts):
        for j, n in enumerate(lens):
            offsets.append(((i * len(lens) + j) * 5) * 4096 + 8192 + s)
            lengths.append(n)
    offsets = np.array(offsets, dtype=np.uint64)
    lengths = np.array(lengths, dtype=np.uint32)
    buf = rng.integers(0, 256, int((offsets + lengths).max()) + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, lengths.size, dtype=np.uint32)
    return buf, offsets, lengths, inits


@FORMS
def test_direct_alignment_sweep(engine, oracle, monkeypatch, lite):
    """Every start residue (step 3) and starts around 4 KiB edges, lengths at
    row, group and chunk edges up to the direct kernel's 16 KiB limit."""
    monkeypatch.setenv("MI_CRC32C_DIRECT_LITE", lite)
    buf, offsets, lengths, inits = _sweep()
    assert np.array_equal(engine.crc32c_batch(buf, offsets, lengths),
                          oracle.batch(buf, offsets, lengths))
    assert np.array_equal(engine.crc32c_batch(buf, offsets, lengths, inits),
                          oracle.batch(buf, offsets, lengths, inits))


@FORMS
@pytest.mark.parametrize("done_word", ["1", "0"], ids=["spin", "sync"])
def test_direct_zero_copy_frames(engine, oracle, monkeypatch, lite, done_word):
    """Durable-log frames in mapped pinned memory: read in place, CRCs back
    through the completion word (or a stream sync), 1 .. 4096 frames."""
    monkeypatch.setenv("MI_CRC32C_DIRECT_LITE", lite)
    monkeypatch.setenv("MI_CRC32C_DONE_WORD", done_word)
    rng = np.random.default_rng(92)
    pinned = engine.PinnedBuffer(4 << 20)
    try:
        before = engine.stats()["zero_copy_batches"]
        calls = 0
        for nbytes in (64, 2000, 40000, 300000, 2 << 20, 4 << 20):
            buf, off, ln = make_frames(rng, nbytes, 1024)
            if off.size == 0:
                continue
            pinned.array[:buf.size] = buf
            view = pinned.array[:buf.size]
            for inits in (None, rng.integers(0, 2**32, off.size, dtype=np.uint32)):
                got = engine.crc32c_batch(view, off, ln, inits)
                assert np.array_equal(got, oracle.batch(buf, off, ln, inits)), (nbytes, inits is None)
                calls += 1
        assert engine.stats()["zero_copy_batches"] - before == calls
    finally:
        pinned.free()


@FORMS
def test_direct_many_records_team_loop(engine, oracle, monkeypatch, lite):
    """More records than the grid has teams (each team takes several): 200k
    records of 0 - 300 B, plus a wave whose records span 1 - 128 rows."""
    monkeypatch.setenv("MI_CRC32C_DIRECT_LITE", lite)
    rng = np.random.default_rng(93)
    count = 200_000
    lengths = rng.integers(0, 300, count).astype(np.uint32)
    lengths[1000:1064] = rng.integers(1, 16385, 64)
    offsets = np.zeros(count, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    buf = rng.integers(0, 256, int(lengths.sum()) + 16, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32)
    assert np.array_equal(engine.crc32c_batch(buf, offsets, lengths, inits),
                          oracle.batch(buf, offsets, lengths, inits))


def test_direct_tiny_packed_batches(engine, oracle, monkeypatch):
    """Batches whose packed inputs fit 8 KiB are read in place from the
    engine's pinned staging (completion word): 1 - 60 records, many calls."""
    rng = np.random.default_rng(94)
    buf = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    for k in range(300):
        n = int(rng.integers(1, 60))
        lens = rng.integers(0, 100, n).astype(np.uint32)
        offs = rng.integers(0, buf.size - 100, n).astype(np.uint64)
        got = engine.crc32c_batch(buf, offs, lens)
        assert np.array_equal(got, oracle.batch(buf, offs, lens, threads=1)), k


def _hip():
    import ctypes as C
    for name in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
        try:
            lib = C.CDLL(name)
            break
        except OSError:
            continue
    lib.hipHostRegister.restype = C.c_int
    lib.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
    lib.hipHostUnregister.restype = C.c_int
    lib.hipHostUnregister.argtypes = [C.c_void_p]
    return lib


def test_zero_copy_needs_the_whole_span_mapped(engine, oracle):
    """a host batch whose span starts in mapped pinned
    memory but runs on into pageable memory must not be read in place (the
    kernel would read past the mapping); it is staged, bit-exact.  A batch
    wholly inside the mapped part still is read in place.  The mapped part
    is the first 1 MiB of a 2 MiB anonymous mapping, registered with
    hipHostRegister(Mapped | Portable); the rest stays pageable."""
    import mmap

    hip = _hip()
    size, half = 2 << 20, 1 << 20
    mm = mmap.mmap(-1, size)
    buf = np.frombuffer(mm, dtype=np.uint8)
    rng = np.random.default_rng(95)
    buf[:] = rng.integers(0, 256, size, dtype=np.uint8)
    addr = buf.ctypes.data
    assert hip.hipHostRegister(addr, half, 0x3) == 0
    try:
        # inside the mapped half: zero-copy
        off = np.arange(64, dtype=np.uint64) * 4096 + 100
        ln = np.full(64, 3000, dtype=np.uint32)
        before = engine.stats()["zero_copy_batches"]
        assert np.array_equal(engine.crc32c_batch(buf, off, ln), oracle.batch(buf, off, ln))
        assert engine.stats()["zero_copy_batches"] - before == 1
        # the same records plus one that crosses into the pageable half, and
        # one wholly in it: staged, not zero-copy
        for extra in ((half - 1000, 5000), (half + 300000, 9000)):
            off2 = np.append(off, np.uint64(extra[0]))
            ln2 = np.append(ln, np.uint32(extra[1]))
            before = engine.stats()["zero_copy_batches"]
            assert np.array_equal(engine.crc32c_batch(buf, off2, ln2),
                                  oracle.batch(buf, off2, ln2)), extra
            assert engine.stats()["zero_copy_batches"] == before, extra
    finally:
        assert hip.hipHostUnregister(addr) == 0
        del buf


def test_zero_copy_two_registrations_with_a_pageable_gap(engine, oracle):
    """ROCm reports hipHostRegister'ed memory with a null
    allocation base, so the span check cannot bound a batch by one
    allocation.  Two separately registered 1 MiB regions with a pageable
    1 MiB gap between them, both ends of the batch mapped at device addresses
    the right distance apart: the batch must be staged (its middle is not
    mapped), bit-exact; batches inside either region stay zero-copy."""
    import mmap

    hip = _hip()
    mib = 1 << 20
    mm = mmap.mmap(-1, 3 * mib)
    buf = np.frombuffer(mm, dtype=np.uint8)
    buf[:] = np.random.default_rng(96).integers(0, 256, 3 * mib, dtype=np.uint8)
    addr = buf.ctypes.data
    assert hip.hipHostRegister(addr, mib, 0x3) == 0
    try:
        assert hip.hipHostRegister(addr + 2 * mib, mib, 0x3) == 0
        try:
            for lo in (0, 2 * mib):  # inside one registration: zero-copy
                off = np.arange(32, dtype=np.uint64) * 8192 + np.uint64(lo + 77)
                ln = np.full(32, 4000, dtype=np.uint32)
                before = engine.stats()["zero_copy_batches"]
                assert np.array_equal(engine.crc32c_batch(buf, off, ln), oracle.batch(buf, off, ln))
                assert engine.stats()["zero_copy_batches"] - before == 1, lo
            # first record in region 1, last in region 2, the gap between
            # them untouched by any record but inside the batch's span
            off = np.array([100, 2 * mib + 5000], dtype=np.uint64)
            ln = np.array([6000, 9000], dtype=np.uint32)
            before = engine.stats()["zero_copy_batches"]
            assert np.array_equal(engine.crc32c_batch(buf, off, ln), oracle.batch(buf, off, ln))
            assert engine.stats()["zero_copy_batches"] == before
        finally:
            assert hip.hipHostUnregister(addr + 2 * mib) == 0
    finally:
        assert hip.hipHostUnregister(addr) == 0
        del buf
