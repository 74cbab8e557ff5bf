"""Error behaviour of the C ABI on a live device (include/consus_crc32c.h):
bad arguments return MI_CRC32C_EINVAL with a message in
mi_crc32c_last_error(), nothing is launched, and the engine keeps working
for the next valid call.  The reference function has no error channel
(common/crc32c.h:40-41); these are the status codes of the batch ABI."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture()
def L(engine):
    return engine.lib()


def _u32(a):
    return a.ctypes.data_as(C.c_void_p)


def _still_works(engine):
    assert engine.crc32c(0, b"123456789") == 0xE3069283


def _einval(engine, L, st):
    assert st == engine.EINVAL
    assert L.mi_crc32c_last_error()  # a message, not empty
    _still_works(engine)


def test_strerror_names_every_status(L, engine):
    for st in (0, engine.EINVAL, engine.ENODEV, -12, -5, -71):
        assert L.mi_crc32c_strerror(st)


def test_batch_argument_errors(L, engine):
    out = np.zeros(4, dtype=np.uint32)
    off = np.zeros(4, dtype=np.uint64)
    ln = np.full(4, 8, dtype=np.uint32)
    buf = np.zeros(64, dtype=np.uint8)
    # count == 0 is a no-op whatever the pointers
    assert L.mi_crc32c_batch(None, None, None, None, 0, 0, None, 0) == 0
    _einval(engine, L, L.mi_crc32c_batch(_u32(buf), None, _u32(ln), None, 4, 0, _u32(out), 0))
    _einval(engine, L, L.mi_crc32c_batch(_u32(buf), _u32(off), _u32(ln), None, 4, 0, None, 0))
    _einval(engine, L, L.mi_crc32c_batch(None, _u32(off), _u32(ln), None, 4, 0, _u32(out), 0))
    # a record whose end wraps the 64-bit address space
    bad = np.array([2**64 - 4], dtype=np.uint64)
    _einval(engine, L, L.mi_crc32c_batch(_u32(buf), _u32(bad), _u32(ln[:1]), None, 1, 0,
                                         _u32(out), 0))
    _einval(engine, L, L.mi_crc32c_batch_fixed(_u32(buf), 16, 8, None, 4, None, 0))
    _einval(engine, L, L.mi_crc32c_batch_fixed(None, 16, 8, None, 4, _u32(out), 0))
    _einval(engine, L, L.mi_crc32c_batch_fixed(_u32(buf), 16, 1 << 32, None, 2, _u32(out), 0))


def test_buffer_argument_errors(L, engine):
    o = C.c_uint32(7)
    _einval(engine, L, L.mi_crc32c_buffer(0, None, 0, None, 0))
    _einval(engine, L, L.mi_crc32c_buffer(0, None, 5, C.byref(o), 0))
    assert L.mi_crc32c_buffer(0xABCD, None, 0, C.byref(o), 0) == 0 and o.value == 0xABCD
    z = np.zeros(4, dtype=np.uint32)
    _einval(engine, L, L.mi_crc32c_combine_batch(None, _u32(z), _u32(z), 4, _u32(z), 0))


def test_pipeline_argument_errors(L, engine):
    p = C.c_void_p()
    _einval(engine, L, L.mi_crc32c_pipeline_create(1 << 20, 0, 2, C.byref(p)))
    _einval(engine, L, L.mi_crc32c_pipeline_create(1 << 20, 16, 0, C.byref(p)))
    assert L.mi_crc32c_pipeline_create(1 << 20, 16, 2, C.byref(p)) == 0
    try:
        seg = np.arange(4096, dtype=np.uint8)
        off = np.array([0, 100], dtype=np.uint64)
        ln = np.array([100, 200], dtype=np.uint32)
        out = np.zeros(2, dtype=np.uint32)
        t = C.c_uint64()
        # larger than the pipeline's segment limit
        big = np.zeros((1 << 20) + 1, dtype=np.uint8)
        _einval(engine, L, L.mi_crc32c_pipeline_submit(p, _u32(big), big.size, _u32(off),
                                                       _u32(ln), None, 2, _u32(out), C.byref(t)))
        # a record past the segment end, and one whose end wraps 64 bits
        for o2 in (4000, 2**64 - 50):
            off2 = np.array([0, o2], dtype=np.uint64)
            _einval(engine, L, L.mi_crc32c_pipeline_submit(p, _u32(seg), seg.size, _u32(off2),
                                                           _u32(ln), None, 2, _u32(out),
                                                           C.byref(t)))
        _einval(engine, L, L.mi_crc32c_pipeline_submit(p, None, seg.size, _u32(off), _u32(ln),
                                                       None, 2, _u32(out), C.byref(t)))
        # refused submits took no ticket: the next good one completes normally
        assert L.mi_crc32c_pipeline_submit(p, _u32(seg), seg.size, _u32(off), _u32(ln), None, 2,
                                           _u32(out), C.byref(t)) == 0
        assert L.mi_crc32c_pipeline_wait(p, t.value) == 0
        assert list(out) == [engine.crc32c(0, seg[0:100]), engine.crc32c(0, seg[100:300])]
    finally:
        assert L.mi_crc32c_pipeline_destroy(p) == 0


def test_device_helper_errors(L, engine):
    buf = engine.DeviceBuffer(4096)
    _einval(engine, L, L.mi_fill_splitmix64(C.c_void_p(buf.ptr + 3), 64, 1, 0))
    _einval(engine, L, L.mi_fill_splitmix64(C.c_void_p(buf.ptr), 64, 1, 5))
    recv = engine.DeviceBuffer(4096)
    _einval(engine, L, L.mi_comm_allgather_u32(C.c_void_p(buf.ptr), 16, C.c_void_p(recv.ptr)))
    # a second device while the engine is bound to device 0
    assert L.mi_crc32c_init(1) != 0
    _still_works(engine)
    buf.free()
    recv.free()


def test_understated_size_hint_is_recovered(engine, oracle):
    """A total_bytes hint below the true sum sizes the workspace too small:
    no kernel accesses out of bounds, and a synchronous call sees the
    overflow and recomputes the batch with the plan size read back, so its
    results are exact -- on the piece path and on the sorted path (ADVICE
    r2: the sorted path used to return OK with partial results).  The calls
    run in fresh threads: their own contexts, so their workspaces are sized by
    the understated hint alone (grow-only buffers of earlier calls would fit)."""
    import threading
    rng = np.random.default_rng(3)
    count = 64
    lengths = np.full(count, 1 << 20, dtype=np.uint32)   # 256+ pieces per record
    offsets = (np.arange(count, dtype=np.uint64) << np.uint64(20)) + np.uint64(5)
    size = (count << 20) + 4096
    buf = rng.integers(0, 256, size, dtype=np.uint8)
    data = engine.DeviceBuffer(size)
    data.upload(buf)
    d_off, d_len, d_out = (engine.DeviceBuffer(count * 8), engine.DeviceBuffer(count * 4),
                           engine.DeviceBuffer(count * 4))
    d_off.upload(offsets)
    d_len.upload(lengths)
    want = oracle.batch(buf, offsets, lengths)
    # a 4 KiB hint on the piece path and on the window path (which sizes its
    # grid from it and loops); a 4 MiB hint (room for 129 descriptors) on the
    # sorted path, whose split records need 64 + 960 of them
    for hint, path in ((4096, "pieces"), (4096, "window"), (4 << 20, "sorted")):
        d_out.upload(np.full(count, 0xABABABAB, dtype=np.uint32))
        errors = []

        def understated():
            try:
                if path:
                    os.environ["MI_CRC32C_VARPATH"] = path
                engine.device_batch(data, d_off, d_len, count, d_out, total_bytes=hint)
            except Exception as e:  # noqa: BLE001
                errors.append(e)
            finally:
                os.environ.pop("MI_CRC32C_VARPATH", None)
        t = threading.Thread(target=understated)
        t.start()
        t.join()
        assert not errors, errors[0]
        assert np.array_equal(d_out.download(np.uint32, count), want), (hint, path)
    for hint in (int(lengths.sum()), 0):
        engine.device_batch(data, d_off, d_len, count, d_out, total_bytes=hint)
        assert np.array_equal(d_out.download(np.uint32, count), want)
    for b in (data, d_off, d_len, d_out):
        b.free()


def test_understated_hint_on_an_async_batch_fails_the_next_sync(engine, oracle):
    """an ASYNCHRONOUS sorted batch whose total_bytes hint
    understates its records cannot be recomputed (nothing waits for it), and
    its out[] is incomplete; the kernel sets a sticky word, and the calling
    thread's next mi_crc32c_stream_sync reports it (EINVAL, counted in
    hint_overflows) and clears it.  The sync after that, and a batch with a
    true hint, are clean.  Runs in a fresh thread: a context whose
    workspace the understated hint alone sizes."""
    import threading
    count = 64
    lengths = np.full(count, 1 << 20, dtype=np.uint32)
    offsets = (np.arange(count, dtype=np.uint64) << np.uint64(20)) + np.uint64(5)
    size = (count << 20) + 4096
    buf = np.random.default_rng(4).integers(0, 256, size, dtype=np.uint8)
    data = engine.DeviceBuffer(size)
    data.upload(buf)
    d_off, d_len, d_out = (engine.DeviceBuffer(count * 8), engine.DeviceBuffer(count * 4),
                           engine.DeviceBuffer(count * 4))
    d_off.upload(offsets)
    d_len.upload(lengths)
    want = oracle.batch(buf, offsets, lengths)
    seen = {}

    def run():
        try:
            os.environ["MI_CRC32C_VARPATH"] = "sorted"
            before = engine.stats()["hint_overflows"]
            engine.device_batch(data, d_off, d_len, count, d_out, total_bytes=4 << 20,
                                asynchronous=True)
            try:
                engine.sync()
                seen["first"] = "ok"
            except engine.EngineError as e:
                seen["first"] = e.status
            seen["counted"] = engine.stats()["hint_overflows"] - before
            engine.sync()  # cleared: clean
            engine.device_batch(data, d_off, d_len, count, d_out, total_bytes=int(lengths.sum()),
                                asynchronous=True)
            engine.sync()
            seen["second"] = "ok"
        except Exception as e:  # noqa: BLE001
            seen["error"] = e
        finally:
            os.environ.pop("MI_CRC32C_VARPATH", None)
    t = threading.Thread(target=run)
    t.start()
    t.join()
    assert "error" not in seen, seen["error"]
    assert seen["first"] == engine.EINVAL and seen["counted"] == 1 and seen["second"] == "ok", seen
    assert np.array_equal(d_out.download(np.uint32, count), want)
    for b in (data, d_off, d_len, d_out):
        b.free()


def _in_thread(fn):
    """Run fn in a fresh thread (its own engine context); re-raise its error."""
    import threading
    box = {}

    def run():
        try:
            box["v"] = fn()
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            box["e"] = e
    t = threading.Thread(target=run)
    t.start()
    t.join()
    if "e" in box:
        raise box["e"]
    return box.get("v")


def _split_batch(engine, seed):
    count = 64
    lengths = np.full(count, 1 << 20, dtype=np.uint32)
    offsets = (np.arange(count, dtype=np.uint64) << np.uint64(20)) + np.uint64(5)
    size = (count << 20) + 4096
    buf = np.random.default_rng(seed).integers(0, 256, size, dtype=np.uint8)
    data = engine.DeviceBuffer(size)
    data.upload(buf)
    d_off, d_len, d_out = (engine.DeviceBuffer(count * 8), engine.DeviceBuffer(count * 4),
                           engine.DeviceBuffer(count * 4))
    d_off.upload(offsets)
    d_len.upload(lengths)
    return count, buf, offsets, lengths, (data, d_off, d_len, d_out)


@pytest.mark.parametrize("async_hint_ok", [True, False])
def test_async_state_survives_a_recovered_sync_batch(engine, oracle, async_hint_ok):
    """an unchecked asynchronous sorted batch, then a synchronous
    sorted batch whose understated hint overflows and is recomputed.  The
    next stream sync reports exactly the asynchronous batch's state: clean
    when its hint was true (round 5 reported a false EINVAL: the sync batch
    left the sticky word set), EINVAL when it was understated (the word as
    the asynchronous batch left it is read before the synchronous batch
    runs).  The synchronous batch's results are exact either way."""
    count, buf, offsets, lengths, (data, d_off, d_len, d_out) = _split_batch(engine, 5)
    want = oracle.batch(buf, offsets, lengths)
    d_out2 = engine.DeviceBuffer(count * 4)

    def run():
        os.environ["MI_CRC32C_VARPATH"] = "sorted"
        try:
            engine.device_batch(data, d_off, d_len, count, d_out2,
                                total_bytes=int(lengths.sum()) if async_hint_ok else 4 << 20,
                                asynchronous=True)
            engine.device_batch(data, d_off, d_len, count, d_out, total_bytes=4 << 20)
            got = d_out.download(np.uint32, count)
            try:
                engine.sync()
                first = "ok"
            except engine.EngineError as e:
                first = e.status
            engine.sync()
            return got, first
        finally:
            os.environ.pop("MI_CRC32C_VARPATH", None)
    got, first = _in_thread(run)
    assert np.array_equal(got, want)
    assert first == ("ok" if async_hint_ok else engine.EINVAL)
    if async_hint_ok:
        assert np.array_equal(d_out2.download(np.uint32, count), want)
    for b in (data, d_off, d_len, d_out, d_out2):
        b.free()


def test_window_record_of_4gib_minus_one(engine, oracle):
    """the window path counted a record's windows in 32 bits, so a
    record of 0xFFFFFFFF bytes wrapped to no window and its CRC was never
    stored.  One such record (bytes [1, 2^32) of the splitmix64 stream
    0xC0DE), forced onto the window path, against the oracle over the same
    bytes."""
    n = 0xFFFFFFFF
    data = engine.DeviceBuffer((1 << 32) + 64)
    data.fill_splitmix64(0xC0DE)
    d_off, d_len, d_out = engine.DeviceBuffer(8), engine.DeviceBuffer(4), engine.DeviceBuffer(4)
    d_off.upload(np.array([1], dtype=np.uint64))
    d_len.upload(np.array([n], dtype=np.uint32))
    d_out.upload(np.array([0xABABABAB], dtype=np.uint32))
    before = engine.stats()["window_batches"]
    os.environ["MI_CRC32C_VARPATH"] = "window"
    try:
        engine.device_batch(data, d_off, d_len, 1, d_out, total_bytes=n)
    finally:
        os.environ.pop("MI_CRC32C_VARPATH", None)
    assert engine.stats()["window_batches"] == before + 1
    host = data.download(np.uint8, 1 << 32)
    data.free()
    want = oracle.crc32c(0, host[1:])
    del host
    assert int(d_out.download(np.uint32, 1)[0]) == want
    for b in (d_off, d_len, d_out):
        b.free()


def test_window_task_overflow_on_an_async_batch_fails_the_next_sync(engine, oracle):
    """1,100 aliased records of 0xFFFFFFFF bytes are 9.2e9 windows,
    past the window path's 2^31 task bound, with a hint of 1 byte (which
    routes them to the window path).  The kernel hashes nothing and sets the
    sticky word; the next stream sync reports EINVAL (counted), and a true
    batch after it on the same context is exact."""
    count = 1100
    data = engine.DeviceBuffer((1 << 32) + 64)
    d_off, d_len, d_out = (engine.DeviceBuffer(count * 8), engine.DeviceBuffer(count * 4),
                           engine.DeviceBuffer(count * 4))
    d_off.upload(np.zeros(count, dtype=np.uint64))
    d_len.upload(np.full(count, 0xFFFFFFFF, dtype=np.uint32))
    rng = np.random.default_rng(9)
    small = rng.integers(0, 256, 5000, dtype=np.uint8)

    def run():
        before = engine.stats()
        engine.device_batch(data, d_off, d_len, count, d_out, total_bytes=1, asynchronous=True)
        try:
            engine.sync()
            first = "ok"
        except engine.EngineError as e:
            first = e.status
        after = engine.stats()
        got = engine.crc32c_batch(small, np.array([0, 7], dtype=np.uint64),
                                  np.array([4000, 900], dtype=np.uint32))
        engine.sync()
        return first, after["window_batches"] - before["window_batches"], \
            after["hint_overflows"] - before["hint_overflows"], got
    first, nwin, nover, got = _in_thread(run)
    assert first == engine.EINVAL and nwin == 1 and nover == 1
    assert np.array_equal(got, oracle.batch(small, np.array([0, 7], dtype=np.uint64),
                                            np.array([4000, 900], dtype=np.uint32)))
    for b in (data, d_off, d_len, d_out):
        b.free()
