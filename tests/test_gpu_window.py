"""GPU parity of the window path (crc32c_kernels.hip "window path", DESIGN.md
section 4.3): mid-size device batches (at most kWinMaxCount = 8192 records,
26 MiB by default) in one launch.  Each record is cut into windows of 4, 8
or 16 rows (512 B - 2 KiB, by batch size) counted back from its end, one
window per team; a record over several waves is combined through one 64-bit
word per record (XOR and segment mask; acc[] / cnt[] past 32 segments), the
last segment storing the CRC and zeroing the words.  Every result is compared with the
CPU oracle, bit-exact; the path is checked to have run
(mi_crc32c_stats().window_batches).  MI_CRC32C_VARPATH=window forces the path
up to 8192 records; without it, the engine takes it by size.  Each forced
test runs with the workgroup and window the engine picks by count and size,
and with one-wave / four-wave / one-per-CU twelve-wave workgroups
(MI_CRC32C_WIN_BLOCK=64 / 256 / 768) and 8 / 16-row
windows (MI_CRC32C_WIN_ROWS, also 4) forced.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[{}, {"MI_CRC32C_WIN_BLOCK": "64"}, {"MI_CRC32C_WIN_BLOCK": "256"},
                        {"MI_CRC32C_WIN_BLOCK": "768"},
                        {"MI_CRC32C_WIN_ROWS": "4"}, {"MI_CRC32C_WIN_ROWS": "8"},
                        {"MI_CRC32C_WIN_ROWS": "16"}],
                ids=["by_size", "block_64", "block_256", "block_768", "rows_4", "rows_8", "rows_16"])
def window_path(engine, request):
    old = os.environ.get("MI_CRC32C_VARPATH")
    os.environ["MI_CRC32C_VARPATH"] = "window"
    os.environ.update(request.param)
    before = engine.stats()["window_batches"]
    yield lambda: engine.stats()["window_batches"] - before
    for k in request.param:
        os.environ.pop(k, None)
    if old is None:
        del os.environ["MI_CRC32C_VARPATH"]
    else:
        os.environ["MI_CRC32C_VARPATH"] = old


def _packed(rng, lengths, gap=0, start=0):
    offsets = np.zeros(lengths.size, dtype=np.uint64)
    if lengths.size > 1:
        steps = lengths[:-1].astype(np.uint64)
        if gap:
            steps = steps + rng.integers(0, gap + 1, lengths.size - 1).astype(np.uint64)
        offsets[1:] = np.cumsum(steps)
    offsets += np.uint64(start)
    end = int(offsets[-1]) + int(lengths[-1]) if lengths.size else start
    return offsets, end


class _Batch:
    """A device batch kept resident, so that it can run several times."""

    def __init__(self, engine, buf, offsets, lengths, inits=None):
        self.e, self.count = engine, lengths.size
        n = max(self.count, 1)
        self.data = engine.DeviceBuffer(max(buf.size, 16))
        self.data.upload(buf)
        self.off, self.len, self.out = (engine.DeviceBuffer(n * 8), engine.DeviceBuffer(n * 4),
                                        engine.DeviceBuffer(n * 4))
        self.off.upload(offsets)
        self.len.upload(lengths)
        self.ini = None
        if inits is not None:
            self.ini = engine.DeviceBuffer(n * 4)
            self.ini.upload(inits)
        self.total = int(lengths.sum(dtype=np.uint64))

    def run(self, hint=None):
        self.out.upload(np.full(max(self.count, 1), 0xABABABAB, dtype=np.uint32))
        self.e.device_batch(self.data, self.off, self.len, self.count, self.out, inits=self.ini,
                            total_bytes=max(self.total, 1) if hint is None else hint)
        return self.out.download(np.uint32, self.count)

    def free(self):
        for b in (self.data, self.off, self.len, self.out, self.ini):
            if b is not None:
                b.free()


def _check(engine, oracle, buf, offsets, lengths, inits=None, hint=None, runs=1):
    b = _Batch(engine, buf, offsets, lengths, inits)
    try:
        want = oracle.batch(buf, offsets, lengths, inits)
        for _ in range(runs):
            assert np.array_equal(b.run(hint), want)
    finally:
        b.free()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_window_random_lengths(engine, oracle, window_path, seed):
    """Lengths 0..20000 (with many 0-5 B records: the seed form below 4 B),
    unaligned starts, small gaps, with and without inits."""
    rng = np.random.default_rng(500 + seed)
    count = 3000
    lengths = rng.integers(0, 20_000, count).astype(np.uint32)
    lengths[rng.integers(0, count, 400)] = rng.integers(0, 6, 400)
    offsets, end = _packed(rng, lengths, gap=9, start=int(rng.integers(0, 128)))
    buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32)
    _check(engine, oracle, buf, offsets, lengths)
    _check(engine, oracle, buf, offsets, lengths, inits)
    assert window_path() == 2


@pytest.mark.parametrize("start", [0, 1, 61, 124, 125, 127])
def test_window_edges_and_long_records(engine, oracle, window_path, start):
    """Every length class around the window and row edges (2047/2048/2049,
    127/128/129, 1-5 B), records of 64 windows and more (the shift past the
    Z_{2048 k} tables, k >= 64), up to 3 MiB; starts at every alignment class
    (125-127: the init word spills into the next row)."""
    rng = np.random.default_rng(60 + start)
    edge = [0, 1, 2, 3, 4, 5, 15, 16, 17, 127, 128, 129, 255, 256, 257, 2047, 2048, 2049,
            4095, 4096, 4097, 32767, 65535, 65536, 65537, 131071, 131072, 131073,
            131072 + 2048, 200 << 10, 1 << 20, 3 << 20]
    lengths = np.array(edge * 2 + list(rng.integers(0, 9000, 200)), dtype=np.uint32)
    rng.shuffle(lengths)
    offsets, end = _packed(rng, lengths, gap=3, start=start)
    buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, lengths.size, dtype=np.uint32)
    _check(engine, oracle, buf, offsets, lengths)
    _check(engine, oracle, buf, offsets, lengths, inits)
    assert window_path() == 2


def test_window_overlapping_and_unordered_records(engine, oracle, window_path):
    """Offsets in any order, records overlapping each other and sharing rows."""
    rng = np.random.default_rng(7)
    count = 2500
    size = 1 << 20
    lengths = rng.integers(0, 40_000, count).astype(np.uint32)
    offsets = rng.integers(0, size - 40_000, count).astype(np.uint64)
    buf = rng.integers(0, 256, size, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32)
    _check(engine, oracle, buf, offsets, lengths, inits)
    assert window_path() == 1


@pytest.mark.parametrize("count", [1, 2, 4095, 4096, 8191, 8192])
def test_window_record_counts(engine, oracle, window_path, count):
    """One record to the 8192-record bound."""
    rng = np.random.default_rng(count)
    lengths = rng.integers(0, 6000, count).astype(np.uint32)
    offsets, end = _packed(rng, lengths, start=3)
    buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
    _check(engine, oracle, buf, offsets, lengths)
    assert window_path() == 1


def test_window_above_the_count_bound_takes_the_sorted_path(engine, oracle, window_path):
    """8193 records: the window path declines even when forced."""
    rng = np.random.default_rng(8193)
    lengths = rng.integers(0, 3000, 8193).astype(np.uint32)
    offsets, end = _packed(rng, lengths)
    buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
    before = engine.stats()["sorted_batches"]
    _check(engine, oracle, buf, offsets, lengths)
    assert window_path() == 0
    assert engine.stats()["sorted_batches"] == before + 1


@pytest.mark.parametrize("count", [8193, 12000, 16384, 16385])
def test_window_raised_count_bound(engine, oracle, window_path, count):
    """MI_CRC32C_WIN_MAX_COUNT raises the record bound up to the 64 KiB LDS
    prefix (16384 records); 16385 records decline."""
    rng = np.random.default_rng(count)
    lengths = rng.integers(0, 4000, count).astype(np.uint32)
    offsets, end = _packed(rng, lengths, gap=2, start=5)
    buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32)
    os.environ["MI_CRC32C_WIN_MAX_COUNT"] = "100000"  # clamped to 16384
    try:
        _check(engine, oracle, buf, offsets, lengths, inits)
    finally:
        del os.environ["MI_CRC32C_WIN_MAX_COUNT"]
    assert window_path() == (1 if count <= 16384 else 0)


@pytest.mark.parametrize("hint", [1, 4096])
def test_window_understated_hint_loops(engine, oracle, window_path, hint):
    """A total_bytes hint far below the batch sizes a smaller grid, whose
    teams loop over the remaining windows: slower, never wrong (the window
    path keeps no size-bounded workspace)."""
    rng = np.random.default_rng(11)
    lengths = np.array([1 << 20] * 6 + list(rng.integers(0, 5000, 300)), dtype=np.uint32)
    rng.shuffle(lengths)
    offsets, end = _packed(rng, lengths, start=9)
    buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
    _check(engine, oracle, buf, offsets, lengths, hint=hint)
    assert window_path() == 1


def test_window_counters_stay_zero_across_launches(engine, oracle, window_path):
    """Multi-window records leave acc[] / cnt[] zero: the same batch three
    times, then other batches (more records, other splits) on the same
    context, all exact."""
    rng = np.random.default_rng(12)
    for count, hi in ((400, 70_000), (1200, 9000), (50, 300_000)):
        lengths = rng.integers(0, hi, count).astype(np.uint32)
        offsets, end = _packed(rng, lengths, start=int(rng.integers(0, 128)))
        buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
        inits = rng.integers(0, 2**32, count, dtype=np.uint32)
        _check(engine, oracle, buf, offsets, lengths, inits, runs=3)
    assert window_path() == 9


def test_window_empty_records_only(engine, oracle, window_path):
    lengths = np.zeros(100, dtype=np.uint32)
    offsets = np.arange(100, dtype=np.uint64)
    buf = np.zeros(256, dtype=np.uint8)
    inits = np.arange(100, dtype=np.uint32) * np.uint32(0x01010101)
    _check(engine, oracle, buf, offsets, lengths, inits, hint=1)
    assert window_path() == 1


def test_window_default_routing_by_size(engine, oracle):
    """Without MI_CRC32C_VARPATH: configs[2]-like batches (Zipf 64 B - 64 KiB)
    of 1 / 8 / 16 / 20 MiB take the window path (four-wave, one-per-CU, ...
    workgroups by size), one of 6513 records (28 MiB) the sorted path."""
    assert "MI_CRC32C_VARPATH" not in os.environ
    rng = np.random.default_rng(13)
    for count, path in ((230, "window_batches"), (1961, "window_batches"), (3811, "window_batches"),
                        (4727, "window_batches"), (6513, "sorted_batches")):
        lengths = engine.zipf_lengths(0xDA7A5EED, count).astype(np.uint32)
        offsets, end = _packed(rng, lengths)
        buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
        before = engine.stats()[path]
        _check(engine, oracle, buf, offsets, lengths)
        assert engine.stats()[path] == before + 1, (count, end)


def test_window_host_batch_with_long_records(engine, oracle):
    """A host batch with a record past the direct kernel's 16 KiB bound is
    staged and takes the window path by size."""
    rng = np.random.default_rng(14)
    lengths = np.array(list(rng.integers(0, 3000, 500)) + [100_000, 40_000], dtype=np.uint32)
    offsets, end = _packed(rng, lengths, start=5)
    buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
    before = engine.stats()["window_batches"]
    got = engine.crc32c_batch(buf, offsets, lengths)
    assert np.array_equal(got, oracle.batch(buf, offsets, lengths))
    assert engine.stats()["window_batches"] == before + 1


def test_window_concurrent_threads(engine, oracle):
    """Eight threads, each with its own engine context (stream and acc
    words), run window-path batches with records split over several waves
    at once; every result exact, and every context's words left zero (the
    second batch of each thread checks that)."""
    import threading
    errors = []

    def worker(t):
        r = np.random.default_rng(300 + t)
        try:
            for _ in range(2):
                count = int(r.integers(50, 1500))
                lengths = r.integers(0, 20_000, count).astype(np.uint32)  # <= 26 MiB a batch
                offsets, end = _packed(r, lengths, gap=5, start=int(r.integers(0, 128)))
                buf = r.integers(0, 256, end + 16, dtype=np.uint8)
                inits = r.integers(0, 2**32, count, dtype=np.uint32)
                b = _Batch(engine, buf, offsets, lengths, inits)
                try:
                    if not np.array_equal(b.run(), oracle.batch(buf, offsets, lengths, inits, threads=1)):
                        errors.append(("mismatch", t, count))
                finally:
                    b.free()
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(("exception", t, repr(e)))

    assert "MI_CRC32C_VARPATH" not in os.environ
    before = engine.stats()["window_batches"]
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:5]
    assert engine.stats()["window_batches"] >= before + 16
