"""GPU parity of the sorted variable-length path:
one team per whole record, records binned by row count inside each
workgroup's cost-balanced share, split records XORed together from their
pieces.  The piece is sized by the batch (engine.hip sorted_piece_log2: 2 KiB
below 32 MiB, 4 KiB below 112 MiB, 8 KiB below 224 MiB, 16 KiB below 1.5 GiB,
32 KiB below 3 GiB, 64 KiB above); every
test runs with the size's own
piece ("auto", 4-row ring, whole records finished in the loop), with the
2-row ring (the finish pass), and with 64 KiB pieces forced
(MI_CRC32C_SORT_PIECE_LOG2=16, the configs[2] piece, 2-row ring), the last
also with lane items off (MI_CRC32C_SORT_LANE_ROWS=0: records of <= 2 rows
take teams too).  MI_CRC32C_VARPATH=sorted makes the default explicit;
every result is compared with the CPU oracle, bit-exact, and the path is
checked to have run (mi_crc32c_stats().sorted_batches).  The hash kernel
computes the cost blocks itself behind a grid barrier (one launch, round 5)
with MI_CRC32C_SORT_FUSED=1 (the "one launch" parameter; measured slower than
sorted_cost_kernel + the hash kernel, the default) while no other thread's
context uses the sorted path on the device.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["auto", "auto-1launch", "auto-ring2", "16", "16-nolane"],
                ids=["piece_auto", "piece_auto_one_launch", "piece_auto_ring2", "piece_64k",
                     "piece_64k_teams_only"])
def sorted_path(engine, request):
    old = os.environ.get("MI_CRC32C_VARPATH")
    os.environ["MI_CRC32C_VARPATH"] = "sorted"
    if request.param == "auto-1launch":
        os.environ["MI_CRC32C_SORT_FUSED"] = "1"  # cost blocks + a grid barrier in the hash kernel
    elif request.param == "auto-ring2":
        os.environ["MI_CRC32C_SORT_RING"] = "2"
    elif request.param == "16-nolane":
        os.environ["MI_CRC32C_SORT_PIECE_LOG2"] = "16"
        os.environ["MI_CRC32C_SORT_LANE_ROWS"] = "0"
    elif request.param != "auto":
        os.environ["MI_CRC32C_SORT_PIECE_LOG2"] = request.param
    before = engine.stats()["sorted_batches"]
    yield lambda: engine.stats()["sorted_batches"] - before
    os.environ.pop("MI_CRC32C_SORT_PIECE_LOG2", None)
    os.environ.pop("MI_CRC32C_SORT_RING", None)
    os.environ.pop("MI_CRC32C_SORT_LANE_ROWS", None)
    os.environ.pop("MI_CRC32C_SORT_FUSED", None)
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


def _device_run(engine, buf, offsets, lengths, inits=None):
    count = lengths.size
    data = engine.DeviceBuffer(max(buf.size, 16))
    data.upload(buf)
    d_off, d_len, d_out = (engine.DeviceBuffer(max(count, 1) * 8), engine.DeviceBuffer(max(count, 1) * 4),
                           engine.DeviceBuffer(max(count, 1) * 4))
    d_off.upload(offsets)
    d_len.upload(lengths)
    d_in = None
    if inits is not None:
        d_in = engine.DeviceBuffer(count * 4)
        d_in.upload(inits)
    total = int(lengths.sum(dtype=np.uint64))
    engine.device_batch(data, d_off, d_len, count, d_out, inits=d_in, total_bytes=max(total, 1))
    got = d_out.download(np.uint32, count)
    for b in (data, d_off, d_len, d_out, d_in):
        if b is not None:
            b.free()
    return got


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_sorted_random_lengths(engine, oracle, sorted_path, seed):
    """Lengths 0..20000 (including 0-3 B records, finished by the cost
    kernel), unaligned starts, small gaps, with and without inits."""
    rng = np.random.default_rng(100 + seed)
    count = 40_000
    lengths = rng.integers(0, 20_000, count).astype(np.uint32)
    lengths[rng.integers(0, count, 2000)] = rng.integers(0, 5, 2000)
    offsets, end = _packed(rng, lengths, gap=9, start=int(rng.integers(0, 128)))
    buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32)
    assert np.array_equal(_device_run(engine, buf, offsets, lengths),
                          oracle.batch(buf, offsets, lengths))
    assert np.array_equal(_device_run(engine, buf, offsets, lengths, inits),
                          oracle.batch(buf, offsets, lengths, inits))
    assert sorted_path() == 2


def test_sorted_zipf_host_and_device(engine, oracle, sorted_path):
    """configs[2]'s length distribution (Zipf 64 B - 64 KiB), packed, as a
    device batch and as a host batch (staged)."""
    rng = np.random.default_rng(5)
    count = 30_000
    lengths = engine.zipf_lengths(0xDA7A5EED, count).astype(np.uint32)
    offsets, end = _packed(rng, lengths)
    buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
    exp = oracle.batch(buf, offsets, lengths)
    assert np.array_equal(_device_run(engine, buf, offsets, lengths), exp)
    assert np.array_equal(engine.crc32c_batch(buf, offsets, lengths, planned=True), exp)
    assert sorted_path() == 2


@pytest.mark.parametrize("start", [0, 1, 64, 127])
def test_sorted_split_records(engine, oracle, sorted_path, start):
    """Records around and beyond the 64 KiB piece: 65535, 65536, 65537,
    65536 + 127/128/129, 200 KiB, 1 MiB, 3 MiB at every alignment class,
    mixed with short ones; inits chain through the first piece."""
    rng = np.random.default_rng(40 + start)
    big = [65535, 65536, 65537, 65536 + 127, 65536 + 128, 65536 + 129, 131072, 131073,
           200 << 10, 1 << 20, 3 << 20, 4, 5, 3, 0, 1000]
    lengths = np.array(big * 3 + list(rng.integers(0, 9000, 300)), dtype=np.uint32)
    rng.shuffle(lengths)
    offsets, end = _packed(rng, lengths, gap=3, start=start)
    buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, lengths.size, dtype=np.uint32)
    assert np.array_equal(_device_run(engine, buf, offsets, lengths),
                          oracle.batch(buf, offsets, lengths))
    assert np.array_equal(_device_run(engine, buf, offsets, lengths, inits),
                          oracle.batch(buf, offsets, lengths, inits))


@pytest.mark.parametrize("grid", ["1", "3"])
def test_sorted_one_workgroup_mixed_groups(engine, oracle, sorted_path, grid):
    """One (or three) workgroups: every item of the batch in one sorted list,
    so groups mix pieces of one record with short items and row counts far
    apart (a 1-row last piece beside a 513-row piece: rows before the item's
    first row must stay zero, init word included)."""
    rng = np.random.default_rng(int(grid))
    lengths = np.array([65537, 65536 + 60000, 131073, 5, 100, 4000, 65535, 200 << 10] +
                       list(rng.integers(0, 3000, 40)), dtype=np.uint32)
    rng.shuffle(lengths)
    offsets, end = _packed(rng, lengths, gap=7, start=3)
    buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, lengths.size, dtype=np.uint32)
    os.environ["MI_CRC32C_SORTED_GRID"] = grid
    try:
        assert np.array_equal(_device_run(engine, buf, offsets, lengths),
                              oracle.batch(buf, offsets, lengths))
        assert np.array_equal(_device_run(engine, buf, offsets, lengths, inits),
                              oracle.batch(buf, offsets, lengths, inits))
    finally:
        del os.environ["MI_CRC32C_SORTED_GRID"]


@pytest.mark.parametrize("grid", ["1", "2"])
def test_sorted_second_pass(engine, oracle, sorted_path, grid):
    """More than 8 records per thread in a workgroup's range (one or two
    workgroups for 30K records): the binning takes its second pass instead
    of holding the ranks in registers; split records included."""
    rng = np.random.default_rng(50 + int(grid))
    lengths = rng.integers(0, 3000, 30_000).astype(np.uint32)
    lengths[rng.integers(0, lengths.size, 12)] = rng.integers(65_537, 300_000, 12)
    offsets, end = _packed(rng, lengths, gap=5, start=11)
    buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, lengths.size, dtype=np.uint32)
    os.environ["MI_CRC32C_SORTED_GRID"] = grid
    try:
        assert np.array_equal(_device_run(engine, buf, offsets, lengths, inits),
                              oracle.batch(buf, offsets, lengths, inits))
    finally:
        del os.environ["MI_CRC32C_SORTED_GRID"]


@pytest.mark.parametrize("grid", ["1", "2", None])
def test_sorted_513_row_records_beside_512_row_pieces(engine, oracle, sorted_path, grid):
    """Whole records of 513 rows (<= 64 KiB but straddling 513 windows) in the
    same workgroup as split records with 128-B-aligned starts, whose full
    pieces have 512 rows: the full pieces are listed first, so a group can
    hold a 512-row piece before a 513-row record (found by the fuzz rounds;
    the group's shape must come from its largest item wherever it sits)."""
    rng = np.random.default_rng(77)
    recs = []  # (alignment within 128 B, length)
    for _ in range(40):
        recs.append((0, int(rng.integers(65537, 300_000))))     # split, aligned: 512-row pieces
        recs.append((int(rng.integers(64, 128)), 65536 - int(rng.integers(0, 60))))  # 513 rows
        recs.append((int(rng.integers(0, 128)), int(rng.integers(4, 9000))))
    rng.shuffle(recs)
    offsets, pos = [], 4096
    for a, L in recs:
        pos = (pos + 127) // 128 * 128 + a
        offsets.append(pos)
        pos += L + int(rng.integers(0, 300))
    offsets = np.array(offsets, dtype=np.uint64)
    lengths = np.array([L for _, L in recs], dtype=np.uint32)
    buf = rng.integers(0, 256, pos + 256, dtype=np.uint8)
    inits = rng.integers(0, 2**32, lengths.size, dtype=np.uint32)
    if grid:
        os.environ["MI_CRC32C_SORTED_GRID"] = grid
    try:
        assert np.array_equal(_device_run(engine, buf, offsets, lengths, inits),
                              oracle.batch(buf, offsets, lengths, inits))
        assert np.array_equal(_device_run(engine, buf, offsets, lengths),
                              oracle.batch(buf, offsets, lengths))
    finally:
        os.environ.pop("MI_CRC32C_SORTED_GRID", None)


def test_sorted_one_huge_record(engine, oracle, sorted_path):
    """One 40 MiB record and a few short ones: the record's 641 pieces are
    spread over many workgroups (the cost split falls inside it)."""
    rng = np.random.default_rng(9)
    lengths = np.array([17, 40 << 20, 300, 5], dtype=np.uint32)
    offsets, end = _packed(rng, lengths, start=3)
    buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
    inits = np.array([1, 0xDEADBEEF, 7, 9], dtype=np.uint32)
    assert np.array_equal(_device_run(engine, buf, offsets, lengths, inits),
                          oracle.batch(buf, offsets, lengths, inits))


@pytest.mark.parametrize("plog", ["9", "12", "14"])
def test_sorted_piece_shift_forms(engine, oracle, plog, monkeypatch):
    """Round 6: a piece's shift to its record's end, P jj, comes from its
    descriptor (jj in the address word's top 16 bits): one Z_{512 k} lookup
    while P jj / 512 < 256, the G^{2^k} chain beyond, and off/len re-read
    when jj does not fit 16 bits.  A 40 MiB record cut into 512 B pieces has
    81,920 of them (jj up to 81,919: all three forms); 4 and 16 KiB pieces
    take the first two.  Records of 64-300 KiB beside
    it, with inits."""
    monkeypatch.setenv("MI_CRC32C_VARPATH", "sorted")
    monkeypatch.setenv("MI_CRC32C_SORT_PIECE_LOG2", plog)
    rng = np.random.default_rng(int(plog))
    lengths = np.array([40 << 20, 65 << 10, 300 << 10, 129 << 10, 7, 100, 513, 2049],
                       dtype=np.uint32)
    offsets, end = _packed(rng, lengths, start=int(rng.integers(0, 128)))
    buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
    inits = rng.integers(0, 2**32, lengths.size, dtype=np.uint32)
    before = engine.stats()["sorted_batches"]
    assert np.array_equal(_device_run(engine, buf, offsets, lengths, inits),
                          oracle.batch(buf, offsets, lengths, inits))
    assert engine.stats()["sorted_batches"] > before


@pytest.mark.parametrize("count", [1, 2, 7, 8, 9, 255, 257, 4097])
def test_sorted_few_records(engine, oracle, sorted_path, count):
    """Fewer records than workgroups (most ranges empty) and partial groups."""
    rng = np.random.default_rng(count)
    lengths = rng.integers(4, 5000, count).astype(np.uint32)
    offsets, end = _packed(rng, lengths, gap=40, start=5)
    buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
    assert np.array_equal(_device_run(engine, buf, offsets, lengths),
                          oracle.batch(buf, offsets, lengths))


def test_sorted_only_tiny_records(engine, oracle, sorted_path):
    """Every record shorter than 4 B: the cost kernel finishes them all and
    the hash kernel has no items (total cost 0)."""
    rng = np.random.default_rng(11)
    count = 10_000
    lengths = rng.integers(0, 4, count).astype(np.uint32)
    offsets, end = _packed(rng, lengths, gap=2)
    buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32)
    assert np.array_equal(_device_run(engine, buf, offsets, lengths, inits),
                          oracle.batch(buf, offsets, lengths, inits))


def test_sorted_unordered_overlapping(engine, oracle, sorted_path):
    """Records in any order, overlapping each other, equal lengths (large
    bins of one row count)."""
    rng = np.random.default_rng(13)
    buf = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    count = 20_000
    lengths = np.where(rng.random(count) < 0.5, 4096, rng.integers(0, 70_000, count)).astype(np.uint32)
    offsets = rng.integers(0, buf.size - 70_000, count).astype(np.uint64)
    assert np.array_equal(_device_run(engine, buf, offsets, lengths),
                          oracle.batch(buf, offsets, lengths))


def test_sorted_matches_piece_path(engine, oracle):
    """The two variable-length paths agree on the same device batch."""
    rng = np.random.default_rng(17)
    count = 50_000
    lengths = engine.zipf_lengths(0x5EED, count).astype(np.uint32)
    offsets, end = _packed(rng, lengths, gap=5, start=33)
    buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
    old = os.environ.get("MI_CRC32C_VARPATH")
    try:
        os.environ["MI_CRC32C_VARPATH"] = "pieces"
        a = _device_run(engine, buf, offsets, lengths)
        os.environ["MI_CRC32C_VARPATH"] = "sorted"
        b = _device_run(engine, buf, offsets, lengths)
    finally:
        if old is None:
            os.environ.pop("MI_CRC32C_VARPATH", None)
        else:
            os.environ["MI_CRC32C_VARPATH"] = old
    assert np.array_equal(a, b)
    assert np.array_equal(b, oracle.batch(buf, offsets, lengths))


def _device_run_no_hint(engine, buf, offsets, lengths):
    count = lengths.size
    data = engine.DeviceBuffer(max(buf.size, 16))
    data.upload(buf)
    d_off, d_len, d_out = (engine.DeviceBuffer(count * 8), engine.DeviceBuffer(count * 4),
                           engine.DeviceBuffer(count * 4))
    d_off.upload(offsets)
    d_len.upload(lengths)
    engine.device_batch(data, d_off, d_len, count, d_out)
    got = d_out.download(np.uint32, count)
    for b in (data, d_off, d_len, d_out):
        b.free()
    return got


@pytest.mark.parametrize("mib", [1, 64, 300, 400])
def test_sorted_default_with_known_total(engine, oracle, mib):
    """Without the knob, a device batch whose total is given takes the sorted
    path above 26 MiB or 8192 records (round 4: with batch-sized pieces it is
    the faster path from 1 MiB up; round 5: below that bound the one-launch
    window path, tests/test_gpu_window.py); without the total, the piece path
    (its plan reads the item count back)."""
    rng = np.random.default_rng(19 + mib)
    count = (mib << 20) // 3400 + 1
    lengths = rng.integers(3300, 3500, count).astype(np.uint32)
    lengths[rng.integers(0, count, 8)] = rng.integers(20_000, 200_000, 8)
    offsets, end = _packed(rng, lengths)
    buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
    want = oracle.batch(buf, offsets, lengths)
    path = "window_batches" if end <= (26 << 20) and count <= 8192 else "sorted_batches"
    before = engine.stats()[path]
    assert np.array_equal(_device_run(engine, buf, offsets, lengths), want)
    assert engine.stats()[path] == before + 1
    if mib <= 64:
        before = engine.stats()["sorted_batches"]
        assert np.array_equal(_device_run_no_hint(engine, buf, offsets, lengths), want)
        assert engine.stats()["sorted_batches"] == before


@pytest.mark.parametrize("seed", range(10))
def test_sorted_fuzz_large(engine, oracle, sorted_path, seed):
    """Seeded batches of 5K-60K records (at most ~200 MB) through the sorted
    path at random grids, so that one workgroup's share holds more than 8
    records per thread (the binning's second pass) as well as fewer; every
    length class of the GPU fuzz rounds, packed or scattered, with and
    without inits."""
    from test_gpu_fuzz import random_lengths
    rng = np.random.default_rng(5150 + seed)
    count = int(rng.integers(5_000, 60_000))
    lengths = np.clip(random_lengths(rng, count), 0, None).astype(np.uint32)
    while int(lengths.sum(dtype=np.uint64)) > 200 << 20:
        lengths = (lengths // 2).astype(np.uint32)
    if rng.integers(0, 2):
        offsets, end = _packed(rng, lengths, gap=int(rng.integers(0, 9)), start=int(rng.integers(0, 4096)))
        size = end + 64
    else:
        size = int(lengths.max()) + int(rng.integers(1, 64 << 20))
        offsets = (rng.random(count) * (size - lengths.astype(np.float64))).astype(np.uint64)
    buf = rng.integers(0, 256, size, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32) if rng.integers(0, 2) else None
    grid = [None, "1", "2", "3", "16"][int(rng.integers(0, 5))]
    if grid:
        os.environ["MI_CRC32C_SORTED_GRID"] = grid
    try:
        got = _device_run(engine, buf, offsets, lengths, inits)
    finally:
        os.environ.pop("MI_CRC32C_SORTED_GRID", None)
    assert np.array_equal(got, oracle.batch(buf, offsets, lengths, inits)), grid
    assert sorted_path() == 1


def test_sorted_leading_and_trailing_tiny_records(engine, oracle, sorted_path):
    """Records shorter than 4 B at the very start and end of the batch (zero
    cost: no workgroup's share starts on them; the cost kernel finishes
    them), split records between them."""
    rng = np.random.default_rng(61)
    lengths = np.concatenate([rng.integers(0, 4, 300), rng.integers(4, 20_000, 3000),
                              [70_000, 9000, 200_000], rng.integers(0, 4, 300)]).astype(np.uint32)
    offsets, end = _packed(rng, lengths, gap=3, start=7)
    buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, lengths.size, dtype=np.uint32)
    assert np.array_equal(_device_run(engine, buf, offsets, lengths, inits),
                          oracle.batch(buf, offsets, lengths, inits))
    assert np.array_equal(_device_run(engine, buf, offsets, lengths),
                          oracle.batch(buf, offsets, lengths))


def test_sorted_many_batches_split_records(engine, oracle, sorted_path):
    """Many batches in a row on one stream, split records at varying
    positions (their pieces XOR into out[]), every result exact."""
    rng = np.random.default_rng(62)
    for k in range(12):
        count = int(rng.integers(50, 3000))
        lengths = rng.integers(0, 9000, count).astype(np.uint32)
        lengths[rng.integers(0, count, 5)] = rng.integers(20_000, 150_000, 5)
        offsets, end = _packed(rng, lengths, gap=int(rng.integers(0, 5)), start=int(rng.integers(0, 128)))
        buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
        assert np.array_equal(_device_run(engine, buf, offsets, lengths),
                              oracle.batch(buf, offsets, lengths)), k


@pytest.mark.parametrize("plog", [9, 11, 12, 16])
def test_sorted_end_cut_head_keeps_init_word(engine, oracle, monkeypatch, plog):
    """Pieces are cut from the record's end; the head (the remainder at the
    start) keeps at least 4 bytes so the ~init word stays inside it, and a
    shorter remainder joins the next piece.  Lengths k*P + d for d in -1..5
    around every multiple of the piece P, at every start alignment class,
    with inits."""
    monkeypatch.setenv("MI_CRC32C_VARPATH", "sorted")
    monkeypatch.setenv("MI_CRC32C_SORT_PIECE_LOG2", str(plog))
    P = 1 << plog
    rng = np.random.default_rng(70 + plog)
    lens = [k * P + d for k in (1, 2, 3) for d in range(-1, 6)]
    lengths = np.array(lens * 6 + list(rng.integers(0, 3 * P, 200)), dtype=np.uint32)
    rng.shuffle(lengths)
    offsets, end = _packed(rng, lengths, gap=5, start=int(rng.integers(0, 128)))
    buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, lengths.size, dtype=np.uint32)
    assert np.array_equal(_device_run(engine, buf, offsets, lengths, inits),
                          oracle.batch(buf, offsets, lengths, inits))
    assert np.array_equal(_device_run(engine, buf, offsets, lengths),
                          oracle.batch(buf, offsets, lengths))


@pytest.mark.parametrize("plog", [None, "9"])
def test_sorted_lane_items_every_shape(engine, oracle, sorted_path, plog, monkeypatch):
    """Lane items (records spanning <= 2 rows, one per lane): every length
    4..400 at every start offset mod 16, with and without inits, mixed with
    team items; with 512-B pieces (plog 9) also split records whose short
    heads are lane items (their part shifted by Z_{E - pe} and XORed in)."""
    if plog:
        monkeypatch.setenv("MI_CRC32C_SORT_PIECE_LOG2", plog)
    rng = np.random.default_rng(77)
    lens = [L for L in range(4, 401) for _ in range(2)]
    lens += [512 * k + h for k in (1, 2, 5) for h in range(4, 140, 3)]  # short heads at plog 9
    lens += list(rng.integers(0, 3000, 500))
    lengths = np.array(lens, dtype=np.uint32)
    rng.shuffle(lengths)
    offsets, end = _packed(rng, lengths, gap=15, start=int(rng.integers(0, 16)))
    buf = rng.integers(0, 256, end + 32, dtype=np.uint8)
    inits = rng.integers(0, 2**32, lengths.size, dtype=np.uint32)
    assert np.array_equal(_device_run(engine, buf, offsets, lengths),
                          oracle.batch(buf, offsets, lengths))
    assert np.array_equal(_device_run(engine, buf, offsets, lengths, inits),
                          oracle.batch(buf, offsets, lengths, inits))
    assert sorted_path() == 2


@pytest.mark.parametrize("count", [8500, 9728, 9729, 9900])
def test_sorted_descriptor_staging_limits(engine, oracle, sorted_path, count):
    """One workgroup holding 8,500-9,900 items: the descriptor list is staged
    in LDS up to kLdsBytes / 16 = 9,728 items (above 8,192 records through the
    binning's second pass) and stored directly above that."""
    rng = np.random.default_rng(count)
    lengths = rng.integers(4, 700, count).astype(np.uint32)
    offsets, end = _packed(rng, lengths, gap=3, start=5)
    buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32)
    os.environ["MI_CRC32C_SORTED_GRID"] = "1"
    try:
        assert np.array_equal(_device_run(engine, buf, offsets, lengths, inits),
                              oracle.batch(buf, offsets, lengths, inits))
    finally:
        del os.environ["MI_CRC32C_SORTED_GRID"]


ONE_LAUNCH_SCRIPT = r"""
import os, sys
import numpy as np
import consus_amd as E
from oracle.oracle import Oracle
from tests.test_gpu_sorted import _device_run, _packed
E.init(0)
orc = Oracle()
os.environ["MI_CRC32C_VARPATH"] = "sorted"
# (1) the one-launch form runs (this process's only sorted context) and gives
# the two launches' CRCs: configs[2] lengths, inits, split and 0-3 B records
rng = np.random.default_rng(77)
count = 50_000
lengths = E.zipf_lengths(0x5EED, count).astype(np.uint32)
lengths[rng.integers(0, count, 500)] = rng.integers(0, 4, 500)
lengths[rng.integers(0, count, 20)] = rng.integers(70_000, 300_000, 20)
offsets, end = _packed(rng, lengths, start=3)
buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
inits = rng.integers(0, 2**32, count, dtype=np.uint32)
want = orc.batch(buf, offsets, lengths, inits)
for plog in ("16", "12"):
    os.environ["MI_CRC32C_SORT_PIECE_LOG2"] = plog
    for fused, runs in (("1", 1), ("0", 0)):
        os.environ["MI_CRC32C_SORT_FUSED"] = fused
        before = E.stats()["sorted_one_launch"]
        assert np.array_equal(_device_run(E, buf, offsets, lengths, inits), want), (plog, fused)
        assert E.stats()["sorted_one_launch"] - before == runs, (plog, fused)
del os.environ["MI_CRC32C_SORT_PIECE_LOG2"]
# (2) the barrier's wait is bounded: one arrival too many awaited
# (MI_CRC32C_SORT_BARRIER_SKEW=1), every workgroup times out; a synchronous
# batch recomputes with two launches (exact), an asynchronous one fails the
# next stream sync, after which the engine is clean
os.environ["MI_CRC32C_SORT_FUSED"] = "1"
os.environ["MI_CRC32C_SORT_BARRIER_SKEW"] = "1"
rng = np.random.default_rng(78)
count = 8_000
lengths = E.zipf_lengths(0x5EEE, count).astype(np.uint32)
offsets, end = _packed(rng, lengths)
buf = rng.integers(0, 256, end + 16, dtype=np.uint8)
want = orc.batch(buf, offsets, lengths)
assert np.array_equal(_device_run(E, buf, offsets, lengths), want)
data = E.DeviceBuffer(buf.size)
data.upload(buf)
d_off, d_len, d_out = E.DeviceBuffer(count * 8), E.DeviceBuffer(count * 4), E.DeviceBuffer(count * 4)
d_off.upload(offsets)
d_len.upload(lengths)
total = int(lengths.sum(dtype=np.uint64))
E.device_batch(data, d_off, d_len, count, d_out, total_bytes=total, asynchronous=True)
try:
    E.sync()
    raise SystemExit("the timed-out asynchronous batch was not reported")
except E.EngineError as e:
    assert e.status == E.EINVAL
del os.environ["MI_CRC32C_SORT_BARRIER_SKEW"]
E.sync()
E.device_batch(data, d_off, d_len, count, d_out, total_bytes=total, asynchronous=True)
E.sync()
assert np.array_equal(d_out.download(np.uint32, count), want)
st = E.stats()
assert st["fallback_calls"] == 0 and st["host_routed_calls"] == 0, st
print("one-launch ok", st["sorted_one_launch"])
"""


def test_sorted_one_launch_form_and_its_bounded_barrier():
    """The one-launch form (cost blocks and a grid barrier in the hash
    kernel, MI_CRC32C_SORT_FUSED=1) runs only while one thread context of the
    process uses the sorted path on the device -- the suite's own process
    holds others (multi-device workers, flush threads) -- so it is checked in
    a fresh process: the same CRCs as the two launches, and a barrier that
    times out (MI_CRC32C_SORT_BARRIER_SKEW=1: one arrival too many awaited)
    is recovered on a synchronous batch and reported on an asynchronous one."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if not k.startswith("MI_CRC32C_SORT")}
    r = subprocess.run([sys.executable, "-c", ONE_LAUNCH_SCRIPT], capture_output=True, text=True,
                       cwd=repo, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "one-launch ok" in r.stdout, r.stdout
    assert int(r.stdout.split("one-launch ok")[1].split()[0]) == 5, r.stdout  # 2 + 3 fused launches


@pytest.mark.parametrize("grid", [None, "7", "40"])
def test_sorted_many_lane_items_small_grids(engine, oracle, grid):
    """Lane items (records of <= 2 rows) drained by the waves' grabs of 64,
    each fetching the next grab's descriptors while it hashes this one and
    all of an item's blocks at once (round 5): a 120K-record batch, most of
    it lane items, with inits, split records and 0-3 B records, at the
    default grid and at small ones (a few workgroups with many items each,
    most of them past the LDS descriptor staging), with the one-launch form
    and without."""
    rng = np.random.default_rng(91)
    count = 120_000
    lengths = rng.integers(4, 300, count).astype(np.uint32)
    big = rng.integers(0, count, 3000)
    lengths[big] = engine.zipf_lengths(0x1234, 3000)
    lengths[rng.integers(0, count, 30)] = rng.integers(70_000, 200_000, 30)
    lengths[rng.integers(0, count, 500)] = rng.integers(0, 4, 500)
    offsets, end = _packed(rng, lengths, gap=3, start=5)
    buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32)
    want = oracle.batch(buf, offsets, lengths, inits)
    os.environ["MI_CRC32C_VARPATH"] = "sorted"
    if grid:
        os.environ["MI_CRC32C_SORTED_GRID"] = grid
    try:
        for mode in ("0", "1"):
            os.environ["MI_CRC32C_SORT_FUSED"] = mode
            got = _device_run(engine, buf, offsets, lengths, inits)
            assert np.array_equal(got, want), (grid, mode, int(np.sum(got != want)))
    finally:
        for k in ("MI_CRC32C_VARPATH", "MI_CRC32C_SORTED_GRID", "MI_CRC32C_SORT_FUSED"):
            os.environ.pop(k, None)
