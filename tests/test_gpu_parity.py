"""GPU parity: the HIP kernels (through the C ABI) vs the CPU oracle.

Bit-exact 32-bit CRCs are required on every case (integer GF(2) work).
Cases follow the reference's semantics (common/crc32c.cc:122-126): any
alignment, any length including 0, chaining inits.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_check_value(engine):
    assert engine.crc32c(0, b"123456789") == 0xE3069283
    assert engine.crc32c(0, bytes(32)) == 0x8A9136AA
    assert engine.crc32c(0, b"\xff" * 32) == 0x62A8AB43
    assert engine.crc32c(0, bytes(range(32))) == 0x46DD794E
    assert engine.crc32c(0, bytes(range(31, -1, -1))) == 0x113FDB5C


def test_empty_returns_init(engine):
    for init in (0, 1, 0xDEADBEEF, 0xFFFFFFFF):
        assert engine.crc32c(init, b"") == init


def test_single_buffers_random(engine, oracle):
    rng = np.random.default_rng(7)
    buf = rng.integers(0, 256, 300_000, dtype=np.uint8)
    for _ in range(60):
        off = int(rng.integers(0, 64))
        n = int(rng.integers(0, 200_000))
        init = int(rng.integers(0, 2**32))
        got = engine.crc32c(init, buf[off:off + n])
        assert got == oracle.crc32c(init, buf, n, off), (off, n, init)


def test_fixed_4k_aligned(engine, oracle):
    rng = np.random.default_rng(1)
    count = 5000
    buf = rng.integers(0, 256, count * 4096, dtype=np.uint8)
    got = engine.crc32c_fixed(buf, 4096, 4096, count)
    exp = oracle.fixed(buf, 4096, 4096, count)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("length,stride", [(16, 16), (128, 128), (1008, 1024), (1024, 1024),
                                           (2048, 2048), (3072, 4096), (4096, 4096),
                                           (4000, 4096), (4112, 4112), (8192, 8192),
                                           (256, 272), (5, 7), (33, 64), (100, 100),
                                           (4097, 4099), (65536, 65536)])
def test_fixed_shapes(engine, oracle, length, stride):
    rng = np.random.default_rng(length * 31 + stride)
    count = 777
    buf = rng.integers(0, 256, (count - 1) * stride + length, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32)
    got = engine.crc32c_fixed(buf, stride, length, count)
    assert np.array_equal(got, oracle.fixed(buf, stride, length, count))
    got = engine.crc32c_fixed(buf, stride, length, count, inits=inits)
    assert np.array_equal(got, oracle.fixed(buf, stride, length, count, inits=inits))


# Host batches of short records take the one-launch direct kernel; planned=True
# skips it (the sorted path, the default with the total known), "pieces"
# forces plan -> chunks -> finalize on the same inputs.
PATHS = pytest.mark.parametrize("planned", [False, True, "pieces"],
                                ids=["direct", "sorted", "pieces"])


@pytest.fixture(autouse=True)
def _force_pieces(request, monkeypatch):
    if "planned" in request.fixturenames and request.getfixturevalue("planned") == "pieces":
        monkeypatch.setenv("MI_CRC32C_VARPATH", "pieces")


@PATHS
def test_var_random_lengths(engine, oracle, planned):
    rng = np.random.default_rng(3)
    count = 4000
    lengths = rng.integers(0, 20000 if planned else 16385, count).astype(np.uint32)
    lengths[::7] = rng.integers(0, 40, lengths[::7].size)
    offsets = np.zeros(count, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    buf = rng.integers(0, 256, int(lengths.sum()) + 1, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32)
    got = engine.crc32c_batch(buf, offsets, lengths, planned=planned)
    assert np.array_equal(got, oracle.batch(buf, offsets, lengths))
    got = engine.crc32c_batch(buf, offsets, lengths, inits, planned=planned)
    assert np.array_equal(got, oracle.batch(buf, offsets, lengths, inits))


@PATHS
def test_var_unordered_overlapping(engine, oracle, planned):
    rng = np.random.default_rng(4)
    buf = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    count = 3000
    lengths = rng.integers(0, 70000 if planned else 16385, count).astype(np.uint32)
    offsets = np.array([rng.integers(0, buf.size - L + 1) for L in lengths], dtype=np.uint64)
    got = engine.crc32c_batch(buf, offsets, lengths, planned=planned)
    assert np.array_equal(got, oracle.batch(buf, offsets, lengths))


def test_device_fill_matches_definition(engine, oracle):
    d = engine.DeviceBuffer(1 << 20)
    d.fill_splitmix64(0xC0DE, byte_offset=4096 * 5)
    assert np.array_equal(d.download(), oracle.fill(1 << 20, 0xC0DE, 4096 * 5))


def make_frames(rng, nbytes, max_entry=20000):
    """A durable-log segment: [recno BE][len BE][entry][crc slot] frames."""
    buf = bytearray()
    offs, lens = [], []
    recno = 1
    while True:
        n = int(rng.integers(0, max_entry))
        if len(buf) + 20 + n > nbytes:
            break
        offs.append(len(buf))
        lens.append(16 + n)
        buf += recno.to_bytes(8, "big") + n.to_bytes(8, "big")
        buf += rng.integers(0, 256, n, dtype=np.uint8).tobytes() + b"\0\0\0\0"
        recno += 1
    return np.frombuffer(bytes(buf), dtype=np.uint8), np.array(offs, np.uint64), \
        np.array(lens, np.uint32)


@pytest.mark.parametrize("max_entry", [20000, 2000], ids=["planned", "direct"])
def test_pipeline_segments_pageable_and_pinned(engine, oracle, max_entry):
    """Segments whose entries are all <= 16 KiB take the direct kernel."""
    rng = np.random.default_rng(8)
    segs = [make_frames(rng, 4 << 20, max_entry) for _ in range(5)]
    p = engine.Pipeline(4 << 20, 16384, depth=2)
    outs, tickets = [], []
    pinned = engine.PinnedBuffer(4 << 20)
    for i, (buf, off, ln) in enumerate(segs):
        out = np.zeros(off.size, dtype=np.uint32)
        if i % 2:
            pinned_i = engine.PinnedBuffer(buf.size)
            pinned_i.array[:] = buf
            tickets.append(p.submit(pinned_i, off, ln, out))
            outs.append((out, pinned_i))
        else:
            tickets.append(p.submit(buf, off, ln, out))
            outs.append((out, None))
    for t in tickets:
        p.wait(t)
    for (buf, off, ln), (out, _) in zip(segs, outs):
        assert np.array_equal(out, oracle.batch(buf, off, ln))
    p.close()
    pinned.free()


def test_pipeline_pageable_reuse_after_submit(engine, oracle):
    """The ownership contract of include/consus_crc32c.h: submit() copies a
    pageable segment and the offsets/lengths before it returns, so the caller
    may overwrite all three at once (one buffer refilled for every segment, as
    a log writer does); the CRCs are of the bytes at submit time."""
    rng = np.random.default_rng(81)
    p = engine.Pipeline(4 << 20, 16384, depth=3)
    segs = [make_frames(rng, 2 << 20, 3000) for _ in range(6)]
    work = np.zeros(2 << 20, dtype=np.uint8)
    outs, tickets = [], []
    for buf, off, ln in segs:
        work[:buf.size] = buf
        w_off, w_len = off.copy(), ln.copy()
        out = np.zeros(off.size, dtype=np.uint32)
        tickets.append(p.submit(work[:buf.size], w_off, w_len, out))
        work[:] = rng.integers(0, 256, work.size, dtype=np.uint8)  # refilled at once
        w_off[:] = 0
        w_len[:] = 1
        outs.append(out)
    for t in tickets:
        p.wait(t)
    for (buf, off, ln), out in zip(segs, outs):
        assert np.array_equal(out, oracle.batch(buf, off, ln))
    p.close()


def test_device_batch_var_and_combine(engine, oracle):
    rng = np.random.default_rng(12)
    count = 20000
    lengths = engine.zipf_lengths(0x5EED, count)
    offsets = np.zeros(count, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    total = int(lengths.sum())
    data = engine.DeviceBuffer(total + 16)
    data.fill_splitmix64(0xDA7A5EED)
    d_off, d_len, d_out = (engine.DeviceBuffer(count * 8), engine.DeviceBuffer(count * 4),
                           engine.DeviceBuffer(count * 4))
    d_off.upload(offsets)
    d_len.upload(lengths)
    for hint in (total, 0):
        engine.device_batch(data, d_off, d_len, count, d_out, total_bytes=hint)
        got = d_out.download(np.uint32, count)
        host = data.download(np.uint8, total)
        assert np.array_equal(got, oracle.batch(host, offsets, lengths))
    a = rng.integers(0, 2**32, 1000, dtype=np.uint32)
    b = rng.integers(0, 2**32, 1000, dtype=np.uint32)
    n = rng.integers(0, 1 << 40, 1000, dtype=np.uint64)
    out = np.zeros(1000, dtype=np.uint32)
    st = engine.lib().mi_crc32c_combine_batch(a.ctypes.data, b.ctypes.data, n.ctypes.data, 1000,
                                               out.ctypes.data, 0)
    assert st == 0
    assert list(out) == [oracle.combine(int(x), int(y), int(z)) for x, y, z in zip(a, b, n)]


def test_large_single_buffer(engine, oracle):
    rng = np.random.default_rng(13)
    buf = rng.integers(0, 256, (1 << 30) + 12345, dtype=np.uint8)
    for n in (buf.size, (1 << 30), 3 << 28):
        assert engine.crc32c(0x1234, buf[:n]) == oracle.crc32c(0x1234, buf, n)


def test_rccl_single_rank_allgather(engine, oracle):
    """The RCCL communicator (mi_comm_*) on one rank: the gathered CRC vector
    is the rank's own, and a second init is refused until destroy."""
    count = 4096
    data = engine.DeviceBuffer(count * 256)
    data.fill_splitmix64(0x1)
    out, recv = engine.DeviceBuffer(count * 4), engine.DeviceBuffer(count * 4)
    engine.device_batch_fixed(data, 256, 256, count, out)
    uid = engine.comm_unique_id()
    engine.comm_init(uid, 1, 0)
    try:
        with pytest.raises(engine.EngineError):
            engine.comm_init(uid, 1, 0)
        engine.comm_allgather_u32(out, count, recv)
        got = recv.download(np.uint32, count)
        assert np.array_equal(got, out.download(np.uint32, count))
        assert np.array_equal(got, oracle.fixed(data.download(np.uint8), 256, 256, count))
    finally:
        engine.comm_destroy()


def test_var_many_records_plan(engine, oracle):
    """6.5M short records (1,587 plan blocks): the scatter derives its bin
    bases from the per-block counts, no scan pass."""
    from tests import _plan_forms
    _plan_forms.many_records(engine, oracle)


def test_var_long_records_block_fold(engine, oracle):
    """Records with 65 - 770 interior pieces: interior items written by the
    scatter's wave loop, the interior run folded block-wide by the finalize."""
    from tests import _plan_forms
    _plan_forms.long_records(engine, oracle)


def test_var_plan_scan_pass_forced():
    """The same two batches with the separate scan pass that plans of more
    than 16M records take (MI_CRC32C_PLAN_SCAN=1, one child process)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, MI_CRC32C_PLAN_SCAN="1")
    r = subprocess.run([sys.executable, os.path.join(here, "_plan_forms.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "plan forms ok 1" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


@PATHS
def test_var_alignment_sweep(engine, oracle, planned):
    """Every start residue mod 128 and starts just before 4 KiB boundaries,
    with lengths at row (128 B), group (1 KiB) and chunk (4 KiB) edges, with
    and without inits: the masking, bin and window-shift cases of the plan."""
    rng = np.random.default_rng(22)
    starts = list(range(0, 128)) + [4096 - d for d in (1, 2, 3, 4, 15, 16, 17, 127, 128, 129,
                                                       1023, 1024, 1025)]
    lens = [1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 33, 63, 64, 127, 128, 129, 255, 256, 257, 511,
            512, 513, 1023, 1024, 1025, 2047, 2048, 2049, 3071, 3072, 3073, 4095, 4096, 4097,
            8191, 8192, 8193, 12289, 70000]
    if not planned:  # the direct kernel takes batches whose records are all <= 16 KiB
        lens = [n for n in lens if n <= 16384]
    offsets, lengths = [], []
    for i, s in enumerate(starts):
        for j, n in enumerate(lens):
            offsets.append(((i * len(lens) + j) * 3) * 4096 + 8192 + s)
            lengths.append(n)
    offsets = np.array(offsets, dtype=np.uint64)
    lengths = np.array(lengths, dtype=np.uint32)
    buf = rng.integers(0, 256, int((offsets + lengths).max()) + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, lengths.size, dtype=np.uint32)
    assert np.array_equal(engine.crc32c_batch(buf, offsets, lengths, planned=planned),
                          oracle.batch(buf, offsets, lengths))
    assert np.array_equal(engine.crc32c_batch(buf, offsets, lengths, inits, planned=planned),
                          oracle.batch(buf, offsets, lengths, inits))


def test_single_record_4GiB_golden(engine):
    """One 4 GiB record (and 4 GiB + 4097 B) against the reference's own
    chained crc32c over the same stream (tests/golden/digests.json)."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "digests.json")) as f:
        gold = json.load(f)["single_record_seed0xc0de"]["crc"]
    n = 1 << 32
    data = engine.DeviceBuffer(n + 4097)
    data.fill_splitmix64(0xC0DE)
    assert engine.crc32c_device(data, n) == gold[str(n)]
    assert engine.crc32c_device(data, n + 4097) == gold[str(n + 4097)]
    data.free()


def test_device_single_buffer_sweep(engine, oracle):
    """Device buffers of >= 64 KiB take launch_single (head up to the next
    4 KiB boundary, 4 KiB chunks through the fixed-record kernel, tail, and a
    two-level combine tree).  Starts at every head case (0-3 bytes before a
    boundary push the head past it so ~init lands in the head), tails of 0,
    1 and 4095 bytes, sizes around the 64 KiB threshold and multi-workgroup
    trees, with and without inits."""
    rng = np.random.default_rng(23)
    total = (9 << 20) + 3 * 4096
    data = engine.DeviceBuffer(total)
    data.fill_splitmix64(0x51C6E)
    host = data.download(np.uint8, total)
    base_mod = data.ptr % 4096
    cases = []
    for start in (0, 1, 2, 3, 4, 5, 16, 127, 2048, 4091, 4092, 4093, 4094, 4095):
        off = (start - base_mod) % 4096 + 4096
        h = (4096 - (data.ptr + off) % 4096) % 4096
        h = h + 4096 if h < 4 else h
        for n in (65535, 65536, 65537, h + 16 * 4096, h + 16 * 4096 + 1, h + 16 * 4096 + 4095,
                  (1 << 20) + 7, (4 << 20) + h, (8 << 20) + 12345):
            cases.append((off, n))
    for off, n in cases:
        for init in (0, int(rng.integers(0, 2**32))):
            assert off + n <= total
            got = engine.crc32c_device(data, n, init_crc=init, offset=off)
            assert got == oracle.crc32c(init, host, n, off), (off, n, init)
    data.free()


@pytest.mark.parametrize("shape", ["only_4_group", "only_short", "mixed_tiny"])
def test_var_chunk_roles(engine, oracle, shape, monkeypatch):
    """The chunk launch gives all 16 waves to one role when the other has no
    pieces: batches of 4 KiB-aligned 4 KiB records (only 4-group pieces),
    of records under 1 KiB (only 1- and 2-group pieces), and a tiny mixed
    batch whose grid is smaller than the chip.  (Piece path forced.)"""
    monkeypatch.setenv("MI_CRC32C_VARPATH", "pieces")
    rng = np.random.default_rng(31)
    if shape == "only_4_group":
        count = 3000
        lengths = np.full(count, 4096, dtype=np.uint32)
        offsets = (np.arange(count, dtype=np.uint64) * 4096 + 8192).astype(np.uint64)
    elif shape == "only_short":
        count = 50000
        lengths = rng.integers(32, 1000, count).astype(np.uint32)
        # every record inside one 4 KiB chunk (a single piece of <= 9 rows)
        offsets = (np.arange(count, dtype=np.uint64) * 4096 +
                   rng.integers(0, 4096 - 1000, count).astype(np.uint64))
    else:
        count = 37
        lengths = rng.integers(0, 20000, count).astype(np.uint32)
        offsets = np.zeros(count, dtype=np.uint64)
        offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    buf = rng.integers(0, 256, int((offsets + lengths).max()) + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32)
    assert np.array_equal(engine.crc32c_batch(buf, offsets, lengths, planned=True),
                          oracle.batch(buf, offsets, lengths))
    assert np.array_equal(engine.crc32c_batch(buf, offsets, lengths, inits, planned=True),
                          oracle.batch(buf, offsets, lengths, inits))


def test_concurrent_callers(engine, oracle):
    """consus::crc32c is called concurrently by the network threads
    (txman/durable_log.cc:215-218, txman/main.cc:191-193): 12 threads, each
    with its own engine stream and staging, mixing single buffers, batches
    and fixed batches, every result checked."""
    import threading
    rng = np.random.default_rng(41)
    buf = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    errors = []

    def worker(t):
        r = np.random.default_rng(100 + t)
        try:
            for _ in range(15):
                off = int(r.integers(0, 1 << 20))
                n = int(r.integers(0, 2 << 20))
                init = int(r.integers(0, 2**32))
                got = engine.crc32c(init, buf[off:off + n])
                if got != oracle.crc32c(init, buf, n, off):
                    errors.append(("buffer", t, off, n, init))
                lens = r.integers(0, 9000, 200).astype(np.uint32)
                offs = r.integers(0, (3 << 20) - 9000, 200).astype(np.uint64)
                if not np.array_equal(engine.crc32c_batch(buf, offs, lens),
                                      oracle.batch(buf, offs, lens, threads=1)):
                    errors.append(("batch", t))
                if not np.array_equal(engine.crc32c_fixed(buf, 4096, 4096, 256),
                                      oracle.fixed(buf, 4096, 4096, 256)):
                    errors.append(("fixed", t))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(("exception", t, repr(e)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:5]


def _gold(name):
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "digests.json")) as f:
        return json.load(f)[name]


def test_full_config3_16M_records_one_gpu(engine):
    """BASELINE configs[3]'s whole record set (16M x 4 KiB = 64 GiB) in one
    launch on one GPU: record offsets past 2^32 and 2^36 bytes, 16 golden
    block digests (crc32c of each 1M-record block's CRC vector)."""
    g = _gold("fixed_4096_seed0xc0de_per_1048576")
    n = 16 << 20
    data = engine.DeviceBuffer(n * 4096)
    out = engine.DeviceBuffer(n * 4)
    data.fill_splitmix64(0xC0DE)
    engine.device_batch_fixed(data, 4096, 4096, n, out)
    per = (1 << 20) * 4
    got = [engine.crc32c_device(out, per, offset=k * per) for k in range(16)]
    assert got == g["block_digests"]
    data.free()
    out.free()


def test_full_config2_zipf_golden(engine):
    """BASELINE configs[2] at full size (1M Zipf records, 4.9 GB) through
    the device batch, with and without the size hint, against the golden
    digest of the reference's CRC vector."""
    from consus_amd import workload as W
    g = _gold("zipf_seed0x5eed_data0xda7a5eed_1048576")
    R = 1 << 20
    off, ln, total = W.zipf_records(R)
    assert total == g["total_bytes"]
    data = engine.DeviceBuffer(total + 16)
    data.fill_splitmix64(W.DATA_SEED)
    d_off, d_len, out = engine.DeviceBuffer(R * 8), engine.DeviceBuffer(R * 4), engine.DeviceBuffer(R * 4)
    d_off.upload(off)
    d_len.upload(ln)
    for hint in (total, 0):
        out.memset(0)
        engine.device_batch(data, d_off, d_len, R, out, total_bytes=hint)
        assert engine.crc32c_device(out, R * 4) == g["digest"], hint
    for b in (data, d_off, d_len, out):
        b.free()


def test_split_record_fold_golden(engine):
    """One 4 GiB record split into 2..8 slices as if over 2..8 GPUs (here
    all on one): per-slice device CRCs folded with crc32c_combine equal the
    golden CRC of the whole record, with and without an init."""
    from consus_amd import shard
    gold = _gold("single_record_seed0xc0de")["crc"]
    n = 1 << 32
    data = engine.DeviceBuffer(n)
    data.fill_splitmix64(0xC0DE)
    for world in (2, 3, 8):
        sl = shard.record_slices(n, world)
        crcs = [engine.crc32c_device(data, L, offset=s) for s, L in sl]
        assert shard.fold_slice_crcs(crcs, [L for _, L in sl]) == gold[str(n)]
    init = 0x9E3779B9
    sl = shard.record_slices(n, 4, align=1 << 20)
    crcs = [engine.crc32c_device(data, L, offset=s) for s, L in sl]
    assert shard.fold_slice_crcs(crcs, [L for _, L in sl], init) == \
        engine.crc32c_device(data, n, init_crc=init)
    data.free()


def test_short_lived_threads_release_contexts(engine, oracle):
    """Each calling thread gets its own stream and workspaces, released when
    the thread exits: 48 threads in turn, each with host and device batches
    (workspaces grown to several MiB), then the calling thread again."""
    import threading
    rng = np.random.default_rng(77)
    lengths = rng.integers(0, 70000, 300).astype(np.uint32)
    offsets = np.zeros(lengths.size, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    buf = rng.integers(0, 256, int(lengths.sum()) + 64, dtype=np.uint8)
    want = oracle.batch(buf, offsets, lengths)
    errors = []

    def work():
        try:
            assert np.array_equal(engine.crc32c_batch(buf, offsets, lengths, planned=True), want)
            assert engine.crc32c(0, buf[:100000]) == oracle.crc32c(0, buf[:100000])
        except Exception as e:  # noqa: BLE001
            errors.append(e)
    for _ in range(48):
        t = threading.Thread(target=work)
        t.start()
        t.join()
    assert not errors, errors[0]
    work()
    assert not errors


def test_config1_golden(engine):
    """BASELINE configs[0] (1K x 256 B records, the reference's CPU case)
    through the GPU: one fixed-stride host batch and per-record drop-in
    calls, against the CRCs the compiled reference produced."""
    import base64
    g = _gold("cfg1_fixed_256_seed0x1_1024")
    want = np.frombuffer(base64.b64decode(g["crcs_b64_le_u32"]), dtype="<u4")
    data = engine.DeviceBuffer(1024 * 256)
    data.fill_splitmix64(1)
    host = data.download(np.uint8)
    assert np.array_equal(engine.crc32c_fixed(host, 256, 256, 1024), want)
    for i in range(0, 1024, 97):
        assert engine.crc32c(0, host[256 * i:256 * (i + 1)]) == int(want[i])
    data.free()


def test_config4_log_segments_golden(engine):
    """BASELINE configs[4]: real durable-log frames packed into 64 MiB
    segments, through the streaming pipeline (H2D + CRC + D2H), each
    segment's CRC vector digested against the reference's golden digest."""
    from consus_amd import workload as W
    gold = _gold("log_segments_64MiB")["segments"][:2]
    filler = engine.DeviceBuffer(W.SEGMENT_BYTES + 64)

    def fill(nbytes, byte_off):
        a = byte_off & ~7
        n = nbytes + (byte_off - a)
        filler.fill_splitmix64(W.DATA_SEED, byte_offset=a, nbytes=(n + 7) & ~7)
        return filler.download(np.uint8, n)[byte_off - a:]
    pipe = engine.Pipeline(W.SEGMENT_BYTES, 20000, depth=2)
    dev = engine.DeviceBuffer(20000 * 4)
    try:
        for (buf, fo, fl), g in zip(W.log_segments(len(gold), fill), gold):
            assert fo.size == g["frames"] and buf.size == g["bytes"]
            out = np.zeros(fo.size, dtype=np.uint32)
            pipe.wait(pipe.submit(buf, fo, fl, out))
            assert int(out[0]) == g["first_crc"]
            dev.upload(out)
            assert engine.crc32c_device(dev, out.size * 4) == g["digest"]
    finally:
        pipe.close()
        dev.free()
        filler.free()
