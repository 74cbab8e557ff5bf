"""The stream path for batches of records in address order:
the batch hashed as aligned 4 KiB chunks of one stream, chain snapshots at
record-boundary rows, boundary prefixes, per-record chaining.  Bit-exact
against the oracle on the same seeded inputs:

  * packed device batches (MI_CRC32C_PACKED) of Zipf lengths, at unaligned
    and aligned stream starts, with and without inits;
  * records of every awkward length (0, 1, 3, 4, 31, 32, 127-129, 4095-4097,
    chunk- and row-aligned boundaries, > 64 interior chunks for the long
    kernel) in one packed batch;
  * host batches in address order with gaps between records (durable-log
    frames with their 4-byte CRC slots), whose order the engine checks;
  * a host batch out of order with the flag: the piece path, exact;
  * a PACKED promise that does not hold: still exact (byte-serial);
  * configs[2] itself against the reference's golden digest.
Each test checks that the stream path actually ran (stream_batches)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "digests.json")


def packed(lengths, start=0):
    off = np.zeros(len(lengths), dtype=np.uint64)
    off[1:] = np.cumsum(np.asarray(lengths[:-1], dtype=np.uint64), dtype=np.uint64)
    return off + np.uint64(start), np.asarray(lengths, dtype=np.uint32)


def run_device(engine, buf, off, ln, inits=None, packed_flag=True):
    E = engine
    n = off.size
    data = E.DeviceBuffer(buf.size)
    data.upload(buf)
    d_off, d_len, d_out = E.DeviceBuffer(n * 8), E.DeviceBuffer(n * 4), E.DeviceBuffer(n * 4)
    d_off.upload(off)
    d_len.upload(ln)
    d_ini = None
    if inits is not None:
        d_ini = E.DeviceBuffer(n * 4)
        d_ini.upload(inits)
    E.device_batch(data, d_off, d_len, n, d_out, inits=d_ini,
                   total_bytes=int(ln.sum(dtype=np.uint64)), packed=packed_flag)
    got = d_out.download(np.uint32, n)
    for b in (data, d_off, d_len, d_out) + ((d_ini,) if d_ini else ()):
        b.free()
    return got


def stream_ran(engine, before):
    return engine.stats()["stream_batches"] > before


@pytest.mark.parametrize("start", [0, 5, 4093, 4096 + 128, 127])
def test_packed_zipf_device(engine, oracle, start):
    ln = engine.zipf_lengths(0x5EED, 12000, first=start * 7)
    off, ln = packed(ln, start)
    rng = np.random.default_rng(start)
    buf = rng.integers(0, 256, int(off[-1]) + int(ln[-1]) + 4096, dtype=np.uint8)
    before = engine.stats()["stream_batches"]
    got = run_device(engine, buf, off, ln)
    assert stream_ran(engine, before)
    assert np.array_equal(got, oracle.batch(buf, off, ln))


def test_packed_with_inits(engine, oracle):
    ln = engine.zipf_lengths(0x5EED, 9000, first=77)
    off, ln = packed(ln, 333)
    rng = np.random.default_rng(9)
    buf = rng.integers(0, 256, int(off[-1]) + int(ln[-1]) + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, off.size, dtype=np.uint32)
    before = engine.stats()["stream_batches"]
    got = run_device(engine, buf, off, ln, inits=inits)
    assert stream_ran(engine, before)
    assert np.array_equal(got, oracle.batch(buf, off, ln, inits))


def awkward_lengths(rng):
    base = [0, 1, 3, 4, 31, 32, 127, 128, 129, 4095, 4096, 4097, 8192, 0, 0, 60, 68, 1 << 20,
            64 * 4096 + 4096 * 3 + 17, 100 * 4096, 5, 4096 - 5, 2, 126]
    out = []
    for _ in range(40):
        out += list(rng.permutation(base))
        out += list(rng.integers(0, 9000, 30))
    return np.array(out, dtype=np.uint32)


@pytest.mark.parametrize("start", [0, 1, 4090, 64])
def test_awkward_lengths(engine, oracle, start):
    rng = np.random.default_rng(100 + start)
    off, ln = packed(awkward_lengths(rng), start)
    total = int(ln.sum(dtype=np.uint64))
    assert total >= 32 << 20
    buf = rng.integers(0, 256, start + total + 8192, dtype=np.uint8)
    inits = rng.integers(0, 2**32, off.size, dtype=np.uint32)
    inits[::3] = 0
    before = engine.stats()["stream_batches"]
    got = run_device(engine, buf, off, ln, inits=inits)
    assert stream_ran(engine, before)
    want = oracle.batch(buf, off, ln, inits)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:10], ln[bad[:10]], off[bad[:10]])


def test_host_frames_with_gaps(engine, oracle):
    """Durable-log frames: header + entry covered, a 4-byte CRC slot after
    each; the engine checks the address order itself and takes the stream
    path."""
    rng = np.random.default_rng(4)
    entry = rng.integers(0, 3000, 30000).astype(np.uint64)
    cover = entry + np.uint64(16)
    off = np.zeros(cover.size, dtype=np.uint64)
    off[1:] = np.cumsum(cover[:-1] + np.uint64(4), dtype=np.uint64)
    ln = cover.astype(np.uint32)
    buf = rng.integers(0, 256, int(off[-1]) + int(ln[-1]) + 4, dtype=np.uint8)
    before = engine.stats()["stream_batches"]
    got = engine.crc32c_batch(buf, off, ln, packed=True)
    assert stream_ran(engine, before)
    assert np.array_equal(got, oracle.batch(buf, off, ln))


def test_host_out_of_order_takes_pieces(engine, oracle):
    rng = np.random.default_rng(12)
    off, ln = packed(rng.integers(0, 9000, 9000).astype(np.uint32), 11)
    perm = rng.permutation(off.size)
    off, ln = off[perm], ln[perm]
    buf = rng.integers(0, 256, int(ln.sum(dtype=np.uint64)) + 4096, dtype=np.uint8)
    before = engine.stats()["stream_batches"]
    got = engine.crc32c_batch(buf, off, ln, packed=True)
    assert engine.stats()["stream_batches"] == before
    assert np.array_equal(got, oracle.batch(buf, off, ln))


def test_broken_packing_promise_is_still_exact(engine, oracle):
    """MI_CRC32C_PACKED on records that are not in address order: the device
    check catches it and every record is hashed byte-serially."""
    rng = np.random.default_rng(5)
    off, ln = packed(rng.integers(1, 8000, 12000).astype(np.uint32), 3)
    perm = rng.permutation(off.size)
    off, ln = off[perm], ln[perm]  # the same ranges, out of address order
    buf = rng.integers(0, 256, int(ln.sum(dtype=np.uint64)) + 4096, dtype=np.uint8)
    before = engine.stats()["stream_batches"]
    got = run_device(engine, buf, off, ln)
    assert stream_ran(engine, before)
    assert np.array_equal(got, oracle.batch(buf, off, ln))


def test_config3_golden_digest_stream(engine):
    from consus_amd import workload as W
    g = json.load(open(GOLD))["zipf_seed0x5eed_data0xda7a5eed_1048576"]
    R = 1 << 20
    off, ln, total = W.zipf_records(R)
    assert total == g["total_bytes"]
    data = engine.DeviceBuffer(total + 16)
    data.fill_splitmix64(W.DATA_SEED)
    d_off, d_len, out = engine.DeviceBuffer(R * 8), engine.DeviceBuffer(R * 4), \
        engine.DeviceBuffer(R * 4)
    d_off.upload(off)
    d_len.upload(ln)
    before = engine.stats()["stream_batches"]
    engine.device_batch(data, d_off, d_len, R, out, total_bytes=total, packed=True)
    assert stream_ran(engine, before)
    assert engine.crc32c_device(out, R * 4) == g["digest"]
    for b in (data, d_off, d_len, out):
        b.free()
