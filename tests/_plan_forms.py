"""Variable-length plans in both forms (run by tests/test_gpu_parity.py, also
as a subprocess with MI_CRC32C_PLAN_SCAN=1): the scatter deriving its bin
bases from the per-block counts, or the separate scan pass that plans of more
than 16M records take.  Long records (> 64 interior pieces) are folded by the
finalize's block-wide pass.  The piece path is forced (MI_CRC32C_VARPATH=
pieces): with the total known the engine takes the sorted path by default.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def _pieces(fn):
    """Run fn with the piece path forced, restoring the environment after."""
    def wrapped(*a, **k):
        old = os.environ.get("MI_CRC32C_VARPATH")
        os.environ["MI_CRC32C_VARPATH"] = "pieces"
        try:
            return fn(*a, **k)
        finally:
            if old is None:
                os.environ.pop("MI_CRC32C_VARPATH", None)
            else:
                os.environ["MI_CRC32C_VARPATH"] = old
    return wrapped


@_pieces
def many_records(engine, oracle):
    """6.5M short records, a few multi-chunk ones: 1,587 plan blocks (the
    scan pass, when forced, runs over several LDS tiles)."""
    rng = np.random.default_rng(21)
    count = 6_500_000
    lengths = rng.integers(0, 97, count, dtype=np.uint32)
    lengths[rng.integers(0, count, 64)] = 70_000
    offsets = np.zeros(count, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    total = int(lengths.sum(dtype=np.uint64))
    data = engine.DeviceBuffer(total + 16)
    data.fill_splitmix64(0x5CA1E)
    d_off, d_len, d_out = (engine.DeviceBuffer(count * 8), engine.DeviceBuffer(count * 4),
                           engine.DeviceBuffer(count * 4))
    d_off.upload(offsets)
    d_len.upload(lengths)
    engine.device_batch(data, d_off, d_len, count, d_out, total_bytes=total)
    got = d_out.download(np.uint32, count)
    host = data.download(np.uint8, total)
    for b in (data, d_off, d_len, d_out):
        b.free()
    assert np.array_equal(got, oracle.batch(host, offsets, lengths)), "many records"


@_pieces
def long_records(engine, oracle):
    """2,000 records, 70 of them 264 KiB - 3 MiB (65 - 770 interior pieces),
    at unaligned starts, with and without inits."""
    rng = np.random.default_rng(24)
    count = 2000
    lengths = rng.integers(0, 9000, count).astype(np.uint32)
    big = rng.choice(count, 70, replace=False)
    lengths[big] = rng.integers(66 * 4096, 3 << 20, big.size)
    offsets = np.zeros(count, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1].astype(np.uint64) + rng.integers(0, 5, count - 1).astype(np.uint64))
    offsets += np.uint64(1237)
    buf = rng.integers(0, 256, int(offsets[-1]) + int(lengths[-1]) + 64, dtype=np.uint8)
    inits = rng.integers(0, 2**32, count, dtype=np.uint32)
    assert np.array_equal(engine.crc32c_batch(buf, offsets, lengths, planned=True),
                          oracle.batch(buf, offsets, lengths)), "long records"
    assert np.array_equal(engine.crc32c_batch(buf, offsets, lengths, inits, planned=True),
                          oracle.batch(buf, offsets, lengths, inits)), "long records, inits"


if __name__ == "__main__":
    import consus_amd as E
    from oracle.oracle import Oracle
    E.init(0)
    orc = Oracle()
    many_records(E, orc)
    long_records(E, orc)
    st = E.stats()
    assert st["fallback_calls"] == 0, st
    print("plan forms ok", os.environ.get("MI_CRC32C_PLAN_SCAN", "0"))
