"""The oracle (oracle/crc32c_oracle.c) pinned against the reference's answers.

The reference has no CRC tests; the pins are the CRC-32C
check value, RFC 3720 B.4, the golden fixtures generated from the reference
compiled unmodified (tests/golden/make_golden.py), and -- when oracle/_ref
is built -- the reference itself on random inputs.
"""
import base64
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def u32(b64):
    return np.frombuffer(base64.b64decode(b64), dtype="<u4")


def splitmix64(x):
    M = (1 << 64) - 1
    z = (x + 0x9E3779B97F4A7C15) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


@pytest.mark.parametrize("impl", ["api", "bitwise", "sb8", "sse42"])
def test_known_answers(oracle, impl):
    for v in load("kat.json")["vectors"]:
        assert oracle.crc32c(v["init"], bytes.fromhex(v["hex"]), impl=impl) == v["crc"], v["name"]


def test_align_sweep_golden(oracle):
    g = load("align_sweep.json")
    crcs = u32(g["crcs_b64_le_u32"]).reshape(g["shape"])
    buf = oracle.fill(g["buffer"]["bytes"], g["buffer"]["stream_seed"], 0)
    for ii, init in enumerate(g["inits"]):
        for off in range(g["offsets"]):
            for n in range(0, g["lengths"], 7):
                assert oracle.crc32c(init, buf, n, off) == crcs[ii, off, n]
                assert oracle.crc32c(init, buf, n, off, impl="sb8") == crcs[ii, off, n]


def test_records_4096_golden(oracle):
    g = load("records_4096.json")
    n = g["count"]
    lens = np.array([splitmix64(0x4096 ^ i) % 8192 for i in range(n)], dtype=np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    inits = np.array([splitmix64(0x1A17 ^ i) & 0xFFFFFFFF for i in range(n)], dtype=np.uint32)
    data = oracle.fill(int(lens.sum()), g["stream_seed"], 0)
    assert np.array_equal(oracle.batch(data, offs, lens), u32(g["crc_init0_b64_le_u32"]))
    assert np.array_equal(oracle.batch(data, offs, lens, inits), u32(g["crc_inits_b64_le_u32"]))


def test_cfg1_golden(oracle):
    g = load("digests.json")["cfg1_fixed_256_seed0x1_1024"]
    data = oracle.fill(1024 * 256, 1, 0)
    c = oracle.fixed(data, 256, 256, 1024)
    assert np.array_equal(c, u32(g["crcs_b64_le_u32"]))
    assert oracle.digest(c) == (g["digest"], g["xor"])


def test_cfg2_block_prefix_golden(oracle):
    g = load("digests.json")["fixed_4096_seed0xc0de_per_1048576"]
    for k in (0, 5, 15):
        data = oracle.fill(16 * 4096, 0xC0DE, k * (1 << 20) * 4096)
        assert list(oracle.fixed(data, 4096, 4096, 16)) == g["block_first16"][k]


def test_frame_example(oracle):
    g = load("digests.json")["frame_example"]
    frame = bytes.fromhex(g["frame_hex"])
    n = len(bytes.fromhex(g["entry_hex"]))
    # the stored CRC is big-endian right after the entry (txman/durable_log.cc:220-224)
    assert int.from_bytes(frame[16 + n:20 + n], "big") == g["crc"]
    assert oracle.crc32c(oracle.crc32c(0, frame[:16]), frame[16:16 + n]) == g["crc"]
    assert oracle.crc32c(0, frame[:16 + n]) == g["crc"]


def test_combine_identity(oracle):
    rng = np.random.default_rng(11)
    buf = rng.integers(0, 256, 200_000, dtype=np.uint8)
    for _ in range(200):
        n = int(rng.integers(0, 150_000))
        s = int(rng.integers(0, n + 1))
        a, b = oracle.crc32c(0, buf[:s]), oracle.crc32c(0, buf[s:n])
        assert oracle.combine(a, b, n - s) == oracle.crc32c(0, buf[:n])


def test_sb8_length_truncation_quirk(oracle):
    # common/crc32c.cc:598 takes the size_t length as uint32_t: n >= 4 GiB wraps.
    n = (1 << 32) + 16
    z = np.zeros(n, dtype=np.uint8)
    assert oracle.crc32c(0, z, n, impl="sb8") == oracle.crc32c(0, z, 16, impl="sb8")
    assert oracle.crc32c(0, z, n, impl="sse42") != oracle.crc32c(0, z, 16, impl="sse42")


def test_tables_match_reference(oracle, reference):
    assert np.array_equal(oracle.tables()[:8], reference.tables())


def test_random_vs_reference(oracle, reference):
    rng = np.random.default_rng(99)
    buf = rng.integers(0, 256, 100_000, dtype=np.uint8)
    for _ in range(2000):
        off = int(rng.integers(0, 64))
        n = int(rng.integers(0, 70_000))
        init = int(rng.integers(0, 2**32))
        exp = reference.crc32c(init, buf, n, off)
        assert oracle.crc32c(init, buf, n, off) == exp
        assert oracle.crc32c(init, buf, n, off, impl="sb8") == exp
        assert reference.crc32c(init, buf, n, off, impl="sw") == exp


def test_zipf_block_goldens_extend_the_1M_golden():
    """The 8 x 1M-record Zipf block digests (bench.py --config zipf at N > 1)
    start with the configs[2] golden itself."""
    d = load("digests.json")
    blocks = d["zipf_seed0x5eed_data0xda7a5eed_blocks"]["block_digests"]
    assert len(blocks) == 8
    assert blocks[0] == d["zipf_seed0x5eed_data0xda7a5eed_1048576"]["digest"]
