"""Synthetic-input definitions agree across implementations."""
import numpy as np

import consus_amd as E
from tests.golden.make_golden import zipf_lengths_py
import json, os


def test_zipf_lengths_restatement():
    got = E.zipf_lengths(0x5EED, 3000, first=123456)
    assert np.array_equal(got, zipf_lengths_py(0x5EED, 3000, first=123456))


def test_zipf_lengths_golden_summary(oracle):
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "digests.json")))
    z = g["zipf_seed0x5eed_data0xda7a5eed_1048576"]
    lz = E.zipf_lengths(0x5EED, 1 << 20)
    assert int(lz.sum(dtype=np.uint64)) == z["total_bytes"]
    assert oracle.digest(lz)[0] == z["length_digest"]
    assert lz.min() == 64 and lz.max() <= 65536


def test_stream_fill_matches_definition(oracle):
    def sm(x):
        M = (1 << 64) - 1
        z = (x + 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)
    words = np.array([sm(0xC0DE ^ j) for j in range(64, 96)], dtype="<u8")
    assert np.array_equal(oracle.fill(256, 0xC0DE, 512), words.view(np.uint8))
    # unaligned start
    assert np.array_equal(oracle.fill(100, 0xC0DE, 515), words.view(np.uint8)[3:103])
