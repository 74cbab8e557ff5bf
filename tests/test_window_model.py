"""The window path's decomposition, restated on the CPU (host logic; the HIP
kernel is tested against the oracle in tests/test_gpu_window.py).

crc32c_kernels.hip, "window path": a record [a, E) covers the 128-B rows
[Rs, Re); window k (k = 0 at the record's end) is rows
[Re - 16 (k + 1), Re - 16 k) (or 8-row windows, the same with 8).  A team's fold value W_k is the raw CRC (from a
zero register) of the window's bytes with everything outside the record
zeroed and ~init XORed over the record's first four bytes (records of >= 4
bytes; shorter ones take the seed Z_L(~init)), evaluated at the window's last
row end.  Claim: XOR_k Z_{2048 k}(W_k) = Z_m(raw), m = 128 Re - E, where raw is
the register the reference reaches over the record (crc = ~raw).  This test
checks the claim with the oracle's CRC and shift on random records at every
alignment, including windows whose first row holds only the init word's
spill.
"""
import numpy as np
import pytest

ROW = 128


def _raw0(oracle, data):
    """Register after `data` from a zero register (crc32c(~0) = ~proc(0))."""
    return (~oracle.crc32c(0xFFFFFFFF, data)) & 0xFFFFFFFF


def _windows(oracle, buf, base, off, L, init, WIN):
    a = base + off
    E = a + L
    Rs, Re = a // ROW, (E + ROW - 1) // ROW
    K = (Re - Rs + WIN - 1) // WIN
    acc = 0
    for k in range(K):
        lo, hi = (Re - WIN * (k + 1)) * ROW, (Re - WIN * k) * ROW
        w = np.zeros(hi - lo, dtype=np.uint8)
        s, e = max(lo, a), min(hi, E)
        if e > s:
            w[s - lo:e - lo] = buf[s - base:e - base]
        if L >= 4:
            ninit = (~init) & 0xFFFFFFFF
            for j in range(4):
                p = a + j
                if lo <= p < hi:
                    w[p - lo] ^= (ninit >> (8 * j)) & 0xFF
        acc ^= oracle.shift(_raw0(oracle, w), WIN * ROW * k)
    return acc, Re * ROW - E, K


@pytest.mark.parametrize("seed,win", [(1, 16), (2, 16), (3, 8), (4, 4)])
def test_window_decomposition_matches_the_oracle(oracle, seed, win):
    rng = np.random.default_rng(seed)
    base = 0x10000
    size = 1 << 18
    buf = rng.integers(0, 256, size, dtype=np.uint8)
    lens = list(rng.integers(0, 9000, 60)) + [0, 1, 2, 3, 4, 5, 127, 128, 129, 2047, 2048,
                                              2049, 4096, 20000, 40000]
    seen_k = 0
    for L in lens:
        L = int(L)
        for off in (int(rng.integers(0, size - L - 1)), 125, 126, 127, 128 * 40 - 1):
            if off + L > size:
                continue
            init = int(rng.integers(0, 2**32))
            crc = oracle.crc32c(init, buf[off:off + L])
            acc, m, K = _windows(oracle, buf, base, off, L, init, win)
            seen_k = max(seen_k, K)
            if L == 0:  # the kernel gives it one task, which stores init
                continue
            if L >= 4:
                raw = (~crc) & 0xFFFFFFFF
            else:
                seed_ = oracle.shift((~init) & 0xFFFFFFFF, L)
                raw = ((~crc) & 0xFFFFFFFF) ^ seed_
            assert oracle.shift(raw, m) == acc, (L, off, init)
    assert seen_k >= 20
