"""CPU model checks of the sorted path's piece geometry and workspace bound
(consus_amd/csrc/crc32c_kernels.hip: sort_cost, the descriptor of piece k,
sorted_fpw).  No GPU: the kernel's integer formulas restated in Python and
checked by brute force over random batches.

* Pieces are cut from the record's end: the full pieces are exactly P bytes
  and end a multiple of P before the record's end (so a piece's shift is
  Z_{P j}); the head is the remainder at the start, 4 .. P + 3 bytes (the
  ~init word stays inside it); the pieces tile the record exactly.
* sorted_fpw(C) bounds the full pieces any workgroup's share holds: a share is
  the items whose cost starts in [T_b, T_b+1) with the XCD-weighted targets.
"""
import random

ROW = 128
FOLD = 2     # kSortFold
XCDW = 15    # kSortXcdw


def pieces(a, L, plog):
    """(start, end, is_head) of each piece in cost order, or [] for L < 4."""
    if L < 4:
        return []
    P = 1 << plog
    n = (L + P - 1) >> plog
    if n > 1 and L - ((n - 1) << plog) < 4:
        n -= 1
    E = a + L
    out = []
    for k in range(n):
        head = k + 1 == n
        pe = E - (((n - 1) if head else (n - 2 - k)) << plog)
        ps = a if head else pe - P
        out.append((ps, pe, head))
    return out


def rows(ps, pe):
    return ((pe + ROW - 1) >> 7) - (ps >> 7)


def fpw(C, plog, grid):
    share = C // (1000 * grid) * (1000 + XCDW) + (C % (1000 * grid)) * (1000 + XCDW) // (1000 * grid) + 2
    return share // ((1 << plog) // ROW + FOLD) + 3


def test_end_cut_pieces_tile_the_record():
    rnd = random.Random(1)
    for _ in range(30_000):
        plog = rnd.choice([9, 10, 11, 12, 14, 16])
        P = 1 << plog
        a = rnd.randrange(0, 1 << 20)
        L = rnd.choice([rnd.randrange(0, 4 * P), max(0, P * rnd.randrange(1, 5) + rnd.randrange(-4, 6))])
        ps = pieces(a, L, plog)
        if L < 4:
            assert ps == []
            continue
        span = sorted((p[0], p[1]) for p in ps)
        assert span[0][0] == a and span[-1][1] == a + L
        assert all(x[1] == y[0] for x, y in zip(span, span[1:]))
        head = [p for p in ps if p[2]]
        assert len(head) == 1 and ps[-1][2] and head[0][0] == a
        assert 4 <= head[0][1] - head[0][0] <= P + 3
        for p in ps[:-1]:
            assert p[1] - p[0] == P and (a + L - p[1]) % P == 0
        assert all(rows(p[0], p[1]) <= P // ROW + 2 for p in ps)


def test_full_piece_regions_hold_every_share():
    rnd = random.Random(5)
    for _ in range(120):
        plog = rnd.choice([9, 10, 12, 13, 14, 16])
        grid = rnd.choice([1, 2, 3, 5, 16, 64, 256])
        P = 1 << plog
        items, a = [], rnd.randrange(0, 1000)
        for _ in range(rnd.randint(1, 2500)):
            L = rnd.choice([rnd.randrange(0, 5000), rnd.randrange(0, 300_000),
                            P * rnd.randrange(1, 6) + rnd.randrange(-5, 5)])
            L = max(L, 0)
            for ps, pe, head in pieces(a, L, plog):
                items.append((not head, rows(ps, pe) + FOLD))
            a += L + rnd.randrange(0, 9)
        C = sum(c for _, c in items)
        if C == 0:
            continue

        def target(x):  # sort_find_blocks' targets
            if x >= grid:
                return C
            if grid % 2 == 0:
                return int(C * (x * 1000.0 + XCDW * (x & 1)) / (grid * 1000.0))
            return C // grid * x + (C % grid) * x // grid
        starts, s = [], 0
        for full, c in items:
            starts.append((s, full))
            s += c
        bound = fpw(C, plog, grid)
        for b in range(grid):
            t0, t1 = target(b), target(b + 1)
            assert sum(1 for st, full in starts if full and t0 <= st < t1) <= bound


# --- lane items: one record per lane, slice-by-16 over its aligned 16-B blocks

POLY = 0x82F63B78


def _tables():
    t0 = []
    for b in range(256):
        c = b
        for _ in range(8):
            c = (c >> 1) ^ (POLY if c & 1 else 0)
        t0.append(c)
    T = [t0]
    for _ in range(15):
        T.append([(v >> 8) ^ t0[v & 0xFF] for v in T[-1]])
    return T


def _bitwise_crc(init, data):
    c = init ^ 0xFFFFFFFF
    for byte in data:
        c ^= byte
        for _ in range(8):
            c = (c >> 1) ^ (POLY if c & 1 else 0)
    return c ^ 0xFFFFFFFF


def lane_item(T, buf, a, L, init):
    """The lane loop of crc32c_sorted_kernel, restated: blocks [a & ~15, ...),
    bytes before a zeroed, ~init over bytes a..a+3, the last block's t-byte
    step (lane_tail_step)."""
    e = a + L
    q = a & 15
    K = ((e + 15) >> 4) - (a >> 4)
    t = ((e - 1) & 15) + 1
    c0 = a & ~15
    ninit = init ^ 0xFFFFFFFF

    def block(j):
        x = bytearray(buf[c0 + 16 * j: c0 + 16 * j + 16])
        x += bytes(16 - len(x))
        for p in range(16):  # head: zero before a, ~init over the first 4 bytes
            pos = c0 + 16 * j + p
            if pos < a:
                x[p] = 0
            elif pos < a + 4:
                x[p] ^= (ninit >> (8 * (pos - a))) & 0xFF
        return x

    st = 0
    for j in range(K - 1):
        x = block(j)
        w0 = int.from_bytes(x[:4], "little") ^ st
        x[:4] = w0.to_bytes(4, "little")
        st = 0
        for p in range(16):
            st ^= T[15 - p][x[p]]
    x = block(K - 1)
    for p in range(t, 16):
        x[p] = 0
    w0 = int.from_bytes(x[:4], "little") ^ st
    x[:4] = w0.to_bytes(4, "little")
    r = (w0 >> (8 * t)) if t < 4 else 0
    for p in range(t):
        r ^= T[t - 1 - p][x[p]]
    return r ^ 0xFFFFFFFF


def test_lane_item_step_matches_crc32c():
    T = _tables()
    rnd = random.Random(11)
    buf = bytes(rnd.randrange(256) for _ in range(2048))
    for _ in range(3000):
        L = rnd.choice([rnd.randrange(4, 40), rnd.randrange(4, 400)])
        a = rnd.randrange(0, len(buf) - L)
        init = rnd.choice([0, 0xFFFFFFFF, rnd.randrange(1 << 32)])
        assert lane_item(T, buf, a, L, init) == _bitwise_crc(init, buf[a:a + L]), (a, L, init)


def test_lane_and_team_bins_are_disjoint_and_ordered():
    """sort_key: team items by rows (kSortRows - rows), lane items after them
    by 16-B blocks (kSortRows + 7 lrows - K), inside kSortBins = kSortRows +
    7 * 3 bins; K <= 8 * rows, so a lane key never meets a team key."""
    k_rows, lmax = 65536 // ROW + 2, 3
    bins = k_rows + 7 * lmax
    rnd = random.Random(3)
    for _ in range(20_000):
        lrows = rnd.randrange(0, lmax + 1)
        a = rnd.randrange(0, 1 << 20)
        L = rnd.randrange(4, 1200)
        e = a + L
        rows = ((e + ROW - 1) >> 7) - (a >> 7)
        K = ((e + 15) >> 4) - (a >> 4)
        assert K <= 8 * rows
        if rows <= lrows:
            key = k_rows + 7 * lrows - K
            assert k_rows - lrows <= key < bins
        else:
            key = k_rows - rows
            assert 0 <= key < k_rows - lrows
