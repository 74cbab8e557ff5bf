#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Every expected CRC below is computed by consus::crc32c from
/root/reference/common/crc32c.cc compiled unmodified (oracle/_ref, built by
oracle/Makefile), and cross-checked against the C restatement
(oracle/crc32c_oracle.c).  The reference has no CRC tests or fixtures of its
own, so these vectors plus RFC 3720 B.4 and the CRC-32C
check value pin the oracle.  Inputs are recipes (splitmix64 streams, Zipf
lengths) so the fixtures stay small; tests regenerate the inputs.

Run in the build container (needs /root/reference):  python tests/golden/make_golden.py
"""
from __future__ import annotations

import base64
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle.oracle import Oracle, Reference  # noqa: E402

import consus_amd  # noqa: E402  (host-only workload generator; no GPU needed)

THREADS = os.cpu_count() or 8


def b64u32(a) -> str:
    return base64.b64encode(np.ascontiguousarray(a, dtype="<u4").tobytes()).decode()


def splitmix64(x: int) -> int:
    M = (1 << 64) - 1
    z = (x + 0x9E3779B97F4A7C15) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def iroot5(x: int) -> int:
    lo, hi = 0, 1 << 26
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if mid ** 5 <= x:
            lo = mid
        else:
            hi = mid - 1
    return lo


def zipf_lengths_py(seed: int, count: int, first: int = 0) -> np.ndarray:
    """Independent restatement of consus_amd/csrc/workload.cc (config 3)."""
    cdf, acc = [], 0
    for k in range(1, 1025):
        acc += (1 << 40) // iroot5((k ** 6) << 50)
        cdf.append(acc)
    cdf = np.array(cdf, dtype=np.uint64)
    out = np.zeros(count, dtype=np.uint32)
    for n in range(count):
        i = first + n
        x = splitmix64(seed ^ (2 * i)) % int(cdf[-1])
        j = splitmix64(seed ^ (2 * i + 1)) & 63
        k = int(np.searchsorted(cdf, x, side="right")) + 1
        out[n] = max(64, 64 * k - j)
    return out


def main() -> None:
    ref, orc = Reference(), Oracle()
    assert ref.lib.ref_dispatch_is_sse42() == 1, "expected the crc32q dispatch on this host"
    t0 = time.time()

    # ---- known answers ---------------------------------------------------------
    kats = [
        ("check_123456789", 0, b"123456789".hex(), 0xE3069283),   # CRC-32C check value
        ("rfc3720_zeros32", 0, (b"\x00" * 32).hex(), 0x8A9136AA),  # RFC 3720 B.4
        ("rfc3720_ones32", 0, (b"\xff" * 32).hex(), 0x62A8AB43),
        ("rfc3720_incr32", 0, bytes(range(32)).hex(), 0x46DD794E),
        ("rfc3720_decr32", 0, bytes(range(31, -1, -1)).hex(), 0x113FDB5C),
        ("empty_init0", 0, "", 0),
        ("empty_init_dead", 0xDEADBEEF, "", 0xDEADBEEF),
    ]
    out_kat = []
    for name, init, hexd, published in kats:
        d = bytes.fromhex(hexd)
        got = ref.crc32c(init, d)
        assert got == published, (name, hex(got))
        assert orc.crc32c(init, d) == got
        out_kat.append({"name": name, "init": init, "hex": hexd, "crc": got})
    # chaining: crc32c(crc32c(0, A), B) == crc32c(0, A||B) (common/crc32c.cc:122-126)
    a, b = b"12345", b"6789"
    chained = ref.crc32c(ref.crc32c(0, a), b)
    assert chained == 0xE3069283
    out_kat.append({"name": "chain_12345_6789", "init": ref.crc32c(0, a), "hex": b.hex(),
                    "crc": chained})

    # ---- alignment sweep ---------------------------------------------------------
    buf = orc.fill(512, 0xA11A, 0)
    inits = [0, 0x9E3779B9]
    sweep = np.zeros((len(inits), 16, 301), dtype=np.uint32)
    for ii, init in enumerate(inits):
        for off in range(16):
            for n in range(301):
                c = ref.crc32c(init, buf, n, off)
                assert c == orc.crc32c(init, buf, n, off, impl="sb8") == \
                    orc.crc32c(init, buf, n, off, impl="sse42")
                sweep[ii, off, n] = c
    align = {"buffer": {"stream_seed": 0xA11A, "bytes": 512}, "inits": inits, "offsets": 16,
             "lengths": 301, "shape": list(sweep.shape), "crcs_b64_le_u32": b64u32(sweep)}

    # ---- 4096 packed records with lengths 0..8191 --------------------------------
    n = 4096
    lens = np.array([splitmix64(0x4096 ^ i) % 8192 for i in range(n)], dtype=np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    rec_init = np.array([splitmix64(0x1A17 ^ i) & 0xFFFFFFFF for i in range(n)], dtype=np.uint32)
    data = orc.fill(int(lens.sum()), 0x4096, 0)
    c0 = ref.batch(data, offs, lens)
    ci = ref.batch(data, offs, lens, rec_init)
    assert np.array_equal(c0, orc.batch(data, offs, lens))
    assert np.array_equal(ci, orc.batch(data, offs, lens, rec_init))
    records = {"stream_seed": 0x4096, "count": n,
               "lengths": "splitmix64(0x4096 ^ i) % 8192, packed back to back from offset 0",
               "inits": "splitmix64(0x1A17 ^ i) & 0xFFFFFFFF",
               "crc_init0_b64_le_u32": b64u32(c0), "crc_inits_b64_le_u32": b64u32(ci)}

    # ---- config digests ------------------------------------------------------------
    digests = {}
    # cfg 1: 1K x 256 B, stream seed 1 (plumbing case, CPU)
    c1 = ref.splitmix_fixed(1, 256, 0, 1024, threads=THREADS)
    digests["cfg1_fixed_256_seed0x1_1024"] = {
        "crcs_b64_le_u32": b64u32(c1), "digest": orc.digest(c1)[0], "xor": orc.digest(c1)[1]}
    # cfg 2 / cfg 4: 16 blocks of 1M x 4 KiB, stream seed 0xC0DE
    block = 1 << 20
    blocks, xors, first16 = [], [], []
    allc = np.zeros(16 * block, dtype=np.uint32)
    for k in range(16):
        c = ref.splitmix_fixed(0xC0DE, 4096, k * block, block, threads=THREADS)
        allc[k * block:(k + 1) * block] = c
        d, x = orc.digest(c)
        blocks.append(d)
        xors.append(x)
        first16.append([int(v) for v in c[:16]])
    g16, gx = orc.digest(allc)
    digests["fixed_4096_seed0xc0de_per_1048576"] = {
        "definition": "record i = bytes [4096 i, 4096 (i+1)) of the splitmix64 stream 0xC0DE; "
                      "block k = records [k 2^20, (k+1) 2^20); digest = crc32c(0, LE bytes of "
                      "the block's CRC vector)",
        "block_digests": blocks, "block_xors": xors, "block_first16": first16,
        "global_16M_digest": g16, "global_16M_xor": gx,
        "global_8M_digest": orc.digest(allc[:8 * block])[0],
        "global_2M_blocks_digests": [orc.digest(allc[k * 2 * block:(k + 1) * 2 * block])[0]
                                     for k in range(8)],
    }
    # cfg 3: 1M Zipf records, packed, lengths seed 0x5EED, bytes from stream 0xDA7A5EED
    lz = consus_amd.zipf_lengths(0x5EED, block)
    assert np.array_equal(lz[:2000], zipf_lengths_py(0x5EED, 2000)), "zipf restatement"
    assert np.array_equal(lz[-500:], zipf_lengths_py(0x5EED, 500, first=block - 500))
    oz = np.zeros(block, dtype=np.uint64)
    oz[1:] = np.cumsum(lz[:-1], dtype=np.uint64)
    cz = ref.splitmix_var(0xDA7A5EED, oz, lz, threads=THREADS)
    dz, xz = orc.digest(cz)
    digests["zipf_seed0x5eed_data0xda7a5eed_1048576"] = {
        "definition": "lengths = mi_workload_zipf_lengths(0x5EED, 0, 2^20); records packed back "
                      "to back from offset 0 of the splitmix64 stream 0xDA7A5EED",
        "total_bytes": int(lz.sum(dtype=np.uint64)), "length_digest": orc.digest(lz)[0],
        "digest": dz, "xor": xz, "first16": [int(v) for v in cz[:16]],
    }
    # the same Zipf record stream continued to 8M records, as 8 blocks of 1M
    # (bench.py --config zipf at N > 1 shards it by bytes across the ranks)
    nz = 8 * block
    lz8 = consus_amd.zipf_lengths(0x5EED, nz)
    assert np.array_equal(lz8[:block], lz)
    oz8 = np.zeros(nz, dtype=np.uint64)
    oz8[1:] = np.cumsum(lz8[:-1], dtype=np.uint64)
    zblocks = []
    for k in range(8):
        ck = cz if k == 0 else ref.splitmix_var(0xDA7A5EED, oz8[k * block:(k + 1) * block],
                                                 lz8[k * block:(k + 1) * block], threads=THREADS)
        zblocks.append(orc.digest(ck)[0])
    assert zblocks[0] == dz
    digests["zipf_seed0x5eed_data0xda7a5eed_blocks"] = {
        "definition": "records [k 2^20, (k+1) 2^20) of the config-3 stream (lengths "
                      "mi_workload_zipf_lengths(0x5EED, 0, 8 x 2^20), packed back to back from offset "
                      "0 of the splitmix64 stream 0xDA7A5EED); digest = crc32c(0, LE CRC vector)",
        "block_digests": zblocks,
        "total_bytes_8M": int(lz8.sum(dtype=np.uint64)),
    }
    # cfg 5: 64 MiB durable-log segments (consus_amd/workload.py recipe)
    from consus_amd.workload import log_segments
    segs = []
    for buf, fo, fl in log_segments(4, lambda n, o: orc.fill(n, 0xDA7A5EED, o)):
        c = ref.batch(buf, fo, fl, threads=THREADS)
        segs.append({"frames": int(fo.size), "bytes": int(buf.size), "digest": orc.digest(c)[0],
                     "first_crc": int(c[0])})
    digests["log_segments_64MiB"] = {
        "definition": "consus_amd.workload.log_segments: frames [recno BE][len BE][entry][crc] "
                      "with config-3 entry lengths and stream 0xDA7A5EED entries, greedily packed "
                      "into 64 MiB segments; digest = crc32c(0, LE CRC vector) per segment",
        "segments": segs}
    # one huge record (bench.py --config single): the whole
    # first 4 GiB (and 4 GiB + 4097 B) of stream 0xC0DE as ONE crc32c; 8, 16
    # and 32 GiB for the record split across 2, 4 and 8 GPUs
    single = {}
    for nbytes in (1 << 32, (1 << 32) + 4097, 1 << 33, 1 << 34, 1 << 35):
        single[str(nbytes)] = ref.splitmix_stream(0xC0DE, 0, nbytes)
    digests["single_record_seed0xc0de"] = {
        "definition": "crc32c(0, bytes [0, n) of the splitmix64 stream 0xC0DE) as one record, "
                      "keyed by n", "crc": single,
        "check_1MiB": ref.splitmix_stream(0xC0DE, 0, 1 << 20)}
    assert digests["single_record_seed0xc0de"]["check_1MiB"] == \
        orc.crc32c(0, orc.fill(1 << 20, 0xC0DE, 0))
    # durable-log framing example (txman/durable_log.cc:54-61, 215-224)
    hdr = (1).to_bytes(8, "big") + (5).to_bytes(8, "big")
    crc = ref.crc32c(ref.crc32c(0, hdr), b"hello")
    assert crc == 0x189BA4C0
    digests["frame_example"] = {"recno": 1, "entry_hex": b"hello".hex(), "crc": crc,
                                "frame_hex": (hdr + b"hello" + crc.to_bytes(4, "big")).hex()}

    meta = {"generator": "tests/golden/make_golden.py",
            "reference": "/root/reference/common/crc32c.cc (consus::crc32c, sse42 crc32q dispatch)",
            "restatement": "oracle/crc32c_oracle.c (agrees on every vector)"}
    for name, obj in (("kat.json", {"meta": meta, "vectors": out_kat}),
                      ("align_sweep.json", {"meta": meta, **align}),
                      ("records_4096.json", {"meta": meta, **records}),
                      ("digests.json", {"meta": meta, **digests})):
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=1)
            f.write("\n")
    print(f"golden fixtures written in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
