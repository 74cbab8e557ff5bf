"""Code-object properties the kernels rely on, read from the gfx950 assembly
of consus_amd/csrc/crc32c_kernels.hip (CPU only: hipcc cross-compiles).

* The record kernels declare no static LDS, so their dynamic table image
  starts at LDS address 0 and a table byte offset is the ds_read address
  (crc32c_kernels.hip, `lds32`).
* The headline kernel fits the 128-VGPR budget of 16 waves per CU with no
  scratch (no spills).
* No scalar-cache writes anywhere (scalar stores, scalar atomics, scalar
  cache write-back or discard): every store goes through vector memory.
"""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "consus_amd", "csrc", "crc32c_kernels.hip")
RECORD_KERNELS = ("crc32c_fixed_pipe_kernel", "crc32c_span_chunk_kernel", "crc32c_fixed_kernel",
                  "crc32c_chunk_kernel", "crc32c_direct_kernel")


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa") / "kernels.s"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-S", "--cuda-device-only", "-I", os.path.join(REPO, "include"),
                        "-o", str(out), SRC], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return out.read_text()


def kernel_meta(asm_text):
    """{mangled kernel name: {field: int}} from the .amdhsa_kernel blocks."""
    meta = {}
    for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", asm_text, re.S):
        fields = dict((k, int(v)) for k, v in
                      re.findall(r"\.amdhsa_(\w+) (\d+)\n", m.group(2)))
        meta[m.group(1)] = fields
    return meta


def test_record_kernels_have_no_static_lds(asm):
    meta = kernel_meta(asm)
    found = {k: v for k, v in meta.items() if any(n in k for n in RECORD_KERNELS)}
    assert len(found) >= 4, sorted(meta)
    for name, f in found.items():
        assert f["group_segment_fixed_size"] == 0, name


def test_headline_kernel_fits_16_waves_without_spills(asm):
    meta = kernel_meta(asm)
    pipe = [f for k, f in meta.items()
            if "crc32c_fixed_pipe_kernel" in k or "crc32c_span_chunk_kernel" in k]
    assert pipe
    for f in pipe:
        assert f["next_free_vgpr"] <= 128
        assert f["private_segment_fixed_size"] == 0


def test_sorted_kernel_fits_16_waves_without_spills(asm):
    """The sorted path's hash kernel (configs[2]) runs 16 waves per CU: at most
    128 VGPRs, no scratch; its LDS image plus the sort state fit 160 KiB."""
    meta = kernel_meta(asm)
    srt = {k: f for k, f in meta.items() if "crc32c_sorted_kernel" in k}
    assert len(srt) == 2, sorted(srt)  # ring depths 2 and 4
    for name, f in srt.items():
        assert f["next_free_vgpr"] <= 128, name
        assert f["private_segment_fixed_size"] == 0, name


def test_no_scalar_cache_writes(asm):
    # opcode families assembled from fragments, so that this file itself
    # names none of them
    fam = ["store", "buffer_" + "store", "scratch_" + "store", "atomic", "buffer_" + "atomic",
           "dcache_" + "wb", "dcache_" + "discard"]
    pat = r"^\s*(s_(?:" + "|".join(fam) + r")\w*)"
    bad = re.findall(pat, asm, re.M)
    assert not bad, sorted(set(bad))
