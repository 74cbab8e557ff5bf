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


def test_clean_tree_build_from_source(tmp_path):
    """build() runs `make`, which may reuse an up-to-date in-tree library.  This
    proves the sources compile: the engine library rebuilt from scratch
    (`make -B`) into a temporary directory, its gfx950 code object unbundled
    from the library's fat binary and its kernel metadata checked, and every
    symbol the headers declare exported by the fresh library."""
    import ctypes

    from test_abi import declared_functions

    obj, lib = tmp_path / "obj", tmp_path / "lib" / "libconsus_crc32c.so"
    r = subprocess.run(["make", "-s", "-B", "-j8", "-C", os.path.join(REPO, "consus_amd", "csrc"),
                        f"BUILD={obj}", f"OUT={lib}", str(lib)],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    assert lib.exists() and sorted(p.name for p in obj.iterdir()) == sorted(
        ["api.o", "crc32c_kernels.o", "durable_log.o", "engine.o", "host_crc.o", "workload.o"])
    llvm = "/opt/rocm/lib/llvm/bin/"
    fat, co = tmp_path / "fat.bin", tmp_path / "co.elf"
    subprocess.run([llvm + "llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", str(lib), os.devnull],
                   check=True, timeout=120)
    bundles = subprocess.run([llvm + "clang-offload-bundler", "--list", "--type=o", f"--input={fat}"],
                             capture_output=True, text=True, check=True, timeout=120).stdout.split()
    assert "hipv4-amdgcn-amd-amdhsa--gfx950" in bundles, bundles
    assert not [b for b in bundles if "amdgcn" in b and not b.endswith("gfx950")], bundles
    subprocess.run([llvm + "clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                   check=True, timeout=120)
    notes = subprocess.run([llvm + "llvm-readelf", "--notes", str(co)], capture_output=True,
                           text=True, check=True, timeout=120).stdout
    assert "amdgcn-amd-amdhsa--gfx950" in notes
    # one metadata map per kernel: name, VGPRs, scratch, static LDS
    kern = {}
    for blk in re.split(r"\n\s+- \.", notes):
        name = re.search(r"\.name:\s+(\S+)", blk)
        if name and "_ZN6mi_crc" in name.group(1):
            kern[name.group(1)] = {k: int(v) for k, v in re.findall(
                r"\.(vgpr_count|private_segment_fixed_size|group_segment_fixed_size):\s+(\d+)", blk)}
    for must in ("crc32c_fixed_pipe_kernel", "crc32c_sorted_kernel", "crc32c_direct_kernel",
                 "sorted_cost_kernel", "crc32c_combine_kernel"):
        assert any(must in k for k in kern), (must, sorted(kern))
    for k, f in kern.items():
        if any(n in k for n in ("crc32c_fixed_pipe_kernel", "crc32c_sorted_kernel")):
            assert f["vgpr_count"] <= 128 and f["private_segment_fixed_size"] == 0, (k, f)
            assert f["group_segment_fixed_size"] == 0, (k, f)  # dynamic LDS image only
    fresh = ctypes.CDLL(str(lib))
    missing = [n for n in declared_functions() if not hasattr(fresh, n)]
    assert not missing, missing
