"""C ABI: the library loads, exports every symbol include/lcrc.h declares, the scalar host API (the
crc32fast::Hasher drop-in) agrees with the oracle, and batched calls fail loudly without a device."""
import os
import re
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    with open(os.path.join(ROOT, "include", "lcrc.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(lcrc\w*)\s*\(", src))
    return sorted(names)


def test_exports_every_declared_symbol(lcrc):
    L = lcrc.lib()
    declared = _header_functions()
    assert len(declared) >= 30
    for name in declared:
        assert hasattr(L, name), f"{name} declared in include/lcrc.h but not exported"
    assert sorted(lcrc.ABI_SYMBOLS) == declared


def test_kernel_image_is_gfx950(lcrc):
    with open(lcrc.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # offload bundle entry of the code object


def test_struct_layouts(lcrc):
    assert lcrc.DESC_DTYPE.itemsize == 16
    assert lcrc.WAL_REC_DTYPE.itemsize == 24
    import ctypes
    assert ctypes.sizeof(lcrc._GJob) == 48 and lcrc._GJob.out_mismatch.offset == 40  # lcrc_gjob
    assert ctypes.sizeof(lcrc._UJob) == 40  # lcrc_ujob
    assert ctypes.sizeof(lcrc._WJob) == 40 and lcrc._WJob.n_recs.offset == 32  # lcrc_wjob


def test_ctx_options_mirror(lcrc):
    """The ctypes mirror of lcrc_ctx_options has the header's fields in the header's order (every field a 32-bit
    integer), so Engine(**options) sets what lcrc_ctx_create_ex reads."""
    with open(os.path.join(ROOT, "include", "lcrc.h")) as f:
        src = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    body = re.search(r"typedef struct lcrc_ctx_options \{(.*?)\} lcrc_ctx_options;", src, flags=re.S).group(1)
    fields = re.findall(r"(u?int32_t)\s+(\w+)(?:\[(\d+)\])?;", body)
    assert [n for _, n, _c in fields] == [n for n, _ in lcrc._CtxOptions._fields_]
    import ctypes
    assert ctypes.sizeof(lcrc._CtxOptions) == 4 * sum(int(c or 1) for _, _n, c in fields)


@pytest.mark.parametrize("n", [0, 1, 3, 7, 8, 9, 16, 100, 4096, 100003])
def test_scalar_value(lcrc, orc, n):
    d = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    assert lcrc.value(d) == zlib.crc32(d) == orc.crc(d, 0)
    assert lcrc.crc32c_value(d) == orc.crc_bitwise(d, 1)
    assert lcrc.lib().lcrc32_value(d, len(d)) == zlib.crc32(d)
    assert lcrc.lib().lcrc32c_value(d, len(d)) == orc.crc(d, 1)


def test_hasher_mirrors_crc32fast(lcrc):
    # Hasher::new(); update([type]); update(data); finalize()  (log.rs:61-64)
    h = lcrc.Hasher()
    h.update(bytes([1]))
    h.update(b"foo")
    assert h.finalize() == zlib.crc32(b"\x01foo") == 0xEACA044A
    assert h.amount == 4
    h2 = lcrc.Hasher.new_with_initial(zlib.crc32(b"\x01f"))
    h2.update(b"oo")
    assert h2.finalize() == 0xEACA044A
    assert lcrc.Hasher().finalize() == 0


def test_extend_and_combine(lcrc, orc):
    d = np.random.default_rng(5).integers(0, 256, 9000, dtype=np.uint8).tobytes()
    for mode in (lcrc.MODE_REF, lcrc.MODE_C):
        full = orc.crc(d, mode)
        for cut in (0, 1, 4096, 8999, 9000):
            a, b = d[:cut], d[cut:]
            assert lcrc.extend(lcrc.value(a, mode), b, mode) == full
            assert lcrc.combine(lcrc.value(a, mode), lcrc.value(b, mode), len(b), mode) == full


def test_mask(lcrc, orc):
    for v in (0, 1, 0xFFFFFFFF, 0xE3069283, 0xDEADBEEF):
        assert lcrc.mask(v) == orc.mask(v)
        assert lcrc.unmask(lcrc.mask(v)) == v


def test_batched_api_fails_loudly_without_device(lcrc):
    if lcrc.device_count() > 0:
        pytest.skip("device present")
    with pytest.raises(lcrc.NoDeviceError):
        lcrc.Engine(0, lcrc.MODE_C)
    assert lcrc.lib().lcrc_batch(None, None, 0, None, 0, None, None, None) == lcrc.EINVAL
    assert lcrc.lib().lcrc_batch_queue(None, None, 0, None) == lcrc.EINVAL
    assert lcrc.lib().lcrc_wal_scan_queue(None, None, 0, None) == lcrc.EINVAL


def test_scalar_extend_every_length_and_register(lcrc, orc):
    """The host CRCs (carry-less-multiply folding from 64 bytes on, tables / crc32 below) against zlib and the
    oracle for every length 0..700, large sizes, unaligned starts and arbitrary running values."""
    rng = np.random.default_rng(77)
    buf = rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
    for n in list(range(0, 700)) + [1023, 1024, 1025, 4096, 4097, 65536 + 13, (1 << 20) - 5]:
        off = int(rng.integers(0, 5))
        d = buf[off:off + n]
        init = int(rng.integers(0, 1 << 32))
        assert lcrc.extend(init, d, lcrc.MODE_REF) == zlib.crc32(d, init)
        if n < 5000:
            assert lcrc.extend(init, d, lcrc.MODE_C) == orc.crc(d, 1, init)


def test_library_built_from_this_tree(lcrc):
    """Build provenance: lcrc_version() carries the hash of the sources and recipe the library was built from,
    and it is this tree's (smoke() makes the same check on the GPU box)."""
    import __graft_entry__ as entry
    assert f"src {entry.source_hash()}" in lcrc.lib().lcrc_version().decode()


def test_build_refuses_diagnostic_flags_and_hashes_flags():
    """The in-tree library is never a diagnostic build: build.py refuses -DLCRC_PROBE_* for it, and any extra
    compile flag changes the source hash compiled into lcrc_version(), so a library built with a define of its
    own fails the provenance check above and smoke()'s."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("lcrc_build_t", os.path.join(ROOT, "leveldb-rust_amd", "build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    with pytest.raises(ValueError):
        b.build(extra_flags=["-DLCRC_PROBE_CLOCK"])
    with pytest.raises(ValueError):
        b.build(extra_flags=["-DLCRC_PROBE_PHASES=1"])
    assert b.source_hash(["-DLCRC_A_WGCU=2"]) != b.source_hash()
    assert b.source_hash(()) == b.source_hash()


def test_product_kernels_carry_no_wrong_crc_ablation():
    """Only clock-stamp diagnostics (which cannot change a CRC) remain behind LCRC_PROBE_* in the shipped
    kernel source."""
    with open(os.path.join(ROOT, "leveldb-rust_amd", "csrc", "lcrc_kernels.hip")) as f:
        src = f.read()
    assert set(re.findall(r"LCRC_PROBE_\w+", src)) <= {"LCRC_PROBE_CLOCK", "LCRC_PROBE_PHASES"}
