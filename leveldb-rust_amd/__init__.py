"""leveldb-rust_amd -- MI355X-native block/record checksum engine for leveldb-rust (Python host mirror).

This package is loaded under the importable name ``leveldb_rust_amd`` (the directory name has a hyphen;
see ``load()`` in ``__graft_entry__.py``). It binds ``_build/liblcrc.so`` (built by ``build.py``) through
ctypes and mirrors the reference's interfaces for the checksum path:

* ``Hasher`` / ``value`` / ``extend``   -- ``crc32fast::Hasher::{new, update, finalize}`` as used at
  src/db/log.rs:61-64, :261-264, src/sstable/table.rs:519-522, src/sstable/format.rs:164-166
* ``crc32c_value`` / ``crc32c_extend`` / ``mask`` / ``unmask`` -- the crc32c value/extend/mask surface
* ``Engine`` -- the batched device API (``lcrc_batch*``, ``lcrc_wal_scan``); GPU only, raises
  ``NoDeviceError`` when no gfx950 device/kernel image is available (there is no CPU fallback)
* ``LogWriter`` / ``LogReader`` / ``BatchLogReader`` -- src/db/log.rs LogWriter / LogReader
* ``TableFile`` -- write_raw_block (table.rs:507-529) and read_block_from_file (format.rs:146-213)
* ``Engine.table_scan`` -- Table::open(paranoid) + verify of every block (table.rs:39-103, format.rs:146-171)
* ``Engine.batch_seal`` -- batched trailer / WAL-header CRCs stored in place (table.rs:519-527, log.rs:61-70)
* ``snappy_frame_decode`` -- the Snappy framing decoder the table walk uses for compressed index blocks
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LCRC_LIB_PATH") or os.path.join(_HERE, "_build", "liblcrc.so")

MODE_REF = 0  # CRC-32/ISO-HDLC (crc32fast)
MODE_C = 1  # CRC-32C
FLAG_MASK = 0x1
FLAG_DIRECT = 0x2
TSCAN_SNAPPY_INDEX = 0x1  # lcrc_table_scan_async_ex: decode a Snappy-framed index block on the device
NO_EXPECT = -0x80000000

OK, EINVAL, ENODEV, EHIP, ENOMEM, ECORRUPT, ERANGE = 0, -1, -2, -3, -4, -5, -6

WAL_OK, WAL_CRC_MISMATCH = 0, 1
WAL_STOP_TRAILER, WAL_STOP_BAD_LENGTH, WAL_STOP_ZERO = 0, 1, 2

BLOCK_SIZE = 32768  # src/db/mod.rs:45
HEADER_SIZE = 7  # src/db/mod.rs:48
BLOCK_TRAILER_SIZE = 5  # src/sstable/format.rs:22


class LcrcError(RuntimeError):
    pass


class TableCorruption(LcrcError):
    """lcrc_table_scan found the table structure corrupt; str() is the reference's message."""


class NoDeviceError(LcrcError):
    pass


DESC_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u4"), ("expect_rel", "<i4")])
TBLK_DTYPE = np.dtype([("offset", "<u8"), ("size", "<u8"), ("crc", "<u4"), ("kind", "u1"), ("type", "u1"),
                       ("status", "u1"), ("reserved", "u1")])
TBLK_DATA, TBLK_FILTER, TBLK_METAINDEX, TBLK_INDEX = 0, 1, 2, 3
TBLK_OK, TBLK_CRC_MISMATCH, TBLK_TRUNCATED, TBLK_BAD_CONTENT, TBLK_BAD_TYPE = 0, 1, 2, 3, 4
WAL_REC_DTYPE = np.dtype([("header", "<u8"), ("length", "<u4"), ("type", "u1"), ("status", "u1"),
                          ("block_end", "<u2"), ("crc", "<u4"), ("stop", "<u4")])


class _Desc(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("length", ctypes.c_uint32), ("expect_rel", ctypes.c_int32)]


class _WalRec(ctypes.Structure):
    _fields_ = [("header", ctypes.c_uint64), ("length", ctypes.c_uint32), ("type", ctypes.c_uint8),
                ("status", ctypes.c_uint8), ("block_end", ctypes.c_uint16), ("crc", ctypes.c_uint32),
                ("stop", ctypes.c_uint32)]


class _UJob(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("n", ctypes.c_uint64), ("expected", ctypes.c_void_p),
                ("out_crc", ctypes.c_void_p), ("out_mismatch", ctypes.c_void_p)]


class _GJob(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("base_len", ctypes.c_uint64), ("descs", ctypes.c_void_p),
                ("n", ctypes.c_uint64), ("out_crc", ctypes.c_void_p), ("out_mismatch", ctypes.c_void_p)]


class _WJob(ctypes.Structure):
    _fields_ = [("file", ctypes.c_void_p), ("file_len", ctypes.c_uint64), ("recs", ctypes.c_void_p),
                ("max_recs", ctypes.c_uint64), ("n_recs", ctypes.c_void_p)]


class _CtxOptions(ctypes.Structure):
    _fields_ = [("size", ctypes.c_uint32), ("general", ctypes.c_int32), ("batch_grid_b", ctypes.c_uint32),
                ("wal_grid_b", ctypes.c_uint32), ("ts_grid", ctypes.c_uint32), ("ts_blocks_div", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32 * 3)]


GENERAL_PATHS = {"auto": 0, "ranges": 1, "blocks": 2}


class _Hasher(ctypes.Structure):
    _fields_ = [("state", ctypes.c_uint32), ("mode", ctypes.c_int32), ("amount", ctypes.c_uint64)]


_lib = None

# every symbol declared in include/lcrc.h (tests check the library exports all of them)
ABI_SYMBOLS = [
    "lcrc32_value", "lcrc32_extend", "lcrc32c_value", "lcrc32c_extend", "lcrc32c_mask", "lcrc32c_unmask",
    "lcrc_extend", "lcrc_combine", "lcrc_hasher_init", "lcrc_hasher_update", "lcrc_hasher_finalize",
    "lcrc_device_count", "lcrc_device_pci_bus_id", "lcrc_ctx_create", "lcrc_ctx_create_ex", "lcrc_ctx_destroy", "lcrc_ctx_reserve", "lcrc_ctx_stream", "lcrc_ctx_join",
    "lcrc_ctx_sync", "lcrc_batch", "lcrc_batch_covered", "lcrc_batch_uniform", "lcrc_batch_uniform_queue", "lcrc_batch_queue", "lcrc_batch_multi", "lcrc_batch_host_uniform", "lcrc_wal_scan", "lcrc_wal_scan_async", "lcrc_wal_scan_queue",
    "lcrc_table_scan", "lcrc_table_scan_async", "lcrc_table_scan_async_ex", "lcrc_table_scan_reserve", "lcrc_table_scan_message",
    "lcrc_batch_seal", "lcrc_snappy_frames",
    "lcrc_tb_create", "lcrc_tb_destroy", "lcrc_tb_add", "lcrc_tb_add_many", "lcrc_tb_flush", "lcrc_tb_finish", "lcrc_tb_size",
    "lcrc_tb_data", "lcrc_tb_blocks", "lcrc_tb_seal_descs",
    "lcrc_dev_alloc", "lcrc_dev_free", "lcrc_host_alloc_pinned", "lcrc_host_free_pinned", "lcrc_memcpy_h2d",
    "lcrc_memcpy_d2h", "lcrc_memset_d", "lcrc_device_sync", "lcrc_timer_start", "lcrc_timer_kernels", "lcrc_timer_stop",
    "lcrc_timer_span",
    "lcrc_graph_begin", "lcrc_graph_end", "lcrc_graph_launch", "lcrc_graph_destroy",
    "lcrc_last_error", "lcrc_version",
]


def lib():
    """Load the native library (fails loudly if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LcrcError(f"{LIB_PATH} missing: run build() (leveldb-rust_amd/build.py) first")
    L = ctypes.CDLL(LIB_PATH)
    u32, u64, sz, vp, i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int
    cp = ctypes.c_char_p

    def sig(name, res, *args):
        f = getattr(L, name)
        f.restype = res
        f.argtypes = list(args)

    sig("lcrc32_value", u32, vp, sz)
    sig("lcrc32_extend", u32, u32, vp, sz)
    sig("lcrc32c_value", u32, vp, sz)
    sig("lcrc32c_extend", u32, u32, vp, sz)
    sig("lcrc32c_mask", u32, u32)
    sig("lcrc32c_unmask", u32, u32)
    sig("lcrc_extend", u32, i32, u32, vp, sz)
    sig("lcrc_combine", u32, i32, u32, u32, u64)
    sig("lcrc_hasher_init", None, ctypes.POINTER(_Hasher), i32)
    sig("lcrc_hasher_update", None, ctypes.POINTER(_Hasher), vp, sz)
    sig("lcrc_hasher_finalize", u32, ctypes.POINTER(_Hasher))
    sig("lcrc_device_count", i32, ctypes.POINTER(ctypes.c_int))
    sig("lcrc_device_pci_bus_id", i32, i32, ctypes.c_char_p, i32)
    sig("lcrc_ctx_create", i32, ctypes.POINTER(vp), i32, i32, u32)
    sig("lcrc_ctx_create_ex", i32, ctypes.POINTER(vp), i32, i32, u32, ctypes.POINTER(_CtxOptions))
    sig("lcrc_ctx_destroy", i32, vp)
    sig("lcrc_ctx_reserve", i32, vp, u64)
    sig("lcrc_ctx_stream", vp, vp)
    sig("lcrc_ctx_sync", i32, vp)
    sig("lcrc_batch", i32, vp, vp, u64, vp, sz, vp, vp, vp)
    sig("lcrc_batch_covered", i32, vp, vp, u64, vp, sz, u64, vp, vp, vp)
    sig("lcrc_batch_uniform", i32, vp, vp, sz, u32, u64, vp, vp, vp, vp)
    sig("lcrc_batch_uniform_queue", i32, vp, ctypes.POINTER(_UJob), sz, u32, u64, vp)
    sig("lcrc_batch_queue", i32, vp, ctypes.POINTER(_GJob), sz, vp)
    sig("lcrc_wal_scan_queue", i32, vp, ctypes.POINTER(_WJob), sz, vp)
    sig("lcrc_batch_host_uniform", i32, vp, vp, sz, u32, u64, vp, vp, vp, sz)
    sig("lcrc_batch_multi", i32, vp, ctypes.c_int, vp, u64, vp, sz, vp, vp)
    sig("lcrc_wal_scan", i32, vp, vp, u64, vp, sz, ctypes.POINTER(ctypes.c_size_t), vp)
    sig("lcrc_wal_scan_async", i32, vp, vp, u64, vp, sz, vp, vp)
    sig("lcrc_table_scan", i32, vp, vp, u64, cp, vp, sz, ctypes.POINTER(ctypes.c_size_t), vp, sz)
    sig("lcrc_batch_seal", i32, vp, vp, u64, vp, sz, vp, vp)
    sig("lcrc_table_scan_async", i32, vp, vp, u64, cp, vp, sz, vp, vp, vp)
    sig("lcrc_table_scan_async_ex", i32, vp, vp, u64, cp, vp, sz, vp, vp, u32, vp)
    sig("lcrc_table_scan_reserve", i32, vp, u64, sz, u64)
    sig("lcrc_table_scan_message", cp, u32)
    sig("lcrc_snappy_frames", i32, vp, vp, vp, sz, vp, u64, vp, vp, ctypes.POINTER(ctypes.c_uint64))
    sig("lcrc_snappy_frame_decode", ctypes.c_int64, vp, sz, vp, sz)
    sig("lcrc_dev_alloc", i32, i32, sz, ctypes.POINTER(vp))
    sig("lcrc_dev_free", i32, vp)
    sig("lcrc_host_alloc_pinned", i32, sz, ctypes.POINTER(vp))
    sig("lcrc_host_free_pinned", i32, vp)
    sig("lcrc_memcpy_h2d", i32, vp, vp, sz)
    sig("lcrc_memcpy_d2h", i32, vp, vp, sz)
    sig("lcrc_memset_d", i32, vp, i32, sz)
    sig("lcrc_device_sync", i32)
    sig("lcrc_timer_start", i32, vp)
    sig("lcrc_ctx_join", i32, vp, vp)
    sig("lcrc_timer_kernels", i32, vp, i32)
    sig("lcrc_timer_stop", i32, vp, ctypes.POINTER(ctypes.c_float))
    sig("lcrc_timer_span", i32, vp, vp, ctypes.POINTER(ctypes.c_float))
    sig("lcrc_graph_begin", i32, vp)
    sig("lcrc_graph_end", i32, vp, ctypes.POINTER(vp))
    sig("lcrc_graph_launch", i32, vp, vp)
    sig("lcrc_graph_destroy", i32, vp)
    sig("lcrc_last_error", cp)
    sig("lcrc_version", cp)
    # C++ restatement of the reference call sites (lcrc_leveldb.cpp)
    sig("lcrc_logw_create", vp, u64)
    sig("lcrc_logw_destroy", None, vp)
    sig("lcrc_logw_add", None, vp, vp, sz)
    sig("lcrc_logw_size", sz, vp)
    sig("lcrc_logw_data", vp, vp)
    sig("lcrc_logw_prepend", None, vp, vp, sz)
    sig("lcrc_logr_create", vp, vp, sz)
    sig("lcrc_logr_create_batch", vp, vp, sz, vp, sz)
    sig("lcrc_logr_destroy", None, vp)
    sig("lcrc_logr_force_error", None, vp)
    sig("lcrc_logr_read", i32, vp)
    sig("lcrc_logr_record", sz, vp, ctypes.POINTER(vp))
    sig("lcrc_logr_dropped", sz, vp)
    sig("lcrc_logr_message", cp, vp)
    sig("lcrc_logr_consistency_errors", i32, vp)
    sig("lcrc_tbl_create", vp)
    sig("lcrc_tbl_destroy", None, vp)
    sig("lcrc_tbl_write_raw_block", None, vp, vp, sz, ctypes.c_uint8, ctypes.POINTER(u64), ctypes.POINTER(u64))
    sig("lcrc_tbl_size", sz, vp)
    sig("lcrc_tbl_data", vp, vp)
    sig("lcrc_tbl_append", None, vp, vp, sz)
    sig("lcrc_tbl_read_block", cp, vp, sz, u64, u64, i32, ctypes.POINTER(ctypes.c_uint8))
    # C++ restatement of the reference's TableBuilder (lcrc_tbuild.cpp)
    sig("lcrc_tb_create", vp, u32, i32, ctypes.c_uint8, i32, u32, i32)
    sig("lcrc_tb_destroy", None, vp)
    sig("lcrc_tb_add", i32, vp, vp, sz, vp, sz)
    sig("lcrc_tb_add_many", i32, vp, vp, sz, vp, sz, sz)
    sig("lcrc_tb_flush", None, vp)
    sig("lcrc_tb_finish", i32, vp, cp, vp, sz)
    sig("lcrc_tb_size", sz, vp)
    sig("lcrc_tb_data", vp, vp)
    sig("lcrc_tb_blocks", sz, vp, vp, sz)
    sig("lcrc_tb_seal_descs", sz, vp, vp, sz)
    _lib = L
    return L


def _buf(data):
    """(pointer, length, keepalive) for bytes / bytearray / numpy array."""
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data)
        return a.ctypes.data_as(ctypes.c_void_p), a.nbytes, a
    if isinstance(data, (bytes, bytearray, memoryview)):
        a = np.frombuffer(bytes(data) if isinstance(data, memoryview) else data, dtype=np.uint8)
        return a.ctypes.data_as(ctypes.c_void_p), a.nbytes, a
    raise TypeError(type(data))


def _check(rc, what):
    if rc == OK:
        return
    msg = f"{what} failed ({rc}): {lib().lcrc_last_error().decode(errors='replace')}"
    if rc == ENODEV:
        raise NoDeviceError(msg)
    raise LcrcError(msg)


# ---------------------------------------------------------------------------------------------------
# scalar API (host)
# ---------------------------------------------------------------------------------------------------
def value(data, mode=MODE_REF):
    p, n, _k = _buf(data)
    return lib().lcrc_extend(mode, 0, p, n)


def extend(crc, data, mode=MODE_REF):
    p, n, _k = _buf(data)
    return lib().lcrc_extend(mode, crc, p, n)


def crc32c_value(data):
    return value(data, MODE_C)


def crc32c_extend(crc, data):
    return extend(crc, data, MODE_C)


def mask(crc):
    return lib().lcrc32c_mask(crc)


def unmask(m):
    return lib().lcrc32c_unmask(m)


def combine(crc_a, crc_b, len_b, mode=MODE_REF):
    return lib().lcrc_combine(mode, crc_a, crc_b, len_b)


class Hasher:
    """Mirror of ``crc32fast::Hasher``: ``Hasher()``, ``update(bytes)``, ``finalize() -> int``."""

    def __init__(self, mode=MODE_REF, initial=0):
        self._h = _Hasher()
        lib().lcrc_hasher_init(ctypes.byref(self._h), mode)
        self._h.state = initial

    @classmethod
    def new_with_initial(cls, crc, mode=MODE_REF):
        return cls(mode, crc)

    def update(self, data):
        p, n, _k = _buf(data)
        lib().lcrc_hasher_update(ctypes.byref(self._h), p, n)

    def finalize(self):
        return lib().lcrc_hasher_finalize(ctypes.byref(self._h))

    @property
    def amount(self):
        return self._h.amount


# ---------------------------------------------------------------------------------------------------
# device memory + batched engine
# ---------------------------------------------------------------------------------------------------
def device_count():
    n = ctypes.c_int(0)
    lib().lcrc_device_count(ctypes.byref(n))
    return n.value


def pci_bus_id(device):
    """The device's PCI bus ID ("dddd:bb:dd.f", lcrc_device_pci_bus_id)."""
    buf = ctypes.create_string_buffer(64)
    _check(lib().lcrc_device_pci_bus_id(int(device), buf, 64), "lcrc_device_pci_bus_id")
    return buf.value.decode()


class DeviceBuffer:
    """Raw device allocation owned by Python (freed on close/GC)."""

    def __init__(self, nbytes, device=0):
        self.nbytes = int(nbytes)
        self.device = device
        p = ctypes.c_void_p()
        _check(lib().lcrc_dev_alloc(device, self.nbytes, ctypes.byref(p)), "lcrc_dev_alloc")
        self.ptr = p.value

    @classmethod
    def from_host(cls, data, device=0, pad=0):
        p, n, _k = _buf(data)
        b = cls(n + pad, device)
        if n:
            _check(lib().lcrc_memcpy_h2d(b.ptr, p, n), "lcrc_memcpy_h2d")
        return b

    def upload(self, data, offset=0):
        p, n, _k = _buf(data)
        assert offset + n <= self.nbytes
        if n:
            _check(lib().lcrc_memcpy_h2d(self.ptr + offset, p, n), "lcrc_memcpy_h2d")

    def download(self, dtype=np.uint8, count=None, offset=0):
        dtype = np.dtype(dtype)
        if count is None:
            count = (self.nbytes - offset) // dtype.itemsize
        out = np.empty(count, dtype=dtype)
        if out.nbytes:
            _check(lib().lcrc_memcpy_d2h(out.ctypes.data_as(ctypes.c_void_p), self.ptr + offset, out.nbytes),
                   "lcrc_memcpy_d2h")
        return out

    def zero(self):
        _check(lib().lcrc_memset_d(self.ptr, 0, self.nbytes), "lcrc_memset_d")

    def close(self):
        if getattr(self, "ptr", None):
            lib().lcrc_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PinnedBuffer:
    def __init__(self, nbytes):
        p = ctypes.c_void_p()
        _check(lib().lcrc_host_alloc_pinned(int(nbytes), ctypes.byref(p)), "lcrc_host_alloc_pinned")
        self.ptr = p.value
        self.nbytes = int(nbytes)
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr))

    def close(self):
        if getattr(self, "ptr", None):
            self.array = None
            lib().lcrc_host_free_pinned(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, (DeviceBuffer, PinnedBuffer)):
        return x.ptr
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):  # torch tensor
        return x.data_ptr()
    raise TypeError(type(x))


class Engine:
    """One device + one CRC mode (``lcrc_ctx``). All batched calls are GPU-only.

    Keyword options (``lcrc_ctx_create_ex``, tests and measurement only): ``general`` ("auto" | "ranges" |
    "blocks"), ``batch_grid_b``, ``wal_grid_b``, ``ts_grid``, ``ts_blocks_div``; unset = the library default."""

    def __init__(self, device=0, mode=MODE_C, flags=0, **options):
        self.device, self.mode, self.flags = device, mode, flags
        ctx = ctypes.c_void_p()
        if options:
            o = _CtxOptions()
            o.size = ctypes.sizeof(_CtxOptions)
            for k, v in options.items():
                if k == "general":
                    v = GENERAL_PATHS[v] if isinstance(v, str) else int(v)
                elif k not in ("batch_grid_b", "wal_grid_b", "ts_grid", "ts_blocks_div"):
                    raise TypeError(f"Engine: unknown option {k!r}")
                setattr(o, k, int(v))
            _check(lib().lcrc_ctx_create_ex(ctypes.byref(ctx), device, mode, flags, ctypes.byref(o)),
                   "lcrc_ctx_create_ex")
        else:
            _check(lib().lcrc_ctx_create(ctypes.byref(ctx), device, mode, flags), "lcrc_ctx_create")
        self.ctx = ctx.value

    def close(self):
        if getattr(self, "ctx", None):
            lib().lcrc_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return lib().lcrc_ctx_stream(self.ctx)

    def sync(self):
        _check(lib().lcrc_ctx_sync(self.ctx), "lcrc_ctx_sync")

    def reserve(self, max_span):
        _check(lib().lcrc_ctx_reserve(self.ctx, int(max_span)), "lcrc_ctx_reserve")

    def batch(self, base, base_len, descs, n, out_crc, out_mismatch=None, stream=None, covered=None):
        """lcrc_batch; with covered (sum of the lengths, or a bound) lcrc_batch_covered, which verifies a
        sparse set reading only its own bytes."""
        if covered is None:
            _check(lib().lcrc_batch(self.ctx, _ptr(base), int(base_len), _ptr(descs), int(n), _ptr(out_crc),
                                    _ptr(out_mismatch), stream), "lcrc_batch")
        else:
            _check(lib().lcrc_batch_covered(self.ctx, _ptr(base), int(base_len), _ptr(descs), int(n), int(covered),
                                            _ptr(out_crc), _ptr(out_mismatch), stream), "lcrc_batch_covered")

    def batch_uniform(self, base, n, length, stride, out_crc, expected=None, out_mismatch=None, stream=None):
        _check(lib().lcrc_batch_uniform(self.ctx, _ptr(base), int(n), int(length), int(stride), _ptr(expected),
                                        _ptr(out_crc), _ptr(out_mismatch), stream), "lcrc_batch_uniform")

    def batch_uniform_queue(self, jobs, length, stride, stream=None):
        """lcrc_batch_uniform_queue: jobs = [(base, n, out_crc[, expected[, out_mismatch]])] (or the array
        ujobs() made of them), each one lcrc_batch_uniform batch; the 4 KiB layout streams up to 32 of them per
        launch."""
        arr = jobs if isinstance(jobs, UJobs) else ujobs(jobs)
        _check(lib().lcrc_batch_uniform_queue(self.ctx, arr.arr, arr.n, int(length), int(stride), stream),
               "lcrc_batch_uniform_queue")

    def batch_queue(self, jobs, stream=None):
        """lcrc_batch_queue: jobs = [(base, base_len, descs, n, out_crc[, out_mismatch])] (or the array gjobs()
        made of them), each one lcrc_batch batch; the window pass of each batch streams while the previous
        batch's range pass finishes beside it."""
        arr = jobs if isinstance(jobs, GJobs) else gjobs(jobs)
        _check(lib().lcrc_batch_queue(self.ctx, arr.arr, arr.n, stream), "lcrc_batch_queue")

    def batch_host_uniform(self, base, n, length, stride, expected=None, chunk_bytes=0):
        """Host-resident input (numpy / PinnedBuffer). Returns (crc array, mismatch bitmap)."""
        bp, _nb, keep = (base.ptr, base.nbytes, base) if isinstance(base, PinnedBuffer) else _buf(base)
        out = np.empty(n, np.uint32)
        mm = np.empty((n + 31) // 32, np.uint32)
        ep, _, keep2 = _buf(np.ascontiguousarray(expected, np.uint32)) if expected is not None else (None, 0, None)
        _check(lib().lcrc_batch_host_uniform(self.ctx, bp, int(n), int(length), int(stride), ep,
                                             out.ctypes.data_as(ctypes.c_void_p), mm.ctypes.data_as(ctypes.c_void_p),
                                             int(chunk_bytes)), "lcrc_batch_host_uniform")
        del keep, keep2
        return out, mm

    def wal_scan_async(self, file_dev, file_len, recs_dev, max_recs, count_dev, stream=None):
        """lcrc_wal_scan_async: enqueue the scan; the record count lands in count_dev (device u64)."""
        _check(lib().lcrc_wal_scan_async(self.ctx, _ptr(file_dev), int(file_len), _ptr(recs_dev), int(max_recs),
                                         _ptr(count_dev), stream), "lcrc_wal_scan_async")

    def wal_scan_queue(self, jobs, stream=None):
        """lcrc_wal_scan_queue: jobs = [(file_dev, file_len, recs_dev, max_recs, count_dev)] (or the array wjobs()
        made of them), each one lcrc_wal_scan_async; the header walks of all the logs first, then the window
        passes back to back with each log's range pass beside the next one."""
        arr = jobs if isinstance(jobs, WJobs) else wjobs(jobs)
        _check(lib().lcrc_wal_scan_queue(self.ctx, arr.arr, arr.n, stream), "lcrc_wal_scan_queue")

    def wal_scan_device(self, file_dev, file_len, recs_dev, max_recs):
        """lcrc_wal_scan leaving the records on the device (recs_dev); returns the record count."""
        n = ctypes.c_size_t(0)
        _check(lib().lcrc_wal_scan(self.ctx, _ptr(file_dev), int(file_len), _ptr(recs_dev), int(max_recs),
                                   ctypes.byref(n), None), "lcrc_wal_scan")
        return n.value

    def wal_scan(self, file_dev, file_len, max_recs=None, recs_dev=None):
        """Parse + verify every physical record of a device-resident log. Returns a WAL_REC_DTYPE array."""
        if max_recs is None:
            max_recs = max(1, file_len // HEADER_SIZE + 1)
        own = recs_dev is None
        if own:
            recs_dev = DeviceBuffer(max_recs * WAL_REC_DTYPE.itemsize, self.device)
        n = ctypes.c_size_t(0)
        _check(lib().lcrc_wal_scan(self.ctx, _ptr(file_dev), int(file_len), _ptr(recs_dev), int(max_recs),
                                   ctypes.byref(n), None), "lcrc_wal_scan")
        self.sync()
        out = recs_dev.download(WAL_REC_DTYPE, n.value)
        if own:
            recs_dev.close()
        return out

    def table_scan(self, file_dev, file_len, filter_name=None):
        """Whole-table verify scan of a device-resident SSTable. Returns a TBLK_DTYPE array sorted by
        offset; raises TableCorruption(reference message) when the structure is corrupt."""
        n = ctypes.c_size_t(0)
        err = ctypes.create_string_buffer(256)
        fname = filter_name.encode() if isinstance(filter_name, str) else filter_name
        rc = lib().lcrc_table_scan(self.ctx, _ptr(file_dev), int(file_len), fname, None, 0, ctypes.byref(n), err, 256)
        if rc == ECORRUPT:
            raise TableCorruption(err.value.decode())
        if rc != ERANGE:
            _check(rc, "lcrc_table_scan")
        out = np.zeros(n.value, TBLK_DTYPE)
        rc = lib().lcrc_table_scan(self.ctx, _ptr(file_dev), int(file_len), fname,
                                   out.ctypes.data_as(ctypes.c_void_p), n.value, ctypes.byref(n), err, 256)
        if rc == ECORRUPT:
            raise TableCorruption(err.value.decode())
        _check(rc, "lcrc_table_scan")
        return out

    def table_scan_into(self, file_dev, file_len, out, filter_name=None):
        """lcrc_table_scan into a preallocated TBLK_DTYPE array; returns the block count."""
        n = ctypes.c_size_t(0)
        err = ctypes.create_string_buffer(256)
        fname = filter_name.encode() if isinstance(filter_name, str) else filter_name
        rc = lib().lcrc_table_scan(self.ctx, _ptr(file_dev), int(file_len), fname, out.ctypes.data_as(ctypes.c_void_p),
                                   len(out), ctypes.byref(n), err, 256)
        if rc == ECORRUPT:
            raise TableCorruption(err.value.decode())
        _check(rc, "lcrc_table_scan")
        return n.value

    def table_scan_reserve(self, max_file_len, max_blocks, decoded_cap=0):
        _check(lib().lcrc_table_scan_reserve(self.ctx, int(max_file_len), int(max_blocks), int(decoded_cap)),
               "lcrc_table_scan_reserve")

    def table_scan_async(self, file_dev, file_len, blocks_dev, max_blocks, count_dev, status_dev, filter_name=None,
                         stream=None, snappy_index=False):
        """lcrc_table_scan_async: enqueued, device-only; results, count (u64) and status (2 x u32) stay where
        the caller points them (device or pinned memory). snappy_index: lcrc_table_scan_async_ex with
        LCRC_TSCAN_SNAPPY_INDEX (a table written with compression: its Snappy-framed index decoded on the device)."""
        fname = filter_name.encode() if isinstance(filter_name, str) else filter_name
        if snappy_index:
            _check(lib().lcrc_table_scan_async_ex(self.ctx, _ptr(file_dev), int(file_len), fname, _ptr(blocks_dev),
                                                  int(max_blocks), _ptr(count_dev), _ptr(status_dev),
                                                  TSCAN_SNAPPY_INDEX, stream), "lcrc_table_scan_async_ex")
            return
        _check(lib().lcrc_table_scan_async(self.ctx, _ptr(file_dev), int(file_len), fname, _ptr(blocks_dev),
                                           int(max_blocks), _ptr(count_dev), _ptr(status_dev), stream),
               "lcrc_table_scan_async")

    def snappy_frames_into(self, base, frames_dev, n, out, out_cap, out_off, status):
        """lcrc_snappy_frames with caller-owned device buffers; returns the decoded size."""
        total = ctypes.c_uint64(0)
        _check(lib().lcrc_snappy_frames(self.ctx, _ptr(base), _ptr(frames_dev), int(n), _ptr(out), int(out_cap),
                                        _ptr(out_off), _ptr(status), ctypes.byref(total)), "lcrc_snappy_frames")
        return total.value

    def batch_seal(self, base, base_len, descs, n, out_crc=None, stream=None):
        """Compute each descriptor's CRC and store it at base[offset + expect_rel] (device, in place)."""
        _check(lib().lcrc_batch_seal(self.ctx, _ptr(base), int(base_len), _ptr(descs), int(n), _ptr(out_crc), stream),
               "lcrc_batch_seal")

    def snappy_frames(self, base, frames_dev, n, out=None, out_cap=0):
        """lcrc_snappy_frames: (decoded bytes per frame as a list, status array). base / frames_dev / out are
        device buffers; with out None the decoded size is queried first and a buffer allocated."""
        total = ctypes.c_uint64(0)
        off = DeviceBuffer(8 * (n + 1), self.device)
        st = DeviceBuffer(max(1, n), self.device)
        own = out is None
        if own:
            rc = lib().lcrc_snappy_frames(self.ctx, _ptr(base), _ptr(frames_dev), int(n), None, 0, off.ptr, st.ptr,
                                          ctypes.byref(total))
            if rc not in (OK, ERANGE):
                _check(rc, "lcrc_snappy_frames")
            out = DeviceBuffer(max(1, total.value), self.device)
            out_cap = total.value
        _check(lib().lcrc_snappy_frames(self.ctx, _ptr(base), _ptr(frames_dev), int(n), _ptr(out), int(out_cap),
                                        off.ptr, st.ptr, ctypes.byref(total)), "lcrc_snappy_frames")
        offs = off.download(np.uint64, n + 1)
        data = out.download(np.uint8, int(offs[n])) if n else np.zeros(0, np.uint8)
        status = st.download(np.uint8, n)
        frames_out = [data[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(n)]
        for b in (off, st) + ((out,) if own else ()):
            b.close()
        return frames_out, status

    def graph_capture(self, fn):
        """Capture the context-stream calls made by fn() into a replayable HIP graph (returns a handle)."""
        _check(lib().lcrc_graph_begin(self.ctx), "lcrc_graph_begin")
        try:
            fn()
        finally:
            ge = ctypes.c_void_p()
            rc = lib().lcrc_graph_end(self.ctx, ctypes.byref(ge))
        _check(rc, "lcrc_graph_end")
        return ge.value

    def graph_launch(self, graph):
        _check(lib().lcrc_graph_launch(self.ctx, graph), "lcrc_graph_launch")

    @staticmethod
    def graph_destroy(graph):
        lib().lcrc_graph_destroy(graph)

    def join(self, other):
        """lcrc_ctx_join: this engine's stream waits (on the device) for the work enqueued on other's so far."""
        _check(lib().lcrc_ctx_join(self.ctx, other.ctx), "lcrc_ctx_join")

    def timer_start(self):
        _check(lib().lcrc_timer_start(self.ctx), "lcrc_timer_start")

    def timer_kernels(self, edge):
        """Fast-path launches carry the timer's events: edge 0 = the next launch records the start, edge 1 = the
        launches from the next one on record the end, edge 2 = disarm."""
        _check(lib().lcrc_timer_kernels(self.ctx, int(edge)), "lcrc_timer_kernels")

    def timer_stop(self):
        ms = ctypes.c_float(0)
        _check(lib().lcrc_timer_stop(self.ctx, ctypes.byref(ms)), "lcrc_timer_stop")
        return ms.value

    def timer_span(self, last):
        """ms from this engine's kernel-carried start event to `last`'s stop event (lcrc_timer_span)."""
        ms = ctypes.c_float(0)
        _check(lib().lcrc_timer_span(self.ctx, last.ctx, ctypes.byref(ms)), "lcrc_timer_span")
        return ms.value

    # convenience: host numpy in, host numpy out (copies; for tests)
    def crc_ranges(self, data, offsets, lengths, expect_rel=None, covered_hint=False):
        data = np.ascontiguousarray(np.frombuffer(data, np.uint8) if not isinstance(data, np.ndarray) else data)
        n = len(offsets)
        d = np.zeros(n, DESC_DTYPE)
        d["offset"] = offsets
        d["length"] = lengths
        d["expect_rel"] = NO_EXPECT if expect_rel is None else expect_rel
        base = DeviceBuffer.from_host(data, self.device)
        dd = DeviceBuffer.from_host(d.view(np.uint8), self.device)
        out = DeviceBuffer(max(4 * n, 4), self.device)
        mm = DeviceBuffer(max(4 * ((n + 31) // 32), 4), self.device)
        self.batch(base, data.nbytes, dd, n, out, mm,
                   covered=int(np.asarray(lengths, np.uint64).sum()) if covered_hint else None)
        self.sync()
        crcs = out.download(np.uint32, n)
        bits = mm.download(np.uint32, (n + 31) // 32)
        return crcs, unpack_bits(bits, n)


def batch_multi(engines, data, offsets, lengths, expect_rel=None):
    """lcrc_batch_multi: a host-resident file (numpy / bytes) and its descriptors sharded over the engines (one
    per GPU, or several on one); returns (crc array, mismatch bool array) as lcrc_batch over the whole file."""
    data = np.ascontiguousarray(np.frombuffer(data, np.uint8) if not isinstance(data, np.ndarray) else data)
    n = len(offsets)
    d = np.zeros(n, DESC_DTYPE)
    d["offset"], d["length"] = offsets, lengths
    d["expect_rel"] = NO_EXPECT if expect_rel is None else expect_rel
    ctxs = (ctypes.c_void_p * len(engines))(*[e.ctx for e in engines])
    out = np.empty(max(n, 1), np.uint32)
    mm = np.empty(max((n + 31) // 32, 1), np.uint32)
    _check(lib().lcrc_batch_multi(ctxs, len(engines), data.ctypes.data_as(ctypes.c_void_p), data.nbytes,
                                  d.ctypes.data_as(ctypes.c_void_p), n, out.ctypes.data_as(ctypes.c_void_p),
                                  mm.ctypes.data_as(ctypes.c_void_p)), "lcrc_batch_multi")
    return out[:n], unpack_bits(mm, n)


class UJobs:
    """A prepared lcrc_ujob array (the queue's jobs, built once, submitted any number of times)."""

    def __init__(self, jobs):
        self.n = len(jobs)
        self.arr = (_UJob * max(1, self.n))()
        self.keep = list(jobs)
        for k, j in enumerate(jobs):
            exp = j[3] if len(j) > 3 else None
            mm = j[4] if len(j) > 4 else None
            self.arr[k] = _UJob(_ptr(j[0]), int(j[1]), _ptr(exp), _ptr(j[2]), _ptr(mm))


def ujobs(jobs):
    return UJobs(jobs)


class GJobs:
    """A prepared lcrc_gjob array (lcrc_batch_queue's jobs, built once, submitted any number of times)."""

    def __init__(self, jobs):
        self.n = len(jobs)
        self.arr = (_GJob * max(1, self.n))()
        self.keep = list(jobs)
        for k, j in enumerate(jobs):
            mm = j[5] if len(j) > 5 else None
            self.arr[k] = _GJob(_ptr(j[0]), int(j[1]), _ptr(j[2]), int(j[3]), _ptr(j[4]), _ptr(mm))


def gjobs(jobs):
    return GJobs(jobs)


class WJobs:
    """A prepared lcrc_wjob array (lcrc_wal_scan_queue's logs, built once, submitted any number of times)."""

    def __init__(self, jobs):
        self.n = len(jobs)
        self.arr = (_WJob * max(1, self.n))()
        self.keep = list(jobs)
        for k, j in enumerate(jobs):
            self.arr[k] = _WJob(_ptr(j[0]), int(j[1]), _ptr(j[2]), int(j[3]), _ptr(j[4]))


def wjobs(jobs):
    return WJobs(jobs)


def unpack_bits(words, n):
    w = np.asarray(words, np.uint32)
    bits = (w[:, None] >> np.arange(32, dtype=np.uint32)[None, :]) & 1
    return bits.reshape(-1)[:n].astype(bool)


# ---------------------------------------------------------------------------------------------------
# reference call-site mirrors (C++ restatement in csrc/lcrc_leveldb.cpp)
# ---------------------------------------------------------------------------------------------------
class LogWriter:
    """src/db/log.rs LogWriter over an in-memory file. ``offset`` = dest length (new_with_dest_len)."""

    def __init__(self, offset=0, existing=b""):
        self._w = lib().lcrc_logw_create(offset)
        if existing:
            p, n, _k = _buf(existing)
            lib().lcrc_logw_prepend(self._w, p, n)

    def add_record(self, data):
        p, n, _k = _buf(data)
        lib().lcrc_logw_add(self._w, p, n)

    def contents(self):
        n = lib().lcrc_logw_size(self._w)
        if n == 0:
            return b""
        return ctypes.string_at(lib().lcrc_logw_data(self._w), n)

    def __len__(self):
        return lib().lcrc_logw_size(self._w)

    def __del__(self):
        try:
            lib().lcrc_logw_destroy(self._w)
        except Exception:
            pass


class EofError(Exception):
    """StatusError::Eof("meet a eof")"""

    def __str__(self):
        return "meet a eof"


class _ReaderBase:
    def read_record(self):
        rc = lib().lcrc_logr_read(self._r)
        if rc != 0:
            raise EofError()
        p = ctypes.c_void_p()
        n = lib().lcrc_logr_record(self._r, ctypes.byref(p))
        return ctypes.string_at(p, n) if n else b""

    def records(self):
        out = []
        while True:
            try:
                out.append(self.read_record())
            except EofError:
                return out

    @property
    def dropped_bytes(self):
        return lib().lcrc_logr_dropped(self._r)

    @property
    def report_message(self):
        return lib().lcrc_logr_message(self._r).decode()

    def __del__(self):
        try:
            lib().lcrc_logr_destroy(self._r)
        except Exception:
            pass


class LogReader(_ReaderBase):
    """src/db/log.rs LogReader; per-record host checksum (call site 2)."""

    def __init__(self, data):
        p, n, _k = _buf(data)
        self._r = lib().lcrc_logr_create(p, n)

    def force_error(self):
        lib().lcrc_logr_force_error(self._r)


class BatchLogReader(_ReaderBase):
    """Same reader contract; all physical-record checksums of the file verified in one device scan."""

    def __init__(self, data, engine):
        arr = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
        dev = DeviceBuffer.from_host(arr, engine.device)
        self.records_scanned = engine.wal_scan(dev, arr.nbytes)
        dev.close()
        p, n, _k = _buf(arr)
        rp, rn, _k2 = _buf(self.records_scanned.view(np.uint8))
        self._r = lib().lcrc_logr_create_batch(p, n, rp, len(self.records_scanned))

    @property
    def consistency_errors(self):
        return lib().lcrc_logr_consistency_errors(self._r)


class TableFile:
    """SSTable block trailers: write_raw_block (table.rs:507-529) / read_block (format.rs:146-213)."""

    def __init__(self):
        self._t = lib().lcrc_tbl_create()

    def write_raw_block(self, content, block_type):
        p, n, _k = _buf(content)
        off, size = ctypes.c_uint64(), ctypes.c_uint64()
        lib().lcrc_tbl_write_raw_block(self._t, p, n, block_type, ctypes.byref(off), ctypes.byref(size))
        return off.value, size.value

    def append(self, data):
        p, n, _k = _buf(data)
        lib().lcrc_tbl_append(self._t, p, n)

    def contents(self):
        n = lib().lcrc_tbl_size(self._t)
        return ctypes.string_at(lib().lcrc_tbl_data(self._t), n) if n else b""

    @staticmethod
    def read_block(file_bytes, offset, size, verify_checksum):
        """Returns (block_type, None) or (None, error string) exactly as format.rs:146-213."""
        p, n, _k = _buf(file_bytes)
        t = ctypes.c_uint8()
        err = lib().lcrc_tbl_read_block(p, n, offset, size, 1 if verify_checksum else 0, ctypes.byref(t))
        return (None, err.decode()) if err else (t.value, None)

    def __del__(self):
        try:
            lib().lcrc_tbl_destroy(self._t)
        except Exception:
            pass


class TableBuilder:
    """src/sstable/table.rs TableBuilder (C++ restatement, lcrc_tbuild.cpp): add(key, value) in key order,
    finish(filter_name, filter_block) -> the table file's bytes. host_seal=True computes every trailer CRC
    on the host as the reference does; host_seal=False leaves them zero and seal_descs() gives one
    {offset, n + 1, n + 1} descriptor per block (data, filter, metaindex, index) for Engine.batch_seal."""

    def __init__(self, block_size=4096, restart_interval=16, compression=0, mode=MODE_REF, flags=0, host_seal=True):
        self._t = lib().lcrc_tb_create(block_size, restart_interval, compression, mode, flags, 1 if host_seal else 0)
        if not self._t:
            raise LcrcError("lcrc_tb_create: bad arguments")

    def add(self, key, value):
        kp, kn, _k1 = _buf(key)
        vp, vn, _k2 = _buf(value)
        _check(lib().lcrc_tb_add(self._t, kp, kn, vp, vn), "TableBuilder.add (keys must increase)")

    def add_many(self, keys, values):
        """keys: (n, klen) u8 array, values: (n, vlen) u8 array -- n entries in one call (keys ascending)."""
        keys = np.ascontiguousarray(keys, np.uint8)
        values = np.ascontiguousarray(values, np.uint8)
        assert keys.ndim == 2 and values.ndim == 2 and len(keys) == len(values)
        _check(lib().lcrc_tb_add_many(self._t, keys.ctypes.data_as(ctypes.c_void_p), keys.shape[1],
                                      values.ctypes.data_as(ctypes.c_void_p), values.shape[1], len(keys)),
               "TableBuilder.add_many (keys must increase)")

    def flush(self):
        lib().lcrc_tb_flush(self._t)

    def finish(self, filter_name=None, filter_block=b""):
        fp, fn, _k = _buf(filter_block) if filter_block else (None, 0, None)
        name = filter_name.encode() if isinstance(filter_name, str) else filter_name
        _check(lib().lcrc_tb_finish(self._t, name, fp, fn), "TableBuilder.finish")
        n = lib().lcrc_tb_size(self._t)
        return ctypes.string_at(lib().lcrc_tb_data(self._t), n) if n else b""

    def blocks(self):
        n = lib().lcrc_tb_blocks(self._t, None, 0)
        out = np.zeros(n, TBLK_DTYPE)
        lib().lcrc_tb_blocks(self._t, out.ctypes.data_as(ctypes.c_void_p), n)
        return out

    def seal_descs(self):
        n = lib().lcrc_tb_seal_descs(self._t, None, 0)
        out = np.zeros(n, DESC_DTYPE)
        lib().lcrc_tb_seal_descs(self._t, out.ctypes.data_as(ctypes.c_void_p), n)
        return out

    def __del__(self):
        try:
            lib().lcrc_tb_destroy(self._t)
        except Exception:
            pass


def snappy_frame_decode(data):
    """Snappy framing decoder of the table walk (host): bytes, or None when corrupt."""
    data = bytes(data)
    buf = ctypes.create_string_buffer(data, len(data)) if data else None
    n = lib().lcrc_snappy_frame_decode(buf, len(data), None, 0)
    if n < 0:
        return None
    out = ctypes.create_string_buffer(max(1, n))
    lib().lcrc_snappy_frame_decode(buf, len(data), out, n)
    return out.raw[:n]
