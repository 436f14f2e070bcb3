"""TEST INFRASTRUCTURE -- CPU oracle for the leveldb-rust checksum path.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import this module, and
only as the checker / CPU baseline. It is never on the product path.

Contents:
* ctypes binding of ``_build/liboracle.so`` (crc_oracle.c): the bitwise CRC definition, slice-by-16,
  the PCLMULQDQ folding path of crc32fast and the SSE4.2 path of snap, multi-threaded timing.
* A pure-Python restatement of the reference's framing (small cases only):
    - ``log_write``  <- LogWriter::add_record / emit_physical_record, src/db/log.rs:21-52, :58-80
    - ``log_read_all`` <- LogReader::read_record / read_physical_record, src/db/log.rs:106-279
    - ``raw_block`` / ``read_block`` <- src/sstable/table.rs:507-529, src/sstable/format.rs:146-213
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
POLY_REF, POLY_C = 0xEDB88320, 0x82F63B78
ALGO_BITWISE_REF, ALGO_BITWISE_C, ALGO_S16_REF, ALGO_S16_C, ALGO_PCLMUL_REF, ALGO_SSE42_C = range(6)

_L = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _L
    if _L is not None:
        return _L
    if not os.path.exists(LIB):
        build()
    L = ctypes.CDLL(LIB)
    u32, sz, vp = ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p
    L.orc_crc_bitwise.restype = u32
    L.orc_crc_bitwise.argtypes = [u32, u32, u32, vp, sz]
    L.orc_crc_s16.restype = u32
    L.orc_crc_s16.argtypes = [ctypes.c_int, u32, vp, sz]
    L.orc_crc_pclmul.restype = u32
    L.orc_crc_pclmul.argtypes = [u32, vp, sz]
    L.orc_crc_sse42.restype = u32
    L.orc_crc_sse42.argtypes = [u32, vp, sz]
    L.orc_mask.restype = u32
    L.orc_mask.argtypes = [u32]
    L.orc_unmask.restype = u32
    L.orc_unmask.argtypes = [u32]
    L.orc_crc_ranges.restype = None
    L.orc_crc_ranges.argtypes = [ctypes.c_int, vp, vp, vp, sz, vp]
    L.orc_crc_uniform_mt.restype = ctypes.c_double
    L.orc_crc_uniform_mt.argtypes = [ctypes.c_int, vp, sz, sz, sz, ctypes.c_int, vp]
    L.orc_splitmix_fill.restype = None
    L.orc_splitmix_fill.argtypes = [ctypes.c_uint64, vp, sz]
    _L = L
    return L


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _arr(data):
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, dtype=np.uint8)
    return np.frombuffer(bytes(data), dtype=np.uint8)


def crc_bitwise(data, mode=0):
    a = _arr(data)
    return lib().orc_crc_bitwise(POLY_C if mode else POLY_REF, 0xFFFFFFFF, 0xFFFFFFFF, _p(a), a.nbytes)


def crc(data, mode=0, initial=0):
    """Fast oracle (slice-by-16), pinned against crc_bitwise and zlib in tests/test_oracle.py."""
    a = _arr(data)
    return lib().orc_crc_s16(1 if mode else 0, initial, _p(a), a.nbytes)


def crc_pclmul(data):
    a = _arr(data)
    return lib().orc_crc_pclmul(0, _p(a), a.nbytes)


def crc_sse42(data):
    a = _arr(data)
    return lib().orc_crc_sse42(0, _p(a), a.nbytes)


def mask(c):
    return lib().orc_mask(c)


def unmask(m):
    return lib().orc_unmask(m)


def crc_ranges(data, offsets, lengths, mode=0, algo=None):
    a = _arr(data)
    offs = np.ascontiguousarray(offsets, np.uint64)
    lens = np.ascontiguousarray(lengths, np.uint32)
    out = np.empty(len(offs), np.uint32)
    if algo is None:
        algo = ALGO_S16_C if mode else ALGO_S16_REF
    lib().orc_crc_ranges(algo, _p(a), _p(offs), _p(lens), len(offs), _p(out))
    return out


def crc_uniform_mt(data, nblocks, blen, stride, threads, algo):
    """Returns (crcs, seconds) -- the CPU baseline timing primitive."""
    a = _arr(data)
    out = np.empty(nblocks, np.uint32)
    secs = lib().orc_crc_uniform_mt(algo, _p(a), nblocks, blen, stride, threads, _p(out))
    return out, secs


def splitmix_bytes(seed, n):
    out = np.empty(n, np.uint8)
    lib().orc_splitmix_fill(seed, _p(out), n)
    return out


# ---------------------------------------------------------------------------------------------------
# Pure-Python restatement of the reference framing (small inputs)
# ---------------------------------------------------------------------------------------------------
BLOCK_SIZE, HEADER_SIZE = 32768, 7
FULL, FIRST, MIDDLE, LAST = 1, 2, 3, 4


def _le32(v):
    return bytes([v & 0xFF, (v >> 8) & 0xFF, (v >> 16) & 0xFF, (v >> 24) & 0xFF])


def log_write(records, offset=0):
    """LogWriter::add_record for each record; returns the file bytes (log.rs:21-80)."""
    out = bytearray()
    for rec in records:
        rec = bytes(rec)
        pos, begin = 0, True
        while pos < len(rec):  # empty records emit nothing (log.rs:24-26)
            leftover = BLOCK_SIZE - offset
            if leftover < HEADER_SIZE:
                out += b"\x00" * leftover
                offset = 0
            avail = BLOCK_SIZE - offset - HEADER_SIZE
            left = len(rec) - pos
            if begin:
                t, n = (FULL, left) if left <= avail else (FIRST, avail)
            else:
                t, n = (LAST, left) if left <= avail else (MIDDLE, avail)
            data = rec[pos:pos + n]
            c = crc(bytes([t]) + data)
            out += _le32(c) + bytes([n & 0xFF, n >> 8, t]) + data
            offset += HEADER_SIZE + n
            pos += n
            begin = False
    return bytes(out)


def log_read_all(data):
    """LogReader over an in-memory file (log.rs:106-279). Returns (records, dropped, message)."""
    data = bytes(data)
    st = {"file_pos": 0, "buf": b"", "consumed": 0, "cap": 0, "eof": False, "dropped": 0, "msg": ""}

    def report(n, m):
        st["dropped"] += n
        st["msg"] += m

    def physical(record):
        while True:
            if st["cap"] - st["consumed"] < HEADER_SIZE:
                if not st["eof"]:
                    st["consumed"] = 0
                    chunk = data[st["file_pos"]:st["file_pos"] + BLOCK_SIZE]
                    st["file_pos"] += len(chunk)
                    st["buf"], st["cap"] = chunk, len(chunk)
                    if len(chunk) < BLOCK_SIZE:
                        st["eof"] = True
                    continue
                st["consumed"] = st["cap"] = 0
                return 5, 0  # Eof
            h = st["buf"][st["consumed"]:st["consumed"] + HEADER_SIZE]
            checksum = int.from_bytes(h[0:4], "little")
            length = h[4] | (h[5] << 8)
            t = h[6]
            if HEADER_SIZE + length > st["cap"] - st["consumed"]:
                dropped = st["cap"] - st["consumed"]
                st["consumed"] = st["cap"] = 0
                if not st["eof"]:
                    report(dropped, "bad record length")
                    return 6, 0
                return 5, 0
            if t == 0 and length == 0:
                st["consumed"] = st["cap"] = 0
                return 6, 0
            body = st["buf"][st["consumed"] + HEADER_SIZE:st["consumed"] + HEADER_SIZE + length]
            if checksum != crc(bytes([t]) + body):
                dropped = st["cap"] - st["consumed"]
                st["consumed"] = st["cap"] = 0
                report(dropped, "checksum mismatch")
                return 6, length
            st["consumed"] += HEADER_SIZE + length
            record += body
            return (t if t <= 6 else 7), length

    def read_record():
        record = bytearray()
        in_frag = False
        while True:
            t, n = physical(record)
            if t == FULL:
                if in_frag and record:
                    dropped = len(record) - n
                    if dropped > 0:
                        report(dropped, "partial record without end(1)")
                    del record[:dropped]
                return bytes(record)
            if t == FIRST:
                if in_frag and record:
                    dropped = len(record) - n
                    if dropped > 0:
                        report(dropped, "partial record without end(2)")
                    del record[:dropped]
                in_frag = True
            elif t == MIDDLE:
                if not in_frag:
                    report(n, "missing start of fragmented record(1)")
                    del record[len(record) - n:]
            elif t == LAST:
                if not in_frag:
                    report(n, "missing start of fragmented record(2)")
                    del record[len(record) - n:]
                else:
                    return bytes(record)
            elif t == 5:
                return None
            elif t == 6:
                if in_frag:
                    report(len(record), "error in middle of record")
                    record.clear()
                    in_frag = False
            else:
                report(len(record), "unknown record type")
                in_frag = False
                record.clear()

    out = []
    while True:
        r = read_record()
        if r is None:
            return out, st["dropped"], st["msg"]
        out.append(r)


def raw_block(content, block_type):
    """write_raw_block bytes: content ++ [type][crc32(content ++ type) LE] (table.rs:507-529)."""
    content = bytes(content)
    return content + bytes([block_type]) + _le32(crc(content + bytes([block_type])))


def read_block(file_bytes, offset, n, verify):
    """format.rs:146-213 up to the type dispatch: (type, None) or (None, error)."""
    if offset > len(file_bytes) or n + 5 > len(file_bytes) - offset:
        return None, "truncated block read"
    d = file_bytes[offset:offset + n + 5]
    if verify and int.from_bytes(d[n + 1:n + 5], "little") != crc(d[:n + 1]):
        return None, "block checksum mismatch"
    if d[n] not in (0, 1):
        return None, "bad block type"
    return d[n], None
