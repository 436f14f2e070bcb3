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
    L.orc_crc_ranges_mt.restype = ctypes.c_double
    L.orc_crc_ranges_mt.argtypes = [ctypes.c_int, vp, vp, vp, sz, ctypes.c_int, vp]
    L.orc_splitmix_fill.restype = None
    L.orc_splitmix_fill.argtypes = [ctypes.c_uint64, vp, sz]
    L.orc_table_blocks_mt.restype = ctypes.c_double
    L.orc_table_blocks_mt.argtypes = [ctypes.c_int, vp, vp, vp, sz, ctypes.c_int, vp, vp]
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


def crc_ranges_mt(data, offsets, lengths, threads, algo):
    """CRC of every range on `threads` threads (contiguous shares of about equal bytes); (crcs, seconds)."""
    a = _arr(data)
    offs = np.ascontiguousarray(offsets, np.uint64)
    lens = np.ascontiguousarray(lengths, np.uint32)
    out = np.empty(len(offs), np.uint32)
    secs = lib().orc_crc_ranges_mt(algo, _p(a), _p(offs), _p(lens), len(offs), threads, _p(out))
    return out, secs


def table_blocks_mt(data, offsets, sizes, threads, algo=None):
    """read_block_from_file with verify_checksum over a table's blocks (format.rs:146-213), C restatement, threaded:
    (trailer CRCs, status per block -- 0 ok, 1 checksum mismatch, 3 bad Snappy content, 4 bad type --, seconds).
    algo: the trailers' CRC (default crc32fast, the reference's)."""
    a = _arr(data)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    sizes = np.ascontiguousarray(sizes, dtype=np.uint64)
    out = np.zeros(len(offs), np.uint32)
    st = np.zeros(len(offs), np.uint8)
    secs = lib().orc_table_blocks_mt(ALGO_PCLMUL_REF if algo is None else algo, _p(a), _p(offs), _p(sizes), len(offs),
                                     threads, _p(out), _p(st))
    return out, st, secs


def mask_array(crcs):
    """LevelDB mask of a u32 array (vectorised orc_mask): ((c >> 15) | (c << 17)) + 0xa282ead8."""
    c = np.asarray(crcs, np.uint32).astype(np.uint64)
    return ((((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF).astype(np.uint32)


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


# ---------------------------------------------------------------------------------------------------
# SSTable files (test infrastructure): a restatement of the reference's table writer and the walk of
# Table::open + read_meta + per-block verify, to generate scan inputs and the expected verdicts.
#   BlockBuilder::add / finish      <- src/sstable/block.rs:320-370
#   TableBuilder::add / flush / finish <- src/sstable/table.rs:315-454 (filter-type quirk :383-391)
#   write_block / write_raw_block   <- src/sstable/table.rs:470-529 (snappy kept iff < raw - raw/8)
#   Footer / BlockHandle            <- src/sstable/format.rs:24-118; varints util/coding.rs
#   BitWiseComparator separators    <- the bytewise FindShortestSeparator / FindShortSuccessor contract
#   Snappy framing + raw format     <- the published Snappy formats (snap crate absent)
# ---------------------------------------------------------------------------------------------------
TABLE_MAGIC = 0xdb4775248b80fb57
FOOTER_LEN = 48


def varint(v):
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def block_build(entries, restart_interval=16):
    """entries: [(key bytes, value bytes)] in key order -> block contents (block.rs:320-370)."""
    buf, restarts, last, counter = bytearray(), [0], b"", 0
    for key, value in entries:
        shared = 0
        if counter < restart_interval:
            while shared < min(len(last), len(key)) and last[shared] == key[shared]:
                shared += 1
        else:
            restarts.append(len(buf))
            counter = 0
        buf += varint(shared) + varint(len(key) - shared) + varint(len(value)) + key[shared:] + value
        counter += 1
        last = key
    for r in restarts:
        buf += _le32(r)
    buf += _le32(len(restarts))
    return bytes(buf)


def shortest_separator(start, limit):
    n = min(len(start), len(limit))
    i = 0
    while i < n and start[i] == limit[i]:
        i += 1
    if i < n:
        b = start[i]
        if b < 0xFF and b + 1 < limit[i]:
            return start[:i] + bytes([b + 1])
    return start


def short_successor(key):
    for i, b in enumerate(key):
        if b != 0xFF:
            return key[:i] + bytes([b + 1])
    return key


def snappy_compress_raw(data):
    """A valid (greedy, 4-byte-hash) Snappy raw encoding: literals and 2-byte-offset copies."""
    data = bytes(data)
    out = bytearray(varint(len(data)))
    table, i, lit = {}, 0, 0

    def literal(a, b):
        while a < b:
            n = min(b - a, 1 << 16)
            if n <= 60:
                out.append((n - 1) << 2)
            elif n <= 256:
                out.extend([60 << 2, n - 1])
            else:
                out.extend([61 << 2, (n - 1) & 0xFF, (n - 1) >> 8])
            out.extend(data[a:a + n])
            a += n

    while i + 4 <= len(data):
        k = data[i:i + 4]
        j = table.get(k)
        table[k] = i
        if j is not None and i - j < 65536:
            n = 4
            while i + n < len(data) and data[j + n] == data[i + n] and n < 64:
                n += 1
            literal(lit, i)
            off = i - j
            out.extend([((n - 1) << 2) | 2, off & 0xFF, off >> 8])
            i += n
            lit = i
        else:
            i += 1
    literal(lit, len(data))
    return bytes(out)


def snappy_frame_encode(data):
    """Snappy framing: stream identifier, then <= 64 KiB chunks [type][u24 len][masked crc32c][body]."""
    out = bytearray(b"\xff\x06\x00\x00sNaPpY")
    for a in range(0, len(data), 65536):
        chunk = bytes(data[a:a + 65536])
        c = _le32(mask(crc(chunk, 1)))
        z = snappy_compress_raw(chunk)
        typ, body = (0, c + z) if len(z) < len(chunk) - len(chunk) // 8 else (1, c + chunk)
        out += bytes([typ, len(body) & 0xFF, (len(body) >> 8) & 0xFF, len(body) >> 16]) + body
    return bytes(out)


def table_build(kvs, block_size=4096, restart_interval=16, compression=0, filter_name=None, filter_block=b"",
                mode=0, masked=False, index_restart_interval=1):
    """TableBuilder over sorted kvs -> (file bytes, [(offset, size, kind)]); kind 0 data, 1 filter,
    2 metaindex, 3 index. Trailer CRCs in `mode` (0 = crc32fast, the reference), optionally masked."""
    f = bytearray()
    blocks = []

    def raw_write(content, typ, kind):
        off = len(f)
        c = crc(bytes(content) + bytes([typ]), mode)
        if masked:
            c = mask(c)
        f.extend(content)
        f.append(typ)
        f.extend(_le32(c))
        blocks.append((off, len(content), kind))
        return off, len(content)

    def write_block(raw, kind):
        if compression == 1:
            z = snappy_frame_encode(raw)
            if len(z) < len(raw) - len(raw) // 8:
                return raw_write(z, 1, kind)
        return raw_write(raw, 0, kind)

    data, index, pending, last_key = [], [], None, b""
    for key, value in kvs:
        if pending is not None:
            index.append((shortest_separator(last_key, key), varint(pending[0]) + varint(pending[1])))
            pending = None
        data.append((key, value))
        last_key = key
        est = len(block_build(data, restart_interval))
        if est >= block_size:
            pending = write_block(block_build(data, restart_interval), 0)
            data = []
    if data:
        pending = write_block(block_build(data, restart_interval), 0)
    meta = []
    if filter_name is not None:
        fh = raw_write(filter_block, compression, 1)  # the reference's quirk: type = options.compression_type
        meta.append((b"filter" + filter_name.encode(), varint(fh[0]) + varint(fh[1])))
    mh = write_block(block_build(meta, restart_interval), 2)
    if pending is not None:
        index.append((short_successor(last_key), varint(pending[0]) + varint(pending[1])))
    # the reference's index block restarts at every entry (table.rs:272); other intervals for tests
    ih = write_block(block_build(index, index_restart_interval), 3)
    foot = bytearray(varint(mh[0]) + varint(mh[1]) + varint(ih[0]) + varint(ih[1]))
    foot += bytes(40 - len(foot)) + _le32(TABLE_MAGIC & 0xFFFFFFFF) + _le32(TABLE_MAGIC >> 32)
    f += foot
    return bytes(f), blocks


def _get_varint(buf, p, limit, bits):
    result, shift = 0, 0
    while shift <= bits - 4:
        if p >= limit:
            return None, p
        b = buf[p]
        p += 1
        result |= (b & 127) << shift
        if not b & 128:
            return result, p
        shift += 7
    return None, p


SNAPPY_MAX_BLOCK = 65536         # snap's frame.rs MAX_BLOCK_SIZE: a chunk's decoded bytes
SNAPPY_MAX_COMPRESS_BLOCK = 76490  # snap's MAX_COMPRESS_BLOCK_SIZE: FrameDecoder's body buffer, any chunk type


def _snap_varu64(z):
    """snap's bytes::read_varu64 (snap "1", Cargo.toml:15): (value mod 2**64, bytes used), or (None, 0) when no byte
    below 0x80 comes within 10 bytes (an 11th byte's shift of 70 fails checked_shl)."""
    v = 0
    for i in range(min(len(z), 10)):
        v |= (z[i] & 127) << (7 * i)
        if z[i] < 128:
            return v & ((1 << 64) - 1), i + 1
    return None, 0


def snappy_frame_decode(data):
    """Snappy framing decode with chunk CRC check as snap's read::FrameDecoder does it (format.rs:196); None when corrupt.
    Restated from the snap crate's published behaviour (the crate is absent here): the first chunk must be the stream
    identifier; a chunk longer than MAX_COMPRESS_BLOCK_SIZE (any type) is an error; a data chunk has a 4-byte masked
    CRC-32C; its decoded bytes are at most MAX_BLOCK_SIZE; 0x02..0x7f are unskippable, 0x80..0xfe skipped."""
    data, p, out, seen = bytes(data), 0, bytearray(), False
    while p < len(data):
        if len(data) - p < 4:
            return None
        typ, n = data[p], data[p + 1] | (data[p + 2] << 8) | (data[p + 3] << 16)
        p += 4
        if len(data) - p < n or n > SNAPPY_MAX_COMPRESS_BLOCK:
            return None
        body, p = data[p:p + n], p + n
        if typ == 0xFF:
            if body != b"sNaPpY":
                return None
            seen = True
            continue
        if not seen:
            return None
        if typ in (0, 1):
            if n < 4:
                return None
            want = int.from_bytes(body[:4], "little")
            chunk = body[4:] if typ == 1 else _snappy_raw(body[4:])
            if chunk is None or len(chunk) > 65536 or mask(crc(chunk, 1)) != want:
                return None
            out += chunk
        elif typ <= 0x7F:
            return None
    return bytes(out)


def _snappy_raw(z):
    ulen, p = _snap_varu64(z)
    if ulen is None or ulen > SNAPPY_MAX_BLOCK:  # snap: Header::read, then the frame decoder's dn > MAX_BLOCK_SIZE
        return None
    out = bytearray()
    while p < len(z):
        tag = z[p]
        p += 1
        t = tag & 3
        if t == 0:
            n = tag >> 2
            if n >= 60:
                nb = n - 59
                # snap's read_literal reads the length as one 4-byte word: it needs 4 input bytes after the tag
                # whatever nb is ("the literal must have length >= 61"), so a short extended literal at the end of the
                # input is an error even when its own bytes fit
                if len(z) - p < 4:
                    return None
                n = int.from_bytes(z[p:p + nb], "little")
                p += nb
            n += 1
            if len(z) - p < n:
                return None
            out += z[p:p + n]
            p += n
            continue
        if t == 1:
            if p >= len(z):
                return None
            n, off = 4 + ((tag >> 2) & 7), ((tag >> 5) << 8) | z[p]
            p += 1
        elif t == 2:
            if len(z) - p < 2:
                return None
            n, off = 1 + (tag >> 2), z[p] | (z[p + 1] << 8)
            p += 2
        else:
            if len(z) - p < 4:
                return None
            n, off = 1 + (tag >> 2), int.from_bytes(z[p:p + 4], "little")
            p += 4
        if off == 0 or off > len(out):
            return None
        for _ in range(n):
            out.append(out[-off])
    return bytes(out) if len(out) == ulen else None


def _block_entries(d):
    """(entries [(key, value)], error) of block contents d (block.rs:21-41, :124-175)."""
    if len(d) < 4:
        return None, "bad block contents, size smaller than u32"
    nr = int.from_bytes(d[-4:], "little")
    if nr > (len(d) - 4) // 4:
        return None, "bad block contents"
    restarts = len(d) - (1 + nr) * 4
    out, key, off = [], b"", 0
    while off < restarts:
        if restarts - off < 3:
            return None, "bad entry in block"
        p = off
        shared, p = _get_varint(d, p, restarts, 32)
        non_shared, p = _get_varint(d, p, restarts, 32) if shared is not None else (None, p)
        vlen, p = _get_varint(d, p, restarts, 32) if non_shared is not None else (None, p)
        if vlen is None or restarts - p < non_shared + vlen or len(key) < shared:
            return None, "bad entry in block"
        key = key[:shared] + d[p:p + non_shared]
        out.append((key, d[p + non_shared:p + non_shared + vlen]))
        off = p + non_shared + vlen
    return out, None


def table_scan_expect(f, filter_name=None, mode=0, masked=False):
    """Expected lcrc_table_scan result: ([(offset, size, kind, type, status, crc)] sorted by offset, None)
    or (None, reference error message)."""
    f = bytes(f)

    def trailer_crc(off, n):
        c = crc(f[off:off + n + 1], mode)
        return mask(c) if masked else c

    def contents(off, n, verify):
        if off > len(f) or n + 5 > len(f) - off:
            return None, "truncated block read"
        if verify and trailer_crc(off, n) != int.from_bytes(f[off + n + 1:off + n + 5], "little"):
            return None, "block checksum mismatch"
        t = f[off + n]
        if t == 0:
            return f[off:off + n], None
        if t == 1:
            d = snappy_frame_decode(f[off:off + n])
            return (d, None) if d is not None else (None, "corrupted compressed block content")
        return None, "bad block type"

    def handle(v):
        a, p = _get_varint(v, 0, len(v), 64)
        b, p = _get_varint(v, p, len(v), 64) if a is not None else (None, p)
        return (a, b) if b is not None else None

    if len(f) < FOOTER_LEN:
        return None, "file is too short to be an sstable"
    foot = f[-FOOTER_LEN:]
    if int.from_bytes(foot[40:48], "little") != TABLE_MAGIC:
        return None, "not an sstable (bad magic number)"
    mo, p = _get_varint(foot, 0, 48, 64)
    ms, p = _get_varint(foot, p, 48, 64)
    io_, p = _get_varint(foot, p, 48, 64)
    is_, p = _get_varint(foot, p, 48, 64)
    if None in (mo, ms, io_, is_):
        return None, "Error when decoding varint64"
    d, err = contents(io_, is_, True)
    if err:
        return None, err
    ents, err = _block_entries(d)
    if err:
        return None, err
    found = []
    for _, v in ents:
        h = handle(v)
        if h is None:
            return None, "Error when decoding varint64"
        found.append((h[0], h[1], 0))
    if filter_name is not None:
        md, err = contents(mo, ms, True)
        if not err:
            mes, err = _block_entries(md)
            if not err:
                want = b"filter" + filter_name.encode()
                for k, v in mes:
                    if k < want:
                        continue
                    if k == want and handle(v) is not None:
                        found.append((*handle(v), 1))
                    break
    found += [(mo, ms, 2), (io_, is_, 3)]
    found.sort(key=lambda b: b[0])
    out = []
    for off, n, kind in found:
        if off > len(f) or n + 5 > len(f) - off:
            out.append((off, n, kind, 0xFF, 2, 0))
            continue
        c = trailer_crc(off, n)
        st = 0 if c == int.from_bytes(f[off + n + 1:off + n + 5], "little") else 1
        # read_block_from_file's type dispatch after a good checksum (format.rs:175-210)
        if st == 0 and f[off + n] == 1 and snappy_frame_decode(f[off:off + n]) is None:
            st = 3  # "corrupted compressed block content"
        elif st == 0 and f[off + n] > 1:
            st = 4  # "bad block type"
        out.append((off, n, kind, f[off + n], st, c))
    return out, None
