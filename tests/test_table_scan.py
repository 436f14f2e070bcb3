"""Whole-table verify scan and the writer-side batch seal (rank 3).

lcrc_table_scan restates Table::open with paranoid_checks (src/sstable/table.rs:39-103: footer, index
block verified, read_meta's metaindex + "filter"<name> entry) followed by read_block_from_file with
verify_checksum for every block (src/sstable/format.rs:146-171); the checksums run in one batched device
pass. Expected results come from the oracle's restatement (oracle.table_scan_expect) on tables written by
the oracle's TableBuilder restatement (oracle.table_build). Snappy framing (the `snap` crate is absent,
SURVEY §8(c)): the C++ decoder is checked against the oracle's independent encoder and decoder --
parity with snap itself is unpinned.
"""
import os

import numpy as np
import pytest

FILTER = "leveldb.BuiltinBloomFilter2"  # src/util/filter.rs:56-58


def _kvs(n, seed, vlen=40):
    rng = np.random.default_rng(seed)
    keys = sorted({bytes(rng.integers(97, 123, int(rng.integers(4, 24)), dtype=np.uint8)) for _ in range(n)})
    out = []
    for k in keys:
        v = rng.integers(0, 256, int(rng.integers(0, vlen)), dtype=np.uint8).tobytes()
        out.append((k, v + b"x" * int(rng.integers(0, vlen))))  # compressible tails
    return out


# ---------------------------------------------------------------------------------------------------
# CPU: Snappy framing decoder and the oracle's table writer / walk
# ---------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n", [0, 1, 59, 60, 61, 255, 256, 257, 65535, 65536, 65537, 200000])
def test_snappy_frame_roundtrip(lcrc, orc, n):
    rng = np.random.default_rng(n)
    a = rng.integers(0, 256, n // 2, dtype=np.uint8).tobytes()
    data = (a + b"leveldb" * (n // 14 + 1))[:n]
    z = orc.snappy_frame_encode(data)
    assert orc.snappy_frame_decode(z) == data
    assert lcrc.snappy_frame_decode(z) == data


def test_snappy_frame_corruption(lcrc, orc):
    data = b"abcdefgh" * 5000 + os.urandom(1000)
    z = bytearray(orc.snappy_frame_encode(data))
    assert lcrc.snappy_frame_decode(bytes(z)) == data
    bad = bytearray(z)
    bad[12] ^= 1  # chunk CRC (masked CRC-32C of the uncompressed chunk)
    assert lcrc.snappy_frame_decode(bytes(bad)) is None and orc.snappy_frame_decode(bytes(bad)) is None
    assert lcrc.snappy_frame_decode(bytes(z[10:])) is None  # no stream identifier
    pad = bytes(z[:10]) + b"\xfe\x03\x00\x00abc" + bytes(z[10:])  # padding chunk is skipped
    assert lcrc.snappy_frame_decode(pad) == data
    skip = bytes(z[:10]) + b"\x80\x01\x00\x00q" + bytes(z[10:])  # reserved skippable
    assert lcrc.snappy_frame_decode(skip) == data
    unskip = bytes(z[:10]) + b"\x02\x01\x00\x00q" + bytes(z[10:])  # reserved unskippable
    assert lcrc.snappy_frame_decode(unskip) is None and orc.snappy_frame_decode(unskip) is None
    assert lcrc.snappy_frame_decode(bytes(z[:-1])) is None  # truncated


def test_oracle_table_walk_is_consistent(orc):
    kvs = _kvs(3000, 1)
    for compression in (0, 1):
        f, blocks = orc.table_build(kvs, compression=compression, filter_name=FILTER, filter_block=b"F" * 77)
        got, err = orc.table_scan_expect(f, FILTER)
        assert err is None
        assert [(b[0], b[1], b[2]) for b in got] == sorted(blocks)
        assert [b[3] for b in got if b[2] == 1] == [compression]  # filter type quirk (table.rs:383-391)
        # ... which makes the raw filter block of a Snappy table unreadable for read_block_from_file:
        # "corrupted compressed block content" (status 3); every other block is clean
        assert [b[4] for b in got if b[2] == 1] == [3 if compression else 0]
        assert all(b[4] == 0 for b in got if b[2] != 1)


# ---------------------------------------------------------------------------------------------------
# GPU: the scan and the seal through the C ABI
# ---------------------------------------------------------------------------------------------------
def _scan(lcrc, eng, f, filter_name=None):
    dev = lcrc.DeviceBuffer.from_host(np.frombuffer(f, np.uint8).copy() if len(f) else np.zeros(1, np.uint8))
    try:
        return eng.table_scan(dev, len(f), filter_name), None
    except lcrc.TableCorruption as e:
        return None, str(e)
    finally:
        dev.close()


def _as_tuples(arr):
    return [(int(b["offset"]), int(b["size"]), int(b["kind"]), int(b["type"]), int(b["status"]),
             int(b["crc"]) if b["status"] != 2 else 0) for b in arr]


@pytest.mark.gpu
@pytest.mark.parametrize("compression", [0, 1])
@pytest.mark.parametrize("filt", [None, FILTER])
@pytest.mark.parametrize("block_size", [256, 4096, 65536])
def test_table_scan_clean(lcrc, orc, engines, compression, filt, block_size):
    kvs = _kvs(4000, block_size + compression)
    f, _ = orc.table_build(kvs, block_size=block_size, compression=compression, filter_name=filt,
                           filter_block=os.urandom(300))
    got, err = _scan(lcrc, engines[lcrc.MODE_REF], f, filt)
    want, werr = orc.table_scan_expect(f, filt)
    assert err is None and werr is None
    assert _as_tuples(got) == want
    # clean, except the raw filter block of a Snappy table (table.rs:383-391: unreadable, status 3)
    quirk = (got["kind"] == 1) & (compression == 1)
    assert (got["status"][~quirk] == 0).all() and (got["status"][quirk] == 3).all()


@pytest.mark.gpu
def test_table_scan_masked_crc32c(lcrc, orc):
    """A table whose trailers are LevelDB-masked CRC-32C, scanned by a C-mode masked context."""
    eng = lcrc.Engine(0, lcrc.MODE_C, lcrc.FLAG_MASK)
    try:
        f, _ = orc.table_build(_kvs(2000, 7), compression=1, filter_name=FILTER, filter_block=b"q" * 64,
                               mode=1, masked=True)
        got, err = _scan(lcrc, eng, f, FILTER)
        want, _ = orc.table_scan_expect(f, FILTER, mode=1, masked=True)
        assert err is None and _as_tuples(got) == want and (got["status"][got["kind"] != 1] == 0).all()
        # a crc32fast context sees every block as a mismatch, and the index first of all
        _, err = _scan(lcrc, lcrc.Engine(0, lcrc.MODE_REF), f, FILTER)
        assert err == "block checksum mismatch"
    finally:
        eng.close()


@pytest.mark.gpu
def test_table_scan_block_corruption(lcrc, orc, engines):
    f, blocks = orc.table_build(_kvs(3000, 11), block_size=1024, compression=1, filter_name=FILTER,
                                filter_block=b"z" * 200)
    data = [b for b in blocks if b[2] == 0]
    g = bytearray(f)
    hit = [data[0], data[len(data) // 2], data[-1]]
    for off, n, _ in hit:
        g[off + n // 2] ^= 0x10  # payload byte
    fb = [b for b in blocks if b[2] == 1][0]
    g[fb[0] + fb[1] + 2] ^= 0x01  # the filter block's stored crc
    got, err = _scan(lcrc, engines[lcrc.MODE_REF], bytes(g), FILTER)
    want, werr = orc.table_scan_expect(bytes(g), FILTER)
    assert err is None and werr is None and _as_tuples(got) == want
    bad = {(int(b["offset"]), int(b["kind"])) for b in got if b["status"] == 1}
    assert bad == {(h[0], 0) for h in hit} | {(fb[0], 1)}


@pytest.mark.gpu
def test_table_scan_structural_errors(lcrc, orc, engines):
    eng = engines[lcrc.MODE_REF]
    f, blocks = orc.table_build(_kvs(1500, 5), compression=1, filter_name=FILTER, filter_block=b"y" * 10)
    cases = {"short": f[-47:], "magic": f[:-1] + bytes([f[-1] ^ 1])}
    ih = [b for b in blocks if b[2] == 3][0]
    g = bytearray(f)
    g[ih[0] + 1] ^= 0x20
    cases["index crc"] = bytes(g)
    g = bytearray(f)
    g[ih[0] + ih[1]] = 7  # index type byte (also breaks its crc -> mismatch is reported first)
    cases["index type"] = bytes(g)
    for name, case in cases.items():
        got, err = _scan(lcrc, eng, case, FILTER)
        want, werr = orc.table_scan_expect(case, FILTER)
        assert got is None and err == werr, name
    assert _scan(lcrc, eng, cases["short"])[1] == "file is too short to be an sstable"
    assert _scan(lcrc, eng, cases["magic"])[1] == "not an sstable (bad magic number)"
    assert _scan(lcrc, eng, cases["index crc"])[1] == "block checksum mismatch"


def _handcrafted(orc, index_entries, meta_entries=(), index_type=0):
    """A table whose index block is built directly from (key, value bytes) -- for malformed handles."""
    f = bytearray(orc.raw_block(b"D" * 100, 0))
    meta = orc.block_build(list(meta_entries))
    moff = len(f)
    f += orc.raw_block(meta, 0)
    idx = orc.block_build(list(index_entries))
    if index_type == 1:
        idx = orc.snappy_frame_encode(idx)
    ioff = len(f)
    f += orc.raw_block(idx, index_type)
    foot = orc.varint(moff) + orc.varint(len(meta)) + orc.varint(ioff) + orc.varint(len(idx))
    foot += bytes(40 - len(foot)) + (orc.TABLE_MAGIC).to_bytes(8, "little")
    return bytes(f + foot)


@pytest.mark.gpu
def test_table_scan_handles(lcrc, orc, engines):
    eng = engines[lcrc.MODE_REF]
    v = orc.varint
    # a handle past the end of the file is reported TRUNCATED, the others are verified
    f = _handcrafted(orc, [(b"a", v(0) + v(100)), (b"b", v(10 ** 6) + v(50))])
    got, err = _scan(lcrc, eng, f)
    want, _ = orc.table_scan_expect(f)
    assert err is None and _as_tuples(got) == want
    assert [int(b["status"]) for b in got] == [0, 0, 0, 2]
    # a malformed handle varint in the index
    f = _handcrafted(orc, [(b"a", b"\xff\xff")])
    assert _scan(lcrc, eng, f)[1] == orc.table_scan_expect(f)[1] == "Error when decoding varint64"
    # a snappy-compressed index block
    f = _handcrafted(orc, [(b"a", v(0) + v(100))], index_type=1)
    got, err = _scan(lcrc, eng, f)
    assert err is None and _as_tuples(got) == orc.table_scan_expect(f)[0]
    # compressed index whose crc is right but whose framing is not
    ih = [b for b in _as_tuples(got) if b[2] == 3][0]
    body = bytearray(orc.snappy_frame_encode(orc.block_build([(b"a", v(0) + v(100))])))
    body[-1] ^= 0xFF
    g = bytearray(f[:ih[0]]) + orc.raw_block(bytes(body), 1) + bytes(f[-48:])  # same sizes, same footer
    assert _scan(lcrc, eng, bytes(g))[1] == orc.table_scan_expect(bytes(g))[1] == "corrupted compressed block content"
    # metaindex without the filter entry, and a metaindex that is corrupt: read_meta's errors are swallowed
    f = _handcrafted(orc, [(b"a", v(0) + v(100))], meta_entries=[(b"filterother", v(0) + v(1))])
    got, err = _scan(lcrc, eng, f, FILTER)
    assert err is None and [int(b["kind"]) for b in got] == [0, 2, 3]
    # a block whose entries overrun the restart array
    bad_index = bytes([0, 5, 9]) + b"ab" + (0).to_bytes(4, "little") + (1).to_bytes(4, "little")
    g = bytearray(orc.raw_block(b"D" * 10, 0))
    ioff = len(g)
    g += orc.raw_block(bad_index, 0)
    foot = orc.varint(0) + orc.varint(10) + orc.varint(ioff) + orc.varint(len(bad_index))
    g += foot + bytes(40 - len(foot)) + orc.TABLE_MAGIC.to_bytes(8, "little")
    assert _scan(lcrc, eng, bytes(g))[1] == orc.table_scan_expect(bytes(g))[1] == "bad entry in block"


@pytest.mark.gpu
def test_table_scan_query_and_range(lcrc, orc, engines):
    import ctypes
    f, blocks = orc.table_build(_kvs(800, 3))
    dev = lcrc.DeviceBuffer.from_host(np.frombuffer(f, np.uint8).copy())
    n = ctypes.c_size_t(0)
    rc = lcrc.lib().lcrc_table_scan(engines[lcrc.MODE_REF].ctx, dev.ptr, len(f), None, None, 0, ctypes.byref(n),
                                    None, 0)
    assert rc == lcrc.ERANGE and n.value == len(blocks)
    dev.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode,flags", [(0, 0), (1, 1)])
def test_seal_table_trailers(lcrc, orc, mode, flags):
    """Writer side: trailers computed and stored by one device call equal write_raw_block's bytes."""
    eng = lcrc.Engine(0, mode, flags)
    try:
        f, blocks = orc.table_build(_kvs(3000, 21), block_size=2048, compression=1, filter_name=FILTER,
                                    filter_block=b"w" * 99, mode=mode, masked=bool(flags))
        blank = np.frombuffer(f, np.uint8).copy()
        for off, n, _ in blocks:
            blank[off + n + 1:off + n + 5] = 0
        d = np.zeros(len(blocks), lcrc.DESC_DTYPE)
        d["offset"] = [b[0] for b in blocks]
        d["length"] = [b[1] + 1 for b in blocks]
        d["expect_rel"] = [b[1] + 1 for b in blocks]
        dev = lcrc.DeviceBuffer.from_host(blank)
        dd = lcrc.DeviceBuffer.from_host(d.view(np.uint8))
        out = lcrc.DeviceBuffer(4 * len(blocks))
        eng.batch_seal(dev, len(f), dd, len(blocks), out)
        eng.sync()
        assert dev.download(np.uint8, len(f)).tobytes() == f
        got = out.download(np.uint32, len(blocks))
        want = [int.from_bytes(f[o + n + 1:o + n + 5], "little") for o, n, _ in blocks]
        assert got.tolist() == want
        for b in (dev, dd, out):
            b.close()
    finally:
        eng.close()


@pytest.mark.gpu
def test_seal_wal_headers(lcrc, orc, engines):
    """Writer side, WAL group commit: every header crc of a log (log.rs:61-70) filled in by one call."""
    rng = np.random.default_rng(4)
    recs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 70000, 60)]
    f = orc.log_write(recs)
    heads = []
    p = 0
    while p + 7 <= len(f):
        blk_left = 32768 - p % 32768
        if blk_left < 7:
            p += blk_left
            continue
        n = f[p + 4] | (f[p + 5] << 8)
        if f[p + 6] == 0 and n == 0:
            break
        heads.append((p, n))
        p += 7 + n
    blank = np.frombuffer(f, np.uint8).copy()
    for h, _ in heads:
        blank[h:h + 4] = 0
    d = np.zeros(len(heads), lcrc.DESC_DTYPE)
    d["offset"] = [h + 6 for h, _ in heads]
    d["length"] = [n + 1 for _, n in heads]
    d["expect_rel"] = -6
    dev = lcrc.DeviceBuffer.from_host(blank)
    dd = lcrc.DeviceBuffer.from_host(d.view(np.uint8))
    eng = engines[lcrc.MODE_REF]
    eng.batch_seal(dev, len(f), dd, len(heads))
    eng.sync()
    assert dev.download(np.uint8, len(f)).tobytes() == f
    dev.close()
    dd.close()


# ---------------------------------------------------------------------------------------------------
# Snappy framing on the device (§8(f) rank 4): decode + masked CRC-32C of every chunk
# ---------------------------------------------------------------------------------------------------
def _frames_on_device(lcrc, streams):
    blob = b"".join(streams)
    offs = np.cumsum([0] + [len(x) for x in streams])[:-1]
    d = np.zeros(len(streams), lcrc.DESC_DTYPE)
    d["offset"], d["length"], d["expect_rel"] = offs, [len(x) for x in streams], lcrc.NO_EXPECT
    base = lcrc.DeviceBuffer.from_host(np.frombuffer(blob, np.uint8) if blob else np.zeros(1, np.uint8))
    dd = lcrc.DeviceBuffer.from_host(d.view(np.uint8) if len(d) else np.zeros(16, np.uint8))
    return base, dd


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_snappy_frames_device(lcrc, orc, engines, mode):
    rng = np.random.default_rng(9)
    raw = []
    for k in range(300):
        n = int(rng.integers(0, 3 * 65536)) if k % 50 == 0 else int(rng.integers(0, 6000))
        a = rng.integers(0, 256, n // 2, dtype=np.uint8).tobytes()
        raw.append((a + b"leveldb-rust " * (n // 13 + 1))[:n])
    streams = [orc.snappy_frame_encode(x) for x in raw]
    # uncompressed data chunks, padding, skippable chunks and a repeated stream identifier
    streams.append(bytes(streams[1][:10]) + b"\x01\x09\x00\x00" + orc.mask(orc.crc(b"abcde", 1)).to_bytes(4, "little")
                   + b"abcde" + b"\xfe\x02\x00\x00zz" + b"\x85\x01\x00\x00q" + bytes(streams[1][:10]))
    raw.append(b"abcde")
    base, dd = _frames_on_device(lcrc, streams)
    got, status = engines[mode].snappy_frames(base, dd, len(streams))
    assert status.tolist() == [0] * len(streams)
    assert got == raw


@pytest.mark.gpu
def test_snappy_frames_device_corruption(lcrc, orc, engines):
    good = orc.snappy_frame_encode(b"abcdefgh" * 3000 + bytes(range(256)) * 10)
    cases = {
        "chunk crc": bytearray(good),
        "no stream id": bytearray(good[10:]),
        "truncated": bytearray(good[:-3]),
        "unskippable": bytearray(good[:10] + b"\x02\x01\x00\x00q" + good[10:]),
        "bad literal": bytearray(good),
    }
    cases["chunk crc"][12] ^= 1
    cases["bad literal"][len(good) - 5] ^= 0x40
    streams = [good] + [bytes(v) for v in cases.values()] + [good]
    base, dd = _frames_on_device(lcrc, streams)
    got, status = engines[lcrc.MODE_REF].snappy_frames(base, dd, len(streams))
    want = [0 if orc.snappy_frame_decode(s) is not None else 1 for s in streams]
    assert [int(x != 0) for x in status] == want
    assert want[1:-1] == [1] * len(cases)
    assert got[0] == got[-1] == orc.snappy_frame_decode(good)


@pytest.mark.gpu
def test_table_scan_compressed_content(lcrc, orc, engines):
    """Snappy-framed data blocks whose trailer crc is right but whose frames are not: the device decode
    reports "corrupted compressed block content" (status 3), a type byte > 1 "bad block type" (4)."""
    f, blocks = orc.table_build(_kvs(3000, 31), block_size=2048, compression=1)
    data = [b for b in blocks if b[2] == 0]
    g = bytearray(f)
    comp = [b for b in data if g[b[0] + b[1]] == 1]
    assert len(comp) >= 3
    for off, n, _ in comp[:2]:
        g[off + n - 3] ^= 0x5A  # inside the frame
        c = orc.crc(bytes(g[off:off + n + 1]), 0)
        g[off + n + 1:off + n + 5] = c.to_bytes(4, "little")  # ... and a trailer that matches it
    off, n, _ = comp[2]
    g[off + n] = 7
    g[off + n + 1:off + n + 5] = orc.crc(bytes(g[off:off + n + 1]), 0).to_bytes(4, "little")
    got, err = _scan(lcrc, engines[lcrc.MODE_REF], bytes(g))
    want, werr = orc.table_scan_expect(bytes(g))
    assert err is None and werr is None and _as_tuples(got) == want
    st = {int(b["offset"]): int(b["status"]) for b in got}
    assert [st[b[0]] for b in comp[:3]] == [3, 3, 4]


@pytest.mark.gpu
@pytest.mark.parametrize("interval", [1, 16, 1000])
def test_table_scan_index_restart_intervals(lcrc, orc, engines, interval):
    """Index blocks with several entries per restart segment (walked per segment on the device) and one
    with a single huge segment (the host walk)."""
    f, _ = orc.table_build(_kvs(6000, 41), block_size=512, compression=1, index_restart_interval=interval)
    got, err = _scan(lcrc, engines[lcrc.MODE_REF], f)
    want, werr = orc.table_scan_expect(f)
    assert err is None and werr is None and _as_tuples(got) == want
    assert (got["status"] == 0).all()


def _snappy_elements(rng, target):
    """A valid Snappy raw stream of random elements in every encoding the format has (literals with 0-4
    extra length bytes, 1-, 2- and 4-byte-offset copies, overlapping copies with offsets 1..8); returns
    (compressed, decoded)."""
    out, z = bytearray(), bytearray()
    while len(out) < target:
        if not out or rng.random() < 0.25:
            n = int(rng.choice([rng.integers(1, 61), rng.integers(61, 300), rng.integers(256, 2000)]))
            need = 0 if n <= 60 else 1 if n <= 256 else 2
            nb = need if rng.random() < 0.6 else int(rng.integers(max(need, 1), 5))
            if nb == 0:
                z.append((n - 1) << 2)
            else:
                z.append((59 + nb) << 2)
                z += (n - 1).to_bytes(nb, "little")
            lit = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            z += lit
            out += lit
            continue
        kind = int(rng.integers(1, 4))
        near = rng.random() < 0.3
        if kind == 1:
            n = int(rng.integers(4, 12))
            off = int(rng.integers(1, min(len(out), 8 if near else 2047) + 1))
            z += bytes([((off >> 8) << 5) | ((n - 4) << 2) | 1, off & 0xFF])
        else:
            n = int(rng.integers(1, 65))
            off = int(rng.integers(1, min(len(out), 8 if near else 65535) + 1))
            z += bytes([((n - 1) << 2) | kind]) + off.to_bytes(2 if kind == 2 else 4, "little")
        for _ in range(n):
            out.append(out[-off])
    return orc_varint(len(out)) + bytes(z), bytes(out)


def orc_varint(v):
    b = bytearray()
    while v >= 128:
        b.append((v & 127) | 128)
        v >>= 7
    b.append(v)
    return bytes(b)


@pytest.mark.gpu
def test_snappy_frames_device_all_element_forms(lcrc, orc, engines):
    """Every element encoding, overlapping copies, chunks on both sides of the LDS staging (8 KiB), and
    random single-byte corruptions: status and contents against the oracle's decoder."""
    rng = np.random.default_rng(2024)
    streams, want = [], []
    for k in range(400):
        target = int(rng.integers(1, 20000)) if k % 7 == 0 else int(rng.integers(1, 6000))
        z, raw = _snappy_elements(rng, target)
        assert orc._snappy_raw(z) == raw
        body = orc.mask(orc.crc(raw, 1)).to_bytes(4, "little") + z
        s = bytearray(b"\xff\x06\x00\x00sNaPpY" + bytes([0, len(body) & 0xFF, (len(body) >> 8) & 0xFF,
                                                          len(body) >> 16]) + body)
        if k % 3 == 2:  # corrupt one element byte (the oracle says whether the frame still decodes)
            p = 18 + int(rng.integers(0, len(z)))
            s[p] ^= 1 << int(rng.integers(0, 8))
        streams.append(bytes(s))
        want.append(orc.snappy_frame_decode(bytes(s)))
    base, dd = _frames_on_device(lcrc, streams)
    got, status = engines[lcrc.MODE_C].snappy_frames(base, dd, len(streams))
    assert [int(x != 0) for x in status] == [int(w is None) for w in want]
    for g_, w_ in zip(got, want):
        if w_ is not None:
            assert g_ == w_
    assert sum(w is None for w in want) > 20


@pytest.mark.gpu
@pytest.mark.parametrize("compression", [0, 1])
def test_table_scan_long_filter_policy_name(lcrc, orc, engines, compression):
    """A filter policy name longer than the device-only scan's metaindex key (124 B): read_meta opens such a
    table (table.rs:86-112), so the synchronous lcrc_table_scan leaves it to the host-assisted walk instead of
    failing -- the same blocks, crcs and statuses as the oracle's walk, the filter block found."""
    name = "leveldb.LongFilterPolicy." + "x" * 150
    f, _ = orc.table_build(_kvs(2500, 31 + compression), compression=compression, filter_name=name,
                           filter_block=os.urandom(200))
    got, err = _scan(lcrc, engines[lcrc.MODE_REF], f, name)
    want, werr = orc.table_scan_expect(f, name)
    assert err is None and werr is None
    assert _as_tuples(got) == want
    assert (got["kind"] == 1).sum() == 1


def test_oracle_table_blocks_c_matches_python_walk(orc):
    """The C restatement the bench times as the table scan's CPU baseline (orc_table_blocks_mt: trailer CRC, type
    dispatch, Snappy frame decode and chunk CRCs, format.rs:146-213) gives the Python walk's verdict for every block of
    a compressed table, clean and with corrupted trailers, frames and types, on 1 and 4 threads."""
    f, blocks = orc.table_build(_kvs(3000, 17), block_size=1024, compression=1, filter_name=FILTER,
                                filter_block=b"c" * 100)
    g = bytearray(f)
    data = [b for b in blocks if b[2] == 0]
    comp = [b for b in data if g[b[0] + b[1]] == 1]
    off, n, _ = data[3]
    g[off + n // 2] ^= 0x01  # trailer mismatch
    for off, n, _ in comp[5:7]:  # a frame that does not decode or check, trailer re-sealed
        g[off + n - 2] ^= 0x40
        g[off + n + 1:off + n + 5] = orc.crc(bytes(g[off:off + n + 1]), 0).to_bytes(4, "little")
    off, n, _ = comp[9]
    g[off + n] = 9  # bad type, re-sealed
    g[off + n + 1:off + n + 5] = orc.crc(bytes(g[off:off + n + 1]), 0).to_bytes(4, "little")
    for case in (f, bytes(g)):
        want, err = orc.table_scan_expect(case, FILTER)
        assert err is None
        offs = [w[0] for w in want]
        sizes = [w[1] for w in want]
        for threads in (1, 4):
            crcs, st, _ = orc.table_blocks_mt(case, offs, sizes, threads)
            assert [(int(c), int(s)) for c, s in zip(crcs, st)] == [(w[5], w[4]) for w in want]
    assert {w[4] for w in orc.table_scan_expect(bytes(g), FILTER)[0]} >= {0, 1, 3, 4}
