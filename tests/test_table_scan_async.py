"""The device-only whole-table scan (lcrc_table_scan_async): Table::open with paranoid_checks
(src/sstable/table.rs:39-103) + read_block_from_file with verify_checksum for every block
(src/sstable/format.rs:146-171), enqueued with no host round trip. Results, verdicts and the reference's
messages against the oracle's restatement (oracle.table_scan_expect) on tables from the oracle's writer; the
cases the device walk hands back to the host (LCRC_TSCAN_HOST) are checked to be exactly those it documents;
and the scan captured in a HIP graph and replayed.
"""
import os

import numpy as np
import pytest

from test_table_scan import FILTER, _as_tuples, _handcrafted, _kvs

OK, CORRUPT, HOST, CAPACITY = 0, 1, 2, 3


def _seq_kvs(n, vlen=24, seed=5):
    """db_bench-style sequential keys: the index block compresses, so a table written with compression=1 gets a
    Snappy-framed index block (table.rs:430, write_block)."""
    rng = np.random.default_rng(seed)
    return [(b"%016d" % i, rng.integers(0, 256, vlen, dtype=np.uint8).tobytes()) for i in range(n)]


class _Scan:
    """Device buffers for one async scan: the file, the result array, the count and the status words."""

    def __init__(self, lcrc, f, cap):
        self.lcrc = lcrc
        self.n = len(f)
        self.file = lcrc.DeviceBuffer.from_host(np.frombuffer(f, np.uint8).copy() if f else np.zeros(1, np.uint8))
        self.cap = cap
        self.blocks = lcrc.DeviceBuffer(max(cap, 1) * lcrc.TBLK_DTYPE.itemsize)
        self.count = lcrc.DeviceBuffer(8)
        self.status = lcrc.DeviceBuffer(8)

    def run(self, eng, filter_name=None, snappy_index=False):
        eng.table_scan_async(self.file, self.n, self.blocks, self.cap, self.count, self.status, filter_name,
                             snappy_index=snappy_index)
        eng.sync()
        return self.read()

    def read(self):
        st = self.status.download(np.uint32, 2)
        n = int(self.count.download(np.uint64, 1)[0])
        got = self.blocks.download(self.lcrc.TBLK_DTYPE, n) if st[0] == OK and n else None
        return int(st[0]), int(st[1]), n, got

    def close(self):
        for b in (self.file, self.blocks, self.count, self.status):
            b.close()


def _expect_async(lcrc, eng, orc, f, filt=None, cap=None, decoded=1 << 22, mode=0, masked=False, snappy_index=False):
    """Run the async scan and compare with the oracle; returns the status."""
    want, werr = orc.table_scan_expect(f, filt, mode, masked)
    eng.table_scan_reserve(len(f), cap if cap is not None else 4096, decoded)
    s = _Scan(lcrc, f, cap if cap is not None else 4096)
    try:
        st, code, n, got = s.run(eng, filt, snappy_index)
        if st == OK:
            assert werr is None
            assert sorted(_as_tuples(got)) == want
        elif st == CORRUPT:
            assert lcrc.lib().lcrc_table_scan_message(code).decode() == werr
        elif st == CAPACITY:
            assert werr is None and n == len(want)
        return st
    finally:
        s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("compression", [0, 1])
@pytest.mark.parametrize("filt", [None, FILTER])
@pytest.mark.parametrize("block_size", [256, 4096, 65536])
def test_async_clean(lcrc, orc, engines, compression, filt, block_size):
    f, _ = orc.table_build(_kvs(4000, block_size + compression), block_size=block_size, compression=compression,
                           filter_name=filt, filter_block=os.urandom(300))
    assert _expect_async(lcrc, engines[lcrc.MODE_REF], orc, f, filt) == OK


@pytest.mark.gpu
@pytest.mark.parametrize("block_size", [256, 4096])
def test_async_exact_decoded_reservation(lcrc, orc, block_size):
    """lcrc_table_scan_reserve's decoded_cap is the Snappy frames' decoded bytes (lcrc.h): a caller reserving
    exactly the oracle's decoded total of a compressed table (small blocks: the per-chunk alignment and stored CRCs
    the device adds are a large fraction of it) gets the device scan (LCRC_TSCAN_OK), not LCRC_TSCAN_HOST."""
    f, blocks = orc.table_build(_kvs(3000, 23 + block_size), block_size=block_size, compression=1,
                                filter_name=FILTER, filter_block=b"f" * 80)
    decoded = 0
    for off, n, kind in blocks:
        if kind == 0 and f[off + n] == 1:  # a Snappy-framed data block (format.rs:194-206; the filter block carries
            # type 1 over raw bytes, table.rs:383-391)
            decoded += len(orc.snappy_frame_decode(f[off:off + n]))
    assert decoded > 0
    eng = lcrc.Engine(0, lcrc.MODE_REF)
    try:
        assert _expect_async(lcrc, eng, orc, f, FILTER, cap=len(blocks) + 4, decoded=decoded) == OK
    finally:
        eng.close()


@pytest.mark.gpu
def test_async_masked_c(lcrc, orc):
    eng = lcrc.Engine(0, lcrc.MODE_C, lcrc.FLAG_MASK)
    try:
        f, _ = orc.table_build(_kvs(2000, 7), compression=1, filter_name=FILTER, filter_block=b"q" * 64,
                               mode=1, masked=True)
        assert _expect_async(lcrc, eng, orc, f, FILTER, mode=1, masked=True) == OK
    finally:
        eng.close()


@pytest.mark.gpu
def test_async_block_and_structural_corruption(lcrc, orc, engines):
    eng = engines[lcrc.MODE_REF]
    f, blocks = orc.table_build(_kvs(3000, 11), block_size=1024, compression=1, filter_name=FILTER,
                                filter_block=b"z" * 200)
    data = [b for b in blocks if b[2] == 0]
    g = bytearray(f)
    for off, n, _ in (data[0], data[len(data) // 2], data[-1]):
        g[off + n // 2] ^= 0x10
    assert _expect_async(lcrc, eng, orc, bytes(g), FILTER) == OK  # block-level verdicts, no error
    ih = [b for b in blocks if b[2] == 3][0]
    mh = [b for b in blocks if b[2] == 2][0]
    cases = {"short": f[-47:], "magic": f[:-1] + bytes([f[-1] ^ 1])}
    g = bytearray(f)
    g[ih[0] + 1] ^= 0x20
    cases["index crc"] = bytes(g)
    g = bytearray(f)
    g[ih[0] + ih[1]] = 7
    cases["index type"] = bytes(g)
    g = bytearray(f)
    g[mh[0] + 2] ^= 0x04  # a metaindex that does not verify: read_meta drops the filter
    cases["meta crc"] = bytes(g)
    for name, case in cases.items():
        st = _expect_async(lcrc, eng, orc, case, FILTER)
        assert st in (OK, CORRUPT), name
    assert _expect_async(lcrc, eng, orc, cases["short"]) == CORRUPT
    assert _expect_async(lcrc, eng, orc, cases["index crc"], FILTER) == CORRUPT


@pytest.mark.gpu
def test_async_handles_and_host_cases(lcrc, orc, engines):
    """Handles past the file, a Snappy index, malformed varints: either the device's verdict equals the
    oracle's, or the scan says LCRC_TSCAN_HOST for exactly the cases it documents; the synchronous wrapper
    then gives the oracle's answer in every case."""
    eng = engines[lcrc.MODE_REF]
    v = orc.varint
    cases = {
        "past end": (_handcrafted(orc, [(b"a", v(0) + v(100)), (b"b", v(10 ** 6) + v(50))]), (OK, HOST)),
        "bad varint": (_handcrafted(orc, [(b"a", b"\xff\xff")]), (CORRUPT, HOST)),
        "snappy index": (_handcrafted(orc, [(b"a", v(0) + v(100))], index_type=1), (HOST,)),
        "no filter entry": (_handcrafted(orc, [(b"a", v(0) + v(100))], meta_entries=[(b"filterother", v(0) + v(1))]),
                            (OK,)),
    }
    for name, (f, allowed) in cases.items():
        st = _expect_async(lcrc, eng, orc, f, FILTER)
        assert st in allowed, name
        got, err = _sync(lcrc, eng, f, FILTER)
        want, werr = orc.table_scan_expect(f, FILTER)
        assert err == werr and (got is None or _as_tuples(got) == want), name


def _sync(lcrc, eng, f, filt):
    dev = lcrc.DeviceBuffer.from_host(np.frombuffer(f, np.uint8).copy())
    try:
        return eng.table_scan(dev, len(f), filt), None
    except lcrc.TableCorruption as e:
        return None, str(e)
    finally:
        dev.close()


@pytest.mark.gpu
@pytest.mark.parametrize("interval", [1, 16, 1000])
def test_async_index_restart_intervals(lcrc, orc, engines, interval):
    f, _ = orc.table_build(_kvs(6000, 41), block_size=512, compression=1, index_restart_interval=interval)
    st = _expect_async(lcrc, engines[lcrc.MODE_REF], orc, f)
    assert st == (HOST if interval == 1000 else OK)  # one segment over 4 KiB: the host walk


@pytest.mark.gpu
def test_async_capacity_and_workspace(lcrc, orc, engines):
    eng = engines[lcrc.MODE_REF]
    f, blocks = orc.table_build(_kvs(3000, 13), block_size=512, compression=1, filter_name=FILTER,
                                filter_block=b"k" * 30)
    assert _expect_async(lcrc, eng, orc, f, FILTER, cap=len(blocks) - 1) == CAPACITY
    assert _expect_async(lcrc, eng, orc, f, FILTER, cap=len(blocks)) == OK
    # chunks the decoder's LDS staging holds need no workspace (k_ts_decode checksums them in LDS): OK even with a
    # 16-byte reservation. 64 KiB blocks' chunks are decoded lane-serially into the workspace: over the reservation
    # they are handed to the host, and the sync wrapper grows it
    eng2 = lcrc.Engine(0, lcrc.MODE_REF)
    try:
        assert _expect_async(lcrc, eng2, orc, f, FILTER, decoded=16) == OK
        g, _ = orc.table_build(_kvs(3000, 13 + 65536), block_size=65536, compression=1, filter_name=FILTER,
                               filter_block=b"k" * 30)
        assert _expect_async(lcrc, eng2, orc, g, FILTER, decoded=16) == HOST
        got, err = _sync(lcrc, eng2, g, FILTER)
        assert err is None and _as_tuples(got) == orc.table_scan_expect(g, FILTER)[0]
        assert _expect_async(lcrc, eng2, orc, g, FILTER, decoded=0) == OK  # the grown workspace stays
    finally:
        eng2.close()


@pytest.mark.gpu
def test_async_compressed_content(lcrc, orc, engines):
    f, blocks = orc.table_build(_kvs(3000, 31), block_size=2048, compression=1)
    g = bytearray(f)
    comp = [b for b in blocks if b[2] == 0 and g[b[0] + b[1]] == 1]
    for off, n, _ in comp[:2]:
        g[off + n - 3] ^= 0x5A
        g[off + n + 1:off + n + 5] = orc.crc(bytes(g[off:off + n + 1]), 0).to_bytes(4, "little")
    off, n, _ = comp[2]
    g[off + n] = 7
    g[off + n + 1:off + n + 5] = orc.crc(bytes(g[off:off + n + 1]), 0).to_bytes(4, "little")
    assert _expect_async(lcrc, engines[lcrc.MODE_REF], orc, bytes(g)) == OK


@pytest.mark.gpu
def test_async_graph_replay(lcrc, orc):
    """The whole scan captured in one HIP graph after lcrc_table_scan_reserve and replayed: the same
    blocks, count and status as the direct call, for a clean and (new file contents, same buffers) a corrupt
    table."""
    eng = lcrc.Engine(0, lcrc.MODE_C, lcrc.FLAG_MASK)
    f, blocks = orc.table_build(_kvs(5000, 3), block_size=1024, compression=1, filter_name=FILTER,
                                filter_block=b"p" * 500, mode=1, masked=True)
    want, _ = orc.table_scan_expect(f, FILTER, 1, True)
    cap = len(blocks) + 8
    eng.table_scan_reserve(len(f), cap, 1 << 22)
    s = _Scan(lcrc, f, cap)
    g = None
    try:
        st, _, n, got = s.run(eng, FILTER)
        assert st == OK and sorted(_as_tuples(got)) == want
        g = eng.graph_capture(lambda: eng.table_scan_async(s.file, s.n, s.blocks, s.cap, s.count, s.status, FILTER))
        for _ in range(2):
            s.blocks.zero()
            s.count.zero()
            eng.graph_launch(g)
            eng.sync()
            st, _, n, got = s.read()
            assert st == OK and sorted(_as_tuples(got)) == want
        ih = [b for b in blocks if b[2] == 3][0]
        bad = bytearray(f)
        bad[ih[0] + 3] ^= 1
        s.file.upload(np.frombuffer(bytes(bad), np.uint8))
        eng.graph_launch(g)
        eng.sync()
        st, code, _, _ = s.read()
        assert st == CORRUPT and lcrc.lib().lcrc_table_scan_message(code).decode() == "block checksum mismatch"
    finally:
        if g is not None:
            eng.graph_destroy(g)
        s.close()
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode,masked", [(0, False), (1, True)])
def test_async_long_meta_blocks(lcrc, orc, mode, masked):
    """An index block and a filter block longer than LCRC_TS_PIECE are verified as 64 KiB pieces and combined
    (crc(A || B) = x^(8|B|) crc(A) ^ crc(B)): same CRCs and verdicts as the oracle, clean and corrupted."""
    eng = lcrc.Engine(0, mode, lcrc.FLAG_MASK if masked else 0)
    try:
        kvs = _kvs(40000, 77, vlen=12)
        f, blocks = orc.table_build(kvs, block_size=128, compression=0, filter_name=FILTER,
                                    filter_block=os.urandom(200_003), mode=mode, masked=masked)
        ih = [b for b in blocks if b[2] == 3][0]
        fb = [b for b in blocks if b[2] == 1][0]
        assert ih[1] + 1 > 2 * 65536 and fb[1] + 1 > 3 * 65536  # several pieces each, a partial last one
        assert _expect_async(lcrc, eng, orc, f, FILTER, cap=len(blocks) + 4, mode=mode, masked=masked) == OK
        g = bytearray(f)
        g[fb[0] + 70000] ^= 0x08  # inside the filter's second piece: that block's status only
        assert _expect_async(lcrc, eng, orc, bytes(g), FILTER, cap=len(blocks) + 4, mode=mode, masked=masked) == OK
        g = bytearray(f)
        g[ih[0] + ih[1] - 100] ^= 0x01  # inside the index's last piece: Table::open fails
        assert _expect_async(lcrc, eng, orc, bytes(g), FILTER, cap=len(blocks) + 4, mode=mode, masked=masked) in (
            CORRUPT, HOST)
        got, err = _sync(lcrc, eng, bytes(g), FILTER)
        assert err == "block checksum mismatch"
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("general", ["auto", "ranges"])
@pytest.mark.parametrize("grid", [1, 3])
def test_async_tile_loops(lcrc, orc, grid, general):
    """The index walk with fewer workgroups than 512-segment chunks (the context option ts_grid caps their grid): a
    workgroup walks a range of several chunks, and the ranges' counts meet through the per-ticket words. Beside the
    window pass (k_ts_windows, the default) and alone (general="ranges": the one-pass range kernel verifies, so the
    launch holds only the index workgroups)."""
    eng = lcrc.Engine(0, lcrc.MODE_REF, ts_grid=grid, general=general)
    try:
        f, blocks = orc.table_build(_kvs(6000, 41), block_size=256, compression=1, index_restart_interval=1,
                                    filter_name=FILTER, filter_block=b"z" * 100)
        assert len(blocks) > 256 * grid + 256  # more tiles than workgroups
        assert _expect_async(lcrc, eng, orc, f, FILTER, cap=len(blocks) + 4) == OK
        g = bytearray(f)
        d = [b for b in blocks if b[2] == 0]
        for off, n, _ in (d[300], d[-2]):  # a data block in a later tile, and one near the end
            g[off + n // 2] ^= 0x10
        assert _expect_async(lcrc, eng, orc, bytes(g), FILTER, cap=len(blocks) + 4) == OK
    finally:
        eng.close()


@pytest.mark.gpu
def test_async_multi_chunk_frames(lcrc, orc, engines):
    """Blocks whose Snappy frame holds several chunks: each decoded chunk lands 16-aligned with its stored masked
    CRC-32C after it, compared by the CRC pass; a chunk corrupted in the middle of a frame (block checksum
    recomputed) fails only its block."""
    f, blocks = orc.table_build(_kvs(3000, 59, vlen=400), block_size=200_000, compression=1)
    comp = [b for b in blocks if b[2] == 0 and f[b[0] + b[1]] == 1]
    assert len(comp) >= 3 and all(b[1] > 65536 for b in comp[:3])  # several chunks per frame
    assert _expect_async(lcrc, engines[lcrc.MODE_REF], orc, f) == OK
    g = bytearray(f)
    off, n, _ = comp[1]
    g[off + n // 2] ^= 0x21  # inside a middle chunk's bytes
    g[off + n + 1:off + n + 5] = orc.crc(bytes(g[off:off + n + 1]), 0).to_bytes(4, "little")
    assert _expect_async(lcrc, engines[lcrc.MODE_REF], orc, bytes(g)) == OK


def _index_block(f, blocks):
    return [b for b in blocks if b[2] == 3][0]


@pytest.mark.gpu
@pytest.mark.parametrize("n,block_size", [(3000, 4096), (6000, 256), (40000, 128)])
@pytest.mark.parametrize("filt", [None, FILTER])
def test_async_snappy_index(lcrc, orc, engines, n, block_size, filt):
    """A table written with compression has a Snappy-framed index block (table.rs:430): without
    LCRC_TSCAN_SNAPPY_INDEX the device walk hands it to the host; with it the index is decoded on the device
    (k_ts_open: one chunk of the frame per workgroup; the 40000-key case has several 64 KiB chunks) and the scan is
    the oracle's. The synchronous wrapper (which always sets the flag) agrees."""
    f, blocks = orc.table_build(_seq_kvs(n), block_size=block_size, compression=1, filter_name=filt,
                                filter_block=b"s" * 90)
    off, size, _ = _index_block(f, blocks)
    assert f[off + size] == 1  # the index block is a Snappy frame
    if n == 40000:
        assert len(orc.snappy_frame_decode(f[off:off + size])) > 3 * 65536
    eng = engines[lcrc.MODE_REF]
    assert _expect_async(lcrc, eng, orc, f, filt, cap=len(blocks) + 4) == HOST
    assert _expect_async(lcrc, eng, orc, f, filt, cap=len(blocks) + 4, snappy_index=True) == OK
    got, err = _sync(lcrc, eng, f, filt)
    assert err is None and _as_tuples(got) == orc.table_scan_expect(f, filt)[0]
    # the flag on a table whose index is stored raw: the same scan as without it
    g, gb = orc.table_build(_kvs(2000, 3), block_size=1024, compression=1)
    assert g[sum(_index_block(g, gb)[:2])] == 0
    assert _expect_async(lcrc, eng, orc, g, cap=len(gb) + 4, snappy_index=True) == OK


@pytest.mark.gpu
def test_async_snappy_index_corruption(lcrc, orc, engines):
    """A Snappy-framed index whose chunk does not decode or check (the block trailer re-sealed, so only the frame is
    wrong), and one whose block checksum fails: the device says LCRC_TSCAN_HOST or the oracle's verdict, and the
    synchronous scan gives the oracle's message in every case."""
    f, blocks = orc.table_build(_seq_kvs(5000), block_size=512, compression=1)
    off, size, _ = _index_block(f, blocks)
    eng = engines[lcrc.MODE_REF]

    def reseal(g):
        g[off + size + 1:off + size + 5] = orc.crc(bytes(g[off:off + size + 1]), 0).to_bytes(4, "little")
        return bytes(g)

    cases = {}
    g = bytearray(f)
    g[off + 10 + 8 + 40] ^= 0x01  # inside the first chunk's compressed body
    cases["chunk body"] = reseal(g)
    g = bytearray(f)
    g[off + 10 + 4] ^= 0x80  # the first chunk's stored masked CRC-32C
    cases["chunk crc"] = reseal(g)
    g = bytearray(f)
    g[off + 1] = 0x07  # the stream identifier's length
    cases["framing"] = reseal(g)
    g = bytearray(f)
    g[off + size // 2] ^= 0x04
    cases["block crc"] = bytes(g)  # not resealed
    for name, case in cases.items():
        st = _expect_async(lcrc, eng, orc, case, snappy_index=True)
        assert st in (HOST, CORRUPT), name
        got, err = _sync(lcrc, eng, case, None)
        want, werr = orc.table_scan_expect(case, None)
        assert err == werr and (got is None or _as_tuples(got) == want), name
    # the clean table after the failures: the failure mark does not stick
    assert _expect_async(lcrc, eng, orc, f, snappy_index=True) == OK


@pytest.mark.gpu
def test_async_snappy_index_workspace(lcrc, orc):
    """The decoded index takes the scan's decode workspace (lcrc_table_scan_reserve's decoded_cap): over it the scan
    is LCRC_TSCAN_HOST, the synchronous wrapper grows the workspace and the next async scan decodes on the device."""
    f, blocks = orc.table_build(_seq_kvs(8000), block_size=256, compression=1)
    off, size, _ = _index_block(f, blocks)
    assert f[off + size] == 1 and len(orc.snappy_frame_decode(f[off:off + size])) > 4096
    eng = lcrc.Engine(0, lcrc.MODE_REF)
    try:
        assert _expect_async(lcrc, eng, orc, f, cap=len(blocks) + 4, decoded=16, snappy_index=True) == HOST
        got, err = _sync(lcrc, eng, f, None)
        assert err is None and _as_tuples(got) == orc.table_scan_expect(f, None)[0]
        assert _expect_async(lcrc, eng, orc, f, cap=len(blocks) + 4, decoded=0, snappy_index=True) == OK
    finally:
        eng.close()


@pytest.mark.gpu
def test_async_snappy_index_uncompressed_chunk(lcrc, orc, engines):
    """A framed index whose only chunk is stored uncompressed (type 1: framing saved nothing on a tiny index): decoded
    on the device with LCRC_TSCAN_SNAPPY_INDEX -- the chunk checksummed where it lies and copied out -- and the scan is
    the oracle's; with the chunk's stored CRC broken the device hands the table to the host walk, whose message is
    the oracle's."""
    v = orc.varint
    f = _handcrafted(orc, [(b"a", v(0) + v(100))], index_type=1)
    want, werr = orc.table_scan_expect(f)
    assert werr is None
    eng = engines[lcrc.MODE_REF]
    assert _expect_async(lcrc, eng, orc, f, snappy_index=True) == OK
    ih = [w for w in want if w[2] == 3][0]
    off, size = ih[0], ih[1]
    assert f[off + size] == 1 and f[off + 10] == 1  # the frame's data chunk is type 1
    g = bytearray(f)
    g[off + 14] ^= 0x01  # the chunk's masked CRC-32C
    g[off + size + 1:off + size + 5] = orc.crc(bytes(g[off:off + size + 1]), 0).to_bytes(4, "little")
    assert _expect_async(lcrc, eng, orc, bytes(g), snappy_index=True) in (HOST, CORRUPT)
    got, err = _sync(lcrc, eng, bytes(g), None)
    assert err == orc.table_scan_expect(bytes(g))[1]


@pytest.mark.gpu
def test_async_snappy_index_graph_replay(lcrc, orc):
    """The seven-launch scan of a table with a Snappy-framed index (LCRC_TSCAN_SNAPPY_INDEX) captured in one HIP graph
    after lcrc_table_scan_reserve and replayed: the oracle's blocks each time, and after the file's index frame is
    corrupted in place (same buffers, trailer re-sealed) the replay hands the table to the host walk, and a replay of
    the restored file is clean again (k_ts_open's failure mark does not stick across replays)."""
    eng = lcrc.Engine(0, lcrc.MODE_REF)
    f, blocks = orc.table_build(_seq_kvs(6000), block_size=512, compression=1)
    off, size, _ = _index_block(f, blocks)
    assert f[off + size] == 1
    want, _ = orc.table_scan_expect(f)
    cap = len(blocks) + 8
    eng.table_scan_reserve(len(f), cap, 1 << 22)
    s = _Scan(lcrc, f, cap)
    g = None
    try:
        g = eng.graph_capture(lambda: eng.table_scan_async(s.file, s.n, s.blocks, s.cap, s.count, s.status,
                                                           snappy_index=True))
        for _ in range(2):
            s.blocks.zero()
            s.count.zero()
            eng.graph_launch(g)
            eng.sync()
            st, _, n, got = s.read()
            assert st == OK and sorted(_as_tuples(got)) == want
        bad = bytearray(f)
        bad[off + 10 + 8 + 30] ^= 0x01  # inside the first chunk's compressed body
        bad[off + size + 1:off + size + 5] = orc.crc(bytes(bad[off:off + size + 1]), 0).to_bytes(4, "little")
        s.file.upload(np.frombuffer(bytes(bad), np.uint8))
        eng.graph_launch(g)
        eng.sync()
        assert s.read()[0] == HOST
        s.file.upload(np.frombuffer(f, np.uint8))
        eng.graph_launch(g)
        eng.sync()
        st, _, n, got = s.read()
        assert st == OK and sorted(_as_tuples(got)) == want
    finally:
        if g is not None:
            eng.graph_destroy(g)
        s.close()
        eng.close()


@pytest.mark.gpu
def test_async_snappy_index_multi_chunk(lcrc, orc):
    """The compressed index through k_ts_open2 (16 waves per 64 KiB chunk): a multi-chunk index, clean and with a
    chunk that does not decode, the oracle's result either way."""
    eng = lcrc.Engine(0, lcrc.MODE_REF)
    try:
        f, blocks = orc.table_build(_seq_kvs(40000), block_size=128, compression=1)
        off, size, _ = _index_block(f, blocks)
        assert len(orc.snappy_frame_decode(f[off:off + size])) > 3 * 65536
        assert _expect_async(lcrc, eng, orc, f, cap=len(blocks) + 4, snappy_index=True) == OK
        g = bytearray(f)
        g[off + size // 2] ^= 0x04
        g[off + size + 1:off + size + 5] = orc.crc(bytes(g[off:off + size + 1]), 0).to_bytes(4, "little")
        assert _expect_async(lcrc, eng, orc, bytes(g), cap=len(blocks) + 4, snappy_index=True) in (OK, CORRUPT, HOST)
        got, err = _sync(lcrc, eng, bytes(g), None)
        assert err == orc.table_scan_expect(bytes(g))[1]
    finally:
        eng.close()


def _skewed_kvs(n, seed):
    """Keys whose index entries differ tenfold in size: the first three quarters short, the rest sharing a 200-byte
    prefix (so that the index separators keep it)."""
    rng = np.random.default_rng(seed)
    keys = [b"a%08d" % i for i in range(3 * n // 4)] + [b"z" + b"q" * 200 + b"%08d" % i for i in range(n - 3 * n // 4)]
    return [(k, rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()) for k in keys]


@pytest.mark.gpu
@pytest.mark.parametrize("skew", [False, True])
@pytest.mark.parametrize("grid", [0, 1, 5])
def test_async_index_ranges(lcrc, orc, grid, skew):
    """The index walk beside the window pass (k_ts_windows): each index workgroup stages its range of restart
    segments in LDS with the range's offsets rebased (a range too long for the LDS is walked in place: one workgroup,
    grid 1, over this ~120 KB index). Restart arrays and entries corrupted at range boundaries and inside ranges, the
    index block re-sealed so that the walk must judge them: the verdict, count and blocks equal those of the index
    workgroups launched alone (general="ranges"), and the synchronous scan gives the oracle's answer. The skewed
    table's ranges lie far from where even entries would put them (the walk's speculative load of a range's bytes
    misses, and a second round loads them)."""
    kvs = _skewed_kvs(16000, 17) if skew else _kvs(16000, 17)
    f, blocks = orc.table_build(kvs, block_size=128, compression=0, index_restart_interval=1)
    off, size, _ = _index_block(f, blocks)
    nres = int.from_bytes(f[off + size - 4:off + size], "little")
    assert f[off + size] == 0 and size > 80_000 and nres > 5000
    ra = off + size - 4 * (1 + nres)
    cap = len(blocks) + 4
    opts = {"ts_grid": grid} if grid else {}
    fused, unfused = lcrc.Engine(0, lcrc.MODE_REF, **opts), lcrc.Engine(0, lcrc.MODE_REF, general="ranges", **opts)

    def rst(g, k):
        return int.from_bytes(g[ra + 4 * k:ra + 4 * k + 4], "little")

    def put(g, k, v):
        g[ra + 4 * k:ra + 4 * k + 4] = (v & 0xFFFFFFFF).to_bytes(4, "little")

    def reseal(g):
        g[off + size + 1:off + size + 5] = orc.crc(bytes(g[off:off + size + 1]), 0).to_bytes(4, "little")
        return bytes(g)

    cases = {"clean": f}
    nidx = min(cap // 512 + 1, grid or 256)  # the index workgroups (lcrc_launch_ts_windows)
    per = -(-nres // nidx)  # segments per range
    for k in (1, per - 1, per, per + 1, nres // 2, nres - 1):
        g = bytearray(f)
        put(g, k, rst(g, k - 1) - 1)
        cases[f"rst {k} before its predecessor"] = reseal(g)
        g = bytearray(f)
        put(g, k, rst(g, k) + 1)
        cases[f"rst {k} + 1"] = reseal(g)
    g = bytearray(f)
    put(g, 0, 1)
    cases["rst 0 = 1"] = reseal(g)
    g = bytearray(f)
    put(g, nres - 1, ra - off + 3)
    cases["last rst past the array"] = reseal(g)
    for k in (per, nres // 3):
        g = bytearray(f)
        g[off + rst(g, k) + 1] = 0xFF  # an entry's non_shared varint
        cases[f"entry {k} varint"] = reseal(g)
    try:
        for name, case in cases.items():
            res = []
            for eng in (fused, unfused):
                eng.table_scan_reserve(len(case), cap, 1 << 20)
                s = _Scan(lcrc, case, cap)
                try:
                    res.append(s.run(eng))
                finally:
                    s.close()
            (st, code, n, got), (ust, ucode, un, ugot) = res
            assert (st, code, n) == (ust, ucode, un), name
            assert (got is None and ugot is None) or _as_tuples(got) == _as_tuples(ugot), name
            if name == "clean":
                assert st == OK and _as_tuples(got) == orc.table_scan_expect(case)[0]
            got, err = _sync(lcrc, fused, case, None)
            want, werr = orc.table_scan_expect(case, None)
            assert err == werr and (got is None or _as_tuples(got) == want), name
    finally:
        fused.close()
        unfused.close()


@pytest.mark.gpu
def test_async_last_three_at_tile_edges(lcrc, orc):
    """The last three blocks (filter as a Snappy frame, metaindex, Snappy-framed index) at every position across a
    256-block tile edge: k_ts_decode's last workgroup finishes, decodes and judges them -- fused, also the finish of a
    tile that holds only some of them -- and the workspace offsets of their frames follow the tiles before."""
    eng = lcrc.Engine(0, lcrc.MODE_REF)
    try:
        for k in (1, 2, 252, 253, 254, 255, 256, 257, 509, 510, 511, 512, 513):
            f, blocks = orc.table_build(_seq_kvs(k), block_size=1, compression=1, filter_name=FILTER,
                                        filter_block=b"f" * 300)
            assert [b[2] for b in blocks].count(0) == k and f[sum(blocks[-3][:2])] == 1  # the filter: a frame
            assert _expect_async(lcrc, eng, orc, f, FILTER, cap=len(blocks) + 4, snappy_index=True) == OK, k
            g = bytearray(f)
            off, n, _ = blocks[-3]
            g[off + n // 2] ^= 0x40  # the filter's frame corrupted, its block trailer re-sealed
            g[off + n + 1:off + n + 5] = orc.crc(bytes(g[off:off + n + 1]), 0).to_bytes(4, "little")
            assert _expect_async(lcrc, eng, orc, bytes(g), FILTER, cap=len(blocks) + 4, snappy_index=True) == OK, k
    finally:
        eng.close()


@pytest.mark.gpu
def test_async_two_contexts_concurrent(lcrc, orc):
    """Two contexts scanning on their own streams at once, several rounds back to back (as bench.py's two scanners
    do): each scan's index workgroups wait only for their own launch's words, and the words are zeroed for the next
    scan by the last ticket -- every result equals the oracle's."""
    f1, b1 = orc.table_build(_kvs(5000, 71), block_size=256, compression=0, filter_name=FILTER, filter_block=b"a" * 50)
    f2, b2 = orc.table_build(_kvs(7000, 72), block_size=512, compression=1, filter_name=FILTER, filter_block=b"b" * 70)
    engs = [lcrc.Engine(0, lcrc.MODE_REF), lcrc.Engine(0, lcrc.MODE_REF)]
    scans = []
    try:
        for eng, (f, blocks) in zip(engs, ((f1, b1), (f2, b2))):
            eng.table_scan_reserve(len(f), len(blocks) + 4, 1 << 22)
            scans.append((_Scan(lcrc, f, len(blocks) + 4), f))
        want = [orc.table_scan_expect(f, FILTER)[0] for f in (f1, f2)]
        for _ in range(6):
            for eng, (s, _f) in zip(engs, scans):
                eng.table_scan_async(s.file, s.n, s.blocks, s.cap, s.count, s.status, FILTER)
            for eng in engs:
                eng.sync()
            for (s, _f), w in zip(scans, want):
                st, code, n, got = s.read()
                assert st == OK and sorted(_as_tuples(got)) == w
    finally:
        for s, _f in scans:
            s.close()
        for eng in engs:
            eng.close()


@pytest.mark.gpu
def test_async_four_contexts_full_index_grid(lcrc, orc):
    """Four contexts on four streams, each scanning a table of more than 131,072 blocks (so 256 index workgroups per
    launch, the cap) three times, all enqueued before any synchronisation: 4 x (256 index + the window workgroups)
    is more than the 512 workgroups the CUs hold at once, so the index workgroups of one launch are not all resident
    together. The ticketed look-back (each index workgroup waits only on tickets taken before its own) must still end
    every launch, and every result equals the oracle's (table.rs:39-146, format.rs:146-171). One table has a
    corrupt index entry, so its last ticket writes the index block alone at slot 0 over the handles lower tickets
    wrote there."""
    tables = []
    for k in range(4):
        f, blocks = orc.table_build(_seq_kvs(131_200 + 500 * k, vlen=4 + 3 * k, seed=40 + k), block_size=1,
                                    compression=0, filter_name=FILTER if k % 2 else None, filter_block=b"q" * 64)
        assert sum(1 for b in blocks if b[2] == 0) > 131_072
        tables.append((f, blocks, FILTER if k % 2 else None))
    # table 3: an index entry inside the last range made unreadable and the index block's trailer NOT re-sealed: the
    # device walk cannot vouch for that segment, so the scan verifies the index block alone -- the last ticket's entry
    # at slot 0, over the data handle ticket 0 wrote there -- and must report the reference's checksum message (a
    # data handle left at slot 0 would verify clean and say LCRC_TSCAN_HOST instead)
    f, blocks, filt = tables[3]
    off, size, _ = _index_block(f, blocks)
    nres = int.from_bytes(f[off + size - 4:off + size], "little")
    ra = off + size - 4 * (1 + nres)
    g = bytearray(f)
    e = int.from_bytes(g[ra + 4 * (nres - 10):ra + 4 * (nres - 9)], "little")
    g[off + e + 1] = 0xFF  # the entry's non_shared varint
    tables[3] = (bytes(g), blocks, filt)
    want = [orc.table_scan_expect(f, filt) for f, _b, filt in tables]
    assert want[3][1] == "block checksum mismatch" and all(w[1] is None for w in want[:3])
    engs = [lcrc.Engine(0, lcrc.MODE_REF) for _ in range(4)]
    scans = []
    try:
        for eng, (f, blocks, _filt) in zip(engs, tables):
            cap = len(blocks) + 4
            assert cap // 512 + 1 >= 256  # the index grid is at its cap
            eng.table_scan_reserve(len(f), cap, 1 << 20)
            scans.append(_Scan(lcrc, f, cap))
        for _ in range(3):
            for s in scans:
                s.blocks.zero()
                s.count.zero()
            for eng, s, (_f, _b, filt) in zip(engs, scans, tables):
                eng.table_scan_async(s.file, s.n, s.blocks, s.cap, s.count, s.status, filt)
            for eng in engs:
                eng.sync()
            for k, (s, (w, werr)) in enumerate(zip(scans, want)):
                st, code, n, got = s.read()
                if werr is None:
                    assert st == OK and sorted(_as_tuples(got)) == w, k
                else:
                    assert st == CORRUPT and lcrc.lib().lcrc_table_scan_message(code).decode() == werr, k
    finally:
        for s in scans:
            s.close()
        for eng in engs:
            eng.close()


def _bench_like_tables(lcrc, orc, sizes):
    """Compressed tables of db_bench-style 4 KiB blocks (k_ts_decode's row path: 8 frames a wave, sub-tiles of 128
    frames), written by the library's TableBuilder (synth.compressed_table); the last one with some data frames
    corrupted and their block trailers re-sealed, so only the frames' chunk CRCs or decodes can tell."""
    synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
    out = []
    for k, n in enumerate(sizes):
        f, tb = synth.compressed_table(lcrc, n)
        f = bytearray(f.tobytes())
        blocks = [(int(b["offset"]), int(b["size"]), int(b["kind"])) for b in tb]
        if k == len(sizes) - 1:
            data = [b for b in blocks if b[2] == lcrc.TBLK_DATA and f[b[0] + b[1]] == 1]
            for j in (0, 127, 128, 255, 256, len(data) // 2, len(data) - 1):
                off, size, _ = data[j]
                f[off + size // 2 + j % 7] ^= 0x20
                f[off + size + 1:off + size + 5] = orc.crc(bytes(f[off:off + size + 1]), 0).to_bytes(4, "little")
        out.append((bytes(f), blocks))
    return out


@pytest.mark.gpu
def test_async_compressed_contexts_concurrent(lcrc, orc):
    """Three contexts scanning compressed tables of 4 KiB blocks on their own streams at once, four rounds enqueued
    back to back: the decode's workgroups of one launch share the CUs with the other launches' (a whole CU's LDS
    each), and every result -- the corrupted frames' content verdicts included -- equals the oracle's
    (format.rs:194-206 through read_block_from_file)."""
    tables = _bench_like_tables(lcrc, orc, (700, 1300, 1500))
    want = [orc.table_scan_expect(f)[0] for f, _b in tables]
    assert sum(1 for w in want[2] if w[4] == 3) == 7 and all(w[4] == 0 for w in want[0] + want[1])
    engs = [lcrc.Engine(0, lcrc.MODE_REF) for _ in tables]
    scans = []
    try:
        for eng, (f, blocks) in zip(engs, tables):
            eng.table_scan_reserve(len(f), len(blocks) + 4, 8 << 20)
            scans.append(_Scan(lcrc, f, len(blocks) + 4))
        for _ in range(4):
            for s in scans:
                s.blocks.zero()
            for eng, s in zip(engs, scans):
                eng.table_scan_async(s.file, s.n, s.blocks, s.cap, s.count, s.status, snappy_index=True)
            for eng in engs:
                eng.sync()
            for k, (s, w) in enumerate(zip(scans, want)):
                st, code, n, got = s.read()
                assert st == OK and sorted(_as_tuples(got)) == w, k
    finally:
        for s in scans:
            s.close()
        for eng in engs:
            eng.close()
