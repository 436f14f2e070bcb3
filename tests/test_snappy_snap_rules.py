"""The snap crate's FrameDecoder rules at their edges (snap "1", Cargo.toml:15; the decoder read_block_from_file uses
for a compressed block, src/sstable/format.rs:194-206). The crate is absent here, so these fixtures are
built from its published behaviour and every decoder in the tree must agree on them: the Python oracle, the C oracle
(the table benches' CPU baseline), the library's host decoder (the synchronous scan's fallback walk) and, on the GPU,
lcrc_snappy_frames and the whole-table scan (row decoder, wave decoder, lane-serial decoder, k_ts_open for an index).

The rules (each found to differ somewhere in the tree before round 5):
* the length preamble is bytes::read_varu64 -- up to 10 bytes, the value mod 2^64 -- and the frame decoder rejects a
  decoded length over MAX_BLOCK_SIZE (65,536): a 5-byte preamble of 2^32 used to truncate to 0 on the device and in
  the host decoder, so an empty chunk carrying the CRC of b"" decoded "clean";
* a chunk longer than MAX_COMPRESS_BLOCK_SIZE (76,490), of any type, is an error;
* read_literal reads an extended literal length as one 4-byte word: 4 input bytes must follow the tag whatever the
  number of length bytes is.
"""
import numpy as np
import pytest

from test_table_scan import FILTER, _as_tuples

STREAM = b"\xff\x06\x00\x00sNaPpY"


def _chunk(orc, typ, payload, decoded):
    body = orc.mask(orc.crc(decoded, 1)).to_bytes(4, "little") + payload
    return bytes([typ, len(body) & 0xFF, (len(body) >> 8) & 0xFF, len(body) >> 16]) + body


def _varu(v, nbytes):
    """v as a varint padded to nbytes bytes (continuation bits on every byte but the last)."""
    out = []
    for i in range(nbytes):
        b = (v >> (7 * i)) & 127
        out.append(b | (128 if i < nbytes - 1 else 0))
    return bytes(out)


def _lit(data, nb=None):
    n = len(data)
    if nb is None:
        nb = 0 if n <= 60 else 1 if n <= 256 else 2 if n <= 65536 else 3
    head = bytes([(n - 1) << 2]) if nb == 0 else bytes([(59 + nb) << 2]) + (n - 1).to_bytes(nb, "little")
    return head + data


def _copy4(off, n):
    return bytes([((n - 1) << 2) | 3]) + off.to_bytes(4, "little")


def snap_cases(orc):
    """[(name, frame bytes, decoded bytes or None)] -- the expected outcome is snap's."""
    c = []

    def comp(payload, decoded):
        return STREAM + _chunk(orc, 0, payload, decoded)

    c.append(("preamble 1 byte", comp(_varu(5, 1) + _lit(b"hello"), b"hello"), b"hello"))
    c.append(("preamble 10 bytes", comp(_varu(5, 10) + _lit(b"hello"), b"hello"), b"hello"))
    c.append(("preamble 11 bytes", comp(_varu(5, 11) + _lit(b"hello"), b"hello"), None))
    c.append(("preamble 2^32 empty", comp(b"\x80\x80\x80\x80\x10", b""), None))
    c.append(("preamble 2^32+5", comp(b"\x85\x80\x80\x80\x10" + _lit(b"hello"), b"hello"), None))
    c.append(("preamble 2^64 wraps to 0", comp(b"\x80" * 9 + b"\x02", b""), b""))
    c.append(("preamble 2^63+5", comp(b"\x85" + b"\x80" * 8 + b"\x01" + _lit(b"hello"), b"hello"), None))
    big = bytes(np.random.default_rng(3).integers(0, 256, 65536, dtype=np.uint8))
    c.append(("preamble 65536", comp(_varu(65536, 3) + _lit(big), big), big))
    c.append(("preamble 65537", comp(_varu(65537, 3) + _lit(big + b"x"), big + b"x"), None))
    c.append(("ext literal 1 B at end", comp(_varu(1, 1) + _lit(b"z", 1), b"z"), None))
    c.append(("ext literal 2 B at end, 3 after tag", comp(_varu(2, 1) + _lit(b"zz", 1), b"zz"), None))
    c.append(("ext literal 3 B at end, 4 after tag", comp(_varu(3, 1) + _lit(b"zzz", 1), b"zzz"), b"zzz"))
    c.append(("ext literal 1 B then more", comp(_varu(4, 1) + _lit(b"z", 1) + _lit(b"abc"), b"zabc"), b"zabc"))
    c.append(("ext2 literal 2 B at end", comp(_varu(2, 1) + _lit(b"ab", 2), b"ab"), b"ab"))
    c.append(("ext4 literal 1 B at end", comp(_varu(1, 1) + _lit(b"q", 4), b"q"), b"q"))
    # a valid compressed stream longer than MAX_COMPRESS_BLOCK_SIZE (copies of 1 byte with 4-byte offsets)
    for ncopy in (15295, 15300):
        dec = b"a" * (1 + ncopy)
        payload = _varu(len(dec), 2) + _lit(b"a") + _copy4(1, 1) * ncopy
        frame = comp(payload, dec)
        c.append((f"compressed chunk {len(payload) + 4} B", frame, dec if len(payload) + 4 <= 76490 else None))
    for n in (76490, 76491):
        c.append((f"skippable chunk {n} B", STREAM + bytes([0x80, n & 0xFF, (n >> 8) & 0xFF, n >> 16]) + b"s" * n
                  + _chunk(orc, 1, b"tail", b"tail"), b"tail" if n <= 76490 else None))
    c.append(("padding chunk 76491 B", STREAM + b"\xfe" + (76491).to_bytes(3, "little") + b"\0" * 76491, None))
    c.append(("uncompressed 65536", STREAM + _chunk(orc, 1, big, big), big))
    c.append(("uncompressed 65537", STREAM + _chunk(orc, 1, big + b"x", big + b"x"), None))
    c.append(("compressed empty body", STREAM + _chunk(orc, 0, b"", b""), None))
    c.append(("no stream identifier first", _chunk(orc, 1, b"abc", b"abc") + STREAM, None))
    c.append(("stream identifier repeated", STREAM + _chunk(orc, 1, b"abc", b"abc") + STREAM
              + comp(_varu(3, 1) + _lit(b"def"), b"def")[len(STREAM):], b"abcdef"))
    c.append(("stream identifier only", STREAM, b""))
    c.append(("empty frame", b"", b""))
    return c


def _c_oracle_status(orc, frames):
    """The C oracle's read_block_from_file walk (oracle/crc_oracle.c) over the frames as type-1 blocks: 0 or 3."""
    f = bytearray()
    offs, sizes = [], []
    for fr in frames:
        offs.append(len(f))
        sizes.append(len(fr))
        f += orc.raw_block(fr, 1)
    _, status, _ = orc.table_blocks_mt(bytes(f), np.array(offs, np.uint64), np.array(sizes, np.uint64), 1)
    return [int(s) for s in status]


def test_snap_rules_cpu(lcrc, orc):
    cases = snap_cases(orc)
    for name, frame, want in cases:
        assert orc.snappy_frame_decode(frame) == want, name
        assert lcrc.snappy_frame_decode(frame) == want, name
    st = _c_oracle_status(orc, [fr for _, fr, _ in cases])
    assert st == [0 if w is not None else 3 for _, _, w in cases]


def frames_table(orc, frames, masked=False):
    """A table whose data blocks are the given byte strings stored as Snappy-framed blocks (type 1), keys k0000.. in
    order, restart interval 1 in the index: the scan's verdict on each block is read_block_from_file's."""
    f = bytearray()
    index = []
    for i, fr in enumerate(frames):
        off = len(f)
        f += orc.raw_block(fr, 1)
        index.append((b"k%05d" % i, orc.varint(off) + orc.varint(len(fr))))
    meta = orc.block_build([])
    moff = len(f)
    f += orc.raw_block(meta, 0)
    idx = orc.block_build(index, 1)
    ioff = len(f)
    f += orc.raw_block(idx, 0)
    foot = orc.varint(moff) + orc.varint(len(meta)) + orc.varint(ioff) + orc.varint(len(idx))
    foot += bytes(40 - len(foot)) + orc.TABLE_MAGIC.to_bytes(8, "little")
    return bytes(f + foot)


@pytest.mark.gpu
def test_snap_rules_device_frames(lcrc, orc, engines):
    """lcrc_snappy_frames (k_snappy_size, the wave decoder, the lane-serial decoder) on every case."""
    from test_table_scan import _frames_on_device
    cases = snap_cases(orc)
    base, dd = _frames_on_device(lcrc, [fr for _, fr, _ in cases])
    got, status = engines[lcrc.MODE_REF].snappy_frames(base, dd, len(cases))
    for (name, _, want), g, s in zip(cases, got, status):
        assert int(s != 0) == int(want is None), name
        if want is not None:
            assert g == want, name


@pytest.mark.gpu
def test_snap_rules_device_table_scan(lcrc, orc, engines):
    """The same frames as data blocks of one table: every block's verdict from the device scan (the row decoder for
    small frames, the whole-wave and lane-serial decoders for large ones) equals the oracle's."""
    from test_table_scan import _scan
    cases = snap_cases(orc)
    f = frames_table(orc, [fr for _, fr, _ in cases])
    want, werr = orc.table_scan_expect(f)
    assert werr is None
    data = [w for w in want if w[2] == 0]
    assert [w[4] for w in data] == [0 if w is not None else 3 for _, _, w in cases]
    got, err = _scan(lcrc, engines[lcrc.MODE_REF], f)
    assert err is None and _as_tuples(got) == want


@pytest.mark.gpu
def test_snap_rules_device_index(lcrc, orc, engines):
    """An index block stored as a Snappy frame whose chunk uses the edge encodings snap accepts (10-byte preamble,
    an extended literal with exactly 4 bytes after its tag) decodes on the device (k_ts_open), and the ones snap
    rejects (a 2^32 preamble that truncates to the right length mod 2^32, a short extended literal at the end) are
    "corrupted compressed block content" from the synchronous scan, as from the oracle."""
    from test_table_scan import _scan
    from test_table_scan_async import _expect_async
    v = orc.varint
    blocks = b""
    entries = []
    for i in range(3):
        entries.append((b"key%d" % i, v(len(blocks)) + v(100)))
        blocks += orc.raw_block(bytes([65 + i]) * 100, 0)
    idx = orc.block_build(entries, 1)
    meta = orc.block_build([])

    def table(frame):
        f = bytearray(blocks)
        moff = len(f)
        f += orc.raw_block(meta, 0)
        ioff = len(f)
        f += orc.raw_block(frame, 1)
        foot = v(moff) + v(len(meta)) + v(ioff) + v(len(frame))
        foot += bytes(40 - len(foot)) + orc.TABLE_MAGIC.to_bytes(8, "little")
        return bytes(f + foot)

    def comp(payload):
        return STREAM + _chunk(orc, 0, payload, idx)

    n = len(idx)
    good = {
        "10-byte preamble": comp(_varu(n, 10) + _lit(idx)),
        "ext literals": comp(_varu(n, 2) + _lit(idx[:-3]) + _lit(idx[-3:], 1)),
    }
    bad = {
        "2^32 + n preamble": comp(_varu(n | (1 << 32), 5) + _lit(idx)),
        "short ext literal at end": comp(_varu(n, 2) + _lit(idx[:-2]) + _lit(idx[-2:], 1)),
    }
    eng = engines[lcrc.MODE_REF]
    for name, fr in good.items():
        f = table(fr)
        want, werr = orc.table_scan_expect(f)
        assert werr is None, name
        assert _expect_async(lcrc, eng, orc, f, snappy_index=True) == 0, name
        got, err = _scan(lcrc, eng, f)
        assert err is None and _as_tuples(got) == want, name
    for name, fr in bad.items():
        f = table(fr)
        assert orc.table_scan_expect(f) == (None, "corrupted compressed block content"), name
        assert _expect_async(lcrc, eng, orc, f, snappy_index=True) == 2, name  # LCRC_TSCAN_HOST
        assert _scan(lcrc, eng, f) == (None, "corrupted compressed block content"), name
