"""The product SSTable writer (csrc/lcrc_tbuild.cpp, the reference's TableBuilder: table.rs:295-454,
write_block / write_raw_block :470-529, block.rs:296-377) against the oracle's independent restatement
(oracle.table_build): byte-identical files for every block size, restart interval, compression (the Snappy
keep-if-smaller-than-7/8 decision of table.rs:489), filter block (written with the compression type as its
type byte, table.rs:383-391) and CRC mode; and the device seal of the writer's descriptors
(lcrc_batch_seal, {offset, n + 1, n + 1}) producing the same trailers as the host."""
import numpy as np
import pytest

from test_table_scan import FILTER, _kvs


def _build(lcrc, kvs, block_size=4096, restart_interval=16, compression=0, mode=0, flags=0, host_seal=True,
           filter_name=None, filter_block=b""):
    tb = lcrc.TableBuilder(block_size, restart_interval, compression, mode, flags, host_seal)
    for k, v in kvs:
        tb.add(k, v)
    return tb, tb.finish(filter_name, filter_block)


@pytest.mark.parametrize("block_size,compression,filt", [(4096, 0, False), (4096, 1, True), (1024, 1, False),
                                                         (512, 0, True), (65536, 1, True), (1, 0, False)])
def test_writer_bytes_equal_oracle(lcrc, orc, block_size, compression, filt):
    kvs = _kvs(3000, block_size + compression)
    kw = dict(filter_name=FILTER, filter_block=b"F" * 123) if filt else {}
    tb, got = _build(lcrc, kvs, block_size=block_size, compression=compression, **kw)
    want, blocks = orc.table_build(kvs, block_size=block_size, compression=compression, **kw)
    assert got == want
    b = tb.blocks()
    assert [(int(x["offset"]), int(x["size"]), int(x["kind"])) for x in b] == list(blocks)
    # the trailer slot of every block holds the crc the writer reports
    for x in b:
        o, n = int(x["offset"]), int(x["size"])
        assert got[o + n] == int(x["type"])
        assert int.from_bytes(got[o + n + 1:o + n + 5], "little") == int(x["crc"])


@pytest.mark.parametrize("mode,masked", [(0, False), (1, False), (1, True)])
def test_writer_modes(lcrc, orc, mode, masked):
    kvs = _kvs(1500, 9)
    _, got = _build(lcrc, kvs, compression=1, mode=mode, flags=lcrc.FLAG_MASK if masked else 0,
                    filter_name=FILTER, filter_block=b"z" * 40)
    want, _ = orc.table_build(kvs, compression=1, mode=mode, masked=masked, filter_name=FILTER, filter_block=b"z" * 40)
    assert got == want


def test_writer_restart_interval_and_empty(lcrc, orc):
    kvs = _kvs(800, 4)
    for ri in (1, 2, 16, 100):
        _, got = _build(lcrc, kvs, restart_interval=ri)
        assert got == orc.table_build(kvs, restart_interval=ri)[0]
    _, got = _build(lcrc, [])  # an empty table: empty metaindex and index blocks, then the footer
    assert got == orc.table_build([])[0]


def test_writer_rejects_unsorted_keys(lcrc):
    tb = lcrc.TableBuilder()
    tb.add(b"b", b"1")
    with pytest.raises(lcrc.LcrcError):
        tb.add(b"a", b"2")
    with pytest.raises(lcrc.LcrcError):
        tb.add(b"b", b"2")


def test_writer_seal_descriptors(lcrc):
    tb, f = _build(lcrc, _kvs(2000, 6), compression=1, host_seal=False, filter_name=FILTER, filter_block=b"q" * 9)
    b, d = tb.blocks(), tb.seal_descs()
    assert len(b) == len(d) and (b["crc"] == 0).all()
    assert (d["offset"] == b["offset"]).all()
    assert (d["length"] == b["size"] + 1).all() and (d["expect_rel"] == b["size"] + 1).all()
    kinds = b["kind"].tolist()
    assert kinds[-3:] == [lcrc.TBLK_FILTER, lcrc.TBLK_METAINDEX, lcrc.TBLK_INDEX]


@pytest.mark.gpu
@pytest.mark.parametrize("mode,flags", [(0, 0), (1, 1)])
def test_writer_device_seal_equals_host_seal(lcrc, orc, mode, flags):
    """The writer leaves the trailers zero; ONE lcrc_batch_seal over its descriptors fills every data,
    filter, metaindex and index trailer: the file equals the host-sealed (reference-equivalent) one, and the
    whole-table scan verifies it clean."""
    kvs = _kvs(6000, 8)
    kw = dict(block_size=2048, compression=1, mode=mode, flags=flags, filter_name=FILTER, filter_block=b"f" * 50)
    _, host = _build(lcrc, kvs, host_seal=True, **kw)
    tb, zero = _build(lcrc, kvs, host_seal=False, **kw)
    assert zero != host
    d = tb.seal_descs()
    dev = lcrc.DeviceBuffer.from_host(np.frombuffer(zero, np.uint8))
    dd = lcrc.DeviceBuffer.from_host(d.view(np.uint8))
    eng = lcrc.Engine(0, mode, flags)
    eng.batch_seal(dev, len(zero), dd, len(d))
    eng.sync()
    assert dev.download(np.uint8, len(zero)).tobytes() == host
    out = eng.table_scan(dev, len(zero), FILTER)
    want, err = orc.table_scan_expect(host, FILTER, mode, bool(flags))
    assert err is None
    # every block verifies; the filter block alone is flagged "corrupted compressed block content" (status 3):
    # the reference stores it raw under the Snappy type byte (table.rs:383-391), read_block_from_file then
    # fails to decode it
    assert [(int(r["offset"]), int(r["size"]), int(r["kind"]), int(r["type"]), int(r["status"])) for r in out] == \
        [w[:5] for w in want]
    assert [int(r["status"]) for r in out if r["kind"] != lcrc.TBLK_FILTER] == [0] * (len(out) - 1)
    eng.close()
