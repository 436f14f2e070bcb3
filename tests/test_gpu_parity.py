"""Device parity: every batched path on the gfx950 kernels against the CPU oracle, bit-exact.
Run on the MI355X box with `pytest -m gpu`."""
import json
import os

import numpy as np
import pytest

import logtests

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MODES = [0, 1]


def _gold(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def _uniform(lcrc, eng, data, n, length, stride, expected=None):
    base = lcrc.DeviceBuffer.from_host(data)
    out = lcrc.DeviceBuffer(max(4 * n, 4))
    mm = lcrc.DeviceBuffer(max(4 * ((n + 31) // 32), 4))
    exp = lcrc.DeviceBuffer.from_host(np.asarray(expected, np.uint32)) if expected is not None else None
    eng.batch_uniform(base, n, length, stride, out, expected=exp, out_mismatch=mm)
    eng.sync()
    return out.download(np.uint32, n), lcrc.unpack_bits(mm.download(np.uint32, (n + 31) // 32), n)


@pytest.mark.parametrize("mode", MODES)
def test_config1_golden_fast_path(lcrc, orc, engines, mode):
    g = _gold("config1_golden.json")
    data = orc.splitmix_bytes(g["seed"], g["nblocks"] * g["block_len"])
    got, mm = _uniform(lcrc, engines[mode], data, 1024, 4096, 4096)
    want = [int(x, 16) for x in g["crc_c" if mode else "crc_ref"]]
    assert got.tolist() == want
    assert not mm.any()


def test_config1_masked_and_verify(lcrc, orc):
    g = _gold("config1_golden.json")
    data = orc.splitmix_bytes(g["seed"], g["nblocks"] * g["block_len"])
    eng = lcrc.Engine(0, lcrc.MODE_C, lcrc.FLAG_MASK)
    exp = np.array([int(x, 16) for x in g["crc_c_masked"]], np.uint32)
    bad = [0, 5, 31, 32, 1023]
    exp2 = exp.copy()
    exp2[bad] ^= 1
    got, mm = _uniform(lcrc, eng, data, 1024, 4096, 4096, exp2)
    assert np.array_equal(got, exp)
    assert np.nonzero(mm)[0].tolist() == bad
    eng.close()


@pytest.mark.parametrize("mode", MODES)
def test_config2_full_size(lcrc, orc, engines, mode):
    """64K x 4 KiB (BASELINE configs[1]) -- every CRC against the oracle."""
    n = 65536
    data = orc.splitmix_bytes(0x5EED0001, n * 4096)
    got, _ = _uniform(lcrc, engines[mode], data, n, 4096, 4096)
    want = orc.crc_ranges(data, np.arange(n, dtype=np.uint64) * 4096, np.full(n, 4096), mode)
    assert np.array_equal(got, want)
    # size-independent property: xor of all block crcs
    assert int(np.bitwise_xor.reduce(got)) == int(np.bitwise_xor.reduce(want))


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 63, 64, 65, 1000, 4097])
def test_fast_path_ragged_counts(lcrc, orc, engines, n):
    data = orc.splitmix_bytes(n, n * 4096)
    for mode in MODES:
        got, _ = _uniform(lcrc, engines[mode], data, n, 4096, 4096)
        assert np.array_equal(got, orc.crc_ranges(data, np.arange(n) * 4096, np.full(n, 4096), mode))


@pytest.mark.parametrize("length,stride", [(1, 1), (1, 7), (3, 5), (16, 16), (100, 105), (255, 256), (256, 256),
                                           (257, 300), (4095, 4100), (4096, 4101), (4097, 4097), (8192, 8192),
                                           (20000, 20005), (65536, 65536)])
def test_uniform_general(lcrc, orc, engines, length, stride):
    n = max(1, min(3000, (4 << 20) // stride))
    data = orc.splitmix_bytes(length * 31 + stride, (n - 1) * stride + length)
    for mode in MODES:
        got, _ = _uniform(lcrc, engines[mode], data, n, length, stride)
        want = orc.crc_ranges(data, np.arange(n, dtype=np.uint64) * stride, np.full(n, length), mode)
        assert np.array_equal(got, want), (mode, np.nonzero(got != want)[0][:10])


def test_ranges_golden(lcrc, orc, engines):
    g = _gold("ranges_golden.json")
    data = orc.splitmix_bytes(g["seed"], g["buffer_len"])
    offs = [r["offset"] for r in g["ranges"]]
    lens = [r["length"] for r in g["ranges"]]
    for mode, key in ((0, "crc_ref"), (1, "crc_c")):
        crcs, _ = engines[mode].crc_ranges(data, offs, lens)
        assert [f"{v:08x}" for v in crcs] == [r[key] for r in g["ranges"]]


@pytest.mark.parametrize("seed", range(4))
def test_random_ranges(lcrc, orc, engines, seed):
    rng = np.random.default_rng(seed)
    total = 3 << 20
    data = orc.splitmix_bytes(1000 + seed, total)
    n = 3000
    lens = np.minimum(rng.integers(0, 1 << rng.integers(1, 18, n)), total).astype(np.uint32)
    offs = np.array([int(rng.integers(0, total - l + 1)) for l in lens], np.uint64)  # overlapping, unsorted
    for mode in MODES:
        crcs, _ = engines[mode].crc_ranges(data, offs, lens)
        want = orc.crc_ranges(data, offs, lens, mode)
        assert np.array_equal(crcs, want), np.nonzero(crcs != want)[0][:10]


def test_direct_mode_matches(lcrc, orc):
    rng = np.random.default_rng(9)
    data = orc.splitmix_bytes(77, 1 << 20)
    lens = rng.integers(0, 20000, 500).astype(np.uint32)
    offs = np.array([int(rng.integers(0, (1 << 20) - l + 1)) for l in lens], np.uint64)
    for mode in MODES:
        eng = lcrc.Engine(0, mode, lcrc.FLAG_DIRECT)
        crcs, _ = eng.crc_ranges(data, offs, lens)
        assert np.array_equal(crcs, orc.crc_ranges(data, offs, lens, mode))
        eng.close()


def test_edges_at_buffer_bounds(lcrc, orc, engines):
    data = orc.splitmix_bytes(5, 70000)
    offs, lens = [], []
    for l in range(0, 40):
        offs += [0, 70000 - l]
        lens += [l, l]
    offs += [1, 15, 16, 17, 69999]
    lens += [69999, 100, 69984, 5000, 1]
    for mode in MODES:
        crcs, _ = engines[mode].crc_ranges(data, offs, lens)
        assert np.array_equal(crcs, orc.crc_ranges(data, offs, lens, mode))


def _sstable(lcrc, orc, seed, nblocks):
    rng = np.random.default_rng(seed)
    t = lcrc.TableFile()
    handles = []
    for _ in range(nblocks):
        n = int(rng.integers(0, 70000)) if rng.random() < 0.3 else int(rng.integers(3000, 5000))
        handles.append(t.write_raw_block(rng.integers(0, 256, n, dtype=np.uint8).tobytes(), int(rng.integers(0, 2))))
    return bytearray(t.contents()), handles


def test_sstable_verify_batch(lcrc, orc, engines):
    """Batched read_block_from_file verify (format.rs:162-171): desc {off, n+1, expect_rel n+1}."""
    f, handles = _sstable(lcrc, orc, 3, 400)
    bad = [0, 17, 200, 399]
    for i in bad:
        off, size = handles[i]
        f[off + size // 2 if size else off] ^= 0x10  # corrupt content (or the type byte of an empty block)
    offs = [h[0] for h in handles]
    lens = [h[1] + 1 for h in handles]
    crcs, mm = engines[0].crc_ranges(np.frombuffer(bytes(f), np.uint8), offs, lens, expect_rel=np.array(lens))
    assert np.nonzero(mm)[0].tolist() == bad
    assert np.array_equal(crcs, orc.crc_ranges(bytes(f), offs, lens, 0))
    for i in range(len(handles)):
        _, err = lcrc.TableFile.read_block(bytes(f), handles[i][0], handles[i][1], True)
        assert (err == "block checksum mismatch") == (i in bad) or err == "bad block type"


@pytest.mark.parametrize("length,stride", [(4096, 4096), (1000, 1024), (4096, 4101)])
def test_host_resident_pipeline(lcrc, orc, engines, length, stride):
    n = 20000
    data = orc.splitmix_bytes(length + stride, (n - 1) * stride + length)
    want = orc.crc_ranges(data, np.arange(n, dtype=np.uint64) * stride, np.full(n, length), 1)
    exp = want.copy()
    exp[[3, 9999]] ^= 0xFF
    got, mm = engines[1].batch_host_uniform(data, n, length, stride, expected=exp, chunk_bytes=8 << 20)
    assert np.array_equal(got, want)
    assert np.nonzero(lcrc.unpack_bits(mm, n))[0].tolist() == [3, 9999]


# ---- WAL path -------------------------------------------------------------------------------------
def _batch_reader(lcrc, engines):
    return lambda data: lcrc.BatchLogReader(data, engines[0])


@pytest.mark.parametrize("scenario", [s for s in logtests.SCENARIOS], ids=lambda f: f.__name__)
def test_wal_reference_scenarios_on_device(lcrc, engines, scenario):
    scenario(logtests.Tester(lcrc, _batch_reader(lcrc, engines)))


def test_wal_random_read_on_device(lcrc, engines):
    logtests.t_random_read(logtests.Tester(lcrc, _batch_reader(lcrc, engines)), np.random.default_rng(5))


@pytest.mark.parametrize("seed", range(10))
def test_wal_batch_equals_host_reader_under_corruption(lcrc, orc, engines, seed):
    rng = np.random.default_rng(500 + seed)
    recs = []
    for _ in range(400):
        k = int(rng.integers(1, 17))
        recs.append(rng.integers(0, 256, int(rng.integers(0, 1 << k)), dtype=np.uint8).tobytes())
    data = bytearray(orc.log_write(recs))
    for _ in range(int(rng.integers(0, 8))):
        pos = int(rng.integers(0, len(data)))
        data[pos] ^= 1 << int(rng.integers(0, 8))
    if rng.random() < 0.5:
        del data[len(data) - int(rng.integers(1, 200)):]
    b = lcrc.BatchLogReader(bytes(data), engines[0])
    got = (b.records(), b.dropped_bytes, b.report_message)
    assert b.consistency_errors == 0
    assert got == orc.log_read_all(bytes(data))
    # per-record device crcs equal the oracle over type ++ payload
    sc = b.records_scanned
    for r in sc[:: max(1, len(sc) // 50)]:
        h = int(r["header"])
        body = bytes(data[h + 6:h + 7 + int(r["length"])])
        assert int(r["crc"]) == orc.crc(body, 0)
        assert int(r["status"]) == (int.from_bytes(data[h:h + 4], "little") != orc.crc(body, 0))


def _wal_expect(orc, data):
    """(header, length, type) of every physical record the reader's header walk visits (log.rs:204-279)."""
    out = []
    for b0 in range(0, len(data), 32768):
        blk = data[b0:b0 + 32768]
        at = 0
        while len(blk) - at >= 7:
            n = blk[at + 4] | (blk[at + 5] << 8)
            t = blk[at + 6]
            if 7 + n > len(blk) - at or (t == 0 and n == 0):
                break
            out.append((b0 + at, n, t))
            at += 7 + n
    return out


def test_wal_scan_many_records_per_block(lcrc, orc, engines):
    """Blocks holding far more records than the parse keeps per block (the emit re-walks them)."""
    rng = np.random.default_rng(77)
    recs = [rng.integers(0, 256, int(rng.integers(0, 4)), dtype=np.uint8).tobytes() for _ in range(30000)]
    recs += [rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()]  # and a multi-block record
    data = orc.log_write(recs)
    dev = lcrc.DeviceBuffer.from_host(np.frombuffer(data, np.uint8))
    got = engines[0].wal_scan(dev, len(data))
    want = _wal_expect(orc, data)
    assert [(int(r["header"]), int(r["length"]), int(r["type"])) for r in got] == want
    assert (got["status"] == 0).all()
    for r in got[::997]:
        h = int(r["header"])
        assert int(r["crc"]) == orc.crc(data[h + 6:h + 7 + int(r["length"])], 0)
    # too small a capacity: LCRC_EINVAL and the count
    import ctypes
    small = lcrc.DeviceBuffer(10 * lcrc.WAL_REC_DTYPE.itemsize)
    n = ctypes.c_size_t(0)
    rc = lcrc.lib().lcrc_wal_scan(engines[0].ctx, dev.ptr, len(data), small.ptr, 10, ctypes.byref(n), None)
    assert rc == lcrc.EINVAL and n.value == len(want)
    assert small.download(lcrc.WAL_REC_DTYPE, 10)["header"].tolist() == [h for h, _, _ in want[:10]]


@pytest.mark.parametrize("shift", [0, 1, 3])
def test_wal_scan_file_tail_and_unaligned_base(lcrc, orc, engines, shift):
    """Files cut at every length over the last record headers (the file's last partial dword comes from
    direct loads, not the staged window), with the log at an unaligned device address."""
    import ctypes
    rng = np.random.default_rng(79)
    recs = [rng.integers(0, 256, int(rng.integers(0, 1 << int(rng.integers(1, 10)))), dtype=np.uint8).tobytes()
            for _ in range(400)]
    full = orc.log_write(recs)
    for cut in range(len(full) - 40, len(full) + 1):
        data = full[:cut]
        dev = lcrc.DeviceBuffer.from_host(np.frombuffer(b"\x5a" * shift + data + b"\xa5" * 5, np.uint8))
        cap = len(data) // 7 + 1
        out = lcrc.DeviceBuffer(cap * lcrc.WAL_REC_DTYPE.itemsize)
        n = ctypes.c_size_t(0)
        rc = lcrc.lib().lcrc_wal_scan(engines[0].ctx, ctypes.c_void_p(dev.ptr + shift), len(data), out.ptr, cap,
                                      ctypes.byref(n), None)
        assert rc == 0
        got = out.download(lcrc.WAL_REC_DTYPE, n.value)
        assert [(int(r["header"]), int(r["length"]), int(r["type"])) for r in got] == _wal_expect(orc, data), cut


def test_wal_scan_async_matches_sync(lcrc, orc, engines):
    rng = np.random.default_rng(78)
    recs = [rng.integers(0, 256, int(rng.integers(0, 1 << int(rng.integers(1, 17)))), dtype=np.uint8).tobytes()
            for _ in range(300)]
    data = orc.log_write(recs)
    dev = lcrc.DeviceBuffer.from_host(np.frombuffer(data, np.uint8))
    sync = engines[1].wal_scan(dev, len(data))
    cap = len(data) // 7 + 1
    rd = lcrc.DeviceBuffer(cap * lcrc.WAL_REC_DTYPE.itemsize)
    cnt = lcrc.DeviceBuffer(8)
    engines[1].wal_scan_async(dev, len(data), rd, cap, cnt)
    engines[1].sync()
    n = int(cnt.download(np.uint64, 1)[0])
    assert n == len(sync)
    assert rd.download(lcrc.WAL_REC_DTYPE, n).tobytes() == sync.tobytes()
    # an empty log
    empty = lcrc.DeviceBuffer(16)
    assert len(engines[1].wal_scan(empty, 0)) == 0


def test_graph_replay_matches_direct(lcrc, orc):
    """lcrc_graph_begin/end/launch: two reserved uniform batches captured once, replayed twice; the replay
    rewrites the outputs with the same CRCs as the direct calls."""
    eng = lcrc.Engine(0, lcrc.MODE_C)
    n = 3000
    data = [orc.splitmix_bytes(0x6A0 + k, n * 4096) for k in range(2)]
    bufs = [lcrc.DeviceBuffer.from_host(d) for d in data]
    outs = [lcrc.DeviceBuffer(4 * n) for _ in range(2)]
    want = [orc.crc_ranges(d, np.arange(n, dtype=np.uint64) * 4096, np.full(n, 4096), 1) for d in data]
    for k in range(2):  # direct calls first (the fast path allocates nothing)
        eng.batch_uniform(bufs[k], n, 4096, 4096, outs[k])
    eng.sync()
    for k in range(2):
        assert np.array_equal(outs[k].download(np.uint32, n), want[k])
    g = eng.graph_capture(lambda: [eng.batch_uniform(bufs[k], n, 4096, 4096, outs[k]) for k in range(2)])
    try:
        for _ in range(2):
            for o in outs:
                o.zero()
            eng.graph_launch(g)
            eng.sync()
            for k in range(2):
                assert np.array_equal(outs[k].download(np.uint32, n), want[k])
    finally:
        eng.graph_destroy(g)
    eng.close()


def test_graph_replay_general_path_and_wal(lcrc, orc):
    """The general path (k_windows + k_blocks over descriptors) and the device-only WAL scan captured in one
    HIP graph after lcrc_ctx_reserve, replayed: the same CRCs, verdicts, records and counts as direct calls."""
    eng = lcrc.Engine(0, lcrc.MODE_C, lcrc.FLAG_MASK)
    rng = np.random.default_rng(91)
    data = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    offs = np.sort(rng.choice(len(data) - 70000, 500, replace=False)).astype(np.uint64)
    lens = rng.integers(0, 70000, 500).astype(np.uint32)
    d = np.zeros(500, lcrc.DESC_DTYPE)
    d["offset"], d["length"], d["expect_rel"] = offs, lens, lcrc.NO_EXPECT
    base = lcrc.DeviceBuffer.from_host(data)
    dd = lcrc.DeviceBuffer.from_host(d.view(np.uint8))
    out = lcrc.DeviceBuffer(4 * 500)
    recs = [rng.integers(0, 256, int(rng.integers(0, 1 << int(rng.integers(1, 15)))), dtype=np.uint8).tobytes()
            for _ in range(200)]
    log = orc.log_write(recs)
    ldev = lcrc.DeviceBuffer.from_host(np.frombuffer(log, np.uint8))
    cap = len(log) // 7 + 1
    rd = lcrc.DeviceBuffer(cap * lcrc.WAL_REC_DTYPE.itemsize)
    cnt = lcrc.DeviceBuffer(8)
    eng.reserve(max(len(data), len(log)))
    want_wal = eng.wal_scan(ldev, len(log))
    want_crc = np.array([orc.mask(int(c)) for c in orc.crc_ranges(data.tobytes(), offs, lens, 1)], np.uint32)

    def calls():
        eng.batch(base, len(data), dd, 500, out)
        eng.wal_scan_async(ldev, len(log), rd, cap, cnt)

    g = eng.graph_capture(calls)
    try:
        for _ in range(2):
            out.zero()
            cnt.zero()
            eng.graph_launch(g)
            eng.sync()
            assert np.array_equal(out.download(np.uint32, 500), want_crc)
            n = int(cnt.download(np.uint64, 1)[0])
            assert n == len(want_wal)
            assert rd.download(lcrc.WAL_REC_DTYPE, n).tobytes() == want_wal.tobytes()
    finally:
        eng.graph_destroy(g)
    eng.close()


def test_ctx_options_reserved_refused(lcrc):
    """lcrc_ctx_options.reserved[3] held the round-5 measurement variants (wal_onepass, ts_open_v1, ts_unfused),
    removed in round 6: a non-zero word is refused with LCRC_EINVAL and a message; zero words create a context."""
    import ctypes
    for k in range(3):
        o = lcrc._CtxOptions()
        o.size = ctypes.sizeof(lcrc._CtxOptions)
        o.reserved[k] = 1
        ctx = ctypes.c_void_p()
        assert lcrc.lib().lcrc_ctx_create_ex(ctypes.byref(ctx), 0, lcrc.MODE_C, 0, ctypes.byref(o)) == lcrc.EINVAL
        assert not ctx.value and b"reserved" in lcrc.lib().lcrc_last_error()
    o = lcrc._CtxOptions()
    o.size = ctypes.sizeof(lcrc._CtxOptions)
    ctx = ctypes.c_void_p()
    assert lcrc.lib().lcrc_ctx_create_ex(ctypes.byref(ctx), 0, lcrc.MODE_C, 0, ctypes.byref(o)) == 0 and ctx.value
    assert lcrc.lib().lcrc_ctx_destroy(ctx) == 0


@pytest.mark.parametrize("path", ["ranges", "blocks"])
def test_general_path_variants(lcrc, orc, path):
    """Both general-path kernels, forced through the context option `general` (lcrc_ctx_create_ex): k_ranges (one
    streaming pass in 4 KiB chunks) and k_windows + k_blocks, on random ranges (empty, 1-3 bytes, unaligned,
    multi-chunk, long), uniform layouts, and a WAL scan -- bit-exact against the oracle."""
    rng = np.random.default_rng(4242)
    data = rng.integers(0, 256, 6 << 20, dtype=np.uint8)
    n = 3000
    lens = np.concatenate([[0, 1, 2, 3, 4, 5, 4095, 4096, 4097, 8191, 8192, 8193, 300000],
                           rng.integers(0, 70000, n - 13)]).astype(np.uint32)
    offs = np.array([int(rng.integers(0, len(data) - int(L))) for L in lens], np.uint64)
    for mode in MODES:
        eng = lcrc.Engine(0, mode, lcrc.FLAG_MASK if mode else 0, general=path)
        crcs, _ = eng.crc_ranges(data, offs, lens)
        want = orc.crc_ranges(data.tobytes(), offs, lens, mode)
        if mode:
            want = np.array([orc.mask(int(c)) for c in want], np.uint32)
        assert np.array_equal(crcs, want), np.nonzero(crcs != want)[0][:10]
        for length, stride in [(4092, 4096), (4096, 4101), (3000, 3001), (513, 1024)]:
            m_ = min(1500, (len(data) - length) // stride + 1)
            got, _ = _uniform(lcrc, eng, data, m_, length, stride)
            w = orc.crc_ranges(data.tobytes(), np.arange(m_, dtype=np.uint64) * stride, np.full(m_, length), mode)
            if mode:
                w = np.array([orc.mask(int(c)) for c in w], np.uint32)
            assert np.array_equal(got, w), (length, stride)
        eng.close()
    recs = [rng.integers(0, 256, int(rng.integers(0, 1 << int(rng.integers(1, 16)))), dtype=np.uint8).tobytes()
            for _ in range(300)]
    log = orc.log_write(recs)
    eng = lcrc.Engine(0, lcrc.MODE_REF, general=path)
    got = eng.wal_scan(lcrc.DeviceBuffer.from_host(np.frombuffer(log, np.uint8)), len(log))
    want = _wal_expect(orc, log)
    assert [(int(r["header"]), int(r["length"]), int(r["type"])) for r in got] == want
    assert (got["status"] == 0).all()
    assert [int(c) for c in got["crc"]] == [orc.crc(log[h + 6:h + 7 + n], 0) for h, n, _ in want]
    eng.close()


@pytest.mark.parametrize("path", ["ranges", "blocks"])
def test_out_of_bounds_descriptors(lcrc, orc, path):
    """A range outside [0, base_len) is never read: CRC 0 and its mismatch bit set; in-bounds neighbours are
    unaffected. The in-place store of lcrc_batch_seal never writes outside the buffer either."""
    data = bytes(orc.splitmix_bytes(99, 1 << 20))
    n0 = len(data)
    offs = np.array([0, 100, n0 - 10, n0, n0 + 5, 2 ** 40, 5000], np.uint64)
    lens = np.array([4096, 300, 10, 0, 1, 16, 70000], np.uint32)
    ok = (offs <= n0) & (lens.astype(np.uint64) <= n0 - np.minimum(offs, n0))
    eng = lcrc.Engine(0, lcrc.MODE_C, general=path)
    crcs, mm = eng.crc_ranges(data, offs, lens)
    want = orc.crc_ranges(data, offs[ok], lens[ok], 1)
    assert np.array_equal(crcs[ok], want)
    assert (crcs[~ok] == 0).all()
    assert mm.tolist() == (~ok).tolist()
    # seal: the expected-value slot of descriptor 1 lies past the end -> not written
    buf = lcrc.DeviceBuffer.from_host(np.frombuffer(data, np.uint8))
    d = np.zeros(2, lcrc.DESC_DTYPE)
    d["offset"], d["length"], d["expect_rel"] = [0, n0 - 8], [64, 8], [64, 6]
    dd = lcrc.DeviceBuffer.from_host(d.view(np.uint8))
    eng.batch_seal(buf, n0, dd, 2)
    eng.sync()
    after = buf.download(np.uint8, n0).tobytes()
    assert after[:64] == data[:64] and after[68:] == data[68:]
    assert int.from_bytes(after[64:68], "little") == orc.crc(data[:64], 1)
    eng.close()


@pytest.mark.parametrize("path", ["ranges", "blocks", "covered", "direct"])
def test_mismatch_bitmap_not_prefilled(lcrc, orc, path):
    """lcrc_batch / lcrc_batch_covered fill no bitmap before the kernel: every range sets or clears its own
    bit and the last range clears the bits past n. A bitmap full of ones comes back exact (bad ranges only,
    zero past n) and the word after it is untouched, twice in a row."""
    opts = {"general": path} if path in ("ranges", "blocks") else {}
    rng = np.random.default_rng(77)
    for n in (77, 64, 1):
        # ranges back to back, each followed by its 4-byte expected slot; ~70 % hold the right CRC
        lens = rng.integers(1, 9000, n).astype(np.uint32)
        offs = np.zeros(n, np.uint64)
        offs[1:] = np.cumsum(lens.astype(np.uint64) + 4)[:-1] + 3  # unaligned starts
        host = np.frombuffer(bytes(orc.splitmix_bytes(0xB17 + n, int(offs[-1]) + int(lens[-1]) + 8)), np.uint8).copy()
        want_crc = orc.crc_ranges(host.tobytes(), offs, lens, 1)
        want_bad = rng.random(n) < 0.3
        for o, L, c, b in zip(offs, lens, want_crc, want_bad):
            v = int(c) ^ (1 if b else 0)
            host[int(o) + int(L):int(o) + int(L) + 4] = np.frombuffer(v.to_bytes(4, "little"), np.uint8)
        d = np.zeros(n, lcrc.DESC_DTYPE)
        d["offset"], d["length"], d["expect_rel"] = offs, lens, lens.astype(np.int64)
        eng = lcrc.Engine(0, lcrc.MODE_C, lcrc.FLAG_DIRECT if path == "direct" else 0, **opts)
        base = lcrc.DeviceBuffer.from_host(host)
        dd = lcrc.DeviceBuffer.from_host(d.view(np.uint8))
        words = (n + 31) // 32
        out, mm = lcrc.DeviceBuffer(4 * n), lcrc.DeviceBuffer(4 * (words + 1))
        for _ in range(2):
            mm.upload(np.full(words + 1, 0xFFFFFFFF, np.uint32).view(np.uint8))
            eng.batch(base, len(host), dd, n, out, mm, covered=int(lens.sum()) if path == "covered" else None)
            eng.sync()
            assert np.array_equal(out.download(np.uint32, n), want_crc)
            got = mm.download(np.uint32, words + 1)
            assert got[words] == 0xFFFFFFFF
            want_words = np.zeros(words, np.uint32)
            for i in np.nonzero(want_bad)[0]:
                want_words[i >> 5] |= np.uint32(1 << (i & 31))
            assert np.array_equal(got[:words], want_words), (n, got[:words], want_words)
        eng.close()


# ---- round 2: BASELINE configs[2] at full size, the queue API, unaligned bases, large logs ------------------
@pytest.mark.parametrize("path", ["blocks", "ranges"])
def test_config3_mixed_sstable_full_size(lcrc, orc, synth, path):
    """BASELINE configs[2] exactly as bench.py's mixed leg builds it: synth.mixed_sizes(256 MiB) (zipf 1.1 over
    256 B-64 KiB) laid out by synth.sstable_layout, every block's trailer sealed with the oracle's CRC (REF:
    the reference's crc32fast bytes; C: masked CRC-32C), a few blocks corrupted, then ONE lcrc_batch with
    {off, n + 1, expect n + 1} (format.rs:162-171): every CRC equals the oracle's and exactly the corrupted
    blocks are flagged. Both general paths (k_windows + k_blocks, k_ranges)."""
    sizes = synth.mixed_sizes(256 << 20)
    offs, total = synth.sstable_layout(sizes)
    lens = sizes.astype(np.uint64) + 1
    base = synth.splitmix_bytes(synth.SEED_MIXED + 1000, total)
    bad = [0, 1, 777, len(sizes) // 2, len(sizes) - 1]
    for mode, flags, algo in ((0, 0, orc.ALGO_PCLMUL_REF), (1, lcrc.FLAG_MASK, orc.ALGO_SSE42_C)):
        want, _ = orc.crc_ranges_mt(base, offs, lens, 8, algo)
        if mode:
            want = orc.mask_array(want)
        f = base.copy()
        slot = (offs + lens).astype(np.int64)
        for k in range(4):
            f[slot + k] = ((want >> np.uint32(8 * k)) & 0xFF).astype(np.uint8)
        for i in bad:
            f[int(offs[i] + lens[i] // 2)] ^= 0x40
        eng = lcrc.Engine(0, mode, flags, general=path)
        crcs, mm = eng.crc_ranges(f, offs, lens, expect_rel=lens.astype(np.int64))
        eng.close()
        got_want, _ = orc.crc_ranges_mt(f, offs, lens, 8, algo)
        if mode:
            got_want = orc.mask_array(got_want)
        assert np.array_equal(crcs, got_want), (mode, np.nonzero(crcs != got_want)[0][:10])
        assert np.nonzero(mm)[0].tolist() == bad
        assert int(np.bitwise_xor.reduce(crcs)) == int(np.bitwise_xor.reduce(got_want))


def test_uniform_queue_matches_batches(lcrc, orc):
    """lcrc_batch_uniform_queue: 37 independent 4 KiB batches (ragged counts, an empty one, expected values
    with injected mismatches, one at an unaligned address) in one call -- two launches of the queued kernel --
    give exactly the CRCs and mismatch bits of 37 separate batches; a 4,000/4,100 B queue runs batch by batch."""
    eng = lcrc.Engine(0, lcrc.MODE_C, lcrc.FLAG_MASK)
    counts = [4096, 1, 3, 0, 5, 4097, 1000, 2] + [64] * 29
    jobs, want, bad = [], [], []
    keep = []
    for k, n in enumerate(counts):
        shift = 3 if k == 6 else 0
        data = orc.splitmix_bytes(0x9000 + k, n * 4096)
        w = orc.mask_array(orc.crc_ranges(data, np.arange(n, dtype=np.uint64) * 4096, np.full(n, 4096), 1))
        exp = w.copy()
        flip = [i for i in (0, 2, n - 1) if 0 <= i < n][: 1 + k % 2]
        exp[flip] ^= 0x10
        buf = lcrc.DeviceBuffer.from_host(np.concatenate([np.full(shift, 0x5A, np.uint8), data]), pad=16)
        out = lcrc.DeviceBuffer(max(4, 4 * n))
        ed = lcrc.DeviceBuffer.from_host(exp) if n else lcrc.DeviceBuffer(4)
        mm = lcrc.DeviceBuffer(max(4, 4 * ((n + 31) // 32)))
        keep += [buf, out, ed, mm]
        jobs.append((buf.ptr + shift, n, out, ed, mm))
        want.append(w)
        bad.append(sorted(set(flip)))
    eng.batch_uniform_queue(jobs, 4096, 4096)
    eng.sync()
    for k, n in enumerate(counts):
        assert np.array_equal(jobs[k][2].download(np.uint32, n), want[k]), k
        bits = lcrc.unpack_bits(jobs[k][4].download(np.uint32, (n + 31) // 32), n) if n else np.zeros(0, bool)
        assert np.nonzero(bits)[0].tolist() == bad[k], k
    # another layout: the queue runs its batches one by one through lcrc_batch_uniform
    data = orc.splitmix_bytes(0x9999, 300 * 4100)
    w = orc.mask_array(orc.crc_ranges(data, np.arange(300, dtype=np.uint64) * 4100, np.full(300, 4000), 1))
    buf = lcrc.DeviceBuffer.from_host(data)
    outs = [lcrc.DeviceBuffer(4 * 300) for _ in range(3)]
    eng.batch_uniform_queue([(buf, 300, o) for o in outs], 4000, 4100)
    eng.sync()
    for o in outs:
        assert np.array_equal(o.download(np.uint32, 300), w)
    eng.close()


@pytest.mark.parametrize("shift", [1, 2, 3, 5, 13])
def test_fast_path_unaligned_base(lcrc, orc, engines, shift):
    """The 4 KiB fast path (k_windows<true>) over a batch that starts at an arbitrary device address (an
    mmap'd .ldb file's blocks need not be aligned): the same CRCs as the oracle, tail blocks included."""
    n = 1003
    data = orc.splitmix_bytes(0x7700 + shift, n * 4096)
    dev = lcrc.DeviceBuffer.from_host(np.concatenate([np.full(shift, 0xA5, np.uint8), data]), pad=64)
    for mode in MODES:
        out = lcrc.DeviceBuffer(4 * n)
        engines[mode].batch_uniform(dev.ptr + shift, n, 4096, 4096, out)
        engines[mode].sync()
        want = orc.crc_ranges(data, np.arange(n, dtype=np.uint64) * 4096, np.full(n, 4096), mode)
        assert np.array_equal(out.download(np.uint32, n), want), mode


def test_wal_scan_hundreds_of_blocks(lcrc, orc, synth, engines):
    """A log of ~275 32 KiB blocks (not a multiple of the parse's 64 blocks per workgroup): the per-workgroup
    record counts, their prefix and the workgroup-0 total of k_wal_parse / k_wal_emit are all exercised. Every
    (header, length, type) equals the reference reader's header walk (log.rs:204-279) and every crc the
    oracle's, in both modes (REF: the stored crc32fast values verify; C: every record is flagged)."""
    w = lcrc.LogWriter()
    payload = synth.splitmix_bytes(0x4444, 1 << 17)
    for n in synth.wal_lengths(9_000_000, seed=0x4445):
        w.add_record(payload[:n] if n <= len(payload) else np.resize(payload, n))
    data = w.contents()
    nblocks = (len(data) + 32767) // 32768
    assert nblocks > 200 and nblocks % 64 != 0
    dev = lcrc.DeviceBuffer.from_host(np.frombuffer(data, np.uint8))
    want = _wal_expect(orc, data)
    h = np.array([x[0] for x in want], np.uint64)
    ln = np.array([x[1] for x in want], np.uint64)
    for mode in MODES:
        got = engines[mode].wal_scan(dev, len(data))
        assert [(int(r["header"]), int(r["length"]), int(r["type"])) for r in got] == want
        crc = orc.crc_ranges(data, h + 6, ln + 1, mode)
        assert np.array_equal(got["crc"], crc)
        assert (got["status"] == (0 if mode == 0 else 1)).all()


def test_wal_many_blocks_reference_size_on_device(lcrc, engines):
    """The reference's test_many_blocks at its own size (log.rs:535-545): 1,000,000 records written, every
    one read back through the device-verified BatchLogReader."""
    logtests.t_many_blocks(logtests.Tester(lcrc, _batch_reader(lcrc, engines)), 1000000)


def test_sparse_verify_in_a_large_file(lcrc, orc):
    """A few blocks verified inside a 1 GiB device buffer (Table::block_iter_from_index reading single data
    blocks, table.rs:114-146 -> format.rs:162-171): lcrc_batch_covered takes the one-pass range kernel, whose
    cost follows the 100 blocks read, not the buffer. Every CRC and mismatch bit equals the oracle's and the
    dense path's; the launch stays far below one pass over the buffer (~150 us)."""
    size = 1 << 30
    rng = np.random.default_rng(1234)
    base = lcrc.DeviceBuffer(size)
    offs = np.sort(rng.choice(size // 8192 - 1, 100, replace=False)).astype(np.uint64) * 8192 + \
        rng.integers(0, 4000, 100).astype(np.uint64)
    lens = np.full(100, 4097, np.uint32)
    host = {}
    for i, o in enumerate(offs):
        blk = bytearray(orc.splitmix_bytes(0x5A00 + i, 4097))
        c = orc.crc(bytes(blk), 0)
        if i in (7, 50):
            c ^= 1  # stored trailer wrong -> mismatch
        host[int(o)] = bytes(blk) + c.to_bytes(4, "little")
        base.upload(np.frombuffer(host[int(o)], np.uint8), int(o))
    d = np.zeros(100, lcrc.DESC_DTYPE)
    d["offset"], d["length"], d["expect_rel"] = offs, lens, lens
    dd = lcrc.DeviceBuffer.from_host(d.view(np.uint8))
    eng = lcrc.Engine(0, lcrc.MODE_REF)
    out, mm = lcrc.DeviceBuffer(400), lcrc.DeviceBuffer(16)
    eng.batch(base, size, dd, 100, out, mm, covered=int(lens.sum()))
    eng.sync()
    want = np.array([orc.crc(host[int(o)][:4097], 0) for o in offs], np.uint32)
    assert np.array_equal(out.download(np.uint32, 100), want)
    assert np.nonzero(lcrc.unpack_bits(mm.download(np.uint32, 4), 100))[0].tolist() == [7, 50]
    eng.timer_start()
    for _ in range(20):
        eng.batch(base, size, dd, 100, out, mm, covered=int(lens.sum()))
    us = eng.timer_stop() / 20 * 1e3
    print(f"sparse verify: 100 x 4,097 B in a 1 GiB buffer: {us:.1f} us per call")
    assert us < 60.0
    eng.close()


@pytest.mark.parametrize("path", ["auto", "ranges"])
def test_general_queue_matches_batches(lcrc, orc, path):
    """lcrc_batch_queue: 7 independent descriptor batches (different file sizes, an empty batch, a batch of
    zero-length file, expected values with injected mismatches, out-of-bounds descriptors) in one call, the
    window pass of each batch beside the previous batch's range pass on the context's second stream: the CRCs
    and mismatch bits of 7 separate lcrc_batch calls and of the oracle; then the same queue captured in a HIP
    graph (a fork and a join) and replayed twice."""
    rng = np.random.default_rng(0x9E)
    eng = lcrc.Engine(0, lcrc.MODE_C, lcrc.FLAG_MASK, general=path)
    jobs, want, keep = [], [], []
    for k, size in enumerate([3 << 20, 1 << 20, 5 << 20, 0, 2 << 20, 777_777, 4 << 20]):
        data = rng.integers(0, 256, max(size, 1), dtype=np.uint8)[:size]
        n = 0 if k == 1 else int(rng.integers(1, 900))
        lens = rng.integers(0, 70000, n).astype(np.uint32)
        offs = np.array([int(rng.integers(0, max(1, size - int(L) - 4))) for L in lens], np.uint64)
        if size == 0:
            lens[:] = 0
            offs[:] = 0
        rel = (lens.astype(np.int64) if size else np.full(n, lcrc.NO_EXPECT, np.int64)).astype(np.int32)
        ok = (offs + lens.astype(np.uint64) + 4 <= size) if size else np.zeros(n, bool)
        crc = np.array([orc.mask(int(c)) for c in orc.crc_ranges(data.tobytes(), offs, lens, 1)], np.uint32) if n \
            else np.zeros(0, np.uint32)
        f = data.copy()
        good = np.zeros(n, bool)
        for i in range(n):  # store the expected value after each range unless a later range overwrote it
            if ok[i] and rng.random() < 0.8:
                f[int(offs[i] + lens[i]):int(offs[i] + lens[i]) + 4] = np.frombuffer(int(crc[i]).to_bytes(4, "little"),
                                                                                       np.uint8)
        if n > 3 and size:  # two out-of-bounds descriptors
            offs[1], lens[1] = size + 3, 1
            offs[2], lens[2] = size - 2, 9
        inb = offs + lens.astype(np.uint64) <= size
        want_crc = np.zeros(n, np.uint32)
        if inb.any():
            want_crc[inb] = [orc.mask(int(c)) for c in orc.crc_ranges(f.tobytes(), offs[inb], lens[inb], 1)]
        for i in range(n):
            slot = int(offs[i]) + int(rel[i])
            good[i] = bool(inb[i]) and rel[i] != lcrc.NO_EXPECT and 0 <= slot and slot + 4 <= size and \
                int.from_bytes(f[slot:slot + 4].tobytes(), "little") == int(want_crc[i])
        want_mm = ~good if size else np.zeros(n, bool)
        want_mm[~inb] = True
        d = np.zeros(n, lcrc.DESC_DTYPE)
        d["offset"], d["length"], d["expect_rel"] = offs, lens, rel
        base = lcrc.DeviceBuffer.from_host(f if size else np.zeros(1, np.uint8))
        dd = lcrc.DeviceBuffer.from_host(d.view(np.uint8) if n else np.zeros(16, np.uint8))
        out = lcrc.DeviceBuffer(max(4, 4 * n))
        mm = lcrc.DeviceBuffer(max(4, 4 * ((n + 31) // 32)))
        keep += [base, dd, out, mm]
        jobs.append((base, size, dd, n, out, mm))
        want.append((want_crc, want_mm))

    def check():
        for (base, size, dd, n, out, mm), (wc, wm) in zip(jobs, want):
            got = out.download(np.uint32, n)
            assert np.array_equal(got, wc), np.nonzero(got != wc)[0][:10]
            assert lcrc.unpack_bits(mm.download(np.uint32, (n + 31) // 32), n).tolist() == wm.tolist()

    # separate lcrc_batch calls first, then the queue
    for base, size, dd, n, out, mm in jobs:
        eng.batch(base, size, dd, n, out, mm)
    eng.sync()
    check()
    for j in jobs:
        j[4].zero()
        j[5].upload(np.full(max(1, (j[3] + 31) // 32), 0xFFFFFFFF, np.uint32))
    eng.batch_queue(jobs)
    eng.sync()
    check()
    eng.reserve(5 << 20)
    arr = lcrc.gjobs(jobs)
    g = eng.graph_capture(lambda: eng.batch_queue(arr))
    try:
        for _ in range(2):
            for j in jobs:
                j[4].zero()
            eng.graph_launch(g)
            eng.sync()
            check()
    finally:
        eng.graph_destroy(g)
    eng.close()


def test_wal_scan_queue_matches_single_scans(lcrc, orc, engines):
    """lcrc_wal_scan_queue: 5 logs (different sizes, one empty, one with corrupted records, one whose last block
    is partial, one with max_recs 0) in one submission -- header walks in one launch, records in one more, window
    passes back to back, range passes on the side stream -- give exactly the records, verdicts and counts of 5
    separate lcrc_wal_scan_async calls; then the queue again in a HIP graph."""
    rng = np.random.default_rng(0xA11)
    eng = lcrc.Engine(0, lcrc.MODE_REF)
    logs = []
    for k, nrec in enumerate([300, 0, 900, 40, 200]):
        recs = [rng.integers(0, 256, int(rng.integers(0, 1 << int(rng.integers(1, 16)))), dtype=np.uint8).tobytes()
                for _ in range(nrec)]
        log = bytearray(orc.log_write(recs))
        if k == 2:
            for pos in rng.integers(0, len(log), 6):
                log[int(pos)] ^= 0x5A
        if k == 3:
            log = log[:len(log) - 1000] if len(log) > 5000 else log
        logs.append(bytes(log))
    jobs, want = [], []
    for k, log in enumerate(logs):
        dev = lcrc.DeviceBuffer.from_host(np.frombuffer(log, np.uint8) if log else np.zeros(1, np.uint8))
        cap = 0 if k == 4 else len(log) // 7 + 1
        rd = lcrc.DeviceBuffer(max(1, cap) * lcrc.WAL_REC_DTYPE.itemsize)
        cnt = lcrc.DeviceBuffer(8)
        eng.wal_scan_async(dev, len(log), rd, cap, cnt)
        eng.sync()
        n = int(cnt.download(np.uint64, 1)[0])
        want.append((n, rd.download(lcrc.WAL_REC_DTYPE, min(n, cap)).tobytes() if cap else b""))
        jobs.append((dev, len(log), rd, cap, cnt))

    def check():
        for (dev, flen, rd, cap, cnt), (n, recs) in zip(jobs, want):
            assert int(cnt.download(np.uint64, 1)[0]) == n
            if cap:
                assert rd.download(lcrc.WAL_REC_DTYPE, min(n, cap)).tobytes() == recs

    for j in jobs:
        j[2].zero()
        j[4].zero()
    eng.wal_scan_queue(jobs)
    eng.sync()
    check()
    arr = lcrc.wjobs(jobs)
    g = eng.graph_capture(lambda: eng.wal_scan_queue(arr))
    try:
        for _ in range(2):
            for j in jobs:
                j[2].zero()
                j[4].zero()
            eng.graph_launch(g)
            eng.sync()
            check()
    finally:
        eng.graph_destroy(g)
    eng.close()


@pytest.mark.parametrize("nctx", [1, 2, 3])
def test_batch_multi_shards(lcrc, orc, synth, nctx):
    """lcrc_batch_multi: a host-resident SSTable-layout file (BASELINE configs[2] sizes, 24 MiB)
    with corrupted blocks, unsorted and out-of-bounds descriptors appended, sharded over 1-3 contexts (several
    share the one GPU here; each shard has its own device buffer, stream and host thread) -- every CRC and
    mismatch bit equals the oracle's and the single-context lcrc_batch's."""
    sizes = synth.mixed_sizes(24 << 20, seed=synth.SEED_MIXED + 7)
    offs, total = synth.sstable_layout(sizes)
    f = np.frombuffer(bytes(orc.splitmix_bytes(0xABC, total)), np.uint8).copy()
    lens = sizes.astype(np.uint32) + 1
    crc = orc.crc_ranges(f.tobytes(), offs, lens, 1)
    for k, (o, L) in enumerate(zip(offs, lens)):
        v = int(crc[k]) ^ (1 if k % 97 == 5 else 0)
        f[int(o) + int(L):int(o) + int(L) + 4] = np.frombuffer(v.to_bytes(4, "little"), np.uint8)
    rng = np.random.default_rng(3)
    extra = rng.permutation(len(offs))[:200]
    offs2 = np.concatenate([offs, offs[extra], np.array([total - 3, total + 10, 2 ** 40], np.uint64)])
    lens2 = np.concatenate([lens, lens[extra], np.array([100, 1, 5], np.uint32)])
    xr = lens2.astype(np.int64)
    engs = [lcrc.Engine(0, lcrc.MODE_C) for _ in range(nctx)]
    got, bad = lcrc.batch_multi(engs, f, offs2, lens2, xr)
    ok = (offs2 <= total) & (lens2.astype(np.uint64) <= total - np.minimum(offs2, total))
    want = np.zeros(len(offs2), np.uint32)
    want[ok] = orc.crc_ranges(f.tobytes(), offs2[ok], lens2[ok], 1)
    assert np.array_equal(got, want)
    stored = np.array([int.from_bytes(f[int(o) + int(L):int(o) + int(L) + 4].tobytes(), "little")
                       if ok[k] and int(o) + int(L) + 4 <= total else -1
                       for k, (o, L) in enumerate(zip(offs2, lens2))], np.int64)
    assert np.array_equal(bad, ~ok | (stored != want.astype(np.int64)))
    one, one_bad = engs[0].crc_ranges(f, offs2, lens2, expect_rel=xr)
    assert np.array_equal(got, one) and np.array_equal(bad, one_bad)
    for e in engs:
        e.close()



def _wal_file(lcrc, synth, total, seed):
    """The bench's WAL file (BASELINE configs[3]): synth.wal_lengths records through the LogWriter restatement."""
    w = lcrc.LogWriter()
    payload = synth.splitmix_bytes(seed + 1000, 1 << 20)
    for n in synth.wal_lengths(total, seed=seed):
        w.add_record(payload[:n] if n <= len(payload) else np.resize(payload, n))
    return bytearray(w.contents())


def _wal_check_scan(lcrc, orc, eng, data, mode):
    """Every (header, length, type) of the device scan equals the reference reader's header walk
    (log.rs:204-279), every crc the oracle's over type ++ payload, every verdict the stored-vs-computed compare
    (log.rs:260-273); the async form returns the same records and count."""
    dev = lcrc.DeviceBuffer.from_host(np.frombuffer(bytes(data), np.uint8))
    want = _wal_expect(orc, data)
    h = np.array([x[0] for x in want], np.uint64)
    ln = np.array([x[1] for x in want], np.uint64)
    ty = np.array([x[2] for x in want], np.uint8)
    got = eng.wal_scan(dev, len(data))
    assert len(got) == len(want)
    assert np.array_equal(got["header"], h) and np.array_equal(got["length"], ln.astype(np.uint32))
    assert np.array_equal(got["type"], ty)
    crc, _ = orc.crc_ranges_mt(bytes(data), h + 6, ln + 1, 8, orc.ALGO_SSE42_C if mode else orc.ALGO_PCLMUL_REF)
    assert np.array_equal(got["crc"], crc), np.nonzero(got["crc"] != crc)[0][:10]
    a = np.frombuffer(bytes(data), np.uint8)
    stored = (a[h.astype(np.int64)].astype(np.uint32) | (a[h.astype(np.int64) + 1].astype(np.uint32) << 8) |
              (a[h.astype(np.int64) + 2].astype(np.uint32) << 16) | (a[h.astype(np.int64) + 3].astype(np.uint32) << 24))
    assert np.array_equal(got["status"], (stored != crc).astype(np.uint8))
    cap = len(data) // 7 + 1
    rd = lcrc.DeviceBuffer(cap * lcrc.WAL_REC_DTYPE.itemsize)
    cnt = lcrc.DeviceBuffer(8)
    eng.wal_scan_async(dev, len(data), rd, cap, cnt)
    eng.sync()
    n = int(cnt.download(np.uint64, 1)[0])
    assert n == len(got) and rd.download(lcrc.WAL_REC_DTYPE, n).tobytes() == got.tobytes()
    return got


def test_wal_config3_full_size(lcrc, orc, synth, engines):
    """BASELINE configs[3] at its bench size: the 256 MiB log of 8,192 32 KiB blocks that bench.py --config wal
    scans (8,195 blocks: 129 header-walk parts of 64 blocks, so k_wal_emit's part sums run past 64), both modes and the async
    form. REF: the stored crc32fast values verify; C: every record is flagged. Then the same log re-sealed with
    CRC-32C headers on the device (as the bench does) scans clean in mode C."""
    data = _wal_file(lcrc, synth, 256 << 20, synth.SEED_WAL)
    nblocks = (len(data) + 32767) // 32768
    assert nblocks >= 8192 and (nblocks + 63) // 64 > 128
    got = _wal_check_scan(lcrc, orc, engines[0], data, 0)
    assert (got["status"] == 0).all() and len(got) > 70000
    got_c = _wal_check_scan(lcrc, orc, engines[1], data, 1)
    assert (got_c["status"] == 1).all()
    # re-seal every header with the raw CRC-32C (lcrc_batch_seal, {h + 6, 1 + len, -6}): a clean mode-C log
    d = np.zeros(len(got), lcrc.DESC_DTYPE)
    d["offset"], d["length"], d["expect_rel"] = got["header"] + 6, got["length"] + 1, -6
    dev = lcrc.DeviceBuffer.from_host(np.frombuffer(bytes(data), np.uint8))
    dd = lcrc.DeviceBuffer.from_host(d.view(np.uint8))
    engines[1].batch_seal(dev, len(data), dd, len(got))
    engines[1].sync()
    sealed = bytearray(dev.download(np.uint8, len(data)).tobytes())
    got_s = _wal_check_scan(lcrc, orc, engines[1], sealed, 1)
    assert (got_s["status"] == 0).all()


def test_wal_capacity_below_count_after_larger_scan(lcrc, orc, synth):
    """lcrc_wal_scan_async with max_recs below the record count, on a context that has just scanned a larger log with
    the full capacity (so its descriptor and record buffers hold that scan's entries): every record below max_recs --
    including a corrupted one -- has the oracle's header, crc and verdict (log.rs:204-279), the count is the full one,
    and nothing past max_recs is written. Capacities inside the first walk ticket (32 blocks), at a ticket edge and
    inside a later ticket."""
    big = _wal_file(lcrc, synth, 24 << 20, 0x5EED0031)
    data = _wal_file(lcrc, synth, 12 << 20, 0x5EED0032)
    want = _wal_expect(orc, data)
    k_bad = len(want) // 3
    h, n, _ = want[k_bad]
    data[h + 6 + n // 2] ^= 0x08
    eng = lcrc.Engine(0, lcrc.MODE_REF)
    try:
        _wal_check_scan(lcrc, orc, eng, big, 0)
        dev = lcrc.DeviceBuffer.from_host(np.frombuffer(bytes(data), np.uint8))
        hh = np.array([x[0] for x in want], np.uint64)
        ln = np.array([x[1] for x in want], np.uint64)
        crc, _ = orc.crc_ranges_mt(bytes(data), hh + 6, ln + 1, 8, orc.ALGO_PCLMUL_REF)
        a = np.frombuffer(bytes(data), np.uint8)
        stored = np.array([int.from_bytes(bytes(a[int(x):int(x) + 4]), "little") for x in hh], np.uint32)
        edge = sum(1 for x in want if x[0] < 32 * 32768)  # the records of ticket 0's 32 blocks
        for cap in (5, edge, edge + 1, k_bad + 10, len(want) - 1):
            rd = lcrc.DeviceBuffer((cap + 64) * lcrc.WAL_REC_DTYPE.itemsize)
            rd.upload(np.full((cap + 64) * lcrc.WAL_REC_DTYPE.itemsize, 0xEE, np.uint8))
            cnt = lcrc.DeviceBuffer(8)
            eng.wal_scan_async(dev, len(data), rd, cap, cnt)
            eng.sync()
            assert int(cnt.download(np.uint64, 1)[0]) == len(want), cap
            raw = rd.download(np.uint8, (cap + 64) * lcrc.WAL_REC_DTYPE.itemsize)
            assert (raw[cap * lcrc.WAL_REC_DTYPE.itemsize:] == 0xEE).all(), cap
            got = raw[:cap * lcrc.WAL_REC_DTYPE.itemsize].view(lcrc.WAL_REC_DTYPE)
            assert np.array_equal(got["header"], hh[:cap]), cap
            assert np.array_equal(got["crc"], crc[:cap]), cap
            assert np.array_equal(got["status"], (stored[:cap] != crc[:cap]).astype(np.uint8)), cap
            assert (cap <= k_bad) or got["status"][k_bad] == 1
    finally:
        eng.close()


def test_wal_four_contexts_concurrent(lcrc, orc, synth):
    """Four contexts scanning four different logs on their own streams at once, three rounds enqueued back to back:
    each launch's walk workgroups take tickets from their own context's counter and look back only at their own
    launch's words, which the last ticket zeroes for the next scan -- every record, crc and verdict equals the
    oracle's walk (log.rs:204-279) every round."""
    logs = [_wal_file(lcrc, synth, (8 + 6 * k) << 20, 0x5EED0040 + k) for k in range(4)]
    exp = []
    for data in logs:
        want = _wal_expect(orc, data)
        hh = np.array([x[0] for x in want], np.uint64)
        ln = np.array([x[1] for x in want], np.uint64)
        crc, _ = orc.crc_ranges_mt(bytes(data), hh + 6, ln + 1, 8, orc.ALGO_PCLMUL_REF)
        exp.append((hh, ln, crc))
    engs = [lcrc.Engine(0, lcrc.MODE_REF) for _ in logs]
    bufs = []
    try:
        for eng, data in zip(engs, logs):
            cap = len(data) // 7 + 1
            eng.reserve(len(data))
            bufs.append((lcrc.DeviceBuffer.from_host(np.frombuffer(bytes(data), np.uint8)),
                         lcrc.DeviceBuffer(cap * lcrc.WAL_REC_DTYPE.itemsize), lcrc.DeviceBuffer(8), cap))
        for _ in range(3):
            for eng, data, (dev, rd, cnt, cap) in zip(engs, logs, bufs):
                rd.zero()
                eng.wal_scan_async(dev, len(data), rd, cap, cnt)
            for eng in engs:
                eng.sync()
            for (dev, rd, cnt, cap), (hh, ln, crc) in zip(bufs, exp):
                n = int(cnt.download(np.uint64, 1)[0])
                assert n == len(hh)
                got = rd.download(lcrc.WAL_REC_DTYPE, n)
                assert np.array_equal(got["header"], hh) and np.array_equal(got["length"], ln.astype(np.uint32))
                assert np.array_equal(got["crc"], crc) and (got["status"] == 0).all()
    finally:
        for eng in engs:
            eng.close()


def test_wal_just_past_64_parts_with_corruption(lcrc, orc, synth, engines):
    """A log of 4,161 blocks (65 header-walk parts, the last block partial) with corrupted payload bytes, a
    corrupted length field and a zeroed header: every record, crc and verdict against the oracle's walk."""
    data = _wal_file(lcrc, synth, 4161 * 32768, 0x5EED0013)
    data = data[:4160 * 32768 + 1000]
    assert (len(data) + 32767) // 32768 == 4161
    rng = np.random.default_rng(0x65)
    want = _wal_expect(orc, data)
    for k in rng.choice(len(want), 40, replace=False):  # payload / type bytes: checksum mismatches
        h, n, _ = want[int(k)]
        data[h + 6 + int(rng.integers(0, n + 1))] ^= 1 << int(rng.integers(0, 8))
    h, n, _ = want[len(want) // 3]
    data[h + 5] ^= 0x80  # a length field: the walk of that block stops (bad length) or wanders
    h, n, _ = want[2 * len(want) // 3]
    data[h:h + 7] = bytes(7)  # a zero header: type 0, length 0 ends that block's walk
    for mode in MODES:
        got = _wal_check_scan(lcrc, orc, engines[mode], data, mode)
        if mode == 0:
            assert 0 < int(got["status"].sum()) <= 45


def test_first_queued_call_inside_a_graph_capture(lcrc, orc):
    """A fresh context whose very first lcrc_batch_queue is made inside lcrc_graph_begin/end: the queue's side
    streams are created by lcrc_graph_begin before the capture starts, so the capture holds the fork and join
    and its replays give the oracle's CRCs."""
    eng = lcrc.Engine(0, lcrc.MODE_C)
    rng = np.random.default_rng(0xF1)
    jobs, keep, want = [], [], []
    for k in range(3):
        size = (1 + k) << 20
        data = rng.integers(0, 256, size, dtype=np.uint8)
        n = 300
        lens = rng.integers(0, 20000, n).astype(np.uint32)
        offs = np.array([int(rng.integers(0, size - int(L))) for L in lens], np.uint64)
        d = np.zeros(n, lcrc.DESC_DTYPE)
        d["offset"], d["length"], d["expect_rel"] = offs, lens, lcrc.NO_EXPECT
        base, dd = lcrc.DeviceBuffer.from_host(data), lcrc.DeviceBuffer.from_host(d.view(np.uint8))
        out = lcrc.DeviceBuffer(4 * n)
        keep += [base, dd, out]
        jobs.append((base, size, dd, n, out, None))
        want.append(orc.crc_ranges(data.tobytes(), offs, lens, 1))
    eng.reserve(3 << 20)
    arr = lcrc.gjobs(jobs)
    g = eng.graph_capture(lambda: eng.batch_queue(arr))
    try:
        for _ in range(2):
            for j in jobs:
                j[4].zero()
            eng.graph_launch(g)
            eng.sync()
            for j, w in zip(jobs, want):
                assert np.array_equal(j[4].download(np.uint32, j[3]), w)
    finally:
        eng.graph_destroy(g)
        eng.close()


# ---- round 3: the range pass's per-row loop far past its usual ~3 iterations ---------------------------------
@pytest.mark.parametrize("grid", [1, 7])
def test_range_pass_small_grid(lcrc, orc, synth, grid):
    """k_blocks with a grid of 1 or 7 workgroups (context option batch_grid_b, a measurement knob) over a 24 MiB slice of
    BASELINE configs[2]'s zipf SSTable layout (~4,100 blocks): each 16-lane row walks 130 or 18 ranges in turn, so
    the descriptor prefetch, the mismatch-bit set/clear of words shared across iterations and the last range's
    clear of the bits past n all run far beyond the bench's ~3 iterations per row. Every CRC and mismatch bit
    equals the oracle's, both modes (format.rs:162-171)."""
    sizes = synth.mixed_sizes(24 << 20, seed=synth.SEED_MIXED + 7)
    offs, total = synth.sstable_layout(sizes)
    lens = sizes.astype(np.uint64) + 1
    base = synth.splitmix_bytes(synth.SEED_MIXED + 1007, total)
    rng = np.random.default_rng(grid)
    bad = sorted({int(i) for i in rng.choice(len(sizes) - 1, 9, replace=False)} | {len(sizes) - 1})
    for mode, flags, algo in ((0, 0, orc.ALGO_PCLMUL_REF), (1, lcrc.FLAG_MASK, orc.ALGO_SSE42_C)):
        want, _ = orc.crc_ranges_mt(base, offs, lens, 8, algo)
        if mode:
            want = orc.mask_array(want)
        f = base.copy()
        slot = (offs + lens).astype(np.int64)
        for k in range(4):
            f[slot + k] = ((want >> np.uint32(8 * k)) & 0xFF).astype(np.uint8)
        for i in bad:
            f[int(offs[i] + lens[i] // 2)] ^= 0x10
        eng = lcrc.Engine(0, mode, flags, general="blocks", batch_grid_b=grid)
        crcs, mm = eng.crc_ranges(f, offs, lens, expect_rel=lens.astype(np.int64))
        eng.close()
        got_want, _ = orc.crc_ranges_mt(f, offs, lens, 8, algo)
        if mode:
            got_want = orc.mask_array(got_want)
        assert np.array_equal(crcs, got_want), (mode, np.nonzero(crcs != got_want)[0][:10])
        assert np.nonzero(mm)[0].tolist() == bad


@pytest.mark.parametrize("grid", [1, 5])
def test_wal_range_pass_small_grid(lcrc, orc, synth, grid):
    """The WAL scan's range pass with 1 or 5 workgroups (context option wal_grid_b): a 40 MiB log's ~11,000 records, the
    one-window records first, walked ~350 or ~70 per row, with corrupted records; every record, crc and verdict
    against the oracle's walk (log.rs:204-279)."""
    data = _wal_file(lcrc, synth, 40 << 20, 0x5EED0021 + grid)
    rng = np.random.default_rng(0x77 + grid)
    want = _wal_expect(orc, data)
    for k in rng.choice(len(want), 25, replace=False):
        h, n, _ = want[int(k)]
        data[h + 6 + int(rng.integers(0, n + 1))] ^= 1 << int(rng.integers(0, 8))
    for mode in MODES:
        eng = lcrc.Engine(0, mode, wal_grid_b=grid)
        got = _wal_check_scan(lcrc, orc, eng, data, mode)
        eng.close()
        if mode == 0:
            assert 0 < int(got["status"].sum()) <= 25
