"""The one-pass WAL scan (lcrc_ctx_options.wal_onepass): the window pass (k_windows_wal) finishes
every record whose covered bytes lie in one 16 KiB region of the log (up to WAL_RMAX per region), k_blocks only the
others. Every record, crc and verdict must be the reference reader's (log.rs:204-279: the header walk; log.rs:260-273:
the stored-vs-computed compare), through the same checks as the two-pass scan."""
import numpy as np
import pytest

import logtests
from test_gpu_parity import MODES, _wal_check_scan, _wal_expect, _wal_file

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def one(lcrc):
    e = {m: lcrc.Engine(0, m, wal_onepass=1) for m in MODES}
    yield e
    for v in e.values():
        v.close()


def test_onepass_config3_full_size(lcrc, orc, synth, one):
    """BASELINE configs[3] at the bench's size (8,195 log blocks, ~74K records), both modes and the async form."""
    data = _wal_file(lcrc, synth, 256 << 20, synth.SEED_WAL)
    got = _wal_check_scan(lcrc, orc, one[0], data, 0)
    assert (got["status"] == 0).all() and len(got) > 70000
    got_c = _wal_check_scan(lcrc, orc, one[1], data, 1)
    assert (got_c["status"] == 1).all()


def test_onepass_corruption_past_64_parts(lcrc, orc, synth, one):
    data = _wal_file(lcrc, synth, 4161 * 32768, 0x5EED0013)
    data = data[:4160 * 32768 + 1000]
    rng = np.random.default_rng(0x66)
    want = _wal_expect(orc, data)
    for k in rng.choice(len(want), 60, replace=False):
        h, n, _ = want[int(k)]
        data[h + 6 + int(rng.integers(0, n + 1))] ^= 1 << int(rng.integers(0, 8))
    for k in rng.choice(len(want), 20, replace=False):  # stored CRCs
        h, n, _ = want[int(k)]
        data[h + int(rng.integers(0, 4))] ^= 1 << int(rng.integers(0, 8))
    h, n, _ = want[len(want) // 3]
    data[h + 5] ^= 0x80
    for mode in MODES:
        got = _wal_check_scan(lcrc, orc, one[mode], data, mode)
        if mode == 0:
            assert 0 < int(got["status"].sum()) <= 82


@pytest.mark.parametrize("scenario", [s for s in logtests.SCENARIOS], ids=lambda f: f.__name__)
def test_onepass_reference_scenarios(lcrc, one, scenario):
    scenario(logtests.Tester(lcrc, lambda data: lcrc.BatchLogReader(data, one[0])))


@pytest.mark.parametrize("seed", range(6))
def test_onepass_equals_host_reader_under_corruption(lcrc, orc, one, seed):
    rng = np.random.default_rng(900 + seed)
    recs = []
    for _ in range(500):
        k = int(rng.integers(1, 17))
        recs.append(rng.integers(0, 256, int(rng.integers(0, 1 << k)), dtype=np.uint8).tobytes())
    data = bytearray(orc.log_write(recs))
    for _ in range(int(rng.integers(0, 10))):
        pos = int(rng.integers(0, len(data)))
        data[pos] ^= 1 << int(rng.integers(0, 8))
    if rng.random() < 0.5:
        del data[len(data) - int(rng.integers(1, 200)):]
    b = lcrc.BatchLogReader(bytes(data), one[0])
    assert b.consistency_errors == 0
    assert (b.records(), b.dropped_bytes, b.report_message) == orc.log_read_all(bytes(data))
    _wal_check_scan(lcrc, orc, one[0], data, 0)


def test_onepass_region_edges(lcrc, orc, one):
    """Records of 0..3 payload bytes (1..4 covered bytes: the short-message injection), records whose covered bytes
    end exactly at a 256 B window, at the middle of their log block, or start exactly there, regions with more than
    WAL_RMAX records (the rest to k_blocks), and blocks with more records than the parse keeps slots for."""
    rng = np.random.default_rng(0x0E)
    recs = []
    for i in range(6000):
        r = rng.random()
        n = int(rng.integers(0, 4)) if r < 0.4 else int(rng.integers(4, 300)) if r < 0.8 else \
            int(rng.integers(300, 20000))
        recs.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    # a record ending exactly at the middle of the first block: header at h, covered [h + 6, h + 7 + n) = 16384
    head = [b"x" * (16384 - 7 - 7 - 5)]  # covered bytes of record 0: [6, 16372): then record 1 ends at 16384
    head += [b"y" * 5]
    head += [b"z" * 300, b"w" * 100]
    data = bytearray(orc.log_write(head + recs))
    for mode in MODES:
        got = _wal_check_scan(lcrc, orc, one[mode], data, mode)
        if mode == 0:
            assert (got["status"] == 0).all()
    # 200 records corrupted at a random covered byte: exactly those are flagged
    want = _wal_expect(orc, data)
    for k in rng.choice(len(want), 200, replace=False):
        h, n, _ = want[int(k)]
        data[h + 6 + int(rng.integers(0, n + 1))] ^= 0x01
    got = _wal_check_scan(lcrc, orc, one[0], data, 0)
    assert int(got["status"].sum()) == 200


@pytest.mark.parametrize("shift", [0, 1, 3])
def test_onepass_file_tail_and_unaligned_base(lcrc, orc, one, shift):
    import ctypes
    rng = np.random.default_rng(80)
    recs = [rng.integers(0, 256, int(rng.integers(0, 1 << int(rng.integers(1, 10)))), dtype=np.uint8).tobytes()
            for _ in range(400)]
    full = orc.log_write(recs)
    for cut in range(len(full) - 30, len(full) + 1, 3):
        data = full[:cut]
        dev = lcrc.DeviceBuffer.from_host(np.frombuffer(b"\x5a" * shift + data + b"\xa5" * 5, np.uint8))
        cap = len(data) // 7 + 1
        out = lcrc.DeviceBuffer(cap * lcrc.WAL_REC_DTYPE.itemsize)
        n = ctypes.c_size_t(0)
        rc = lcrc.lib().lcrc_wal_scan(one[0].ctx, ctypes.c_void_p(dev.ptr + shift), len(data), out.ptr, cap,
                                      ctypes.byref(n), None)
        assert rc == 0
        got = out.download(lcrc.WAL_REC_DTYPE, n.value)
        want = _wal_expect(orc, data)
        assert [(int(r["header"]), int(r["length"]), int(r["type"])) for r in got] == want, cut
        for r in got:
            h = int(r["header"])
            assert int(r["crc"]) == orc.crc(data[h + 6:h + 7 + int(r["length"])], 0), (cut, h)
            assert int(r["status"]) == 0


def test_onepass_graph_replay(lcrc, orc, synth):
    """The one-pass scan (four launches) captured in a HIP graph and replayed: the direct call's records."""
    eng = lcrc.Engine(0, lcrc.MODE_REF, wal_onepass=1)
    data = _wal_file(lcrc, synth, 8 << 20, 0x5EED0031)
    dev = lcrc.DeviceBuffer.from_host(np.frombuffer(bytes(data), np.uint8))
    want = eng.wal_scan(dev, len(data))
    cap = len(data) // 7 + 1
    rd = lcrc.DeviceBuffer(cap * lcrc.WAL_REC_DTYPE.itemsize)
    cnt = lcrc.DeviceBuffer(8)
    g = eng.graph_capture(lambda: eng.wal_scan_async(dev, len(data), rd, cap, cnt))
    try:
        for _ in range(2):
            rd.zero()
            eng.graph_launch(g)
            eng.sync()
            n = int(cnt.download(np.uint64, 1)[0])
            assert n == len(want) and rd.download(lcrc.WAL_REC_DTYPE, n).tobytes() == want.tobytes()
    finally:
        eng.graph_destroy(g)
        eng.close()
