"""The WAL framing restated in C++ (csrc/lcrc_leveldb.cpp) against the reference's own log tests
(src/db/log.rs:282-811) and against the pure-Python oracle restatement, byte for byte."""
import numpy as np
import pytest

import logtests


@pytest.fixture
def tester(lcrc):
    return logtests.Tester(lcrc, lambda data: lcrc.LogReader(data))


@pytest.mark.parametrize("scenario", logtests.SCENARIOS, ids=lambda f: f.__name__)
def test_reference_scenario(tester, scenario):
    scenario(tester)


def test_many_blocks(tester):
    logtests.t_many_blocks(tester)  # the reference's 1,000,000 records (log.rs:535-545)


def test_random_read(tester):
    logtests.t_random_read(tester, np.random.default_rng(11))


def test_read_error(tester):
    logtests.t_read_error(tester)


def _random_records(rng, n):
    out = []
    for _ in range(n):
        k = int(rng.integers(1, 17))
        m = int(rng.integers(0, 1 << k))
        out.append(rng.integers(0, 256, m, dtype=np.uint8).tobytes())
    return out


@pytest.mark.parametrize("seed", range(6))
def test_writer_matches_oracle(lcrc, orc, seed):
    recs = _random_records(np.random.default_rng(seed), 200)
    w = lcrc.LogWriter()
    for r in recs:
        w.add_record(r)
    assert w.contents() == orc.log_write(recs)


@pytest.mark.parametrize("seed", range(12))
def test_reader_matches_oracle_under_corruption(lcrc, orc, seed):
    rng = np.random.default_rng(100 + seed)
    data = bytearray(orc.log_write(_random_records(rng, 120)))
    for _ in range(int(rng.integers(1, 6))):
        kind = int(rng.integers(0, 3))
        pos = int(rng.integers(0, len(data)))
        if kind == 0:
            data[pos] ^= 1 << int(rng.integers(0, 8))
        elif kind == 1:
            data[pos] = int(rng.integers(0, 256))
        else:
            del data[len(data) - int(rng.integers(0, 64)):]
    want = orc.log_read_all(bytes(data))
    r = lcrc.LogReader(bytes(data))
    got = (r.records(), r.dropped_bytes, r.report_message)
    assert got == want
