"""Snappy element coverage of the whole-table scan's row decoder (k_ts_decode's row_snappy_decode): every element
form the snap crate's decoder accepts (snap "1", the decompressor behind src/sstable/format.rs:194-206) at every
destination alignment -- literals with 0..4 length bytes (minimal and not), 1-, 2- and 4-byte-offset copies, copies
overlapping their own output (offset < length: the repeat), copies closer than a 128 B pass and farther, literals
longer than a pass -- plus invalid streams (offset past the output, output past the preamble's length, a header cut
by the end) and uncompressed chunks of every length mod 4 in rows beside compressed ones (a row the decoder skips
must see none of its stores). Frames are sized for the row staging (<= 2,701 B compressed, <= ROW_OUT decoded), stored as
the data blocks of one table, and the device scan's verdict on each block must equal the oracle's read_block_from_file.

The generator's own decode of each valid stream is checked against the oracle first (CPU), so the cases are what
they claim to be.
"""
import numpy as np
import pytest

from test_snappy_snap_rules import STREAM, _chunk, _varu, frames_table
from test_table_scan import _as_tuples

# a row's decoded chunk in k_ts_decode (TR_OUT = TR_ROW - 16, lcrc_kernels.hip: rows of 4,320 B since round 6's 8-lane
# rows); larger chunks go through the whole-wave decoder
ROW_OUT = 4304


def _lit_el(data, nb):
    n = len(data)
    if nb == 0:
        return bytes([(n - 1) << 2]) + data
    return bytes([(59 + nb) << 2]) + (n - 1).to_bytes(nb, "little") + data


def _copy_el(off, n, kind):
    if kind == 1:  # 1-byte offset: length 4..11, offset < 2048
        return bytes([((off >> 8) << 5) | ((n - 4) << 2) | 1, off & 0xFF])
    if kind == 2:
        return bytes([((n - 1) << 2) | 2]) + off.to_bytes(2, "little")
    return bytes([((n - 1) << 2) | 3]) + off.to_bytes(4, "little")


def gen_stream(rng, target, lit_max=300):
    """(payload after the preamble, decoded bytes or None): random elements until about `target` decoded bytes. None:
    an extended-length literal's tag is followed by fewer than 4 bytes (snap reads its length as one 4-byte word)."""
    out = bytearray()
    pay = bytearray()
    ext_tag = -1
    while len(out) < target:
        r = rng.random()
        if not out or r < 0.35:
            n = int(rng.choice([rng.integers(1, 9), rng.integers(50, 71), rng.integers(120, 140),
                                rng.integers(1, lit_max + 1)]))
            alphabet = int(rng.choice([2, 16, 256]))
            data = bytes(rng.integers(0, alphabet, n, dtype=np.uint8))
            nmin = 0 if n <= 60 else 1 if n <= 256 else 2
            nb = int(rng.integers(nmin, 5)) if rng.random() < 0.3 else nmin
            if nb:
                ext_tag = len(pay)
            pay += _lit_el(data, nb)
            out += data
            continue
        kind = int(rng.choice([1, 2, 4]))
        n = int(rng.integers(4, 12)) if kind == 1 else int(rng.integers(1, 65))
        w = len(out)
        lim = min(w, 2047 if kind == 1 else 65535)
        pick = rng.random()
        if pick < 0.3:
            off = int(rng.integers(1, min(n, lim) + 1))        # overlapping its own output (or touching it)
        elif pick < 0.6:
            off = int(rng.integers(min(n, lim), min(130, lim) + 1))  # within a pass
        else:
            off = int(rng.integers(1, lim + 1))
        pay += _copy_el(off, n, kind)
        for _ in range(n):
            out.append(out[-off])
    return bytes(pay), (bytes(out) if ext_tag < 0 or len(pay) - ext_tag - 1 >= 4 else None)


def _frame(orc, payload, decoded, ulen=None):
    pre = _varu(len(decoded) if ulen is None else ulen, 2)
    return STREAM + _chunk(orc, 0, pre + payload, decoded)


def row_cases(orc, seed=11, count=160):
    """[(frame, decoded or None)]: valid random streams (some frames with two chunks) and invalid ones."""
    rng = np.random.default_rng(seed)
    cases = []
    while len(cases) < count:
        target = int(rng.choice([1, 7, 64, 129, 1000, 3000, 4096, 4250]))
        pay, dec = gen_stream(rng, target, lit_max=int(rng.choice([60, 300])))
        if dec is None:
            continue
        fr = _frame(orc, pay, dec)
        if len(fr) > 2701 or len(dec) > ROW_OUT:
            continue
        r = rng.random()
        if rng.random() < 0.12:  # an uncompressed chunk (copied in the row, beside rows decoding compressed ones)
            data = bytes(rng.integers(0, 256, int(rng.integers(1, 2600)), dtype=np.uint8))
            cases.append((STREAM + _chunk(orc, 1, data, data), data))
            continue
        if r < 0.1 and len(dec) > 10:  # a second chunk
            pay2, dec2 = gen_stream(rng, 200)
            fr2 = _frame(orc, pay2, dec2 or b"")[len(STREAM):]
            if dec2 is not None and len(fr) + len(fr2) <= 2701:
                cases.append((fr + fr2, dec + dec2))
                continue
        if r < 0.2:  # output past the preamble's length
            cases.append((_frame(orc, pay, dec, ulen=len(dec) - 1), None))
        elif r < 0.27:  # a copy reaching before the output's start
            cases.append((_frame(orc, pay + _copy_el(len(dec) + 1, 4, 2), dec + b"\0" * 4), None))
        elif r < 0.32:  # a header cut by the stream's end
            cases.append((_frame(orc, pay + b"\x02\x01", dec), None))
        elif r < 0.36:  # a wrong chunk CRC
            fr = bytearray(fr)
            fr[len(STREAM) + 4] ^= 1
            cases.append((bytes(fr), None))
        else:
            cases.append((fr, dec))
    return cases


def in_place_cases(orc, seed=5):
    """Frames the row decodes in place only up to a point (k_ts_decode stages a frame at its row's end and decodes from
    the row's start): a compressible head then a long literal tail, so the output reaches the literal's unread bytes
    (the row gives the frame to the whole-wave decoder) -- sized near the row (ROW_OUT) so that some decode in place
    and some are given up, by the frame's alignment too; and two-chunk frames. Each must decode as the oracle does."""
    rng = np.random.default_rng(seed)
    cases = []
    for head, total in ((2400, 4285), (2500, 4295), (2600, 4301), (2700, 4303), (2800, 4297), (2900, 4304),
                        (2200, 4304), (3000, 4302), (3200, 4300), (3400, 4290)):
        tail = total - head
        pay = _lit_el(bytes(rng.integers(0, 256, 8, dtype=np.uint8)), 0)
        dec = bytearray(pay[1:])
        while len(dec) + 64 <= head:
            pay += _copy_el(8, 64, 2)
            for _ in range(64):
                dec.append(dec[-8])
        lit = bytes(rng.integers(0, 256, tail, dtype=np.uint8))
        pay += _lit_el(lit, 2)
        dec += lit
        cases.append((_frame(orc, bytes(pay), bytes(dec)), bytes(dec)))
    for first in (2500, 3000, 3500):
        pay = _lit_el(b"abcdefgh", 0)
        dec = bytearray(b"abcdefgh")
        while len(dec) + 64 <= first:
            pay += _copy_el(8, 64, 2)
            dec += dec[-8:] * 8
        second = bytes(rng.integers(0, 256, 2200, dtype=np.uint8))
        fr = _frame(orc, bytes(pay), bytes(dec)) + _frame(orc, _lit_el(second, 2), second)[len(STREAM):]
        cases.append((fr, bytes(dec) + second))
    return cases


def test_in_place_cases_match_oracle(orc, lcrc):
    for fr, want in in_place_cases(orc):
        assert len(fr) <= 2701
        assert orc.snappy_frame_decode(fr) == want
        assert lcrc.snappy_frame_decode(fr) == want


@pytest.mark.gpu
def test_row_decoder_in_place_limits(lcrc, orc, engines):
    from test_table_scan import _scan
    from test_table_scan_async import _expect_async
    cases = in_place_cases(orc) + row_cases(orc, 21, 40)
    f = frames_table(orc, [fr for fr, _ in cases])
    want, werr = orc.table_scan_expect(f)
    assert werr is None and [w[4] for w in want if w[2] == 0] == [0 if d is not None else 3 for _, d in cases]
    assert _expect_async(lcrc, engines[lcrc.MODE_REF], orc, f) == 0
    got, err = _scan(lcrc, engines[lcrc.MODE_REF], f)
    assert err is None and _as_tuples(got) == want


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_row_cases_match_oracle(orc, lcrc, seed):
    """The generator's decode is the oracle's (so each case is the element mix it claims), and the host decoder's."""
    for fr, want in row_cases(orc, seed):
        assert orc.snappy_frame_decode(fr) == want
        assert lcrc.snappy_frame_decode(fr) == want


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12, 13])
def test_row_decoder_elements(lcrc, orc, engines, seed):
    from test_table_scan import _scan
    from test_table_scan_async import _expect_async
    cases = row_cases(orc, seed)
    f = frames_table(orc, [fr for fr, _ in cases])
    want, werr = orc.table_scan_expect(f)
    assert werr is None
    assert [w[4] for w in want if w[2] == 0] == [0 if d is not None else 3 for _, d in cases]
    eng = engines[lcrc.MODE_REF]
    assert _expect_async(lcrc, eng, orc, f) == 0
    got, err = _scan(lcrc, eng, f)
    assert err is None and _as_tuples(got) == want


def over_row_cases(orc, seed=31, count=24):
    """Valid and corrupted frames whose chunk decodes to more than a row holds (ROW_OUT < size <= 5,200 B: the row path
    of rounds 4-5, whose 5,136 B rows held them) but whose frame fits the row staging: k_ts_decode hands each to the
    whole-wave decoder after the rows. Some with a wrong chunk CRC, some with output past the preamble's length."""
    rng = np.random.default_rng(seed)
    cases = []
    while len(cases) < count:
        target = int(rng.integers(ROW_OUT + 1, 5200))
        pay, dec = gen_stream(rng, target, lit_max=60)
        if dec is None or not ROW_OUT < len(dec) <= 5200:
            continue
        fr = _frame(orc, pay, dec)
        if len(fr) > 2701:
            continue
        r = rng.random()
        if r < 0.15:
            fr = bytearray(fr)
            fr[len(STREAM) + 4] ^= 1
            cases.append((bytes(fr), None))
        elif r < 0.25:
            cases.append((_frame(orc, pay, dec, ulen=len(dec) - 1), None))
        else:
            cases.append((fr, dec))
    return cases


def test_over_row_cases_match_oracle(orc, lcrc):
    for fr, want in over_row_cases(orc):
        assert orc.snappy_frame_decode(fr) == want
        assert lcrc.snappy_frame_decode(fr) == want


@pytest.mark.gpu
def test_row_decoder_over_row(lcrc, orc, engines):
    from test_table_scan import _scan
    from test_table_scan_async import _expect_async
    cases = over_row_cases(orc) + row_cases(orc, 41, 24)
    f = frames_table(orc, [fr for fr, _ in cases])
    want, werr = orc.table_scan_expect(f)
    assert werr is None
    assert [w[4] for w in want if w[2] == 0] == [0 if d is not None else 3 for _, d in cases]
    eng = engines[lcrc.MODE_REF]
    assert _expect_async(lcrc, eng, orc, f) == 0
    got, err = _scan(lcrc, eng, f)
    assert err is None and _as_tuples(got) == want


def boundary_cases(orc, seed=51):
    """Frames whose chunk decodes to an exact size at the row decoder's edges: below one 16 B piece, at and around
    whole 1 KiB CRC passes (no zero padding to undo), and at ROW_OUT and one past it (the whole-wave decoder), each
    compressed enough for the row staging (64 literal bytes, then copies of them); plus uncompressed chunks up to the
    staging's limit, and a few of each with a wrong chunk CRC."""
    rng = np.random.default_rng(seed)
    cases = []
    sizes = [1, 3, 4, 5, 15, 16, 17, 63, 64, 65, 1023, 1024, 1025, 2048, 3072, 4095, 4096, 4097,
             ROW_OUT - 16, ROW_OUT - 15, ROW_OUT - 1, ROW_OUT, ROW_OUT + 1]
    for n in sizes:
        head = bytes(rng.integers(0, 256, min(n, 64), dtype=np.uint8))
        pay = bytearray(_lit_el(head, 0 if len(head) <= 60 else 1))
        dec = bytearray(head)
        while len(dec) < n:
            m = min(64, n - len(dec))
            off = 64 if m >= 4 or len(dec) >= 64 else len(dec)
            pay += _copy_el(off, m, 2)
            for _ in range(m):
                dec.append(dec[-off])
        fr = _frame(orc, bytes(pay), bytes(dec))
        assert len(fr) <= 2701
        cases.append((fr, bytes(dec)))
    for n in (1, 4, 16, 1024, 2048, 2683):
        data = bytes(rng.integers(0, 256, n, dtype=np.uint8))
        cases.append((STREAM + _chunk(orc, 1, data, data), data))
    for k in (2, 9, 13, 19, 24):  # wrong chunk CRCs
        fr = bytearray(cases[k][0])
        fr[len(STREAM) + 4] ^= 0x80
        cases.append((bytes(fr), None))
    return cases


def test_boundary_cases_match_oracle(orc, lcrc):
    for fr, want in boundary_cases(orc):
        assert orc.snappy_frame_decode(fr) == want
        assert lcrc.snappy_frame_decode(fr) == want


@pytest.mark.gpu
def test_row_decoder_boundaries(lcrc, orc, engines):
    from test_table_scan import _scan
    from test_table_scan_async import _expect_async
    cases = boundary_cases(orc)
    f = frames_table(orc, [fr for fr, _ in cases])
    want, werr = orc.table_scan_expect(f)
    assert werr is None
    assert [w[4] for w in want if w[2] == 0] == [0 if d is not None else 3 for _, d in cases]
    eng = engines[lcrc.MODE_REF]
    assert _expect_async(lcrc, eng, orc, f) == 0
    got, err = _scan(lcrc, eng, f)
    assert err is None and _as_tuples(got) == want
