"""Randomized corruption sweep of Snappy-compressed tables through the device decoders.

The device decoders read on-disk bytes an attacker can shape: chunk headers, length preambles, literal lengths, copy
offsets and lengths, the stream identifier. Each case below takes one of four tables written with compression (the
reference's default, option.rs:127) -- small framed data blocks (the row decoder), ~10 KB frames (the whole-wave
decoder), 150 KB frames of three chunks (the lane-serial decoder into the workspace) and a multi-chunk Snappy-framed
index block (k_ts_open's two-phase decoder) --, corrupts one field of one frame, optionally re-seals the chunk's masked
CRC-32C when the corrupted chunk still decodes (so the decoder must accept different bytes: for the index, other
handles), and always re-seals the block trailer, so the scan has to walk the corrupted bytes instead of stopping at the
block checksum (format.rs:162-171 checks the trailer before the type dispatch at :175-206).

Every outcome must equal oracle.table_scan_expect: the synchronous lcrc_table_scan gives the oracle's blocks or its
message; the device-only scan (lcrc_table_scan_async_ex with LCRC_TSCAN_SNAPPY_INDEX) gives the oracle's blocks, its
message, or LCRC_TSCAN_HOST. Every tenth case scans on a fresh context with a 16-byte decode reservation, so the
synchronous scan's workspace growth runs too.
"""
import numpy as np
import pytest

from test_table_scan import FILTER, _as_tuples, _scan
from test_table_scan_async import _expect_async

STREAM_LEN = 10
NCASES = 200
PARTS = 8


def _db_values(n, vlen, seed):
    """db_bench-style entries: sequential keys, values half random and half a repeat (Snappy saves ~1/2)."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        a = rng.integers(0, 256, (vlen + 1) // 2, dtype=np.uint8).tobytes()
        out.append((b"%016d" % i, (a + a)[:vlen]))
    return out


@pytest.fixture(scope="module")
def tables(orc):
    return build_tables(orc)


def build_tables(orc):
    t = {}
    t["rows"] = orc.table_build(_db_values(3000, 100, 1), block_size=4096, compression=1, filter_name=FILTER,
                                filter_block=b"f" * 100) + (FILTER,)
    t["wave"] = orc.table_build(_db_values(1500, 100, 2), block_size=10000, compression=1) + (None,)
    t["serial"] = orc.table_build(_db_values(1500, 400, 3), block_size=150000, compression=1) + (None,)
    rng = np.random.default_rng(4)
    t["index"] = orc.table_build([(b"%016d" % i, rng.integers(0, 256, 24, dtype=np.uint8).tobytes())
                                  for i in range(40000)], block_size=128, compression=1) + (None,)
    for name, (f, blocks, filt) in t.items():
        assert orc.table_scan_expect(f, filt)[1] is None, name
        ih = [b for b in blocks if b[2] == 3][0]
        assert name != "index" or (f[ih[0] + ih[1]] == 1 and len(orc.snappy_frame_decode(f[ih[0]:ih[0] + ih[1]]))
                                   > 3 * 65536)
    return t


def _chunks(f, off, size):
    """(header position, type, body position, body length) of every chunk of the frame at f[off, off + size)."""
    out, p, end = [], off, off + size
    while end - p >= 4:
        cl = f[p + 1] | (f[p + 2] << 8) | (f[p + 3] << 16)
        if end - p - 4 < cl:
            break
        out.append((p, f[p], p + 4, cl))
        p += 4 + cl
    return out


def _elements(f, body, cl):
    """The Snappy elements of a compressed chunk's body (after its 4-byte CRC): (position, kind, header bytes) with
    kind 0 literal, 1/2/3 copy with a 1/2/4-byte offset; and the preamble's span."""
    z0, z1 = body + 4, body + cl
    p = z0
    while p < z1 and f[p] & 128:
        p += 1
    pre = (z0, p + 1)
    p += 1
    els = []
    while p < z1:
        t = f[p]
        k = t & 3
        if k == 0:
            L = t >> 2
            nb = L - 59 if L >= 60 else 0
            n = (int.from_bytes(f[p + 1:p + 1 + nb], "little") if nb else L) + 1
            els.append((p, 0, 1 + nb))
            p += 1 + nb + n
        else:
            els.append((p, k, 1 + (1, 2, 4)[k - 1]))
            p += 1 + (1, 2, 4)[k - 1]
    return pre, els


KINDS = ["chunk_len", "preamble", "literal", "copy", "stream_id", "chunk_type", "chunk_crc", "bytes"]


def _corrupt(orc, f, blocks, target, rng):
    """One corruption of one frame of f; returns (new file bytes, description). The block trailer is re-sealed."""
    g = bytearray(f)
    if target == "index":
        off, size, _ = [b for b in blocks if b[2] == 3][0]
    else:
        framed = [b for b in blocks if b[2] == 0 and f[b[0] + b[1]] == 1]
        off, size, _ = framed[int(rng.integers(0, len(framed)))]
    chunks = _chunks(f, off, size)
    data = [c for c in chunks if c[1] in (0, 1)]
    comp = [c for c in chunks if c[1] == 0]
    kind = KINDS[int(rng.integers(0, len(KINDS)))]
    ch = data[int(rng.integers(0, len(data)))] if data else chunks[0]
    desc = kind
    if kind == "chunk_len":
        v = ch[3] + int(rng.choice([-3, -1, 1, 2, 7, 1000, 70000, 1 << 23])) if rng.random() < 0.7 else \
            int(rng.integers(0, 1 << 24))
        v = max(0, min(v, (1 << 24) - 1))
        g[ch[0] + 1:ch[0] + 4] = v.to_bytes(3, "little")
        desc += f" {ch[3]}->{v}"
    elif kind == "preamble" and comp:
        ch = comp[int(rng.integers(0, len(comp)))]
        (a, b), _ = _elements(f, ch[2], ch[3])
        choice = int(rng.integers(0, 4))
        if choice == 0:  # one preamble byte replaced
            g[a + int(rng.integers(0, b - a))] = int(rng.integers(0, 256))
        elif choice == 1:  # the preamble's last byte gains a continuation bit (the length swallows the first element)
            g[b - 1] |= 0x80
        elif choice == 2:  # +-1 on the length
            v, _ = orc._snap_varu64(bytes(f[a:b]))
            w = v + int(rng.choice([-1, 1]))
            enc = orc.varint(max(w, 0))
            if len(enc) == b - a:
                g[a:b] = enc
        else:  # a high bit of the preamble's last byte: a length far past 65,536
            g[b - 1] ^= 0x40
        desc += f" [{a - ch[2]},{b - ch[2]})"
    elif kind in ("literal", "copy") and comp:
        ch = comp[int(rng.integers(0, len(comp)))]
        _, els = _elements(f, ch[2], ch[3])
        pick = [e for e in els if (e[1] == 0) == (kind == "literal")]
        if pick:
            p, k, hl = pick[int(rng.integers(0, len(pick)))]
            if rng.random() < 0.5 or hl == 1:
                g[p] ^= 1 << int(rng.integers(0 if kind == "copy" else 2, 8))  # tag: length bits (or the type)
            else:
                q = p + 1 + int(rng.integers(0, hl - 1))
                g[q] = int(rng.integers(0, 256))  # an extension length byte, or an offset byte
            desc += f" element kind {k} at +{p - ch[2]}"
        else:
            g[ch[2] + 4 + int(rng.integers(0, max(1, ch[3] - 4)))] ^= 0x10
    elif kind == "stream_id":
        g[off + int(rng.integers(0, STREAM_LEN))] ^= 1 << int(rng.integers(0, 8))
    elif kind == "chunk_type":
        g[ch[0]] = int(rng.choice([0, 1, 2, 0x7F, 0x80, 0xFD, 0xFE, 0xFF]))
    elif kind == "chunk_crc":
        g[ch[2] + int(rng.integers(0, 4))] ^= 1 << int(rng.integers(0, 8))
    else:
        for _ in range(int(rng.integers(1, 4))):
            g[off + int(rng.integers(0, size))] ^= 1 << int(rng.integers(0, 8))
    # re-seal the chunk CRC when the corrupted chunk still decodes (different bytes, valid frame): half the time
    if kind not in ("chunk_crc", "stream_id", "chunk_len") and rng.random() < 0.5:
        for hp, t, bp, cl in _chunks(bytes(g), off, size):
            if t == 0 and cl >= 4:
                d = orc._snappy_raw(bytes(g[bp + 4:bp + cl]))
                if d is not None and len(d) <= 65536:
                    g[bp:bp + 4] = orc.mask(orc.crc(d, 1)).to_bytes(4, "little")
        desc += " (chunk crc resealed)"
    g[off + size + 1:off + size + 5] = orc.crc(bytes(g[off:off + size + 1]), 0).to_bytes(4, "little")
    return bytes(g), f"{target} block @{off}: {desc}"


@pytest.mark.gpu
@pytest.mark.parametrize("part", range(PARTS))
def test_corruption_sweep(lcrc, orc, engines, tables, part):
    eng = engines[lcrc.MODE_REF]
    names = ["rows", "wave", "serial", "index"]
    seen = {"ok": 0, "corrupt": 0, "host": 0, "bad_blocks": 0}
    for case in range(part, NCASES, PARTS):
        rng = np.random.default_rng(7000 + case)
        tname = names[int(rng.integers(0, len(names)))]
        f, blocks, filt = tables[tname]
        target = "index" if tname == "index" or rng.random() < 0.3 else "data"
        g, desc = _corrupt(orc, f, blocks, target, rng)
        want, werr = orc.table_scan_expect(g, filt)
        fresh = case % 10 == 0
        e = lcrc.Engine(0, lcrc.MODE_REF) if fresh else eng
        try:
            got, err = _scan(lcrc, e, g, filt)
            assert err == werr, f"case {case} sync: {desc}"
            assert got is None or _as_tuples(got) == want, f"case {case} sync: {desc}"
            st = _expect_async(lcrc, e, orc, g, filt, cap=len(blocks) + 8, decoded=16 if fresh else 1 << 22,
                               snappy_index=True)
            assert st in (0, 1, 2), f"case {case} async: {desc}"
        finally:
            if fresh:
                e.close()
        seen["ok" if st == 0 else "corrupt" if st == 1 else "host"] += 1
        seen["bad_blocks"] += int(want is not None and any(w[4] == 3 for w in want if w[2] == 0))
    n = len(range(part, NCASES, PARTS))
    assert sum(seen[k] for k in ("ok", "corrupt", "host")) == n
    print(f"part {part}: {seen}")


def _frame_of(blocks, g, target, f):
    """The corrupted frame's (offset, size): the index block, or the one data block whose bytes changed."""
    if target == "index":
        off, size, _ = [b for b in blocks if b[2] == 3][0]
        return off, size
    for off, size, kind in blocks:
        if kind == 0 and g[off:off + size + 5] != f[off:off + size + 5]:
            return off, size
    return None


def test_corruption_sweep_cpu_decoders(lcrc, orc, tables):
    """The same 200 corrupted frames through the CPU decoders: the library's host decoder (the synchronous scan's
    fallback walk) and the C oracle (the table benches' CPU baseline) agree with the Python oracle on every one."""
    names = ["rows", "wave", "serial", "index"]
    frames, want = [], []
    for case in range(NCASES):
        rng = np.random.default_rng(7000 + case)
        tname = names[int(rng.integers(0, len(names)))]
        f, blocks, _ = tables[tname]
        target = "index" if tname == "index" or rng.random() < 0.3 else "data"
        g, desc = _corrupt(orc, f, blocks, target, rng)
        loc = _frame_of(blocks, g, target, f)
        if loc is None:  # (a corruption that changed nothing)
            continue
        fr = g[loc[0]:loc[0] + loc[1]]
        w = orc.snappy_frame_decode(fr)
        assert lcrc.snappy_frame_decode(fr) == w, f"case {case}: {desc}"
        frames.append(fr)
        want.append(w)
    from test_snappy_snap_rules import _c_oracle_status
    assert _c_oracle_status(orc, frames) == [0 if w is not None else 3 for w in want]
    assert sum(w is None for w in want) > NCASES // 2 and sum(w is not None for w in want) > 10
