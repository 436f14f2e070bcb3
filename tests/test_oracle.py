"""Pins the CPU oracle: definition vs published check values, RFC 3720 vectors, Python zlib, the
committed golden fixtures, and the crc32fast/snap CPU paths restated in oracle/crc_oracle.c."""
import json
import os
import zlib

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_check_values(orc):
    v = _load("vectors.json")
    assert orc.crc_bitwise(b"123456789", 0) == 0xCBF43926 == int(v["check_ref_123456789"], 16)
    assert orc.crc_bitwise(b"123456789", 1) == 0xE3069283 == int(v["check_c_123456789"], 16)
    for name, case in v["rfc3720_crc32c"].items():
        assert orc.crc_bitwise(bytes.fromhex(case["data"]), 1) == int(case["crc"], 16), name


def test_empty_input(orc):
    for mode in (0, 1):
        assert orc.crc_bitwise(b"", mode) == 0
        assert orc.crc(b"", mode) == 0


@pytest.mark.parametrize("n", list(range(0, 70)) + [127, 128, 129, 255, 256, 1000, 4095, 4096, 4097, 65536 + 7])
def test_all_cpu_paths_agree(orc, n):
    d = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    z = zlib.crc32(d)
    assert orc.crc_bitwise(d, 0) == z
    assert orc.crc(d, 0) == z
    assert orc.crc_pclmul(d) == z
    c = orc.crc_bitwise(d, 1)
    assert orc.crc(d, 1) == c
    assert orc.crc_sse42(d) == c


def test_extend_semantics(orc):
    d = np.random.default_rng(3).integers(0, 256, 5000, dtype=np.uint8).tobytes()
    for cut in (0, 1, 17, 2500, 4999, 5000):
        assert orc.crc(d[cut:], 0, orc.crc(d[:cut], 0)) == zlib.crc32(d)
        assert orc.crc(d[cut:], 1, orc.crc(d[:cut], 1)) == orc.crc(d, 1)


def test_mask_roundtrip(orc):
    v = _load("vectors.json")
    for k, m in v["mask_examples"].items():
        assert orc.mask(int(k, 16)) == int(m, 16)
        assert orc.unmask(int(m, 16)) == int(k, 16)


def test_config1_golden(orc):
    g = _load("config1_golden.json")
    data = orc.splitmix_bytes(g["seed"], g["nblocks"] * g["block_len"])
    assert data[:16].tobytes().hex() == g["first16"]
    offs = np.arange(g["nblocks"], dtype=np.uint64) * g["block_len"]
    lens = np.full(g["nblocks"], g["block_len"], np.uint32)
    assert [f"{v:08x}" for v in orc.crc_ranges(data, offs, lens, 0)] == g["crc_ref"]
    assert [f"{v:08x}" for v in orc.crc_ranges(data, offs, lens, 1)] == g["crc_c"]
    # SURVEY.md 8c anchors
    assert g["crc_ref"][0] == "472faa0d" and g["crc_c"][0] == "076de509" and g["crc_c_masked"][0] == "6c94f9b3"
    assert g["crc_ref"][1023] == "1b48391d" and g["crc_c"][1023] == "38e9cd0a"
    assert (g["xor_ref"], g["xor_c"], g["xor_c_masked"]) == ("8923ef44", "941223fc", "c5846f84")
    assert g["sstable_trailer_ref_type0"][0] == "acf4bc9a"


def test_ranges_golden(orc):
    g = _load("ranges_golden.json")
    data = orc.splitmix_bytes(g["seed"], g["buffer_len"])
    for r in g["ranges"]:
        blk = data[r["offset"]:r["offset"] + r["length"]]
        assert f"{orc.crc(blk, 0):08x}" == r["crc_ref"]
        assert f"{orc.crc(blk, 1):08x}" == r["crc_c"]


def test_framing_literals(orc):
    v = _load("vectors.json")
    assert orc.log_write([b"foo"]).hex() == v["wal_record_foo"] == "4a04caea030001666f6f"
    assert orc.log_write([b"foo", b"", b"bar"]).hex() == v["wal_records_foo_bar_empty"]
    assert orc.raw_block(bytes.fromhex("0000000001000000"), 0)[8:].hex() == v["empty_block_trailer_type0"]
    assert orc.raw_block(bytes.fromhex("0000000001000000"), 1)[8:].hex() == v["empty_block_trailer_type1"]


def test_oracle_log_roundtrip(orc):
    recs = [b"x" * n for n in (1, 100, 32761, 32762, 70000, 3)]
    recs_read, dropped, msg = orc.log_read_all(orc.log_write(recs))
    assert recs_read == recs and dropped == 0 and msg == ""


def test_uniform_mt_matches(orc):
    data = orc.splitmix_bytes(1, 256 * 4096)
    want = orc.crc_ranges(data, np.arange(256) * 4096, np.full(256, 4096), 1)
    for algo in (orc.ALGO_S16_C, orc.ALGO_SSE42_C):
        got, secs = orc.crc_uniform_mt(data, 256, 4096, 4096, 4, algo)
        assert np.array_equal(got, want) and secs > 0
    want_r = orc.crc_ranges(data, np.arange(256) * 4096, np.full(256, 4096), 0)
    got, _ = orc.crc_uniform_mt(data, 256, 4096, 4096, 3, orc.ALGO_PCLMUL_REF)
    assert np.array_equal(got, want_r)


def test_host_clmul_constants():
    """The carry-less-multiply folding constants of csrc/lcrc_scalar.cpp, recomputed from P."""

    def xmod(e, P):
        r = 1
        for _ in range(e):
            r <<= 1
            if r >> 32 & 1:
                r ^= P
        return r

    def refl(v, bits):
        return int(bin(v)[2:].zfill(bits)[::-1], 2)

    for P, ks, mu, p in ((0x104C11DB7, (0x0154442bd4, 0x01c6e41596, 0x01751997d0, 0x00ccaa009e, 0x0163cd6124),
                          0x01f7011641, 0x01db710641),
                         (0x11EDC6F41, (0x00740eef02, 0x009e4addf8, 0x00f20c0dfe, 0x014cd00bd6, 0x00dd45aab8),
                          0x00dea713f1, 0x0105ec76f1)):
        for e, k in zip((128 * 4 + 32, 128 * 4 - 32, 128 + 32, 128 - 32, 64), ks):
            assert refl(xmod(e, P), 32) << 1 == k
        num, q = 1 << 64, 0
        while num.bit_length() >= 33:
            sh = num.bit_length() - 33
            q |= 1 << sh
            num ^= P << sh
        assert refl(q, 33) == mu and refl(P, 33) == p
