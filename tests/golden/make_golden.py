"""Generates tests/golden/*.json from the CPU oracle (bitwise definition) cross-checked with Python's
zlib.crc32 (an independent CRC-32/ISO-HDLC implementation). Run from the repo root:
    python tests/golden/make_golden.py
The reference (Rust, unbuildable here) holds no CRC golden vectors of its own."""
import json
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as orc  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    # config 1: 1024 x 4096 B, seed 0x5EED, one host thread
    seed, n, blen = 0x5EED, 1024, 4096
    data = orc.splitmix_bytes(seed, n * blen)
    ref, c, trailer = [], [], []
    for i in range(n):
        blk = data[i * blen:(i + 1) * blen]
        r = orc.crc_bitwise(blk, 0)
        assert r == zlib.crc32(blk.tobytes())
        ref.append(r)
        c.append(orc.crc_bitwise(blk, 1))
        trailer.append(orc.crc_bitwise(np.concatenate([blk, np.zeros(1, np.uint8)]), 0))
    masked = [orc.mask(v) for v in c]
    x = lambda vs: int(np.bitwise_xor.reduce(np.array(vs, np.uint32)))
    g = {
        "config": "1K x 4 KiB splitmix64 blocks (BASELINE.json configs[0])",
        "seed": seed, "nblocks": n, "block_len": blen,
        "first16": data[:16].tobytes().hex(),
        "crc_ref": [f"{v:08x}" for v in ref],
        "crc_c": [f"{v:08x}" for v in c],
        "crc_c_masked": [f"{v:08x}" for v in masked],
        "sstable_trailer_ref_type0": [f"{v:08x}" for v in trailer],
        "xor_ref": f"{x(ref):08x}", "xor_c": f"{x(c):08x}", "xor_c_masked": f"{x(masked):08x}",
    }
    with open(os.path.join(OUT, "config1_golden.json"), "w") as f:
        json.dump(g, f, indent=0)

    # literal known-answer vectors (published check values + RFC 3720 B.4) and framing bytes
    rfc = {
        "zeros32": ("00" * 32, "8a9136aa"),
        "ones32": ("ff" * 32, "62a8ab43"),
        "incr32": (bytes(range(32)).hex(), "46dd794e"),
        "decr32": (bytes(range(31, -1, -1)).hex(), "113fdb5c"),
    }
    for k, (hx, want) in rfc.items():
        assert f"{orc.crc_bitwise(bytes.fromhex(hx), 1):08x}" == want, k
    lit = {
        "check_ref_123456789": f"{orc.crc_bitwise(b'123456789', 0):08x}",
        "check_c_123456789": f"{orc.crc_bitwise(b'123456789', 1):08x}",
        "rfc3720_crc32c": {k: {"data": hx, "crc": want} for k, (hx, want) in rfc.items()},
        "wal_record_foo": orc.log_write([b"foo"]).hex(),
        "wal_records_foo_bar_empty": orc.log_write([b"foo", b"", b"bar"]).hex(),
        "empty_block_trailer_type0": orc.raw_block(bytes.fromhex("0000000001000000"), 0)[8:].hex(),
        "empty_block_trailer_type1": orc.raw_block(bytes.fromhex("0000000001000000"), 1)[8:].hex(),
        "mask_examples": {f"{v:08x}": f"{orc.mask(v):08x}" for v in (0, 1, 0xFFFFFFFF, 0xE3069283, 0x12345678)},
    }
    assert lit["check_ref_123456789"] == "cbf43926" and lit["check_c_123456789"] == "e3069283"
    with open(os.path.join(OUT, "vectors.json"), "w") as f:
        json.dump(lit, f, indent=1)

    # mixed-length ranges over a 256 KiB buffer (edge lengths around the 16 B / 256 B / 4 KiB structure)
    data2 = orc.splitmix_bytes(0x5EED0010, 262144)
    rng = np.random.default_rng(7)
    lens = [0, 1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 512,
            513, 1023, 1024, 1025, 4095, 4096, 4097, 8191, 8192, 8193, 65535, 65536, 65537]
    offs = [int(rng.integers(0, 262144 - l + 1)) for l in lens]
    offs += [0, 262144 - 1, 255, 256, 257, 4095, 4096, 4097]
    lens += [262144, 1, 1, 256, 3000, 1, 4096, 100000]
    ranges = []
    for o, l in zip(offs, lens):
        blk = data2[o:o + l]
        r = orc.crc_bitwise(blk, 0)
        assert r == zlib.crc32(blk.tobytes())
        ranges.append({"offset": o, "length": l, "crc_ref": f"{r:08x}", "crc_c": f"{orc.crc_bitwise(blk, 1):08x}"})
    with open(os.path.join(OUT, "ranges_golden.json"), "w") as f:
        json.dump({"seed": 0x5EED0010, "buffer_len": 262144, "ranges": ranges}, f, indent=0)
    print("wrote", os.listdir(OUT))


if __name__ == "__main__":
    main()
