"""SSTable block trailers (table.rs:507-529) and read_block_from_file (format.rs:146-213)."""
import numpy as np


def test_write_raw_block_matches_oracle(lcrc, orc):
    rng = np.random.default_rng(1)
    t = lcrc.TableFile()
    want = b""
    handles = []
    for n in (0, 1, 5, 255, 4096, 4097, 70000):
        content = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        btype = int(rng.integers(0, 2))
        handles.append(t.write_raw_block(content, btype))
        want += orc.raw_block(content, btype)
    f = t.contents()
    assert f == want
    for off, size in handles:
        assert lcrc.TableFile.read_block(f, off, size, True) == orc.read_block(f, off, size, True)
        assert lcrc.TableFile.read_block(f, off, size, True)[1] is None


def test_read_block_errors(lcrc, orc):
    t = lcrc.TableFile()
    off, size = t.write_raw_block(b"hello world", 0)
    f = bytearray(t.contents())
    assert lcrc.TableFile.read_block(bytes(f), off, size + 1, True) == (None, "truncated block read")
    f[3] ^= 0x40
    assert lcrc.TableFile.read_block(bytes(f), off, size, True) == (None, "block checksum mismatch")
    # default ReadOption (verify_checksum = false, db/mod.rs:153-160) does not notice
    assert lcrc.TableFile.read_block(bytes(f), off, size, False) == (0, None)
    g = bytearray(orc.raw_block(b"abc", 7))
    assert lcrc.TableFile.read_block(bytes(g), 0, 3, True) == (None, "bad block type")
    for case in (bytes(f), bytes(g)):
        for verify in (True, False):
            n = 11 if case is not g else 3
            assert lcrc.TableFile.read_block(case, 0, n, verify) == orc.read_block(case, 0, n, verify)
