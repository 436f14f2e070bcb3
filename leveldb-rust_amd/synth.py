"""Synthetic inputs for the BASELINE.json configs. Deterministic from committed seeds.

* ``splitmix_bytes(seed, n)``: s += 0x9E3779B97F4A7C15, standard splitmix64 mix, 8 LE bytes per step.
* config 1: 1,024 x 4,096 B, seed 0x5EED (golden CPU vectors)
* config 2: 65,536 x 4,096 B back-to-back, seed 0x5EED0001 (+g per GPU)
* config 3: SSTable-like file, block sizes 256 B-64 KiB zipf(1.1) over classes ordered by closeness to
  4 KiB, each block stored with its 5-byte trailer (table.rs:507-529), seed 0x5EED0002
* config 4: WAL file written by the LogWriter restatement, record lengths k ~ U[1,16], n ~ U[1, 2^k)
  (the distribution of the reference's own test_random_read, src/db/log.rs:641-644)
"""
import numpy as np

GOLDEN = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1
SEED_GOLDEN, SEED_FIXED, SEED_MIXED, SEED_WAL = 0x5EED, 0x5EED0001, 0x5EED0002, 0x5EED0003


def splitmix_u64(seed, n):
    i = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + i * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def splitmix_bytes(seed, n):
    words = splitmix_u64(seed, (n + 7) // 8)
    return words.astype("<u8").view(np.uint8)[:n]


class SplitMix:
    """Scalar splitmix64 stream (for sizes)."""

    def __init__(self, seed):
        self.s = seed & M64

    def next(self):
        self.s = (self.s + GOLDEN) & M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)

    def uniform(self):
        return (self.next() >> 11) * (1.0 / (1 << 53))

    def below(self, n):
        return self.next() % n


MIXED_CLASSES = [4096, 2048, 8192, 1024, 16384, 512, 32768, 256, 65536]  # ranked by closeness to 4 KiB


def mixed_sizes(total_bytes, seed=SEED_MIXED, s=1.1):
    """Zipf(s) class per block, size uniform in (class/2, class], first class floored at 256."""
    rng = SplitMix(seed)
    w = np.array([1.0 / (r ** s) for r in range(1, len(MIXED_CLASSES) + 1)])
    cdf = np.cumsum(w / w.sum())
    sizes, tot = [], 0
    while tot < total_bytes:
        u = rng.uniform()
        cls = MIXED_CLASSES[int(np.searchsorted(cdf, u, side="right").clip(0, len(MIXED_CLASSES) - 1))]
        lo = cls // 2
        sz = lo + 1 + rng.below(cls - lo)
        sz = max(sz, 256)
        sizes.append(sz)
        tot += sz
    return np.array(sizes, dtype=np.uint32)


def sstable_layout(sizes):
    """Offsets of blocks stored back to back with 5-byte trailers. Descriptor covers content+type."""
    sizes = np.asarray(sizes, np.uint64)
    stored = sizes + np.uint64(5)
    offs = np.zeros(len(sizes), np.uint64)
    if len(sizes) > 1:
        offs[1:] = np.cumsum(stored)[:-1]
    total = int(stored.sum())
    return offs, total


def wal_lengths(total_bytes, seed=SEED_WAL):
    rng = SplitMix(seed)
    out, tot = [], 0
    while tot < total_bytes:
        k = 1 + rng.below(16)
        n = 1 + rng.below((1 << k) - 1)
        out.append(n)
        tot += n + 7
    return out


SEED_TABLE, SEED_SNAPPY = 0x5EED0004, 0x5EED0005
TABLE_MAGIC = 0xdb4775248b80fb57  # src/sstable/format.rs:20


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def table_layout(nblk, blen, seed=SEED_TABLE):
    """A synthetic SSTable for the whole-table scan bench: nblk raw data blocks of blen random bytes, each
    followed by its 5-byte trailer slot [type 0][crc: zero, to be sealed], then an (empty) metaindex block and
    an index block with one entry per data block (shared = 0, one restart), trailer slots likewise, and the
    48-byte footer. The index block restarts at every entry, as the reference's (table.rs:272). Returns (file bytes as numpy u8, [(offset, size)] of every block needing a trailer)."""
    import numpy as np
    stride = blen + 5
    data = np.zeros(nblk * stride, np.uint8)
    body = splitmix_bytes(seed, nblk * blen).reshape(nblk, blen)
    data.reshape(nblk, stride)[:, :blen] = body
    blocks = [(i * stride, blen) for i in range(nblk)]
    meta = (0).to_bytes(4, "little") + (1).to_bytes(4, "little")  # restart [0], one restart
    idx = bytearray()
    restarts = []
    for i in range(nblk):  # restart interval 1, as the reference's index blocks (table.rs:272)
        key = i.to_bytes(8, "big")
        val = _varint(i * stride) + _varint(blen)
        restarts.append(len(idx))
        idx += b"\x00" + _varint(len(key)) + _varint(len(val)) + key + val
    idx += np.asarray(restarts, "<u4").tobytes() + len(restarts).to_bytes(4, "little")
    moff = len(data)
    tail = bytearray(meta) + bytes(5)
    ioff = moff + len(tail)
    tail += idx + bytes(5)
    foot = _varint(moff) + _varint(len(meta)) + _varint(ioff) + _varint(len(idx))
    foot += bytes(40 - len(foot)) + TABLE_MAGIC.to_bytes(8, "little")
    tail += foot
    blocks += [(moff, len(meta)), (ioff, len(idx))]
    return np.concatenate([data, np.frombuffer(bytes(tail), np.uint8)]), blocks


def snappy_frame_synthetic(seed=SEED_SNAPPY, unit=64, reps=64):
    """One Snappy frame (stream identifier + one compressed data chunk) of `unit` random bytes repeated
    `reps` times, Snappy-encoded as one literal and reps - 1 two-byte-offset copies; the chunk CRC slot is
    zero (to be filled with the masked CRC-32C of the uncompressed bytes). Returns (frame bytes, raw bytes,
    offset of the CRC slot)."""
    lit = bytes(splitmix_bytes(seed, unit))
    raw = lit * reps
    z = bytearray(_varint(len(raw)))
    z += bytes([60 << 2, unit - 1]) + lit if unit > 60 else bytes([(unit - 1) << 2]) + lit
    for _ in range(reps - 1):
        z += bytes([((unit - 1) << 2) | 2, unit & 0xFF, unit >> 8])
    body = bytes(4) + bytes(z)
    frame = b"\xff\x06\x00\x00sNaPpY" + bytes([0]) + len(body).to_bytes(3, "little") + body
    return frame, raw, 14


SEED_TEXT = 0x5EED0006


def compressible_values(n, vlen, fraction=0.5, seed=SEED_TEXT):
    """n values of vlen bytes as LevelDB's db_bench makes them (CompressibleString: a random printable string of
    vlen * fraction bytes, repeated to fill vlen), so Snappy keeps about `fraction` of each."""
    k = max(1, int(vlen * fraction))
    rng = np.random.default_rng(seed)
    raw = rng.integers(ord(" "), ord("~") + 1, (n, k)).astype(np.uint8)
    reps = -(-vlen // k)
    return np.tile(raw, (1, reps))[:, :vlen]


def compressed_table(m, nblk, block_size=4096, vlen=100):
    """A Snappy-compressed SSTable written by the TableBuilder restatement (table.rs:268-468, compression type 1 =
    the reference's default, option.rs:127): keys k%015d, db_bench-style values (half compressible), about nblk data
    blocks. Returns (file bytes as numpy u8, the builder's block list)."""
    # entries per data block: the index-shared key prefix leaves ~vlen + 6 bytes per entry (flushed at >= block_size)
    per = max(1, -(-block_size // (vlen + 6)))
    n = nblk * per
    vals = compressible_values(n, vlen)
    tb = m.TableBuilder(block_size=block_size, compression=1, mode=m.MODE_REF, host_seal=True)
    digits = np.arange(n, dtype=np.int64)[:, None] // (10 ** np.arange(14, -1, -1, dtype=np.int64))[None, :] % 10
    keys = np.concatenate([np.full((n, 1), ord("k"), np.uint8), (digits + ord("0")).astype(np.uint8)], axis=1)
    tb.add_many(keys, vals)
    f = tb.finish()
    return np.frombuffer(f, np.uint8), tb.blocks()
