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
