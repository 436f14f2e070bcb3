"""Worker for tests/test_multi_rank.py: bench.py's N>1 path (Dist barrier + max-over-ranks + weak-scaling
aggregate) on the gloo backend, with each rank checksumming its own shard on the CPU oracle."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
import __graft_entry__ as entry  # noqa: E402

dist = bench.Dist(backend="gloo")
orc = entry.load_oracle()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"]) if entry.load() else None
nblk, blen = 256, 4096
data = synth.splitmix_bytes(synth.SEED_FIXED + dist.rank, nblk * blen)  # rank-private shard, no exchange
crcs = []


def step(i):
    crcs.append(orc.crc_ranges(data, np.arange(nblk) * blen, np.full(nblk, blen), 1))


elapsed_max, _ = bench.timed_run(dist, step, steps=3, warmup=1)
value = bench.aggregate_gibs(nblk * blen, 3, dist.world, elapsed_max)
with open(os.path.join(os.environ["LCRC_DIST_OUT"], f"rank{dist.rank}.json"), "w") as f:
    json.dump({"rank": dist.rank, "world": dist.world, "elapsed_max": elapsed_max, "value": value,
               "xor": int(np.bitwise_xor.reduce(crcs[-1]))}, f)
dist.close()
