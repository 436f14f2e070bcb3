"""Per-wave timeline of one k_blocks launch on the mixed (SSTable) workload (LCRC_PROBE_CLOCK build)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
sizes = synth.mixed_sizes(256 << 20, seed=synth.SEED_MIXED)
offs, total = synth.sstable_layout(sizes)
data = synth.splitmix_bytes(synth.SEED_MIXED + 1000, total)
d = np.zeros(len(sizes), m.DESC_DTYPE)
d["offset"], d["length"], d["expect_rel"] = offs, sizes.astype(np.uint64) + 1, m.NO_EXPECT
buf = m.DeviceBuffer.from_host(data)
dd = m.DeviceBuffer.from_host(d.view(np.uint8))
out = m.DeviceBuffer(4 * len(sizes))
eng = m.Engine(0, 1)
eng.reserve(total)
for i in range(10):
    eng.batch(buf, total, dd, len(sizes), out)
eng.sync()
if os.environ.get("CORUN"):
    # the measured k_blocks beside another stream's window passes (as in the 2-stream bench): two fast-path
    # launches of 256 MiB enqueued on a second engine first
    fb = m.DeviceBuffer(65536 * 4096)
    fb.upload(synth.splitmix_bytes(0x5EED0001, 65536 * 4096))
    fo = m.DeviceBuffer(65536 * 4)
    e2 = m.Engine(0, 1)
    e2.batch_uniform(fb, 65536, 4096, 4096, fo)
    e2.sync()
    e2.batch_uniform(fb, 65536, 4096, 4096, fo)
    e2.batch_uniform(fb, 65536, 4096, 4096, fo)
    e2.batch_uniform(fb, 65536, 4096, 4096, fo)
eng.batch(buf, total, dd, len(sizes), out)
eng.sync()
if os.environ.get("CORUN"):
    e2.sync()
st = (ctypes.c_ulonglong * (8192 * 8))()
m.lib().lcrc_probe_bstamps(st)
a = np.frombuffer(st, dtype=np.uint64).reshape(8192, 8).astype(np.int64)
a = a[a[:, 0] != 0]
t0 = a[:, 0].min()
r = (a - t0) / 100.0
print(f"k_blocks: ranges {len(sizes)}, waves {len(a)}")
for k, name in enumerate(["entry", "tables", "it1", "it2", "it3", "it4", "it5", "end"]):
    col = r[:, k][a[:, k] != 0]
    if not len(col):
        continue
    print(f"  {name:7s} " + " ".join(f"{x:7.2f}" for x in np.percentile(col, [0, 10, 50, 90, 100])))
# per-iteration durations (each row's range: loads, head walk, fold, tail walk, store)
prev = a[:, 1]
for k in range(5):
    cur = a[:, 2 + k]
    ok = cur != 0
    if ok.any():
        d = (cur[ok] - prev[ok]) / 100.0
        print(f"  iter {k + 1} waves {ok.sum():5d} us " + " ".join(f"{x:6.2f}" for x in np.percentile(d, [10, 50, 90])))
    prev = np.where(ok, cur, prev)
if os.environ.get("PHASES"):
    # LCRC_PROBE_PHASES build: first iteration's phase ends in columns 3..6 (loads, head, fold, tail), 2 = end
    ph = a[:, 3:7]
    ok = (ph != 0).all(1)
    prev = a[ok, 1]
    for k, name in enumerate(["loads", "head walk", "fold", "tail walk"]):
        d = (ph[ok, k] - prev) / 100.0
        print(f"  phase {name:10s} us " + " ".join(f"{x:6.2f}" for x in np.percentile(d, [10, 50, 90])))
        prev = ph[ok, k]
    d = (a[ok, 2] - prev) / 100.0
    print(f"  phase {'store':10s} us " + " ".join(f"{x:6.2f}" for x in np.percentile(d, [10, 50, 90])))
