"""Diagnose lcrc_table_scan_async graph replay on the bench's table (step by step, progress to stdout)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
mode = m.MODE_REF if (len(sys.argv) < 2 or sys.argv[1] == "ref") else m.MODE_C
f, blocks = synth.table_layout(65536, 4096)
dev = m.DeviceBuffer.from_host(f)
d = np.zeros(len(blocks), m.DESC_DTYPE)
d["offset"] = [b[0] for b in blocks]
d["length"] = [b[1] + 1 for b in blocks]
d["expect_rel"] = [b[1] + 1 for b in blocks]
dd = m.DeviceBuffer.from_host(d.view(np.uint8))
seal = m.Engine(0, mode)
seal.batch_seal(dev, len(f), dd, len(blocks))
seal.sync()
cap = len(blocks) + 8
e = m.Engine(0, mode)
if "sync-first" in sys.argv:  # as bench.py: the synchronous scan into pinned memory first
    pinned = m.PinnedBuffer(cap * m.TBLK_DTYPE.itemsize)
    out = pinned.array.view(m.TBLK_DTYPE)
    print("sync scan", e.table_scan_into(dev, len(f), out), flush=True)
e.table_scan_reserve(len(f), cap)
res = (m.DeviceBuffer(cap * m.TBLK_DTYPE.itemsize), m.DeviceBuffer(8), m.DeviceBuffer(8))
e.table_scan_async(dev, len(f), res[0], cap, res[1], res[2])
e.sync()
print("direct ok", res[2].download(np.uint32, 2), int(res[1].download(np.uint64, 1)[0]), flush=True)
gr = e.graph_capture(lambda: e.table_scan_async(dev, len(f), res[0], cap, res[1], res[2]))
print("captured", flush=True)
for k in range(3):
    res[1].zero()
    e.graph_launch(gr)
    e.sync()
    print("replay", k, res[2].download(np.uint32, 2), int(res[1].download(np.uint64, 1)[0]), flush=True)
for k in range(5):
    e.graph_launch(gr)
e.sync()
print("5 back to back ok", flush=True)
# a second context whose first scan is the captured one, then both graphs alternating on their streams
e2 = m.Engine(0, mode)
e2.table_scan_reserve(len(f), cap)
res2 = (m.DeviceBuffer(cap * m.TBLK_DTYPE.itemsize), m.DeviceBuffer(8), m.DeviceBuffer(8))
gr2 = e2.graph_capture(lambda: e2.table_scan_async(dev, len(f), res2[0], cap, res2[1], res2[2]))
print("captured 2", flush=True)
e2.graph_launch(gr2)
e2.sync()
print("replay 2 alone", res2[2].download(np.uint32, 2), int(res2[1].download(np.uint64, 1)[0]), flush=True)
for k in range(6):
    (e if k % 2 == 0 else e2).graph_launch(gr if k % 2 == 0 else gr2)
e.sync()
e2.sync()
print("alternating ok", flush=True)
e.graph_destroy(gr)
e2.graph_destroy(gr2)
e.close()
e2.close()
