"""k_ts_open2 per-workgroup timeline (LCRC_PROBE_CLOCK build): entry, frame walked, chunk reached, staged, phase 1,
decoded, checksummed, end -- microseconds from the earliest entry, one compressed-table async scan run alone."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
f, tb = synth.compressed_table(m, 65536)
dev = m.DeviceBuffer.from_host(f, 0)
eng = m.Engine(0, m.MODE_REF)
cap = len(tb) + 8
res = m.DeviceBuffer(cap * m.TBLK_DTYPE.itemsize, 0), m.DeviceBuffer(8, 0), m.DeviceBuffer(8, 0)
eng.table_scan_reserve(len(f), cap, 300 << 20)
for i in range(4):
    eng.table_scan_async(dev, len(f), res[0], cap, res[1], res[2], snappy_index=True)
    eng.sync()
st = (ctypes.c_ulonglong * (4096 * 8))()
m.lib().lcrc_probe_stamps(st)
a = np.frombuffer(st, dtype=np.uint64).reshape(4096, 8)[3072:].astype(np.int64)  # (k_ts_open's rows)
a = a[a[:, 0] != 0]
t0 = a[:, 0].min()
r = np.where(a != 0, (a - t0) / 100.0, np.nan)
print("status", res[2].download(np.uint32, 2), "workgroups", len(a))
names = ["entry", "staged", "A exits", "B entries", "C-F1", "F2 (S)", "F3 jumps", "end"]
for k, name in enumerate(names):
    print(f"  {name:8s} " + " ".join(f"{x:8.2f}" for x in np.nanpercentile(r[:, k], [0, 50, 100])))
for w in range(len(a)):
    print("  wg %2d " % w + " ".join("%7.1f" % x for x in r[w]))
