"""k_ts_decode timeline (LCRC_PROBE_CLOCK build), one raw-table (or, argument "z", compressed-table) async scan alone: per workgroup entry, gate passed,
content judged, end -- microseconds from the earliest entry."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
Z = len(sys.argv) > 1 and sys.argv[1] == "z"  # "z": the bench's compressed table (framed index decoded on the device)
eng = m.Engine(0, m.MODE_REF)
if Z:
    f, blocks = synth.compressed_table(m, 65536)
    dev = m.DeviceBuffer.from_host(f, 0)
else:
    f, blocks = synth.table_layout(65536, 4096)
    dev = m.DeviceBuffer.from_host(f, 0)
    d = np.zeros(len(blocks), m.DESC_DTYPE)
    d["offset"] = [b[0] for b in blocks]
    d["length"] = [b[1] + 1 for b in blocks]
    d["expect_rel"] = [b[1] + 1 for b in blocks]
    dd = m.DeviceBuffer.from_host(d.view(np.uint8), 0)
    eng.batch_seal(dev, len(f), dd, len(blocks))
    eng.sync()
cap = len(blocks) + 8
res = m.DeviceBuffer(cap * m.TBLK_DTYPE.itemsize, 0), m.DeviceBuffer(8, 0), m.DeviceBuffer(8, 0)
eng.table_scan_reserve(len(f), cap, 300 << 20)
for rep in range(3):
    for i in range(5):
        eng.table_scan_async(dev, len(f), res[0], cap, res[1], res[2], snappy_index=Z)
        eng.sync()
    st = (ctypes.c_ulonglong * (4096 * 8))()
    m.lib().lcrc_probe_stamps(st)
    a = np.frombuffer(st, dtype=np.uint64).reshape(4096, 8).astype(np.int64)
    w = a[2304:2304 + 768]
    w = w[w[:, 0] != 0]
    t0 = w[:, 0].min()
    print(f"status {res[2].download(np.uint32, 2)} workgroups {len(w)}")
    q = lambda v: " ".join(f"{x:7.2f}" for x in np.percentile((v[v != 0] - t0) / 100.0, [0, 10, 50, 90, 100]))
    for k, name in [(0, "entry"), (3, "gate"), (4, "content"), (5, "end")]:
        print(f"  {name:8s}", q(w[:, k]))
    full = a[2304:2304 + 768]
    ids = np.nonzero(full[:, 0])[0]
    ends = (full[ids, 5] - t0) / 100.0
    top = ids[np.argsort(-ends)[:6]]
    print("  latest workgroups (tile: gate, end):", ", ".join(
        f"{int(i)}: {(full[i, 3] - t0) / 100.0:.1f}, {(full[i, 5] - t0) / 100.0:.1f}" for i in top))
