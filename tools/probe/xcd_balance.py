"""Per-XCD end times of k_windows<true> over several single launches (LCRC_PROBE_CLOCK build, via LCRC_LIB_PATH):
is the XCD spread of one launch the same XCDs every time (then a static / feedback share per XCD could balance it)?
Prints, per launch, the last wave's end per XCC_ID relative to the launch's first wave entry (us)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
launches = int(sys.argv[2]) if len(sys.argv) > 2 else 12
bufs = [m.DeviceBuffer(nb * 4096) for _ in range(4)]
for i, b in enumerate(bufs):
    b.upload(synth.splitmix_bytes(0x5EED0001 + i, nb * 4096))
out = m.DeviceBuffer(nb * 4)
eng = m.Engine(0, 1)
for i in range(10):
    eng.batch_uniform(bufs[i % 4], nb, 4096, 4096, out)
rows = []
for k in range(launches):
    eng.timer_start()
    eng.batch_uniform(bufs[k % 4], nb, 4096, 4096, out)
    ms = eng.timer_stop()
    st = (ctypes.c_ulonglong * (4096 * 8))()
    m.lib().lcrc_probe_stamps(st)
    a = np.frombuffer(st, dtype=np.uint64).reshape(4096, 8).astype(np.int64)
    ok = a[:, 0] != 0
    t0 = a[ok, 0].min()
    xcc = a[:, 7] & 0xF
    ends, firsts, cnt = [], [], []
    for x in range(8):
        sel = ok & (xcc == x)
        ends.append((a[sel, 3].max() - t0) / 100.0 if sel.any() else np.nan)
        firsts.append((np.median(a[sel, 1]) - t0) / 100.0 if sel.any() else np.nan)
        cnt.append(int(sel.sum()))
    rows.append(ends)
    print(f"launch {k:2d} event {ms * 1000:6.1f} us  end/XCC " + " ".join(f"{e:6.2f}" for e in ends) +
          f"  spread {np.nanmax(ends) - np.nanmin(ends):5.2f}  tables " + " ".join(f"{f:5.2f}" for f in firsts) +
          f"  waves/XCC {cnt}")
r = np.array(rows)
rank = np.argsort(np.argsort(-r, axis=1), axis=1)  # 0 = latest XCC of that launch
print("mean end per XCC  ", " ".join(f"{v:6.2f}" for v in r.mean(0)))
print("std end per XCC   ", " ".join(f"{v:6.2f}" for v in r.std(0)))
print("mean rank (0=last)", " ".join(f"{v:6.2f}" for v in rank.mean(0)))
# the end of each XCC relative to that launch's mean: a stable pattern shows a small std here
rel = r - r.mean(1, keepdims=True)
print("rel mean          ", " ".join(f"{v:6.2f}" for v in rel.mean(0)))
print("rel std           ", " ".join(f"{v:6.2f}" for v in rel.std(0)))
