"""Per-wave end times of one queued launch (k_windows_q, LCRC_PROBE_CLOCK build via LCRC_LIB_PATH): how far
apart the CUs / XCDs finish inside a Q-batch launch of 64K x 4 KiB batches. Usage: qstamps.py [Q]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
Q = int(sys.argv[1]) if len(sys.argv) > 1 else 5
nb = 65536
bufs = [m.DeviceBuffer(nb * 4096) for _ in range(Q)]
for i, b in enumerate(bufs):
    b.upload(synth.splitmix_bytes(0x5EED0001 + i, nb * 4096))
outs = [m.DeviceBuffer(nb * 4) for _ in range(Q)]
eng = m.Engine(0, 1)
jobs = m.ujobs([(bufs[i], nb, outs[i]) for i in range(Q)])
for i in range(10):
    eng.batch_uniform_queue(jobs, 4096, 4096)
eng.timer_kernels(0)
eng.timer_kernels(1)
eng.batch_uniform_queue(jobs, 4096, 4096)
ms = eng.timer_stop()
st = (ctypes.c_ulonglong * (4096 * 8))()
m.lib().lcrc_probe_stamps(st)
full = np.frombuffer(st, dtype=np.uint64).reshape(4096, 8).astype(np.int64)
ok = full[:, 0] != 0
t0 = full[ok, 0].min()
rr = (full[:, :6] - t0) / 100.0  # 100 MHz ticks -> us: entry, tables, first half, end, loads issued, built
m.lib().lcrc_probe_clock_mhz.restype = ctypes.c_double
m.lib().lcrc_probe_clock_mhz.argtypes = [ctypes.c_int]
print(f"Q {Q}: event {ms * 1000:.1f} us, waves {ok.sum()}, shader clock {m.lib().lcrc_probe_clock_mhz(256):.0f} MHz "
      "(median over workgroups, tile loop)")
for k, name in ((0, "entry"), (4, "issued"), (5, "built"), (1, "tables"), (2, "first"), (3, "end")):
    print(f"  {name:7s}", np.percentile(rr[ok, k], [0, 10, 50, 90, 100]).round(2))
ids = full[:, 6:8]
xcc = ids[:, 1] & 0xF
print("  by XCC (waves, median end, max end)")
for x in range(8):
    sel = ok & (xcc == x)
    if sel.any():
        print(f"    xcc {x}: {sel.sum():5d} {np.median(rr[sel, 3]):8.2f} {rr[sel, 3].max():8.2f}")
key = xcc * 256 + ((ids[:, 0] >> 8) & 0xFF)
ce = np.array([rr[ok & (key == k), 3].max() for k in np.unique(key[ok])])
print(f"  CUs {len(ce)}; per-CU last end percentiles", np.percentile(ce, [0, 10, 50, 90, 100]).round(2))
busy = ce.max() - ce  # idle time of each CU before the launch ends
print(f"  mean CU idle at the end {busy.mean():.2f} us of {ce.max():.2f} ({100 * busy.mean() / ce.max():.1f} %)")
