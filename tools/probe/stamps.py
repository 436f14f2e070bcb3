"""Per-wave timeline of one k_windows launch (LCRC_PROBE_CLOCK build): entry, tables ready, first half
walked, end -- relative to the earliest entry, in microseconds."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as g  # noqa: E402

m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
for nb in (int(a) for a in (sys.argv[1:] or ["65536"])):
    bufs = [m.DeviceBuffer(nb * 4096) for _ in range(4)]
    for i, b in enumerate(bufs):
        b.upload(synth.splitmix_bytes(0x5EED0001 + i, nb * 4096))
    out = m.DeviceBuffer(nb * 4)
    eng = m.Engine(0, 1)
    for i in range(20):
        eng.batch_uniform(bufs[i % 4], nb, 4096, 4096, out)
    eng.timer_start()
    eng.batch_uniform(bufs[1], nb, 4096, 4096, out)
    ms = eng.timer_stop()
    st = (ctypes.c_ulonglong * (4096 * 8))()
    m.lib().lcrc_probe_stamps(st)
    a = np.frombuffer(st, dtype=np.uint64).reshape(4096, 8)[:, [0, 4, 5, 1, 2, 3]].astype(np.int64)
    a = a[a[:, 0] != 0]
    t0 = a[:, 0].min()
    r = (a - t0) / 100.0  # 100 MHz ticks -> us
    print(f"nblk {nb}: event {ms * 1000:.1f} us, waves {len(a)}")
    for k, name in enumerate(["entry", "src", "staged", "tables", "first", "end"]):
        q = np.percentile(r[:, k], [0, 10, 50, 90, 100])
        print(f"  {name:7s} " + " ".join(f"{x:7.2f}" for x in q))
    # grouping: workgroup w runs on XCD w % 8 (round-robin dispatch); wave index inside the workgroup
    full = np.frombuffer(st, dtype=np.uint64).reshape(4096, 8)[:, [0, 1, 2, 3]].astype(np.int64)
    gw = np.arange(4096)
    ok = full[:, 0] != 0
    rr = (full - t0) / 100.0
    wg = gw // 8
    print("  by XCD   (median first / median end / max end)")
    for x in range(8):
        sel = ok & (wg % 8 == x)
        if sel.any():
            print(f"    xcd {x}: {np.median(rr[sel, 2]):7.2f} {np.median(rr[sel, 3]):7.2f} {rr[sel, 3].max():7.2f}")
    print("  by wave-in-WG (median first / median end)")
    for wv in range(8):
        sel = ok & (gw % 8 == wv)
        if sel.any():
            print(f"    wave {wv:2d}: {np.median(rr[sel, 2]):7.2f} {np.median(rr[sel, 3]):7.2f}")
    # CU-level: per workgroup max end
    we = np.array([rr[(wg == w) & ok, 3].max() if ((wg == w) & ok).any() else np.nan for w in range(512)])
    print("  per-WG max end percentiles", np.nanpercentile(we, [0, 10, 50, 90, 100]).round(2))
    # CU-level: key = (XCC_ID, HW_ID[15:8] = cu/sh/se)
    ids = np.frombuffer(st, dtype=np.uint64).reshape(4096, 8)[:, 6:8].astype(np.int64)
    key = (ids[:, 1] & 0xF) * 256 + ((ids[:, 0] >> 8) & 0xFF)
    cus = {}
    for w in range(4096):
        if ok[w]:
            cus.setdefault(int(key[w]), []).append(w)
    ce = np.array([rr[v, 3].max() for v in cus.values()])
    cfirst_wg_end = []
    for v in cus.values():
        wgs = sorted({int(x) // 8 for x in v})
        ends = [rr[[x for x in v if x // 8 == g_], 3].max() for g_ in wgs]
        cfirst_wg_end.append(ends)
    print(f"  CUs seen {len(cus)}; per-CU end percentiles", np.percentile(ce, [0, 10, 50, 90, 100]).round(2))
    wgs_per_cu = [len(e) for e in cfirst_wg_end]
    print("  WGs per CU histogram", np.bincount(wgs_per_cu))
    lo = np.array([min(e) for e in cfirst_wg_end if len(e) == 2])
    hi = np.array([max(e) for e in cfirst_wg_end if len(e) == 2])
    if len(lo):
        print("  2-WG CUs: earlier WG end pct", np.percentile(lo, [10, 50, 90]).round(2),
              " later WG end pct", np.percentile(hi, [10, 50, 90]).round(2))
    # which WG indices share a CU (first few)
    print("  sample CU -> WGs", [sorted({int(x) // 8 for x in v}) for v in list(cus.values())[:6]])
