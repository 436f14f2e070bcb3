"""Time the compressed-table device scan (lcrc_table_scan_async, the bench's tablez workload) alone on one stream,
for each library named on the command line (tools/probe/variants/NAME.so; "prod" = the in-tree one). No result check
beyond printing the scan's status: ablation builds that skip work are timed too. Prints us per scan."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r'''
import os, sys
import numpy as np
sys.path.insert(0, ROOT)
import __graft_entry__ as g
m = g.load()
synth = __import__("leveldb_rust_amd.synth", fromlist=["x"])
f, tb = synth.compressed_table(m, 65536)
dev = m.DeviceBuffer.from_host(f, 0)
cap = len(tb) + 8
dec = int(sum(len(m.snappy_frame_decode(f[int(b["offset"]):int(b["offset"] + b["size"])]))
              for b in tb if f[int(b["offset"] + b["size"])] == 1))
eng = m.Engine(0, m.MODE_REF, **dict(kv.split("=") for kv in os.environ.get("TZ_OPTS", "").split() if kv))
eng.table_scan_reserve(len(f), cap, dec)
res, cnt, st = m.DeviceBuffer(cap * m.TBLK_DTYPE.itemsize, 0), m.DeviceBuffer(8, 0), m.DeviceBuffer(8, 0)
for _ in range(3):
    eng.table_scan_async(dev, len(f), res, cap, cnt, st, snappy_index=True)
eng.sync()
best = 1e9
for rep in range(3):
    eng.timer_start()
    for _ in range(10):
        eng.table_scan_async(dev, len(f), res, cap, cnt, st, snappy_index=True)
    best = min(best, eng.timer_stop() / 10)
s = st.download(np.uint32, 2).tolist()
print(f"{os.environ.get('TZ_NAME', 'prod'):16s} {best * 1000:8.1f} us per scan  status {s}", flush=True)
'''.replace("ROOT", repr(ROOT))
vdir = os.path.join(ROOT, "tools", "probe", "variants")
for v in sys.argv[1:] or ["prod"]:
    env = dict(os.environ, TZ_NAME=v)
    if v != "prod":
        env["LCRC_LIB_PATH"] = os.path.join(vdir, v if v.endswith(".so") else v + ".so")
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, timeout=300)
    if r.returncode:
        sys.exit(r.returncode)
