"""Per-kernel durations and gaps from a rocprofv3 rocpd database (rocprofv3 -d DIR -o run, no csv):
python3 tools/probe/kernel_times.py DIR/run_results.db [LAST_N]"""
import sqlite3
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
last = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = list(c.execute("select name, start, end from kernels order by start"))
prev = None
for name, s, e in rows[-last:]:
    print(f"{name[:48]:48s} {(e - s) / 1e3:8.2f} us  gap {((s - prev) / 1e3) if prev else 0:7.2f}")
    prev = e
agg = defaultdict(list)
for name, s, e in rows:
    agg[name.split("(")[0]].append((e - s) / 1e3)
for k, v in agg.items():
    v.sort()
    print(f"{k[:60]:60s} n={len(v):4d} median {v[len(v) // 2]:8.2f} us  min {v[0]:8.2f}")
