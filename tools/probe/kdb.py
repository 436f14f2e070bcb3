"""Per-kernel durations from a rocprofv3 results database (rocpd sqlite): python3 kdb.py DIR_OR_DB..."""
import glob
import os
import sqlite3
import sys

for a in sys.argv[1:]:
    for f in ([a] if a.endswith(".db") else sorted(glob.glob(os.path.join(a, "**", "*.db"), recursive=True))):
        cur = sqlite3.connect(f).cursor()
        print("==", os.path.relpath(f))
        q = ("select name, count(*), avg(end-start), min(end-start), max(end-start) from kernels group by name "
             "order by sum(end-start) desc")
        for name, n, avg, mn, mx in cur.execute(q):
            name = name.split("(")[0].replace("void ", "").replace("lcrc_dev::", "")
            print(f"  {name:28s} calls {n:4d} avg {avg/1e3:9.2f} us  min {mn/1e3:8.2f}  max {mx/1e3:8.2f}")
