"""Kernel timeline of a rocprofv3 --kernel-trace run: per dispatch the kernel, its queue/stream, start and
end relative to the first timed dispatch (us), and the gap since the previous kernel on the HBM stream.
Usage: python3 timeline.py TRACE_DIR [LAST_N]"""
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = rows[-last:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("lcrc_dev::", "")
    q = r.get("Queue_Id") or r.get("Stream_Id") or ""
    st = r.get("Stream_Id", "")
    print(f"{name:20s} q{q:>3s} s{st:>3s} {s / 1e3:9.2f} -> {e / 1e3:9.2f}  ({(e - s) / 1e3:7.2f} us)")
