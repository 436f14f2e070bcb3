"""Kernel timeline of the last steps of a rocprofv3 --kernel-trace CSV (the window and range passes of consecutive
steps on two streams): start/end relative to the first listed kernel, and per pair the overlap.
Usage: timeline_mixed.py TRACE_DIR [N]"""
import csv
import glob
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    name = r["Kernel_Name"].split("(")[0].replace("void lcrc_dev::", "")
    print(f"{name:28s} q{r.get('Queue_Id', '?'):>3s} start {s / 1e3:8.2f} end {e / 1e3:8.2f} dur {(e - s) / 1e3:7.2f}")
