"""Kernel averages from rocprofv3 kernel_stats.csv files: python3 kstats.py DIR..."""
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)):
        print("==", os.path.relpath(f))
        for r in csv.DictReader(open(f)):
            name = r["Name"].split("(")[0].replace("void ", "").replace("lcrc_dev::", "")
            print(f"  {name:28s} calls {int(r['Calls']):4d} avg {float(r['AverageNs'])/1e3:8.2f} us"
                  f"  min {float(r['MinNs'])/1e3:7.2f}  max {float(r['MaxNs'])/1e3:7.2f}")
