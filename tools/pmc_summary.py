"""Average per-dispatch counter values of each kernel in a tools/pmc_probe.sh output directory."""
import csv
import glob
import os
import sys


def main(d):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0]
            per.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    for k, cs in per.items():
        print(k)
        for c in sorted(cs):
            v = cs[c]
            print(f"  {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
