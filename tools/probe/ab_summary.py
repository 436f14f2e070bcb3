"""Medians of tools/probe/ab_multi.sh results: value and per-launch kernel time per variant."""
import glob
import json
import os
import statistics
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_multi"
rows = {}
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    name = os.path.basename(f).rsplit("_", 1)[0]
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        continue
    rows.setdefault(name, []).append((j["value"], (j.get("roofline") or {}).get("launch_us")))
for name, v in rows.items():
    vals = [a for a, _ in v]
    lus = [b for _, b in v if b is not None]
    print(f"{name:12s} n={len(v)} value median {statistics.median(vals):8.1f} [{min(vals):.0f}..{max(vals):.0f}]"
          + (f"  launch_us median {statistics.median(lus):.1f}" if lus else ""))
