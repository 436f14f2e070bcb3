"""Medians of tools/probe/ab_multi.sh results: value, per-launch kernel time and the wall time beyond the
launches (ms_per_step x steps - launch_us x launches) per variant."""
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
    r = j.get("roofline") or {}
    over = j["ms_per_step"] * j["steps"] * 1e3 - r["launch_us"] * r["launches"] if r.get("launch_us") else None
    rows.setdefault(name, []).append((j["value"], r.get("launch_us"), over))
for name, v in rows.items():
    vals = [a for a, _, _ in v]
    lus = [b for _, b, _ in v if b is not None]
    ov = [c for _, _, c in v if c is not None]
    print(f"{name:12s} n={len(v)} value median {statistics.median(vals):8.1f} [{min(vals):.0f}..{max(vals):.0f}]"
          + (f"  launch_us median {statistics.median(lus):.1f}" if lus else "")
          + (f"  wall beyond launches median {statistics.median(ov):.1f} us" if ov else ""))
