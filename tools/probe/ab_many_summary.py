"""Summarize gpurun_out/ab_many: mean value per (config, build)."""
import collections
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_many"
r = collections.defaultdict(list)
single = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    c, k, _ = os.path.basename(f)[:-5].rsplit("_", 2)
    try:
        line = json.loads(open(f).read().strip().splitlines()[-1])
        r[(c, k)].append(line["value"])
        sl = (line.get("roofline") or {}).get("single_launch")
        if sl:
            single[(c, k)].append(sl["launch_us_median"])
    except Exception:
        pass
for (c, k), v in sorted(r.items()):
    s = single.get((c, k))
    extra = f"  single-launch median us {sum(s) / len(s):6.2f} {s}" if s else ""
    print(f"{c:8s} {k:8s} mean {sum(v) / len(v):8.1f}  {v}{extra}")
