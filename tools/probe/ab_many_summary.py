"""Summarize gpurun_out/ab_many: mean value per (config, build)."""
import collections
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_many"
r = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    c, k, _ = os.path.basename(f)[:-5].rsplit("_", 2)
    try:
        r[(c, k)].append(json.loads(open(f).read().strip().splitlines()[-1])["value"])
    except Exception:
        pass
for (c, k), v in sorted(r.items()):
    print(f"{c:8s} {k:8s} mean {sum(v) / len(v):8.1f}  {v}")
