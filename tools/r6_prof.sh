#!/bin/bash
# GPU box: rocprofv3 kernel trace (+ stats) of one bench config: tools/r6_prof.sh TAG "BENCH ARGS"
# -> gpurun_out/r6p_<TAG>/ (stats csv, bench line)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=$1
shift
OUT=gpurun_out/r6p_$T
rm -rf "$OUT"
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline "$@" --extra-out "$OUT/bench.json" > "$OUT/log" 2>&1 || { tail -5 "$OUT/log"; exit 1; }
f=$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)
cp "$f" "$OUT/stats.csv"
python3 - "$OUT" <<'PY'
import csv, json, sys
o = sys.argv[1]
b = json.load(open(o + "/bench.json"))
print(o, b["value"], "ms/step", b["ms_per_step"])
for r in csv.DictReader(open(o + "/stats.csv")):
    print("  %-40s calls %4s avg %8.2f us min %8.2f max %8.2f" % (r["Name"].split("(")[0][-40:], r["Calls"],
          float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
PY
