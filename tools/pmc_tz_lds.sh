#!/bin/bash
# GPU box: LDS-side SQ counters of the compressed-table scan, one stream (one --pmc pass):
# tools/pmc_tz_lds.sh [LIB]  -> gpurun_out/pmc_lds/ (LIB: a variant build; default the in-tree one)
set -e
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
[ -n "$1" ] && export LCRC_LIB_PATH=$(realpath "$1")
OUT=gpurun_out/pmc_lds${2:+_$2}
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL --output-format csv -d "$OUT" -o run -- python3 bench.py --config table --compression 1 --steps 4 --warmup 1 --no-cpu-baseline --streams 1 > "$OUT/log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].split("::")[-1]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, c in acc.items():
    if "decode" not in k and "open2" not in k: continue
    v = {x: c[x] / n[(k, x)] for x in c}
    wc = v.get("SQ_WAVE_CYCLES", 1)
    print(k, {x: round(y) for x, y in v.items()})
    print("   wait_any %.3f wait_inst %.3f active %.3f  bank_conflict/lds_active %.3f" % (
        v.get("SQ_WAIT_ANY", 0) / wc, v.get("SQ_WAIT_INST_ANY", 0) / wc, v.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        v.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, v.get("SQ_LDS_IDX_ACTIVE", 1))))
PY
