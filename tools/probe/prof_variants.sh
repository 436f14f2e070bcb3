#!/bin/bash
# PMC passes over ablation variants: rocprofv3 --pmc (no tracing domains), one counter group per pass.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_INSTS_VALU SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
for v in ${VARIANTS:-noload l2 base}; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    LCRC_LIB_PATH=$PWD/tools/probe/variants/$v.so timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d $OUT/$v.p$i -o run -- python3 tools/probe/one_variant.py 10 > $OUT/$v.p$i.log 2>&1 || { echo "fail $v $i"; tail -5 $OUT/$v.p$i.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, os, collections
for f in sorted(glob.glob("gpurun_out/pmc/*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        if "k_windows" not in row.get("Kernel_Name", ""):
            continue
        agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
    print(f.split("/")[2], {k: round(sum(v) / len(v)) for k, v in agg.items()})
PY
