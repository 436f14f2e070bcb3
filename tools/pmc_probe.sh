#!/bin/bash
# SQ counter passes over the 4 KiB fast path (one rocprofv3 --pmc pass per counter group, each bounded).
# Usage (GPU box): tools/pmc_probe.sh [LIB.so ...]   -> gpurun_out/pmc_<lib>/g<i>/...
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
LIBS="$*"
[ -z "$LIBS" ] && LIBS=leveldb-rust_amd/_build/liblcrc.so
for lib in $LIBS; do
  name=$(basename "$lib" .so)
  OUT=gpurun_out/pmc_$name
  rm -rf "$OUT"; mkdir -p "$OUT"
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    LCRC_LIB_PATH=$(realpath "$lib") timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/g$i" -o run -- python3 tools/probe/one_variant.py 20 1 > "$OUT/g$i.log" 2>&1 || { echo "pass $i failed for $name"; tail -5 "$OUT/g$i.log"; exit 1; }
  done
  python3 tools/pmc_summary.py "$OUT"
done
