#!/bin/bash
# SQ counter passes over one bench.py workload (one rocprofv3 --pmc pass per group, each bounded).
# Usage (GPU box): tools/pmc_bench.sh CONFIG   -> gpurun_out/pmcb_<config>/g<i>/..., summary on stdout
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
CFG=${1:-mixed}
OUT=gpurun_out/pmcb_$CFG
rm -rf "$OUT"; mkdir -p "$OUT"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/g$i" -o run -- python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --streams 1 --queue 1 > "$OUT/g$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/g$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT"
