#!/bin/bash
# A/B of the async table scan's verify pass (k_blocks grid divisor) beside the mixed config's k_blocks, with
# kernel traces: tools/probe/table_ab.sh  (GPU box; results under gpurun_out/table_ab)
set -e
cd "$(dirname "$0")/../.."
R=$PWD
O=$R/gpurun_out/table_ab
mkdir -p $O
for d in 1 2; do
  LCRC_TS_BLOCKS_DIV=$d timeout -k 10 200 python -u bench.py --config table --streams 1 > $O/t_div$d.json 2>> $O/err.log
  LCRC_TS_BLOCKS_DIV=$d timeout -k 10 200 python -u bench.py --config table --streams 2 > $O/t2_div$d.json 2>> $O/err.log
done
cd /tmp && export TMPDIR=/tmp
for d in 1 2; do
  LCRC_TS_BLOCKS_DIV=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t$d -o run -- python3 $R/bench.py --config table --steps 20 --streams 1 > $O/tp$d.json 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_m -o run -- python3 $R/bench.py --config mixed --steps 20 --streams 1 > $O/mp.json 2>&1
