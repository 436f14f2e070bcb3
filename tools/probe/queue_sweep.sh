#!/bin/bash
# The driver's bench command at several queue depths (steps per submission), alternated.
cd "$(dirname "$0")/../.."
O=gpurun_out/qsweep; mkdir -p $O; rm -f $O/*.json
for r in $(seq 1 ${NR:-3}); do
  for q in ${QS:-5 10 0}; do
    timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --queue $q > $O/q${q}_$r.json 2>> $O/err.log || exit 1
  done
done
