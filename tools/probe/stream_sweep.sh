#!/bin/bash
# The driver's bench command (fixed config) with one launch per step over S streams (--queue 1 --streams S)
# and the queued default, alternated NR times, STEPS timed steps.  -> gpurun_out/ssweep_<STEPS>/
cd "$(dirname "$0")/../.."
O=gpurun_out/ssweep_${STEPS:-20}; mkdir -p $O; rm -f $O/*.json
for r in $(seq 1 ${NR:-3}); do
  for s in ${SS:-2 3 4}; do
    timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 5 --queue 1 --streams $s > $O/s${s}_$r.json 2>> $O/err.log || exit 1
  done
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 5 > $O/q5_$r.json 2>> $O/err.log || exit 1
done
