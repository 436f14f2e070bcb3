#!/bin/bash
# A/B of bench.py's roofline timer on one box (the driver's command): events carried by the launches vs event
# markers after the first submission, alternated three times.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/timer_ab
rm -f gpurun_out/timer_ab/*.json
for r in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/timer_ab/kernel_$r.json 2>> gpurun_out/timer_ab/err.log || exit 1
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --marker-timer > gpurun_out/timer_ab/marker_$r.json 2>> gpurun_out/timer_ab/err.log || exit 1
done
