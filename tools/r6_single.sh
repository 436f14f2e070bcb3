#!/bin/bash
# GPU box: single-launch and two-stream figures of the fixed config for several library builds, alternated.
# Usage: tools/r6_single.sh ROUNDS NAME=LIB ...  (LIB: prod or a .so path)
cd "$(dirname "$0")/.."
N=$1; shift
O=gpurun_out/r6single; mkdir -p $O
for r in $(seq 1 $N); do
  for spec in "$@"; do
    name=${spec%%=*}; libp=${spec#*=}
    if [ "$libp" = prod ]; then unset LCRC_LIB_PATH; else export LCRC_LIB_PATH=$libp; fi
    timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/${name}_$r.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/${name}_$r.json')); s = d['roofline']['single_launch']
print('%-8s r%d value %7.1f  single median %6.2f min %6.2f (frac %.4f)' % ('$name', $r, d['value'], s['launch_us_median'], s['launch_us_min'], d['roofline']['frac_single_launch']))"
  done
done
