#!/bin/bash
# The driver's bench command N times: value, ms/step, kernel time per launch and the wall time beyond the launches.
# Usage (GPU box): tools/probe/bench_rep.sh N [BENCH ARGS]
cd "$(dirname "$0")/../.."
N=$1; shift
O=gpurun_out/bench_rep; mkdir -p $O; rm -f $O/*.json
for r in $(seq 1 $N); do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 "$@" > $O/b_$r.json 2>> $O/err.log || exit 1
  python3 -c "
import json; j = json.loads(open('$O/b_$r.json').read().strip().splitlines()[-1]); r = j['roofline']
print(j['value'], j['ms_per_step'], r['launch_us'], r['launches'], round(j['ms_per_step'] * j['steps'] * 1000 - r['launch_us'] * r['launches'], 1))"
done
