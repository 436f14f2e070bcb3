#!/bin/bash
# bench configs at several stream counts: tools/probe/streams_ab.sh "CONFIGS" "STREAMS" [ROUNDS]
cd "$(dirname "$0")/../.."
O=gpurun_out/streams_ab; mkdir -p $O
for r in $(seq ${3:-1}); do for c in $1; do for s in $2; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --config $c --streams $s --steps 20 --warmup 5 > $O/${c}_s${s}_$r.json 2>> $O/err.log || exit 1
  python3 -c "import json; d=json.load(open('$O/${c}_s${s}_$r.json')); print('$c', 'streams=$s', d['value'], d['roofline']['launch_us'])"
done; done; done
