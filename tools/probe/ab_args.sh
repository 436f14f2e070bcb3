#!/bin/bash
# One bench config under several (environment, bench-argument) settings, alternated per round:
#   tools/probe/ab_args.sh ROUNDS CONFIG "NAME|VAR=V ...|--bench-args" ...   (- for none)
cd "$(dirname "$0")/../.."
N=$1; shift
C=$1; shift
O=gpurun_out/ab_args; mkdir -p $O
for r in $(seq 1 $N); do
  for v in "$@"; do
    IFS='|' read -r name envs bargs <<< "$v"
    [ "$envs" = "-" ] && envs=""
    [ "$bargs" = "-" ] && bargs=""
    env $envs timeout -k 10 120 python -u bench.py --no-cpu-baseline --config $C --steps 40 --warmup 5 $bargs > $O/${C}_${name}_$r.json 2>> $O/err.log || exit 1
    python3 -c "import json;d=json.load(open('$O/${C}_${name}_$r.json'));print('$C', '$name', $r, d['value'], d['ms_per_step'])"
  done
done
