#!/bin/bash
# One bench config under several environment settings, alternated per round:
#   tools/probe/ab_env.sh ROUNDS CONFIG "NAME:VAR=V VAR2=V2" ...   (NAME:- for no extra variable)
# Prints one line per run (name, value, ms_per_step); results in gpurun_out/ab_env/
cd "$(dirname "$0")/../.."
N=$1; shift
C=$1; shift
O=gpurun_out/ab_env; mkdir -p $O
for r in $(seq 1 $N); do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    [ "$envs" = "-" ] && envs=""
    env $envs timeout -k 10 120 python -u bench.py --no-cpu-baseline --config $C --steps 20 --warmup 5 > $O/${C}_${name}_$r.json 2>> $O/err.log || exit 1
    python3 -c "import json,sys;d=json.load(open('$O/${C}_${name}_$r.json'));print('$C', '$name', $r, d['value'], d['ms_per_step'])"
  done
done
