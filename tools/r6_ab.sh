#!/bin/bash
# GPU box: alternated bench lines over library builds and bench arguments.
# Usage: tools/r6_ab.sh ROUNDS "NAME=LIB|BENCH ARGS" ...   (LIB: prod = the in-tree library, else a .so path)
# -> gpurun_out/r6ab/<name>_<round>.json and a summary line per run
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
N=$1; shift
O=gpurun_out/r6ab; mkdir -p $O
for r in $(seq 1 $N); do
  for spec in "$@"; do
    name=${spec%%=*}; rest=${spec#*=}; libp=${rest%%|*}; args=${rest#*|}
    if [ "$libp" = prod ]; then unset LCRC_LIB_PATH; else export LCRC_LIB_PATH=$libp; fi
    timeout -k 10 180 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 $args > $O/${name}_$r.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/${name}_$r.json'))
print('%-14s r%d %9.1f GiB/s  %.4f ms/step' % ('$name', $r, d['value'], d['ms_per_step']))"
  done
done
