#!/bin/bash
# Bench configs over several library builds, alternated: tools/probe/ab_many.sh ROUNDS "CONFIGS" NAME=PATH...
# (NAME=prod for the product library). Results: gpurun_out/ab_many/<config>_<name>_<round>.json
cd "$(dirname "$0")/../.."
N=$1; shift
CONFIGS=$1; shift
O=gpurun_out/ab_many; mkdir -p $O; rm -f $O/*.json
for r in $(seq 1 $N); do
  for v in "$@"; do
    name=${v%%=*}; path=${v#*=}
    if [ "$name" = prod ]; then unset LCRC_LIB_PATH; else export LCRC_LIB_PATH=$path; fi
    for c in $CONFIGS; do
      timeout -k 10 120 python -u bench.py --no-cpu-baseline --config $c --steps 20 --warmup 5 $BENCH_ARGS > $O/${c}_${name}_$r.json 2>> $O/err.log || exit 1
    done
  done
done
