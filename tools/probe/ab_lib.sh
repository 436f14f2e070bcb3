#!/bin/bash
# A/B of bench.py between the product library and a variant build, alternated (order swapped every round).
# Usage (GPU box): tools/probe/ab_lib.sh VARIANT.so ROUNDS [BENCH ARGS]
cd "$(dirname "$0")/../.."
V=$1; shift
N=$1; shift
O=gpurun_out/ab_lib; mkdir -p $O; rm -f $O/*.json
for r in $(seq 1 $N); do
  if [ $((r % 2)) -eq 1 ]; then order="prod var"; else order="var prod"; fi
  for k in $order; do
    if [ $k = var ]; then export LCRC_LIB_PATH=$V; else unset LCRC_LIB_PATH; fi
    timeout -k 10 120 python -u bench.py --no-cpu-baseline "$@" > $O/${k}_$r.json 2>> $O/err.log || exit 1
  done
done
