#!/bin/bash
# A/B of several bench configs between the product library and a variant build (alternated, order swapped).
# Usage (GPU box): tools/probe/ab_configs.sh VARIANT.so ROUNDS CONFIG...
cd "$(dirname "$0")/../.."
V=$1; shift
N=$1; shift
O=gpurun_out/ab_cfg; mkdir -p $O; rm -f $O/*.json
for c in "$@"; do
  for r in $(seq 1 $N); do
    if [ $((r % 2)) -eq 1 ]; then order="prod var"; else order="var prod"; fi
    for k in $order; do
      if [ $k = var ]; then export LCRC_LIB_PATH=$V; else unset LCRC_LIB_PATH; fi
      timeout -k 10 120 python -u bench.py --no-cpu-baseline --config $c --steps 20 --warmup 5 > $O/${c}_${k}_$r.json 2>> $O/err.log || exit 1
    done
  done
done
