#!/bin/bash
# bench.py over several variant builds, rotated each round (variant "prod" = the product library).
# Usage (GPU box): tools/probe/ab_multi.sh "prod tools/probe/variants/q_x.so ..." ROUNDS [BENCH ARGS]
# -> gpurun_out/ab_multi/<name>_<round>.json; summary: tools/probe/ab_summary.py gpurun_out/ab_multi
cd "$(dirname "$0")/../.."
VS=($1); shift
N=$1; shift
O=gpurun_out/ab_multi; mkdir -p $O; rm -f $O/*.json
nv=${#VS[@]}
for r in $(seq 1 $N); do
  for i in $(seq 0 $((nv - 1))); do
    v=${VS[$(((i + r) % nv))]}
    name=$(basename $v .so)
    if [ $v = prod ]; then unset LCRC_LIB_PATH; else export LCRC_LIB_PATH=$v; fi
    timeout -k 10 120 python -u bench.py --no-cpu-baseline "$@" > $O/${name}_$r.json 2>> $O/err.log || exit 1
  done
done
