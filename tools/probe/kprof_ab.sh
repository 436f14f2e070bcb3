#!/bin/bash
# Per-kernel averages (rocprofv3 --kernel-trace --stats) of bench configs for the product library and one
# variant build, then a bench A/B of the same configs.
# Usage (GPU box): tools/probe/kprof_ab.sh VARIANT.so ROUNDS CONFIG...
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
V=$1; shift
N=$1; shift
O=gpurun_out/kprof; rm -rf $O; mkdir -p $O
for c in "$@"; do
  for k in prod var; do
    if [ $k = var ]; then export LCRC_LIB_PATH=$V; else unset LCRC_LIB_PATH; fi
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${k}_$c -o run -- \
      python3 bench.py --no-cpu-baseline --config $c --steps 20 --warmup 5 > $O/${k}_$c.log 2>&1 || exit 1
    f=$(find $O/${k}_$c -name '*kernel_stats.csv' | head -1)
    echo "== $k $c"; cut -d, -f1-4 "$f" | cut -c1-140
  done
done
unset LCRC_LIB_PATH
bash tools/probe/ab_configs.sh "$V" "$N" "$@" && python3 tools/probe/ab_summary.py gpurun_out/ab_cfg
