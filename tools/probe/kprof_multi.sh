#!/bin/bash
# Per-kernel averages (rocprofv3 --kernel-trace --stats) of one bench config for several builds.
# Usage (GPU box): tools/probe/kprof_multi.sh "prod tools/probe/variants/x.so ..." CONFIG [BENCH ARGS]
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
VS=($1); shift
C=$1; shift
O=gpurun_out/kprof_multi; rm -rf $O; mkdir -p $O
for v in "${VS[@]}"; do
  name=$(basename $v .so)
  if [ $v = prod ]; then unset LCRC_LIB_PATH; else export LCRC_LIB_PATH=$v; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- \
    python3 bench.py --no-cpu-baseline --config $C --steps 20 --warmup 5 "$@" > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }
  python3 tools/probe/kstats.py $O/$name
done
