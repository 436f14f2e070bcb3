#!/bin/bash
# Per-kernel durations for bench configs (GPU box): one rocprofv3 kernel trace per config, summarized by kdb.py.
# Usage: tools/ktrace.sh CONFIG...   (aliases as in dev_r5.sh)   -> gpurun_out/kt/<config>.txt
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/kt
mkdir -p $O
for c in "$@"; do
  case "$c" in
    tablez) BC="--config table --compression 1" ;;
    *) BC="--config $c" ;;
  esac
  rm -rf $O/prof_$c
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/prof_$c -o k -- python3 bench.py $BC --steps 10 --warmup 2 \
    --no-cpu-baseline ${EXTRA} > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  python3 tools/probe/kdb.py $O/prof_$c > $O/$c.txt
  echo "### $c"; cat $O/$c.txt
  rm -rf $O/prof_$c
done
