#!/bin/bash
# GPU-box check used during development: parity tests, smoke, the default bench line and the other configs.
# Usage: tools/gpu_check.sh [quick]   (quick: no pytest)
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$1" != "quick" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
  tail -3 gpurun_out/t.log
fi
timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_fixed.json 2> gpurun_out/bench_fixed.err || { tail -20 gpurun_out/bench_fixed.err; exit 1; }
cat gpurun_out/bench_fixed.json
for c in ${CONFIGS:-mixed wal table tablez}; do
  case "$c" in
    tablez) BC="--config table --compression 1" ;;
    *) BC="--config $c" ;;
  esac
  timeout -k 10 300 python -u bench.py $BC > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  cut -c1-1500 gpurun_out/bench_$c.json
done
