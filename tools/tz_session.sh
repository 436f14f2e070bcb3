#!/bin/bash
# Compressed-table scan measurements (GPU box): the kernel trace of the default build's device-only scan, then the
# bench line of each decode-staging variant given as arguments (tools/probe/variants/NAME.so).
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/tz
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$PYTEST_K" > gpurun_out/tz_pytest.log 2>&1 || { tail -60 gpurun_out/tz_pytest.log; exit 1; }
  tail -2 gpurun_out/tz_pytest.log
fi
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o tz -- python3 bench.py --config table --compression 1 \
  --steps 10 --warmup 2 > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
python3 tools/probe/kdb.py $O/prof
for v in prod "$@"; do
  ( [ "$v" != prod ] && export LCRC_LIB_PATH=$R/tools/probe/variants/$v.so
    timeout -k 10 300 python3 -u bench.py --config table --compression 1 > $O/bench_$v.json 2> $O/bench_$v.err ) || { tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
