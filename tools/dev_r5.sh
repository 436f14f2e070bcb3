#!/bin/bash
# Round-5 development check on the GPU box: the -m gpu suite (up to 10 failures reported), then one bench line per
# config of interest (two-pass and one-pass WAL, compressed table with both index decoders, raw table, fixed).
# Usage (GPU box): tools/dev_r5.sh [PYTEST_ARGS]   -> gpurun_out/dev5/
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/dev5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread "$@" > $O/pytest.log 2>&1
rc=$?
tail -15 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # (1: test failures; anything else: a crash or timeout -- stop)
for c in wal walop tablez tablezv1 table fixed; do
  case "$c" in
    tablez) BC="--config table --compression 1" ;;
    tablezv1) BC="--config table --compression 1 --engine-opt ts_open_v1=1" ;;
    walop) BC="--config wal --engine-opt wal_onepass=1" ;;
    *) BC="--config $c" ;;
  esac
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline $BC > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));r=d.get('roofline') or {};print('$c', d['value'], d['ms_per_step'], r.get('frac'), r.get('frac_single_launch'))"
done
