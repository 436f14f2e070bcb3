#!/bin/bash
# WAL scan A/B on the GPU box: parity tests of the WAL path, then the wal bench with the fused window pass + header
# walk (default) and with the separate header walk (LCRC_WAL_FUSED=0), alternated.  Usage: tools/probe/wal_ab.sh [ROUNDS]
set -e
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/wal_ab
timeout -k 10 600 python -u -m pytest tests -m gpu -k "wal or WAL or log" -x -q --timeout 120 --timeout-method thread > gpurun_out/wal_ab/t.log 2>&1 || { tail -40 gpurun_out/wal_ab/t.log; exit 1; }
tail -2 gpurun_out/wal_ab/t.log
for i in $(seq ${1:-2}); do
  for f in 1 0; do
    LCRC_WAL_FUSED=$f timeout -k 10 300 python -u bench.py --config wal --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/wal_ab/w${f}_$i.json 2> gpurun_out/wal_ab/w${f}_$i.err || { tail -20 gpurun_out/wal_ab/w${f}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/wal_ab/w${f}_$i.json')); print('fused=$f', d['value'], d['ms_per_step'], d['roofline']['launch_us'])"
  done
done
