#!/bin/bash
# Kernel trace of the WAL bench on one stream (each kernel alone): tools/probe/wal_prof.sh [EXTRA ENV...]
set -e
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
rm -rf gpurun_out/walprof; mkdir -p gpurun_out/walprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/walprof -o run -- python3 bench.py --config wal --steps 20 --warmup 5 --no-cpu-baseline --streams 1 > gpurun_out/walprof/bench.log 2>&1
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/walprof/run_kernel_stats.csv")):
    print(r["Name"].split("(")[0][:40], r["Calls"], round(float(r["AverageNs"])/1e3, 2), round(float(r["MinNs"])/1e3, 2))
PY
