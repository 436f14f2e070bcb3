#!/bin/bash
# One GPU session's evidence for a round: parity suite, smoke, the driver's bench command and its rocprofv3
# summaries (kernel trace + FETCH/WRITE passes of the SAME command) for the headline and the other configs.
# Usage (GPU box): tools/gpu_round.sh ROUND   -> gpurun_out/round_<ROUND>/... and gpurun_out/prof_<ROUND>_*;
# then, in the container: for c in fixed mixed wal table; do python3 tools/summarize_profile.py \
#   gpurun_out/prof_<ROUND>_${c}_c <ROUND> $c c; cp gpurun_out/round_<ROUND>/bench_$c.json profiles/<ROUND>_bench_${c}_c.json; done
# (gpurun brings back gpurun_out/ only)
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=${1:-r02}
OUT=gpurun_out/round_$R
mkdir -p "$OUT" profiles
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 120 python -u __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
# the driver's headline command, then the other BASELINE configs
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --extra-out "$OUT/bench_fixed_full.json" > "$OUT/bench_fixed.json" 2> "$OUT/bench_fixed.err" || { tail -20 "$OUT/bench_fixed.err"; exit 1; }
cat "$OUT/bench_fixed.json"
for c in mixed wal table; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --config $c --extra-out "$OUT/bench_${c}_full.json" > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail -20 "$OUT/bench_$c.err"; exit 1; }
  cut -c1-400 "$OUT/bench_$c.json"
done
for c in fixed mixed wal table; do
  timeout -k 10 900 bash tools/profile_round.sh $R $c c > "$OUT/prof_$c.log" 2>&1 || { tail -20 "$OUT/prof_$c.log"; exit 1; }
  python3 -c "import json;s=json.load(open('profiles/${R}_${c}_c_summary.json'));print('$c', s.get('kernel'), s.get('avg_us'), s.get('frac'), s.get('bench_line'))"
done
