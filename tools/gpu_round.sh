#!/bin/bash
# One GPU session's evidence for a round: parity suite, smoke, then per config the rocprofv3 profile (kernel trace +
# FETCH/WRITE passes, summarized into profiles/ on the box) FOLLOWED by the driver's bench command, so that the
# bench line embeds the summary of the profile taken just before it in the same session.
# Usage (GPU box): tools/gpu_round.sh ROUND [CONFIGS...]   -> gpurun_out/round_<ROUND>/ (bench lines, logs, and a
# copy of the box's profiles/<ROUND>_* + traffic_*.json to bring back: gpurun returns gpurun_out/ only). Then, in the
# container: cp gpurun_out/round_<ROUND>/profiles/* profiles/
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=${1:-r03}
shift || true
CONFIGS=${@:-fixed mixed wal table tablez}
OUT=gpurun_out/round_$R
mkdir -p "$OUT/profiles" profiles
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
  timeout -k 10 120 python -u __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
for c in $CONFIGS; do
  timeout -k 10 900 bash tools/profile_round.sh $R $c c > "$OUT/prof_$c.log" 2>&1 || { tail -20 "$OUT/prof_$c.log"; exit 1; }
  python3 -c "import json;s=json.load(open('profiles/${R}_${c}_c_summary.json'));print('$c profile:', s.get('kernel'), s.get('avg_us'), s.get('trace_launch_us'), 'agreement (profiled run)', s.get('agreement_profiled_run'))"
  case "$c" in
    tablez) BC="--config table --compression 1" ;;
    *) BC="--config $c" ;;
  esac
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 $BC --extra-out "$OUT/bench_${c}_full.json" > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail -20 "$OUT/bench_$c.err"; exit 1; }
  cut -c1-300 "$OUT/bench_$c.json"
  # the committed line is the profiled run's own line (the trace reproduces it); the un-profiled run of the same
  # command is kept beside it (the profiler's per-dispatch cost slows multi-kernel steps on two streams)
  cp gpurun_out/prof_${R}_${c}_c/bench.json profiles/${R}_bench_${c}_c.json
  cp "$OUT/bench_${c}_full.json" profiles/${R}_bench_${c}_c_unprofiled.json
  python3 tools/summarize_profile.py gpurun_out/prof_${R}_${c}_c $R $c c profiles/${R}_bench_${c}_c.json profiles/${R}_bench_${c}_c_unprofiled.json > /dev/null
  python3 -c "import json;s=json.load(open('profiles/${R}_${c}_c_summary.json'));print('$c agreement vs committed line:', s.get('agreement'), 'wall', s.get('agreement_wall'), 'vs un-profiled run:', s.get('agreement_unprofiled'))"
  cp profiles/${R}_${c}_c_* profiles/${R}_bench_${c}_c*.json profiles/traffic_${c}_c.json "$OUT/profiles/"
done
