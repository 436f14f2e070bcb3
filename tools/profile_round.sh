#!/bin/bash
# Profiles bench.py with rocprofv3 and writes the judged summaries into profiles/:
#   1. --kernel-trace --stats        -> per-kernel average duration (must agree with bench.py's roofline)
#   2. --pmc FETCH_SIZE (own pass)   -> HBM read bytes per launch (gfx950: FETCH_SIZE counts half the bytes of
#   3. --pmc WRITE_SIZE (own pass)      wide coalesced streaming reads -> x2; MI355X_MICROARCH.md HBM section)
# Usage (on the GPU box): tools/profile_round.sh ROUND CONFIG MODE [EXTRA BENCH ARGS]   e.g. tools/profile_round.sh r02 fixed c
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
ROUND=${1:-r01}
CONFIG=${2:-fixed}
MODE=${3:-c}
EXTRA=${4:-}
OUT=gpurun_out/prof_${ROUND}_${CONFIG}_${MODE}
rm -rf "$OUT"
mkdir -p "$OUT" profiles
# the driver's command (bench.py --gpus 1 --steps 20 --warmup 5) for this config, without the CPU leg
# tablez: the Snappy-compressed table (bench.py --config table --compression 1)

case "$CONFIG" in
  tablez) BCONF="--config table --compression 1" ;;
  *) BCONF="--config $CONFIG" ;;
esac
BENCH="bench.py --gpus 1 $BCONF --mode $MODE --steps 20 --warmup 5 --no-cpu-baseline $EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH --extra-out "$OUT/bench.json" > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $BENCH > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $BENCH > "$OUT/write.log" 2>&1
python3 tools/summarize_profile.py "$OUT" "$ROUND" "$CONFIG" "$MODE"
