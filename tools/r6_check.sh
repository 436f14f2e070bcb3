#!/bin/bash
# GPU box: the parity suite (or a selection: PYTEST_K=...), smoke, then one bench line per config given.
# Usage: tools/r6_check.sh TAG [CONFIGS...]   -> gpurun_out/r6_<TAG>/
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=${1:-x}
shift || true
OUT=gpurun_out/r6_$T
mkdir -p "$OUT"
if [ -z "$SKIP_TESTS" ]; then
  K=()
  [ -n "$PYTEST_K" ] && K=(-k "$PYTEST_K")
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread "${K[@]}" \
    > "$OUT/pytest.log" 2>&1
  rc=$?
  tail -25 "$OUT/pytest.log"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -u __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
for c in "$@"; do
  case "$c" in
    tablez) BC="--config table --compression 1" ;;
    *) BC="--config $c" ;;
  esac
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 $BC --extra-out "$OUT/bench_${c}_full.json" \
    > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail -20 "$OUT/bench_$c.err"; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/bench_$c.json'))
print('$c', d['value'], d['unit'][:5], 'ms/step', d['ms_per_step'], 'frac', d.get('roofline', {}).get('frac'),
      'single', d.get('roofline', {}).get('single_launch'))"
done
