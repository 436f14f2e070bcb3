#!/bin/bash
# Development GPU session: the -m gpu suite, smoke, then the probes and bench configs named in $STEPS, each under its
# own time limit; stops at the first failure (nothing more runs on the GPU after a failed step).
# Usage (GPU box): STEPS="glds fixed table tablez" tools/dev_session.sh
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/dev
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
  timeout -k 10 120 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
for s in ${STEPS:-fixed}; do
  case $s in
    glds) timeout -k 10 60 ./tools/probe/probe_glds > $O/glds.log 2>&1 || { cat $O/glds.log; exit 1; }; cat $O/glds.log ;;
    host) timeout -k 10 300 python -u bench.py --host-resident > $O/bench_host.json 2> $O/bench_host.err || { tail -20 $O/bench_host.err; exit 1; }; cut -c1-900 $O/bench_host.json ;;
    sens) timeout -k 10 600 bash tools/probe/ab_many.sh 2 mixed prod=x norange=$PWD/tools/probe/variants/norange.so \
            norangevalu=$PWD/tools/probe/variants/norangevalu.so norangelds=$PWD/tools/probe/variants/norangelds.so \
            > $O/sens.log 2>&1 || { tail -20 $O/sens.log; exit 1; }
          python3 tools/probe/ab_many_summary.py | tee $O/sens_summary.txt ;;
    *) c=${s%@*}; var=""; [ "$c" != "$s" ] && var=${s#*@}
       BC="--config $c"; [ "$c" = tablez ] && BC="--config table --compression 1"
       [ "$c" = tablezsync ] && BC="--config table --compression 1 --table-sync"
       tag=$c${var:+_$var}
       ( [ -n "$var" ] && export LCRC_LIB_PATH=$PWD/tools/probe/variants/$var.so
         timeout -k 10 300 python -u bench.py $BC ${BENCH_ARGS} --extra-out $O/bench_${tag}_full.json > $O/bench_$tag.json 2> $O/bench_$tag.err ) || { tail -20 $O/bench_$tag.err; exit 1; }
       cut -c1-1200 $O/bench_$tag.json ;;
  esac
done
