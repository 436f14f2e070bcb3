#!/bin/bash
# Raw table scan under context options (GPU box): one bench line per option set, value / step / single scan.
# (CONFIG=mixed|wal|...: another bench config)
# Usage: tools/table_opts.sh "general=1" "ts_blocks_div=2" ...   ("" = defaults)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/topts
mkdir -p $O
i=0
for opts in "$@"; do
  i=$((i + 1))
  EO=""
  for kv in $opts; do EO="$EO --engine-opt $kv"; done
  timeout -k 10 300 python -u bench.py --config ${CONFIG:-table} ${TABLEZ:+--compression 1} --no-cpu-baseline $EO > $O/b$i.json 2> $O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$i.json'));r=d['roofline'];print('[$opts]', d['value'], d['ms_per_step'], (r.get('single_launch') or {}).get('launch_us_median'))"
done
# (TABLEZ=1: the compressed table, --compression 1)
