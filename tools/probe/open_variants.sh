#!/bin/bash
# k_ts_open per-variant kernel trace (the compressed-table bench under rocprofv3 --kernel-trace, one run per variant).
set -e
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
R=$PWD; O=gpurun_out/ov
mkdir -p $O
for v in "$@"; do
  ( [ "$v" != prod ] && export LCRC_LIB_PATH=$R/tools/probe/variants/$v.so
    timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/$v -o ov -- python3 bench.py --config table --compression 1 \
      --steps 10 --warmup 2 > $O/$v.json 2> $O/$v.err ) || { tail -20 $O/$v.err; exit 1; }
  echo "== $v $(python3 -c "import json; d=json.load(open('$O/$v.json')); print(d['value'], d['ms_per_step'])")"
  python3 tools/probe/kdb.py $O/$v | grep -E "k_ts_open|k_ts_decode"
done
