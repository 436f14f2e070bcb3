#!/bin/bash
# One config over several library builds and stream counts, alternated:
#   tools/probe/ab_streams.sh ROUNDS CONFIG "STREAMS" NAME=PATH...   (NAME=prod: the product library)
# -> gpurun_out/ab_streams/<config>_<name>_s<streams>_<round>.json, then a summary line per build and stream count
cd "$(dirname "$0")/../.."
N=$1; C=$2; SS=$3; shift 3
O=gpurun_out/ab_streams; mkdir -p $O; rm -f $O/*.json
for r in $(seq 1 $N); do
  for v in "$@"; do
    name=${v%%=*}; path=${v#*=}
    if [ "$name" = prod ]; then unset LCRC_LIB_PATH; else export LCRC_LIB_PATH=$path; fi
    for s in $SS; do
      timeout -k 10 120 python -u bench.py --no-cpu-baseline --config $C --streams $s --steps 20 --warmup 5 > $O/${C}_${name}_s${s}_$r.json 2>> $O/err.log || exit 1
    done
  done
done
python3 - "$O" <<'PY'
import glob, json, os, sys, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    key = os.path.basename(f).rsplit("_", 1)[0]
    acc[key].append((d["value"], d["ms_per_step"] * 1e3))
for k, v in acc.items():
    print(f"{k:28s} GiB/s {sum(a for a, _ in v) / len(v):8.1f}  us/step {sum(b for _, b in v) / len(v):6.1f}  {[round(a) for a, _ in v]}")
PY
