set -e
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for v in base noprio; do echo "== $v"; LCRC_LIB_PATH=$PWD/tools/probe/variants/$v.so timeout -k 10 200 python tools/probe/stamps.py 65536 | grep -v "xcd\|wave \|by "; done
timeout -k 10 200 python tools/probe/time_variants.py base noprio wg1 base noprio wg1
for v in base noprio; do for s in 1 2; do LCRC_LIB_PATH=$PWD/tools/probe/variants/$v.so timeout -k 10 200 python bench.py --config fixed --steps 50 --warmup 5 --no-cpu-baseline --streams $s | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v streams', d['config']['streams'], d['value'], 'GiB/s', d['ms_per_step'], 'ms/step; roofline', d['roofline']['achieved'], d['roofline']['frac'], d['roofline']['launch_us'])"; done; done
