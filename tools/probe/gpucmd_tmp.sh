set -e
export TMPDIR=/tmp
for s in 1 2; do LCRC_BENCH_PRE=1 timeout -k 10 200 python bench.py --config fixed --steps 50 --warmup 5 --no-cpu-baseline --streams $s | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fixed streams', d['config']['streams'], d['value'], 'GiB/s', d['ms_per_step'], 'ms/step; roofline', d['roofline']['achieved'], d['roofline']['frac'], d['roofline']['launch_us'])"; done
LCRC_BENCH_PRE=1 timeout -k 10 200 python bench.py --config fixed --steps 200 --warmup 5 --no-cpu-baseline --streams 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fixed streams', d['config']['streams'], d['value'], 'GiB/s', d['ms_per_step'], 'ms/step; roofline', d['roofline']['achieved'], d['roofline']['frac'], d['roofline']['launch_us'])"
timeout -k 10 200 python tools/probe/size_sweep.py
