set -e
cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_check.sh > gpurun_out/check.log 2>&1 || { tail -30 gpurun_out/check.log; exit 1; }
tail -6 gpurun_out/check.log | cut -c1-600
for q in 1 5 10 20; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --queue $q --no-cpu-baseline > gpurun_out/q$q.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/q$q.json'));print('q=$q',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['launch_us'],d['config']['streams'])"
done
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --queue 5 --streams 2 --no-cpu-baseline > gpurun_out/q5s2.json 2>/dev/null
python -c "import json;d=json.load(open('gpurun_out/q5s2.json'));print('q=5 s2',d['value'],d['ms_per_step'],d['roofline']['frac'])"
timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/k100.json 2>/dev/null
python -c "import json;d=json.load(open('gpurun_out/k100.json'));print('k100',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['launch_us'])"
timeout -k 10 300 python tools/probe/time_queue.py
