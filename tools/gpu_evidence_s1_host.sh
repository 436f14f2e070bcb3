#!/bin/bash
# The one-stream fast-path profile (<round>s1: kernel trace + FETCH/WRITE passes, the line committed beside an
# un-profiled run) and the host-resident end-to-end line (pinned H2D + kernel + D2H), after tools/gpu_round.sh.
# Usage (GPU box): tools/gpu_evidence_s1_host.sh ROUND   -> gpurun_out/round_<ROUND>/
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=${1:-r06}
OUT=gpurun_out/round_$R
mkdir -p $OUT/profiles profiles
cp profiles/traffic_fixed_c.json /tmp/traffic_fixed_c.json  # (the two-stream profile's; the s1 pass must not replace it)
timeout -k 10 600 bash tools/profile_round.sh ${R}s1 fixed c "--streams 1" > $OUT/prof_s1.log 2>&1 || { tail -20 $OUT/prof_s1.log; exit 1; }
cp profiles/traffic_fixed_c.json profiles/traffic_fixeds1_c.json
cp /tmp/traffic_fixed_c.json profiles/traffic_fixed_c.json
timeout -k 10 300 python -u bench.py --streams 1 --extra-out $OUT/bench_fixed_s1_full.json > $OUT/bench_fixed_s1.json 2> $OUT/bench_fixed_s1.err || { tail -20 $OUT/bench_fixed_s1.err; exit 1; }
cp gpurun_out/prof_${R}s1_fixed_c/bench.json profiles/${R}s1_bench_fixed_c.json
cp $OUT/bench_fixed_s1_full.json profiles/${R}s1_bench_fixed_c_unprofiled.json
python3 tools/summarize_profile.py gpurun_out/prof_${R}s1_fixed_c ${R}s1 fixed c profiles/${R}s1_bench_fixed_c.json profiles/${R}s1_bench_fixed_c_unprofiled.json > /dev/null
cp /tmp/traffic_fixed_c.json profiles/traffic_fixed_c.json
cp profiles/${R}s1_* profiles/traffic_fixeds1_c.json $OUT/profiles/
python3 -c "import json;s=json.load(open('profiles/${R}s1_fixed_c_summary.json'));print('s1 fixed:', s.get('avg_us'), s.get('frac'), 'agreement', s.get('agreement'), s.get('agreement_unprofiled'))"
timeout -k 10 300 python -u bench.py --host-resident --extra-out $OUT/bench_host_full.json > $OUT/bench_host.json 2> $OUT/bench_host.err || { tail -20 $OUT/bench_host.err; exit 1; }
cp $OUT/bench_host_full.json profiles/${R}_bench_host_c.json
cp profiles/${R}_bench_host_c.json $OUT/profiles/
cut -c1-400 $OUT/bench_host.json
