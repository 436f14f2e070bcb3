set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "queue or config2 or config1 or unaligned" 2>&1 | tail -3
timeout -k 10 120 python -u __graft_entry__.py smoke | tail -1
for i in 1 2 3; do timeout -k 10 300 python tools/probe/time_queue.py q_shift q_tree; done
