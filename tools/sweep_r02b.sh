set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_table_builder.py -k "sparse or writer or config3 or hundreds or many_blocks_reference" 2>&1 | tail -8
