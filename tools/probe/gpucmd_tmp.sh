set -e
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -3 gpurun_out/t.log
