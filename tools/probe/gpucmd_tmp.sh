set -e
export TMPDIR=/tmp
for v in base; do echo "== $v"; LCRC_LIB_PATH=$PWD/tools/probe/variants/$v.so timeout -k 10 200 python tools/probe/stamps.py 65536 4096 | grep -v "xcd\|wave\|by "; done
