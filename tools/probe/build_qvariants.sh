#!/bin/bash
# Shape builds of liblcrc.so for the queued fast path (tools/probe/variants/q_*.so), timed by
# tools/probe/time_queue.py. Usage: tools/probe/build_qvariants.sh [NAME:FLAGS ...]
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/probe/variants
SRC="leveldb-rust_amd/csrc/lcrc_kernels.hip leveldb-rust_amd/csrc/lcrc_api.cpp leveldb-rust_amd/csrc/lcrc_scalar.cpp leveldb-rust_amd/csrc/lcrc_leveldb.cpp leveldb-rust_amd/csrc/lcrc_table.cpp leveldb-rust_amd/csrc/lcrc_tbuild.cpp"
build() { out=$1; shift; /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-atomic-optimizer-strategy=None -std=c++17 -fPIC -shared -Wno-unused-result "$@" $SRC -o tools/probe/variants/q_$out.so; }
if [ $# -eq 0 ]; then
  set -- "base:" "clock:-DLCRC_PROBE_CLOCK" "wg2:-DLCRC_A_WGCU=2" "t1024:-DLCRC_A_THREADS=1024" "aux0:-DLCRC_LOAD_AUX=0"
fi
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  build $name $flags &
done
wait
ls tools/probe/variants
