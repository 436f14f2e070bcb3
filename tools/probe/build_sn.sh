#!/bin/bash
# Snappy decode probe builds (tools/probe/variants/sn*.so): 0 full, 1 frame overhead only, 2 parse only.
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/probe/variants
SRC="leveldb-rust_amd/csrc/lcrc_kernels.hip leveldb-rust_amd/csrc/lcrc_api.cpp leveldb-rust_amd/csrc/lcrc_scalar.cpp leveldb-rust_amd/csrc/lcrc_leveldb.cpp leveldb-rust_amd/csrc/lcrc_table.cpp"
build() { /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result "$@" $SRC; }
build -o tools/probe/variants/sn0.so &
build -DLCRC_SN_PROBE=1 -o tools/probe/variants/sn1.so &
build -DLCRC_SN_PROBE=2 -o tools/probe/variants/sn2.so &
wait
