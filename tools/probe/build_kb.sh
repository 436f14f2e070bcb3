#!/bin/bash
# k_blocks ablation builds (LCRC_PROBE_KB: 1 table fill only, 2 no head/tail walks, 3 no window fold) and the
# product sources as they are (kb0), into tools/probe/variants/.
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/probe/variants
SRC="leveldb-rust_amd/csrc/lcrc_kernels.hip leveldb-rust_amd/csrc/lcrc_api.cpp leveldb-rust_amd/csrc/lcrc_scalar.cpp leveldb-rust_amd/csrc/lcrc_leveldb.cpp leveldb-rust_amd/csrc/lcrc_table.cpp leveldb-rust_amd/csrc/lcrc_tbuild.cpp"
build() { /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-atomic-optimizer-strategy=None -std=c++17 -fPIC -shared -Wno-unused-result "$@" $SRC; }
for v in ${@:-1 2 3}; do build -DLCRC_PROBE_KB=$v -o tools/probe/variants/kb$v.so & done
wait
