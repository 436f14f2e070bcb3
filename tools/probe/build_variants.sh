#!/bin/bash
# Ablation builds of liblcrc.so for bottleneck analysis (tools/probe/variants/*.so).
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/probe/variants
SRC="leveldb-rust_amd/csrc/lcrc_kernels.hip leveldb-rust_amd/csrc/lcrc_api.cpp leveldb-rust_amd/csrc/lcrc_scalar.cpp leveldb-rust_amd/csrc/lcrc_leveldb.cpp leveldb-rust_amd/csrc/lcrc_table.cpp"
build() { /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-atomic-optimizer-strategy=None -std=c++17 -fPIC -shared -Wno-unused-result "$@" $SRC; }
build -DLCRC_PROBE_CLOCK -o tools/probe/variants/base.so &
build -DLCRC_PROBE_CLOCK -DLCRC_PROBE_L2 -o tools/probe/variants/l2.so &
build -DLCRC_PROBE_CLOCK -DLCRC_PROBE_LDSDATA -o tools/probe/variants/ldsdata.so &
build -DLCRC_PROBE_CLOCK -DLCRC_PROBE_NOLOAD -o tools/probe/variants/noload.so &
build -DLCRC_PROBE_CLOCK -DLCRC_PROBE_NOWALK -o tools/probe/variants/nowalk.so &
wait
ls tools/probe/variants
