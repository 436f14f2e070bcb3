#!/bin/bash
# One variant build of the whole library: tools/probe/build_one.sh NAME [-DFLAG ...] -> tools/probe/variants/NAME.so
set -e
cd "$(dirname "$0")/../.."
N=$1; shift
mkdir -p tools/probe/variants
C=leveldb-rust_amd/csrc
H=$(python3 -c "import sys; sys.path.insert(0, 'leveldb-rust_amd'); import build; print(build.source_hash())")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -amdgpu-atomic-optimizer-strategy=None \
  -Wno-unused-result -DLCRC_SRC_HASH="\"$H-$N\"" "$@" -o tools/probe/variants/$N.so \
  $C/lcrc_kernels.hip $C/lcrc_api.cpp $C/lcrc_scalar.cpp $C/lcrc_leveldb.cpp $C/lcrc_table.cpp $C/lcrc_tbuild.cpp
