#!/bin/bash
# A measurement build of the whole library from a copy of the sources edited by a sed script:
#   tools/probe/build_src_variant.sh NAME 'SED-EXPR' [-DFLAG ...]   (SED-EXPR '' = unchanged sources)  -> tools/probe/variants/NAME.so (LCRC_LIB_PATH=...)
# The in-tree library and sources are left alone; the variant's version string carries NAME.
set -e
cd "$(dirname "$0")/../.."
N=$1; E=$2; shift 2
T=$(mktemp -d)
mkdir -p $T/a/b $T/a/include tools/probe/variants
cp -r leveldb-rust_amd/csrc $T/a/b/ && cp include/lcrc.h $T/a/include/
if [ -n "$E" ]; then  # (an empty expression: the sources as they are, only the -D flags differ)
  sed -i "$E" $T/a/b/csrc/lcrc_kernels.hip
  if cmp -s $T/a/b/csrc/lcrc_kernels.hip leveldb-rust_amd/csrc/lcrc_kernels.hip; then echo "sed changed nothing" >&2; exit 1; fi
fi
C=$T/a/b/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -amdgpu-atomic-optimizer-strategy=None \
  -Wno-unused-result -DLCRC_SRC_HASH="\"variant-$N\"" "$@" -o tools/probe/variants/$N.so \
  $C/lcrc_kernels.hip $C/lcrc_api.cpp $C/lcrc_scalar.cpp $C/lcrc_leveldb.cpp $C/lcrc_table.cpp $C/lcrc_tbuild.cpp
rm -rf $T
echo tools/probe/variants/$N.so
