#!/bin/bash
# Build a tree-encoder A/B variant: spec_amd/libspec_amd_NAME.so with extra -D flags (objects under
# spec_amd/csrc/build/v_NAME), then precompile its pkg1 tree kernels into the shared jit_cache.
# Usage: bash tools/build_tree_variant.sh NAME "-DSPEC_AB_X=0 ..."
set -e
NAME=$1; FLAGS=$2
cd "$(dirname "$0")/.."
make -s -j8 -C spec_amd/csrc BUILD=build/v_$NAME OUT=../libspec_amd_$NAME.so \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $FLAGS"
python3 - "$NAME" <<'PY'
import ctypes as C, sys
import spec_amd
from spec_amd import _lib
L = C.CDLL(_lib.LIB_PATH.replace("libspec_amd.so", f"libspec_amd_{sys.argv[1]}.so"))
_lib._declare(L)
print(L.spec_tree_jit_compile(C.byref(spec_amd.pkg1_tree().c)))
PY
echo built spec_amd/libspec_amd_$NAME.so
