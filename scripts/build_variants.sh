#!/bin/bash
# Diagnostic: build libhhfm.so variants that differ in ONE source file's -D
# flags, into ab/<name>/ (for scripts/ab_libs.sh).  Not part of the product.
#   scripts/build_variants.sh dfm_fused name1:-DX=1 name2:-DX=2 ...
set -e
cd "$(dirname "$0")/.."
src=$1; shift
make -s native
others=$(ls build/*.o | grep -v "build/$src.o")
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  mkdir -p ${AB_DIR:-ab}/$name
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
    -DHHFM_DIAG_BUILD $defs -c hhfm_amd/csrc/$src.hip -o build/var_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ${AB_DIR:-ab}/$name/libhhfm.so $others build/var_$name.o
  cp hhfm_amd/lib/_hhfm*.so ${AB_DIR:-ab}/$name/
  rm build/var_$name.o
done
