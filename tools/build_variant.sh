#!/bin/bash
# Builds a variant of the library under tools/variants/<name>.so with extra
# compile-time flags (solver A/B experiments; never the product library).
# usage: tools/build_variant.sh <name> [-DFLAG=VALUE ...]
set -e
HERE=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p "$HERE/tools/variants"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function \
  -fgpu-flush-denormals-to-zero "$@" -Wl,--version-script="$HERE/bsdb_amd/csrc/exports.map" \
  -o "$HERE/tools/variants/$name.so.tmp.$$" "$HERE/bsdb_amd/csrc/bsdb_capi.hip"
mv -f "$HERE/tools/variants/$name.so.tmp.$$" "$HERE/tools/variants/$name.so"
