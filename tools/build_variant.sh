#!/bin/bash
# A variant of lib/libsrsran_amd.so with one source compiled under extra flags (A/B runs through SRSRAN_AMD_LIB):
#   tools/build_variant.sh <name> <source.hip> <flags...>   -> tools/_build/libsrsran_amd_<name>.so
# <source.hip>: a file of srsran_project_amd/csrc, or a path to an edited copy of one (same base name)
set -e
name=$1; src=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
obj=$root/srsran_project_amd/lib/obj
mkdir -p "$root/tools/_build/var_$name"
base=$(basename "$src" .hip)
path=$root/srsran_project_amd/csrc/$base.hip
[ -f "$src" ] && path=$(cd "$(dirname "$src")" && pwd)/$(basename "$src")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -I"$root/include" -I"$root/srsran_project_amd/csrc" \
  -Wall -Wno-unused-function "$@" -c "$path" -o "$root/tools/_build/var_$name/$base.o"
objs=$(ls "$obj"/*.o | grep -v "/$base.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/tools/_build/libsrsran_amd_$name.so" $objs \
  "$root/tools/_build/var_$name/$base.o" -Wl,--no-undefined
echo "$root/tools/_build/libsrsran_amd_$name.so"
