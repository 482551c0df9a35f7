#!/bin/bash
# build_variant.sh <name> <sed-expr>... : builds abx/<name>/libsrsran_amd.so from the in-tree objects
# (make -C srsran_project_amd first) with csrc/$VFILE (default ldpc_decoder.hip) recompiled after the sed
# edits -- for A/B timing only (tools/ab.sh, tools/gpu_probe.sh).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
VFILE=${VFILE:-ldpc_decoder.hip}
W=$(mktemp -d)
cp -r "$ROOT/srsran_project_amd/csrc" "$W/csrc"
for e in "$@"; do sed -i "$e" "$W/csrc/$VFILE"; done
mkdir -p "$ROOT/abx/$name"
obj=$ROOT/srsran_project_amd/lib/obj
vo="$W/${VFILE%.*}.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -I"$ROOT/include" -I"$W/csrc" -x hip -c "$W/csrc/$VFILE" -o "$vo"
objs=$(ls "$obj"/*.o | grep -v "/${VFILE%.*}.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/abx/$name/libsrsran_amd.so" $objs "$vo"
rm -rf "$W"
echo "built abx/$name"
