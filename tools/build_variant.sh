#!/bin/bash
# build_variant.sh <name> <sed-expr>... : builds srsran_project_amd with a patched
# csrc/$VFILE (default ldpc_decoder.hip) into exp/<name>/libsrsran_amd.so (for A/B timing only).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
W=$(mktemp -d)
cp -r "$ROOT/srsran_project_amd/csrc" "$W/csrc"
for e in "$@"; do sed -i "$e" "$W/csrc/${VFILE:-ldpc_decoder.hip}"; done
mkdir -p "$ROOT/exp/$name"
objs=""
pids=""
for f in "$W"/csrc/*.hip "$W"/csrc/*.cpp; do
  o="$W/$(basename "$f").o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -I"$ROOT/include" -I"$W/csrc" -x hip -c "$f" -o "$o" &
  pids="$pids $!"
  objs="$objs $o"
done
for p in $pids; do wait $p || { echo "variant $name: compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/exp/$name/libsrsran_amd.so" $objs
rm -rf "$W"
echo "built exp/$name"
