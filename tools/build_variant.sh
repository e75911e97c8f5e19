#!/bin/bash
# Build an A/B variant of the engine from the working tree without touching it:
#   tools/build_variant.sh NAME [sed-expression FILE]...
# copies csrc/ and include/ into build/NAME/, applies each sed expression to its
# file there, and builds soft-actor-critic_amd/lib_NAME.so (for tools/ab_bench.sh).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1
shift
B=$R/build/$name
rm -rf "$B" && mkdir -p "$B/x" "$B/include"
cp -r "$R/soft-actor-critic_amd/csrc" "$B/x/csrc"
cp "$R"/include/*.h "$B/include/"
while [ $# -ge 2 ]; do
  before=$(md5sum < "$B/x/csrc/$2")
  sed -i "$1" "$B/x/csrc/$2"
  [ "$before" != "$(md5sum < "$B/x/csrc/$2")" ] || { echo "sed expression changed nothing in $2: $1" >&2; exit 1; }
  shift 2
done
cd "$B/x/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
  -mllvm -amdgpu-kernarg-preload-count=16 ${VARIANT_FLAGS:-} -shared -o "$R/soft-actor-critic_amd/lib_$name.so" sac_engine.hip
echo "built soft-actor-critic_amd/lib_$name.so"
