#!/bin/bash
# Build the engine of a committed revision for same-box A/Bs:
#   tools/build_rev.sh REV NAME  ->  soft-actor-critic_amd/lib_NAME.so
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
rev=$1
name=$2
B=$R/build/rev_$name
rm -rf "$B" && mkdir -p "$B/src" "$B/x" "$B/include"
git -C "$R" archive "$rev" soft-actor-critic_amd/csrc include | tar -x -C "$B/src"
mv "$B/src/soft-actor-critic_amd/csrc" "$B/x/csrc"
cp "$B/src/include/"*.h "$B/include/"
cd "$B/x/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
  -mllvm -amdgpu-kernarg-preload-count=16 -shared -o "$R/soft-actor-critic_amd/lib_$name.so" sac_engine.hip
echo "built soft-actor-critic_amd/lib_$name.so from $rev"
