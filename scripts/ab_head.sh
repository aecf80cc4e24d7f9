#!/bin/bash
# Build a git revision's libdpemu.so (default HEAD) into ab_build/libdpemu_<name>.so
# for a same-process A/B against the working tree's library (scripts/ab.py).
#   scripts/ab_head.sh [rev] [name]
set -e
rev=${1:-HEAD}; name=${2:-head}
repo="$(cd "$(dirname "$0")/.." && pwd)"
tmp=$(mktemp -d)
git -C "$repo" archive "$rev" distributed_processor_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$repo/ab_build"
cd "$tmp/distributed_processor_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -shared \
    -o "$repo/ab_build/libdpemu_$name.so" *.hip capi.cpp
rm -rf "$tmp"
