#!/bin/bash
# Build A/B variants of libdpemu.so from the same sources with extra -D flags
# (build-time A/B only; the product library has no knobs):
#   scripts/ab_libs.sh <name> "<flags>" ...  ->  /tmp/ab/libdpemu_<name>.so
set -e
cd "$(dirname "$0")/../distributed_processor_amd/csrc"
mkdir -p ../../ab_build
while [ $# -ge 2 ]; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $2 -shared \
        -o ../../ab_build/libdpemu_$1.so interp.hip branch.hip branch_demod.hip straight.hip macro.hip dds.hip capi.cpp
    shift 2
done
