#!/bin/bash
# Build the library with extra -D flags into explib/lib<name>.so (kernel A/B experiments).
# Usage: bash tools/build_variant.sh <name> [-DFLAG ...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p explib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -Wall -Wno-unused-function \
    -Wno-unused-variable -mllvm -amdgpu-sched-strategy=iterative-ilp "$@" -o explib/lib$name.so \
    dragg_amd/csrc/mpc_kernel.hip
