#!/bin/bash
# Build the memory-side probe (tools/mem_probe.hip) into exp_libs/ (diagnostic, never loaded by the product).
set -e
cd "$(dirname "$0")/.."
mkdir -p exp_libs
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-inline-asm -fPIC -shared -o exp_libs/libmem_probe.so tools/mem_probe.hip
