#!/bin/bash
# Build an experimental library variant: scripts/build_variant.sh NAME "-DFLAG=1 ..."
# -> libiqo_amd/variants/NAME.so (kernels.hip recompiled with the flags, other objects shared)
set -e
cd "$(dirname "$0")/../libiqo_amd"
make -s build/plan.o build/resizers.o build/abi.o
mkdir -p variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-strict-aliasing -I../include -Icsrc --offload-arch=gfx950 $2 \
    -c csrc/kernels.hip -o variants/$1_kernels.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/$1.so build/plan.o build/resizers.o \
    variants/$1_kernels.o build/abi.o
rm -f variants/$1_kernels.o
echo "variants/$1.so"
