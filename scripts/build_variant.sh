#!/bin/bash
# Build an experimental library variant: scripts/build_variant.sh NAME "-DFLAG=1 ..."
# -> libiqo_amd/variants/NAME.so (kernels.hip, kernels_ratio.hip and abi.hip recompiled with the flags, the host
# objects shared).  -DIQO_VARIANT_DEBUG enables the wrong-output timing flags ("debug_flags").
set -e
cd "$(dirname "$0")/../libiqo_amd"
make -s build/plan.o build/cpu_generic.o build/resizers.o
mkdir -p variants
F="-O3 -std=c++17 -fPIC -fno-strict-aliasing -I../include -Icsrc --offload-arch=gfx950 $2"
/opt/rocm/bin/hipcc $F -c csrc/kernels.hip -o variants/$1_kernels.o &
/opt/rocm/bin/hipcc $F -c csrc/kernels_ratio.hip -o variants/$1_kratio.o &
/opt/rocm/bin/hipcc $F -ffp-contract=off -c csrc/abi.hip -o variants/$1_abi.o
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/$1.so build/plan.o build/cpu_generic.o build/resizers.o \
    variants/$1_kernels.o variants/$1_kratio.o variants/$1_abi.o
rm -f variants/$1_kernels.o variants/$1_kratio.o variants/$1_abi.o
echo "variants/$1.so"
