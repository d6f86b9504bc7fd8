#!/bin/bash
# Build kernel variants for A/B runs: each argument is NAME:"-DFLAG=V ...", or
# NAME@REV:"..." to build git revision REV's kernel source (e.g. head@HEAD:).
# Output: build_variants/liboch_gpu_NAME.so (select with OCH_GPU_LIB=...).
set -e
cd "$(dirname "$0")/.."
make -s -C octree_ray_tracing_amd/csrc
HIPCC=/opt/rocm/bin/hipcc
FLAGS="-std=c++17 -O3 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result --offload-arch=gfx950 -fno-gpu-flush-denormals-to-zero -munsafe-fp-atomics"
mkdir -p build_variants
for spec in "$@"; do
    name=${spec%%:*}; defs=${spec#*:}
    src=octree_ray_tracing_amd/csrc/och_kernels.hip
    if [[ "$name" == *@* ]]; then      # NAME@REV: the kernel source of git revision REV
        src=octree_ray_tracing_amd/csrc/och_kernels_${name%%@*}.hip
        git show "${name#*@}":octree_ray_tracing_amd/csrc/och_kernels.hip > "$src"
    fi
    $HIPCC $FLAGS $defs -c "$src" -o build_variants/k_${name%%@*}.o &
done
wait
for spec in "$@"; do
    name=${spec%%:*}
    [[ "$name" == *@* ]] && rm -f octree_ray_tracing_amd/csrc/och_kernels_${name%%@*}.hip
    name=${name%%@*}
    $HIPCC -shared -fPIC --offload-arch=gfx950 -o build_variants/liboch_gpu_$name.so build_variants/k_$name.o \
        octree_ray_tracing_amd/csrc/build/och_api.o octree_ray_tracing_amd/csrc/build/och_builder.o \
        octree_ray_tracing_amd/csrc/build/och_editor.o octree_ray_tracing_amd/csrc/build/och_group.o \
        octree_ray_tracing_amd/csrc/build/och_comm.o -pthread -ldl
    rm -f build_variants/k_$name.o
done
ls -la build_variants
