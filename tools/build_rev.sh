#!/bin/bash
# Build the whole product library of git revision REV (its own kernel, API and
# headers, so no struct layout is mixed) into build_variants/liboch_gpu_NAME.so,
# for interleaved A/B runs against the working tree (OCH_GPU_LIB=..., or the
# gpu_run.sh step lib=NAME).  usage: tools/build_rev.sh REV NAME
set -e
cd "$(dirname "$0")/.."
REV=${1:?rev}; NAME=${2:?name}
WT=$(mktemp -d /tmp/och_rev_XXXX)
git worktree add -q --detach "$WT" "$REV"
make -s -j8 -C "$WT/octree_ray_tracing_amd/csrc"
mkdir -p build_variants
cp "$WT/octree_ray_tracing_amd/liboch_gpu.so" "build_variants/liboch_gpu_$NAME.so"
git worktree remove --force "$WT"
echo "build_variants/liboch_gpu_$NAME.so <- $(git rev-parse --short "$REV")"
