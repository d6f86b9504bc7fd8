#!/bin/bash
# Interleaved A/B of kernel library variants (tools/build_variants.sh) with
# tools/ab_render.py: serial launch latency and pipelined bench-style steps,
# two rounds per variant, one process per run.  Usage: bash tools/ab_libs.sh TAG NAME...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for round in 1 2; do
  for v in "$@"; do
    OCH_GPU_LIB=build_variants/liboch_gpu_$v.so timeout -k 10 300 python -u tools/ab_render.py --rounds 4 --pipelined 400 \
        --cache /tmp/och_terrain_cache.npz --out gpurun_out/ab_${TAG}_${v}_$round.json --arm "{}" \
        > gpurun_out/ab_${TAG}_${v}_$round.log 2>&1 || { tail -5 gpurun_out/ab_${TAG}_${v}_$round.log; exit 1; }
    echo "$v $round $(grep '^{' gpurun_out/ab_${TAG}_${v}_$round.log)"
  done
done
