#!/bin/bash
set -o pipefail
for round in 1 2; do
  for v in merged mdim top2 top3 top4; do
    OCH_GPU_LIB=build_variants/liboch_gpu_$v.so timeout -k 10 300 python -u tools/ab_render.py --rounds 4 --pipelined 400 \
        --cache /tmp/och_terrain_cache.npz --out gpurun_out/ab_t_${v}_$round.json --arm "{}" --arm '{"block": 256}' \
        > gpurun_out/ab_t_${v}_$round.log 2>&1 || { tail -5 gpurun_out/ab_t_${v}_$round.log; exit 1; }
    grep '^{' gpurun_out/ab_t_${v}_$round.log | sed "s/^/$v $round /" | cut -c1-250
  done
done
