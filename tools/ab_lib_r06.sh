#!/bin/bash
# Library A/B at N = 1: bench.py (the driver's 20 steps, W 5) with each
# build_variants/liboch_gpu_<name>.so and the in-tree library ("new"),
# interleaved; headline, sustained, config 5 and the split arm (on / off).
set -o pipefail
mkdir -p gpurun_out/ablib
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
for round in ${ROUNDS:-1 2 3}; do
  for v in ${VARIANTS:-old new}; do
    lib=build_variants/liboch_gpu_$v.so; [ "$v" = "new" ] && lib=octree_ray_tracing_amd/liboch_gpu.so
    out=gpurun_out/ablib/${v}_r$round
    OCH_GPU_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs \
        --no-cull-off > $out.json 2> $out.err || exit 1
    python -c "
import json;d=json.loads(open('$out.json').read().strip().splitlines()[-1]);s=d['split']
print('$v r$round', d['value'], d['sustained']['value'], d['bounce']['value'], 'split on', s['on']['value'], s['on']['sustained'], 'off', s['off']['value'], s['off']['sustained'], flush=True)"
  done
done
