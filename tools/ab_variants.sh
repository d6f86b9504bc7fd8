#!/bin/bash
# A/B of kernel variants built by tools/build_variants.sh: latency probe and
# bench per variant, interleaved twice.  Usage: bash tools/ab_variants.sh NAME...
set -o pipefail
mkdir -p gpurun_out
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
for round in 1 2; do
  for v in "$@"; do
    lib=build_variants/liboch_gpu_$v.so
    OCH_GPU_LIB=$lib timeout -k 10 200 python -u tools/latency_probe.py --blocks 64 --out gpurun_out/abv_lat_${v}_$round.json \
        > gpurun_out/abv_lat_${v}_$round.log 2>&1 || exit 1
    OCH_GPU_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/abv_bench_${v}_$round.json \
        2> gpurun_out/abv_bench_${v}_$round.err || exit 1
    python - "$v" "$round" <<'PY'
import json, sys
v, r = sys.argv[1:3]
d = json.load(open(f"gpurun_out/abv_bench_{v}_{r}.json"))
lat = json.load(open(f"gpurun_out/abv_lat_{v}_{r}.json"))
print(v, r, "bench", d["value"], "bounce", d["bounce"]["value"], "render2", lat.get("render2_layout1_block64_us"),
      "tile-0.6", lat["pitch-0.6_layout1_block64"]["tile_656_160_us"], "ray", lat["pitch-0.6_layout1_block64"]["ray_663_166"]["us"])
PY
  done
done
