# round 3: merge kernel after the plan fix (tests, block-128 A/B), then the
# PMC profile + window trace of the current bench kernel
set -o pipefail
O=gpurun_out/r03n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_merge.py -m gpu -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_render.py --rounds 4 --pipelined 400 --cache /tmp/och_terrain_cache.npz --out $O/ab.json \
  --arm '{"tile_order": 2}' --arm '{"tile_order": 2, "block": 128}' --arm '{"tile_order": 2, "block": 128, "merge": 8}' \
  --arm '{"tile_order": 2, "block": 128, "merge": 16}' --arm '{"tile_order": 2, "block": 256, "merge": 16}' > $O/ab.log 2>&1 || exit 2
bash tools/profile.sh r03n > $O/profile.log 2>&1 || exit 3
