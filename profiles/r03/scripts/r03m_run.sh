# round 3: in-block wave merging -- parity, interleaved A/B, PMC counters of the two kernels
set -o pipefail
O=gpurun_out/r03m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 90 python -u tools/merge_probe.py > $O/probe.log 2>&1 || exit 9
timeout -k 10 500 python -u -m pytest tests/test_gpu_merge.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/ab_render.py --rounds 4 --pipelined 400 --cache /tmp/och_terrain_cache.npz --out $O/ab.json \
  --arm '{"tile_order": 2}' --arm '{"tile_order": 2, "block": 256}' --arm '{"tile_order": 2, "block": 256, "merge": 4}' \
  --arm '{"tile_order": 2, "block": 256, "merge": 8}' --arm '{"tile_order": 2, "block": 256, "merge": 16}' \
  --arm '{"tile_order": 2, "block": 128, "merge": 8}' > $O/ab.log 2>&1 || exit 2
for arm in base merge8; do
  A='{"tile_order": 2}'; [ $arm = merge8 ] && A='{"tile_order": 2, "block": 256, "merge": 8}'
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"; do
    n=$(echo $grp | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_${arm}_$n -o run -- python -u tools/ab_render.py \
      --rounds 1 --reps 3 --cache /tmp/och_terrain_cache.npz --out $O/pmc_${arm}_$n.json --arm "$A" > /dev/null 2>&1 || exit 3
  done
done
python tools/pmc_arms.py $O > $O/pmc_arms.json || exit 4
find $O -name "run_*.csv" -size +2M -delete
