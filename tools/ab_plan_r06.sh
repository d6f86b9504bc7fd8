#!/bin/bash
# Launch-order plan shape at N = 1 on the final kernel (OCH_OPT_PLAN: the
# costliest P % of the planning frame's workgroups first; 0 = all costliest
# first; 100 = costliest and cheapest alternating) and tile_order 3 (XCD-grouped
# supertiles): the driver's 20-step window and sustained, interleaved rounds.
set -o pipefail
mkdir -p gpurun_out/abpl
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
ARMS=${ARMS:-"plan=10 plan=0 plan=3 plan=30 plan=100 tile_order=3"}
for round in ${ROUNDS:-1 2 3}; do
  for arm in $ARMS; do
    out=gpurun_out/abpl/$(echo $arm | tr '=,' '__')_r$round
    opts=""; for kv in ${arm//,/ }; do opts="$opts --opt $kv"; done      # "a=1,b=2": several options
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-bounce \
        --no-other-configs --no-cull-off --no-split-arm $opts > $out.json 2> $out.err || exit 1
    python -c "import json;d=json.loads(open('$out.json').read().strip().splitlines()[-1]);print('$arm r$round', d['value'], d['sustained']['value'], d['roofline']['kernel_ms_serial'], flush=True)"
  done
done
