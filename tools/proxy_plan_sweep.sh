#!/bin/bash
# The planned order's shape (OCH_OPT_PLAN) in the N = 2 / 4 proxies
# (tools/proxy_rank.py, every shard, bench.py's per-N frames in flight and
# display weight), interleaved.  usage: bash tools/proxy_plan_sweep.sh OUTDIR ROUNDS "P1 P2 ..." "W1 W2 ..."
set -o pipefail
out=${1:?outdir}; rounds=${2:-2}; arms=${3:-"10 3 0"}; worlds=${4:-"2 4"}
mkdir -p "$out"
for r in $(seq "$rounds"); do
  for p in $arms; do
    for w in $worlds; do
      dw=$(python -c "import octree_ray_tracing_amd as o; print(o.display_weight($w, 'all_gather'))")
      timeout -k 10 300 python -u tools/proxy_rank.py --worlds $w --inflight 3 --shards all --events \
        --display-weight $dw --opt plan=$p --out "$out/n${w}_p${p}_r$r.json" > "$out/n${w}_p${p}_r$r.log" 2>&1 \
        || { tail -20 "$out/n${w}_p${p}_r$r.log"; exit 2; }
      echo "n$w plan=$p r$r: $(tail -1 "$out/n${w}_p${p}_r$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['slowest_ms_per_step_20'], d['slowest_ms_per_step_sustained'])")"
    done
  done
done
