#!/bin/bash
# The N = 8 proxy (tools/proxy_rank.py: every shard of the 3840x2160 two-view
# step on this one GPU, six frames in flight on eight hardware queues, the
# display rank at weight 0.5, costliest-first plan -- bench.py's N = 8 setup)
# with and without the heavy-tile split, one fresh process per arm.
# usage: bash tools/proxy_split.sh OUTDIR "ARM_OPTS" ["ARM_OPTS" ...]
#   ARM_OPTS: extra proxy_rank.py --opt flags, "" = the plain plan
set -o pipefail
out=${1:?outdir}; shift
mkdir -p "$out"
i=0
for arm in "$@"; do
  i=$((i + 1))
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/proxy_rank.py --worlds 8 --inflight 6 --shards all \
    --events --display-weight 0.5 --opt plan=0 $arm --out "$out/proxy_$i.json" > "$out/proxy_$i.log" 2>&1 \
    || { tail -20 "$out/proxy_$i.log"; exit $i; }
  echo "arm $i ($arm): $(tail -1 "$out/proxy_$i.log")"
done
