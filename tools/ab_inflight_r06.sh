#!/bin/bash
# Frames in flight / hardware queues at N = 1 on the final kernel: bench.py's
# headline window (the driver's --steps 20 --warmup 5) and sustained, per arm,
# interleaved over rounds.  Arms: "inflight:hwqueues" (hwqueues 0 = the env's).
set -o pipefail
mkdir -p gpurun_out/abif
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
ARMS=${ARMS:-"3:0 2:0 4:0 4:8 5:8 6:8"}
for round in 1 2 3; do
  for arm in $ARMS; do
    n=${arm%%:*}; q=${arm##*:}
    extra=""; [ "$q" != "0" ] && extra="--hw-queues $q"
    out=gpurun_out/abif/if${n}_q${q}_r$round
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-bounce \
        --no-other-configs --no-cull-off --no-split-arm --inflight $n $extra > $out.json 2> $out.err || exit 1
    python -c "import json;d=json.loads(open('$out.json').read().strip().splitlines()[-1]);print('inflight $n q $q r$round', d['value'], d['sustained']['value'], d['ms_per_step'], flush=True)"
  done
done
