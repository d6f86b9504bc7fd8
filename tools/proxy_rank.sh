#!/bin/bash
# tools/proxy_rank.py arms, one fresh process each (see its docstring).
# usage: tools/proxy_rank.sh "1 2 4 8" "2 3 4 6" [rounds] [extra proxy_rank.py args]
set -e
mkdir -p gpurun_out
out=${OUT:-gpurun_out/proxy_rank.jsonl}
: > $out
for r in $(seq ${3:-1}); do
  for w in $1; do
    for f in $2; do
      timeout -k 10 120 python -u tools/proxy_rank.py --worlds $w --inflight $f --out gpurun_out/proxy_arm.json ${4:-} \
        2>>gpurun_out/proxy_rank.err | tee -a $out
    done
  done
done
