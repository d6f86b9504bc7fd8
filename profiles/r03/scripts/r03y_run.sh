# round 3: per-rank proxy of the N-rank step (every shard) after the dispatch-recorded timing
set -o pipefail
O=gpurun_out/r03y; mkdir -p $O
for w in 1 2 4 8; do
  timeout -k 10 300 python -u tools/proxy_rank.py --worlds $w --inflight 3 --shards all --events --out $O/proxy_w$w.json > $O/proxy_w$w.txt 2> $O/proxy_w$w.err || exit 1
done
