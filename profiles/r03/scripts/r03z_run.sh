# round 3: frames in flight x hardware queues, N = 8 proxy (every shard) and N = 1
set -o pipefail
O=gpurun_out/r03z; mkdir -p $O
for q in 4 8; do
  for f in 3 4 6; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/proxy_rank.py --worlds 8 --inflight $f --shards all --events \
      --out $O/p8_q${q}_f$f.json > $O/p8_q${q}_f$f.txt 2> $O/p8_q${q}_f$f.err || exit 1
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/proxy_rank.py --worlds 1 --inflight $f --events \
      --out $O/p1_q${q}_f$f.json > $O/p1_q${q}_f$f.txt 2> $O/p1_q${q}_f$f.err || exit 1
  done
done
