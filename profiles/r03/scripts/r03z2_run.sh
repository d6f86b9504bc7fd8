# round 3: frames in flight x hardware queues at N = 2 and 4 (every shard), N = 8 with 5 / 8 in flight
set -o pipefail
O=gpurun_out/r03z2; mkdir -p $O
for cfg in "2 4 3" "2 8 4" "2 8 6" "4 4 3" "4 8 4" "4 8 6" "8 8 5" "8 8 8"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python -u tools/proxy_rank.py --worlds $1 --inflight $3 --shards all --events \
    --out $O/p$1_q$2_f$3.json > $O/p$1_q$2_f$3.txt 2> $O/p$1_q$2_f$3.err || exit 1
done
