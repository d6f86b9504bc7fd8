# round 3: N = 8 proxy, default (4 queues, 3 in flight) against 8 queues x 6 / 7 in flight, interleaved
set -o pipefail
O=gpurun_out/r03z3; mkdir -p $O
i=0
for cfg in "4 3" "8 6" "4 3" "8 6" "8 7" "8 6"; do
  set -- $cfg; i=$((i+1))
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 python -u tools/proxy_rank.py --worlds 8 --inflight $2 --shards all --events \
    --out $O/p8_q$1_f$2_$i.json > $O/p8_q$1_f$2_$i.txt 2> $O/p8_q$1_f$2_$i.err || exit 1
done
