# round 3: N = 8 display-rank weight at 6 frames on 8 queues (proxy, every shard); the first-step
# issue with the process's other threads moved off the issuing CPU
set -o pipefail
O=gpurun_out/r03ag; mkdir -p $O
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
for w in 0.6 0.45 0.75 0.6 0.45 0.75; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/proxy_rank.py --worlds 8 --inflight 6 --shards all --events \
    --opt plan=0 --display-weight $w --out $O/p8_w$w.json >> $O/p8_w$w.txt 2> $O/p8_w$w.err || exit 1
done
EXTRA="--pin-core --isolate-main" bash tools/r03t_run.sh || exit 2
cp gpurun_out/r03t/stamps.txt $O/stamps_isolate.txt
