# round 3: plan shape at N = 8 (proxy, every shard, 6 frames on 8 queues) and config 5 at N = 1
set -o pipefail
O=gpurun_out/r03ae; mkdir -p $O
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
for i in 1 2; do
  for arm in plan=10 plan=0; do
    GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/proxy_rank.py --worlds 8 --inflight 6 --shards all --events \
      --opt $arm --out $O/p8_${arm/=/_}_$i.json > $O/p8_${arm/=/_}_$i.txt 2> $O/p8_${arm/=/_}_$i.err || exit 1
  done
done
B="--steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --moving-steps 0 --sustain 0.5 --no-cull-off"
for arm in plan=10 plan=0 plan=10 plan=0; do
  timeout -k 10 300 python -u bench.py $B --opt $arm > $O/b_${arm/=/_}_$(date +%s%N).json 2> $O/b.err || exit 2
done
