# round 3: N = 1 frames in flight x hardware queues with the final bench path (interleaved, twice)
set -o pipefail
O=gpurun_out/r03an; mkdir -p $O
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
B="--steps 20 --warmup 5 --extra-windows 2 --no-cpu-baseline --no-other-configs --no-bounce --moving-steps 0 --no-cull-off --sustain 0.5"
for i in 1 2; do
  for cfg in "3 4" "2 4" "4 5" "4 6" "3 8" "5 6"; do
    set -- $cfg
    timeout -k 10 300 python -u bench.py $B --inflight $1 --hw-queues $2 > $O/f$1_q$2_$i.json 2> $O/f$1_q$2_$i.err || exit 1
  done
done
