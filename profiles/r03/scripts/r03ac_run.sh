# round 3: planned launch order (tile_order 2, the bench default) against natural order, interleaved
set -o pipefail
O=gpurun_out/r03ac; mkdir -p $O
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
B="--steps 20 --warmup 5 --extra-windows 2 --no-cpu-baseline --no-other-configs --no-bounce --moving-steps 0 --sustain 0.5"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py $B > $O/plan_$i.json 2> $O/plan_$i.err || exit 1
  timeout -k 10 300 python -u bench.py $B --opt tile_order=0 > $O/natural_$i.json 2> $O/natural_$i.err || exit 1
done
