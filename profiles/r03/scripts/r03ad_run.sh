# round 3: plan shapes (OCH_OPT_PLAN) against costliest-first and natural order, interleaved
set -o pipefail
O=gpurun_out/r03ad; mkdir -p $O
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
B="--steps 20 --warmup 5 --extra-windows 2 --no-cpu-baseline --no-other-configs --no-bounce --moving-steps 0 --sustain 0.5"
for i in 1 2; do
  for arm in plan=0 plan=5 plan=15 plan=40 plan=100 tile_order=0; do
    timeout -k 10 300 python -u bench.py $B --opt $arm > $O/${arm/=/_}_$i.json 2> $O/${arm/=/_}_$i.err || exit 1
  done
done
