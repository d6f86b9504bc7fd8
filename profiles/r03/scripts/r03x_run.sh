# round 3: the N = 2 bench path (gloo on one GPU) with the prepared render issue, and the N = 1 bench
set -o pipefail
O=gpurun_out/r03x; mkdir -p $O
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
bash tools/rehearse_n2.sh > $O/rehearse.txt 2>&1 || exit 4
cp gpurun_out/rehearse_n2.json $O/
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 3
