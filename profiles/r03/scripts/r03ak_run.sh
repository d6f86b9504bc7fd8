# round 3: node order in HBM, breadth-first (builder) vs depth-first preorder (kernel unchanged)
set -o pipefail
O=gpurun_out/r03ak; mkdir -p $O
timeout -k 10 500 python -u tools/reorder_ab.py --depth 12 --rounds 4 --pipelined 400 --out $O/reorder_ab.json > $O/reorder_ab.log 2>&1 || exit 1
