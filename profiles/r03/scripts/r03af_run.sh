# round 3: sorted batches (OCH_OPT_SORT) -- parity tests, then the bench's trace_batch section
set -o pipefail
O=gpurun_out/r03af; mkdir -p $O
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-other-configs --no-bounce --moving-steps 0 --sustain 0.3 > $O/bench.json 2> $O/bench.err || exit 2
