# round 3: eight views per launch
set -o pipefail
O=gpurun_out/r03am; mkdir -p $O
timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_eight_views_per_launch" -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
