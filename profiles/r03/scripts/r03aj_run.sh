# round 3: the new GPU tests (random cameras at depth 12; plan shapes)
set -o pipefail
O=gpurun_out/r03aj; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py::test_random_cameras_d12 "tests/test_gpu_parity.py::test_planned_launch_order" \
  -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
