# native window issue (och_gpu_render_steps_dev) against one C-ABI call per step:
# the timing tests, then the driver's command interleaved with --issue python
set -o pipefail
O=gpurun_out/r03as; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_timing.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/native_$i.json 2> $O/native_$i.err || exit 2
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --issue python > $O/python_$i.json 2> $O/python_$i.err || exit 3
done
