# round 3: in-block wave merging -- probe, then the parity tests
set -o pipefail
O=gpurun_out/r03m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/merge_probe.py > $O/probe.log 2>&1 || exit 9
timeout -k 10 600 python -u -m pytest tests/test_gpu_merge.py -m gpu -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1 || exit 1
