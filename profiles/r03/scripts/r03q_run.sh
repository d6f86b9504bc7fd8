# round 3: step events recorded by the render's own dispatch (och_gpu_set_launch_events)
# vs fence-free records vs torch events; kernel trace of the default window
set -o pipefail
O=gpurun_out/r03q; mkdir -p $O
export TMPDIR=/tmp
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
timeout -k 10 200 python -u -m pytest tests/test_gpu_timing.py -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="--steps 20 --warmup 5 --extra-windows 4 --no-cpu-baseline --no-other-configs --no-bounce --sustain 0.5"
for m in dispatch nofence torch dispatch; do
  timeout -k 10 300 python -u bench.py $B --step-events $m > $O/$m.json 2> $O/$m.err || exit 2
  cp $O/$m.json $O/${m}_$(date +%s).json
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python -u bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --no-parity --sustain 0 --no-other-configs --no-bounce --no-cull-off > $O/trace.json 2> $O/trace.err || exit 3
python tools/window_trace.py $O/trace --steps 20 --bench-json $O/trace.json --config d12_1920x1080_n1 \
  --out $O/window.json --csv $O/window.csv > /dev/null || exit 4
find $O -name "run_*.csv" -delete
