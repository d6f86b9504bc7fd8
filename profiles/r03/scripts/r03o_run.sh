# round 3: the bench window with and without per-step timing events; a kernel
# trace of the window with no events (tools/window_trace.py)
set -o pipefail
O=gpurun_out/r03o; mkdir -p $O
export TMPDIR=/tmp
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --extra-windows 6 --no-cpu-baseline --no-other-configs --no-bounce > $O/bench_extra.json 2> $O/bench_extra.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_noev -o run -- python -u bench.py --steps 20 --warmup 5 --no-step-events \
  --no-cpu-baseline --no-parity --sustain 0 --no-other-configs --no-bounce --no-cull-off > $O/trace_noev.json 2> $O/trace_noev.err || exit 2
python tools/window_trace.py $O/trace_noev --steps 20 --bench-json $O/trace_noev.json --config d12_1920x1080_n1 \
  --out $O/window_noev.json --csv $O/window_noev.csv > /dev/null || exit 3
find $O -name "run_*.csv" -delete
