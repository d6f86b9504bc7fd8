set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiled_batch.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/win -o run -- python -u bench.py --no-cpu-baseline --no-parity --sustain 0 --no-other-configs --no-bounce --no-cull-off > $O/bench_win.json 2> $O/bench_win.err || exit 3
python tools/window_trace.py $O/win --steps 20 --bench-json $O/bench_win.json --out $O/window_summary.json --csv $O/window_trace.csv > /dev/null || exit 4
timeout -k 10 400 python -u tools/proxy_rank.py --worlds 2,4,8 --inflight 3 --shards all --windows 5 --sustain-steps 200 --cache /tmp/och_d12.npz --out $O/proxy_all_shards.json > $O/proxy.log 2>&1 || exit 5
