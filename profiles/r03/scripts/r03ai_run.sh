# round 3: kernel trace of a 200-step window (is the sustained rate's structure different from 20 steps?)
set -o pipefail
O=gpurun_out/r03ai; mkdir -p $O
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python -u bench.py --steps 200 --warmup 5 \
  --no-cpu-baseline --no-parity --sustain 0 --no-other-configs --no-bounce --no-cull-off --moving-steps 0 > $O/trace.json 2> $O/trace.err || exit 3
python tools/window_trace.py $O/trace --steps 200 --bench-json $O/trace.json --config d12_1920x1080_n1_200 \
  --out $O/window.json --csv $O/window.csv > /dev/null || exit 4
find $O -name "run_*.csv" -delete
