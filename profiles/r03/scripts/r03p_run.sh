# round 3: step timing events without the system-scope fence vs torch events vs none;
# stream priorities; a kernel trace of the default (fence-free) window
set -o pipefail
O=gpurun_out/r03p; mkdir -p $O
export TMPDIR=/tmp
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
B="--steps 20 --warmup 5 --extra-windows 4 --no-cpu-baseline --no-other-configs --no-bounce --sustain 0.5"
timeout -k 10 300 python -u bench.py $B > $O/nofence.json 2> $O/nofence.err || exit 1
timeout -k 10 300 python -u bench.py $B --step-events torch > $O/torch.json 2> $O/torch.err || exit 1
timeout -k 10 300 python -u bench.py $B --stream-priority=-1 > $O/prio1.json 2> $O/prio1.err || exit 1
timeout -k 10 300 python -u bench.py $B --stream-priority=-1,-1 > $O/prio2.json 2> $O/prio2.err || exit 1
timeout -k 10 300 python -u bench.py $B > $O/nofence2.json 2> $O/nofence2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python -u bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --no-parity --sustain 0 --no-other-configs --no-bounce --no-cull-off > $O/trace.json 2> $O/trace.err || exit 2
python tools/window_trace.py $O/trace --steps 20 --bench-json $O/trace.json --config d12_1920x1080_n1 \
  --out $O/window.json --csv $O/window.csv > /dev/null || exit 3
find $O -name "run_*.csv" -delete
