# round 3: end of the timed window -- poll the streams then synchronize, vs a blocking
# synchronize; host clock readings of the window lined up with a kernel trace
set -o pipefail
O=gpurun_out/r03r; mkdir -p $O
export TMPDIR=/tmp
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
B="--steps 20 --warmup 5 --extra-windows 3 --no-cpu-baseline --no-other-configs --no-bounce --sustain 0.5"
for m in spin block spin block; do
  timeout -k 10 300 python -u bench.py $B --wait $m > $O/w_$m.json 2> $O/w_$m.err || exit 2
  cp $O/w_$m.json $O/w_${m}_$(date +%s%N).json
done
for m in spin block; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$m -o run -- python -u bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --no-parity --sustain 0 --no-other-configs --no-bounce --no-cull-off --host-stamps --wait $m > $O/trace_$m.json 2> $O/trace_$m.err || exit 3
python tools/window_trace.py $O/trace_$m --steps 20 --bench-json $O/trace_$m.json --config d12_1920x1080_n1 \
  --out $O/window_$m.json --csv $O/window_$m.csv > /dev/null || exit 4
python - $O/trace_$m $O/trace_$m.json > $O/stamps_$m.txt <<'PY' || exit 5
import csv, json, sys
from pathlib import Path
rows = []
for f in Path(sys.argv[1]).rglob("*kernel_trace.csv"):
    rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in csv.DictReader(open(f))]
rows.sort()
st = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])["host_stamps_ns"]
for clock, i in (("monotonic", 0), ("boottime", 1)):
    t0, t1 = st["t0"][i], st["t1"][i]
    print(clock, "host window us", (t1 - t0) / 1e3)
    near = [r for r in rows if t0 - 200000 <= r[0] <= t1 + 200000]
    for s, e, n in near:
        print(f"  {n:40s} start {(s - t0) / 1e3:9.1f} end {(e - t0) / 1e3:9.1f}")
PY
done
find $O -name "run_*.csv" -delete
