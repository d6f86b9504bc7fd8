# round 3: host issue timeline of the headline window against its kernel trace
set -o pipefail
O=gpurun_out/r03t; mkdir -p $O
export TMPDIR=/tmp
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python -u bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --no-parity --sustain 0 --no-other-configs --no-bounce --no-cull-off --host-stamps $EXTRA > $O/trace.json 2> $O/trace.err || exit 3
python - $O/trace $O/trace.json > $O/stamps.txt <<'PY' || exit 5
import csv, json, sys
from pathlib import Path
rows = []
for f in Path(sys.argv[1]).rglob("*kernel_trace.csv"):
    rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in csv.DictReader(open(f))]
rows.sort()
st = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])["host_stamps_ns"]
t0, t1 = st["t0"][0], st["t1"][0]
print("host window us", (t1 - t0) / 1e3)
print("issued us", [round((x - t0) / 1e3, 1) for x in st["issued"]])
print("step parts us", [(n, round((x - t0) / 1e3, 1)) for n, x in st.get("step_parts", [])])
for s, e, n in [r for r in rows if t0 - 500000 <= r[0] <= t1 + 200000]:
    print(f"  {n:40s} start {(s - t0) / 1e3:9.1f} end {(e - t0) / 1e3:9.1f}")
PY
find $O -name "run_*.csv" -delete
