# round 3: HIP API calls of the headline window's first steps (rocprofv3 --hip-trace)
set -o pipefail
O=gpurun_out/r03u; mkdir -p $O
export TMPDIR=/tmp
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/trace -o run -- python -u bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --no-parity --sustain 0 --no-other-configs --no-bounce --no-cull-off --host-stamps > $O/trace.json 2> $O/trace.err || exit 3
ls -R $O/trace > $O/files.txt
python - $O/trace $O/trace.json > $O/api.txt <<'PY' || exit 5
import csv, json, sys
from pathlib import Path
st = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])["host_stamps_ns"]
t0 = st["t0"][0]
rows = []
for f in Path(sys.argv[1]).rglob("*.csv"):
    r0 = next(csv.DictReader(open(f)), None)
    if not r0 or "Start_Timestamp" not in r0:
        continue
    for r in csv.DictReader(open(f)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 - 400000 <= s <= t0 + 400000:
            rows.append((s, e, f.name[:22], (r.get("Function") or r.get("Kernel_Name") or r.get("Operation") or "")[:50],
                         r.get("Thread_Id", "")))
rows.sort()
print("parts", [(n, round((x - t0) / 1e3, 1)) for n, x in st.get("step_parts", [])])
for s, e, f, n, tid in rows:
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {f:22s} {tid:>8s} {n}")
PY
find $O -name "run_*.csv" -delete
