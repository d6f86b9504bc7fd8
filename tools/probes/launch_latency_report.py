"""Line the host clock readings of launch_latency.py up with the rocprofv3
kernel trace: for each launch, the first kernel that starts after its host
reading; prints host issue time and host-to-kernel-start latency per variant."""
import csv
import json
import statistics
import sys
from collections import defaultdict
from pathlib import Path

rows = []
for f in Path(sys.argv[1]).rglob("*kernel_trace.csv"):
    rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))]
rows.sort()
recs = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
lat = defaultdict(list)
for r in recs:
    k = next((x for x in rows if x[0] >= r["h0"]), None)
    if k is None:
        continue
    lat[(r["what"], r["idle_us"], r["stream"])].append(((r["h1"] - r["h0"]) / 1e3, (k[0] - r["h0"]) / 1e3,
                                                       (k[1] - k[0]) / 1e3))
for key in sorted(lat):
    v = lat[key]
    print(f"{key[0]:10s} idle {key[1]:6d} us {key[2]}: issue {statistics.median(a for a, _, _ in v):7.1f} us, "
          f"host->start {statistics.median(b for _, b, _ in v):7.1f} us, kernel {statistics.median(c for _, _, c in v):7.1f} us")
