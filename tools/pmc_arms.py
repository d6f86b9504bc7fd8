"""Per-kernel PMC means of the A/B arms of profiles/r03/scripts/r03m_run.sh (rocprofv3 CSVs under
gpurun_out/r03m/pmc_<arm>_<group>/): the render kernels only (k_trace_grid /
k_trace_grid_merge over CameraSource), per dispatch, with the derived VALU lane
utilisation, VALU per wave and wait fraction."""
import csv
import json
import statistics
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
out = defaultdict(lambda: defaultdict(list))
for d in sorted(root.glob("pmc_*")):
    if not d.is_dir():
        continue
    arm = d.name.split("_")[1]
    for f in d.rglob("*counter_collection.csv"):
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(f)):
            if "CameraSource" not in row["Kernel_Name"]:
                continue
            per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
        for cs in per.values():
            for c, v in cs.items():
                out[arm][c].append(v)
res = {}
for arm, cs in out.items():
    m = {c: statistics.fmean(v) for c, v in cs.items()}
    if m.get("SQ_ACTIVE_INST_VALU"):
        m["valu_lane_utilization"] = round(m.get("SQ_THREAD_CYCLES_VALU", 0) / (64 * m["SQ_ACTIVE_INST_VALU"]), 4)
    if m.get("SQ_WAVES"):
        m["valu_insts_per_wave"] = round(m["SQ_INSTS_VALU"] / m["SQ_WAVES"], 1)
    if m.get("SQ_WAVE_CYCLES"):
        m["wait_inst_frac"] = round(m.get("SQ_WAIT_INST_ANY", 0) / m["SQ_WAVE_CYCLES"], 4)
    res[arm] = m
print(json.dumps(res, indent=1, sort_keys=True))
