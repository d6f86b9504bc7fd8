"""Mean per-dispatch SQ counters of the render kernel from tools/pmc_sq.sh output.
python tools/pmc_show.py gpurun_out/pmc_<variant> ..."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if "CameraSource" in r["Kernel_Name"] and "Bounce" not in r["Kernel_Name"]:
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        for cs in per.values():
            for c, x in cs.items():
                acc[c].append(x)
    print(d, "  ".join(f"{c}={sum(x) / len(x) / 64800:.0f}" for c, x in sorted(acc.items())), "(per wave)")
