#!/bin/bash
# GPU-box routine after a kernel change: parity tests, serial-latency probe,
# bench (no CPU leg).  Each step has its own time limit; a failing step ends
# the script.  Usage: bash tools/gpu_check.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-check}; shift
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
timeout -k 10 200 python -u tools/latency_probe.py --blocks 64 --out gpurun_out/lat_$TAG.json \
    > gpurun_out/lat_$TAG.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
python - "$TAG" <<'EOF'
import json, sys
tag = sys.argv[1]
d = json.load(open(f"gpurun_out/bench_{tag}.json"))
print("bench", d["value"], "Mrays/s", d["ms_per_step"], "ms/step, kernel", d["roofline"]["kernel_ms"],
      "serial kernel", d["roofline"]["kernel_ms_serial"], "| bounce", d["bounce"] and d["bounce"]["value"],
      d["bounce"] and d["bounce"]["ms_per_step"])
for line in open(f"gpurun_out/lat_{tag}.log"):
    if line.startswith("{") or line.startswith("pitch"):
        print(line.strip()[:260])
EOF
