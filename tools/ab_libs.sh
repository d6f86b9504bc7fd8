#!/bin/bash
# Interleaved A/B of whole libraries on one GPU box: R rounds, each arm once per
# round, every run a fresh bench.py process (HIP maps streams to hardware queues
# in creation order, so arms never share a process).
#   bash tools/ab_libs.sh TAG ROUNDS "BENCH ARGS" ARM [ARM ...]
# ARM is LABEL:LIB[:EXTRA BENCH ARGS], LIB a build_variants/liboch_gpu_LIB.so name
# or "default" (the in-tree library).  Outputs gpurun_out/TAG/bench_LABELr.json (r = round),
# and a one-line summary per run on stdout.  The first failing run ends it.
set -o pipefail
TAG=${1:?tag}; R=${2:?rounds}; ARGS=${3:?bench args}; shift 3
O=gpurun_out/$TAG; mkdir -p "$O"
for r in $(seq 1 "$R"); do
  for arm in "$@"; do
    label=${arm%%:*}; rest=${arm#*:}; lib=${rest%%:*}; extra=""
    [[ "$rest" == *:* ]] && extra=${rest#*:}
    if [[ "$lib" == default ]]; then unset OCH_GPU_LIB; else export OCH_GPU_LIB=build_variants/liboch_gpu_$lib.so; fi
    # shellcheck disable=SC2086
    timeout -k 10 300 python -u bench.py $ARGS $extra > "$O/bench_$label$r.json" 2> "$O/bench_$label$r.err" \
      || { echo "run $label$r failed"; tail -20 "$O/bench_$label$r.err"; exit 1; }
    python - "$O/bench_$label$r.json" "$label$r" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
s = d.get("sustained") or {}
rf = d.get("roofline") or {}
print(sys.argv[2], d["value"], s.get("value"), rf.get("kernel_ms_serial"), (d.get("parity") or {}).get("mismatches"),
      (d.get("bounce") or {}).get("ms_per_step"), flush=True)
EOF
  done
done
