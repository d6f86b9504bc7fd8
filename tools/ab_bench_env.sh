#!/bin/bash
# Interleaved bench runs (N = 1, the driver's --steps 20 --warmup 5) for
# environment arms: ARM = "name:VAR=value ...".  One process per run.
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-parity --no-cpu-baseline \
        --no-other-configs --no-bounce > gpurun_out/abe_${name}_$round.json 2> gpurun_out/abe_${name}_$round.err || exit 1
    python -c "
import json,sys; d=json.load(open('gpurun_out/abe_${name}_$round.json'))
print('$name', $round, d['value'], d['ms_per_step'], d['sustained']['value'], d['roofline']['kernel_ms_serial'])"
  done
done
