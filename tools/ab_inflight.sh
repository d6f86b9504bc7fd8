#!/bin/bash
# Frames in flight and tile shape: bench.py (no CPU leg) per setting.
set -o pipefail
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
for n in 2 3 4 6; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity --no-bounce --inflight $n > gpurun_out/bi_$n.json 2> gpurun_out/bi_$n.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bi_$n.json'));print('inflight $n', d['value'], d['sustained']['value'], d['ms_per_step'])"
done
for v in def tw16 tw4; do
  OCH_GPU_LIB=build_variants/liboch_gpu_$v.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity --no-bounce > gpurun_out/bt_$v.json 2> gpurun_out/bt_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bt_$v.json'));print('tile $v', d['value'], d['sustained']['value'], d['roofline']['kernel_ms_serial'])"
done
