#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box: two ranks share the
# GPU, collectives go through gloo on the host (OCH_DIST_BACKEND=gloo).  The
# numbers are not a scaling measurement; the run checks that the sharded
# frame, the exchange, the timing and the JSON line work at world size 2.
set -o pipefail
mkdir -p gpurun_out
OCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/rehearse_n2.json 2> gpurun_out/rehearse_n2.err || { tail -20 gpurun_out/rehearse_n2.err; exit 1; }
cut -c1-400 gpurun_out/rehearse_n2.json
