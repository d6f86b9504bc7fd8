#!/bin/bash
# Rehearsal of bench.py's N = 8 path (the driver's 8-GPU run) on a one-GPU box:
# eight ranks share the GPU, collectives go through gloo on the host
# (OCH_DIST_BACKEND=gloo).  Not a scaling measurement: the run checks that the
# N = 8 settings (six frames in flight, costliest-first plan, the display
# rank's row deal, padded slices, per-rank times, parity on rank 0) run end to
# end at world size 8.  --hw-queues 2 keeps the eight processes' hardware
# queues on the one GPU at 16 (the driver's run gives each rank its own GPU and 8).
# Extra arguments go to bench.py (e.g. --display-weight 0.5, the deal of the
# driver's RCCL gather at N = 8; gloo itself always all-gathers).
set -o pipefail
O=gpurun_out/rehearse_n8; mkdir -p $O
OCH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29557 bench.py --gpus 8 --steps 5 --warmup 2 --no-cpu-baseline --sustain 0.3 \
    --hw-queues 2 "$@" > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
