# round 3: the N >= 8 defaults (6 frames in flight, 8 hardware queues) exercised at N = 2 (gloo on
# one GPU, explicit flags; the N = 8 run itself is the driver's), and the N = 1 bench
set -o pipefail
O=gpurun_out/r03aa; mkdir -p $O
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
OCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29556 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
    --inflight 6 --hw-queues 8 > $O/rehearse_n2_f6q8.json 2> $O/rehearse_n2_f6q8.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 2
