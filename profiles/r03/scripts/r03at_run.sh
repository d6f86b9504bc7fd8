# round 3: rocprofv3 kernel trace + PMC passes of the bench with the native window issue
set -o pipefail
O=gpurun_out/r03at; mkdir -p $O
bash tools/profile.sh r03at > $O/profile.log 2>&1 || exit 5
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29561 tools/nccl_host_cost.py > $O/nccl_host_cost.json 2> $O/nccl_host_cost.err || exit 6
