"""Host cost of one N > 1 bench step's collective issue (diagnostic).

At N = 8 a rank's step lasts ~0.08 ms on the GPU (tools/proxy_rank.py), and
every step issues one `dist.all_gather_into_tensor` from Python.  If issuing it
costs the host as long as the GPU step, the host, not the GPU, sets the pace --
something the one-GPU proxy (which writes the gathered buffer on the device)
cannot see.  This times the issue of the same call on a world-size-1 RCCL group
(the host path is the same; the copy is local), on the bench's frame streams,
with the N = 8 slice size (2 views x 272 rows x 3840 bytes).  It also times
the library's own communicator (och_comm_all_gather, the exchange that
och_gpu_render_sharded_steps_dev issues natively), called from Python here, so
the figure is an upper bound of the native loop's per-frame collective issue.

Run: python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1
     --master-port 29561 tools/nccl_host_cost.py
"""
import json
import os
import time

import torch
import torch.distributed as dist


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    world = dist.get_world_size()
    rows = 272
    sl = torch.zeros((2, rows, 3840), dtype=torch.uint8, device=dev)
    gathered = torch.empty((world, 2, rows, 3840), dtype=torch.uint8, device=dev)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream(device=dev) for _ in range(5)]
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import octree_ray_tracing_amd as ort
    comm = ort.RcclComm.from_process_group()
    out = {}
    for label, use_streams in (("current stream", False), ("six frame streams", True)):
        for rep in range(3):
            n = 200
            for k in range(20):
                comm.all_gather(sl, gathered, streams[k % len(streams)] if use_streams else streams[0])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(n):
                comm.all_gather(sl, gathered, streams[k % len(streams)] if use_streams else streams[0])
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            out.setdefault("library comm, " + label, []).append(
                {"issue_us_per_call": round((t1 - t0) / n * 1e6, 2), "wall_us_per_call": round((t2 - t0) / n * 1e6, 2)})
    comm.close()
    for label, use_streams in (("current stream", False), ("six frame streams", True)):
        for rep in range(3):
            n = 200
            for k in range(20):                                   # warm-up
                dist.all_gather_into_tensor(gathered, sl)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(n):
                if use_streams:
                    with torch.cuda.stream(streams[k % len(streams)]):
                        dist.all_gather_into_tensor(gathered, sl)
                else:
                    dist.all_gather_into_tensor(gathered, sl)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            out.setdefault(label, []).append({"issue_us_per_call": round((t1 - t0) / n * 1e6, 2),
                                              "wall_us_per_call": round((t2 - t0) / n * 1e6, 2)})
    if dist.get_rank() == 0:
        print(json.dumps({"world": world, "slice_bytes": sl.numel(), "calls": out}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
