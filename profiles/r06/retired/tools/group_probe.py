"""Measures cost-sorted wave assembly on the GPU (design probe, not product;
group_model.c (beside this file) prices it in the lockstep model: -13 % / -19 % of the
waves' work for 16x16 / 32x32 blocks).

The bench's two depth-12 1080p views as resident rays (och_gpu_raygen_dev),
traced through the same kernel (och_gpu_trace_batch_dev: 64 consecutive rays
per wave) in different orders of the ray array:
  tiled     one 8x8 pixel tile per wave (what the render launch walks);
  sortB     each BxB pixel block's rays sorted by their walked PUSH count
            (a counting launch of the same rays), longest first, 64 to a wave.
The records must not depend on the order (checked); the question is whether the
waves' shorter lockstep walks beat the lost coherence of their loads.  Timed
lone (one launch, idle GPU) and pipelined (launches round-robin over 3 streams).

Usage (GPU box): python profiles/r06/retired/tools/group_probe.py [--blocks 16,32] [--launches 60]"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[4]))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", default="16,32")
    ap.add_argument("--launches", type=int, default=60)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    import torch
    import octree_ray_tracing_amd as ort

    W, H = 1920, 1080
    t0 = time.time()
    tree = ort.build_terrain(12, use_gpu=True)
    pool = ort.HOctree(tree.nodes, tree.root, 12, device=0)
    print(f"[probe] tree {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    dev = torch.device("cuda", 0)
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in (0.0, -0.6)]
    dirs = torch.empty((2, H * W, 3), dtype=torch.float32, device=dev)
    for v, c in enumerate(cams):
        pool.raygen_dev(c, dirs[v])
    dirs = dirs.reshape(-1, 3)
    n = dirs.shape[0]
    origin = torch.tensor([1.5, 1.5, 1.5], dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream()
    pool.set_stream(stream)

    def outs():
        return (torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
                torch.empty(n, dtype=torch.int32, device=dev))

    # per-ray cost: PUSH tests walked (cull 2: rays the exact cull ends count 0)
    push = torch.zeros(n, dtype=torch.int32, device=dev)
    hd, hv, ht = outs()
    pool.set_option("cull", 2)
    pool.trace_batch_dev(origin, dirs, hd, hv, ht, push=push)
    torch.cuda.synchronize()
    pool.set_option("cull", 1)
    cost = push.cpu().numpy().reshape(2, H, W)
    print(f"[probe] costs: mean {cost.mean():.2f}, walking {np.mean(cost > 0):.3f}", file=sys.stderr, flush=True)

    orders = {}
    tiles = []
    for v in range(2):
        base = v * H * W
        for ty in range(0, H, 8):
            for tx in range(0, W, 8):
                yy, xx = np.mgrid[ty:ty + 8, tx:tx + 8]
                tiles.append(base + (yy * W + xx).ravel())
    orders["tiled"] = np.concatenate(tiles)
    for B in [int(x) for x in a.blocks.split(",")]:
        parts = []
        for v in range(2):
            base = v * H * W
            for by in range(0, H, B):
                for bx in range(0, W, B):
                    yy, xx = np.mgrid[by:min(by + B, H), bx:min(bx + B, W)]
                    idx = (yy * W + xx).ravel()
                    c = cost[v].ravel()[idx]
                    parts.append(base + idx[np.argsort(-c, kind="stable")])
        orders[f"sort{B}"] = np.concatenate(parts)
    # the lockstep work of each order (sum over waves of the longest lane)
    flat = cost.ravel()
    model = {k: int(flat[o].reshape(-1, 64).max(axis=1).sum()) for k, o in orders.items()}

    arms = {}
    ref = None
    for k, o in orders.items():
        assert len(o) == n and len(np.unique(o)) == n
        oi = torch.from_numpy(o.astype(np.int64)).to(dev)
        arms[k] = {"dirs": dirs[oi].contiguous(), "perm": oi, "bufs": [outs() for _ in range(3)]}
        hd, hv, ht = arms[k]["bufs"][0]
        pool.trace_batch_dev(origin, arms[k]["dirs"], hd, hv, ht)
        torch.cuda.synchronize()
        rec = torch.empty((3, n), dtype=torch.int32, device=dev)
        for j, b in enumerate((hd, hv, ht)):
            rec[j, oi] = b
        rec = rec.cpu().numpy()
        if ref is None:
            ref = rec
        arms[k]["records_equal"] = bool(np.array_equal(rec, ref))

    streams = [torch.cuda.Stream(device=dev) for _ in range(3)]
    res = {k: {"lone_ms": [], "pipelined_mrays_s": [], "model_work": model[k],
               "model_vs_tiled": round(model[k] / model["tiled"], 4), "records_equal": arms[k]["records_equal"]}
           for k in orders}
    for rnd in range(a.rounds):
        for k in orders:
            A = arms[k]
            # lone launches
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                hd, hv, ht = A["bufs"][0]
                pool.set_stream(stream)
                e0.record(stream)
                pool.trace_batch_dev(origin, A["dirs"], hd, hv, ht)
                e1.record(stream)
                torch.cuda.synchronize()
                res[k]["lone_ms"].append(round(e0.elapsed_time(e1), 4))
            # pipelined
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i in range(a.launches):
                s = streams[i % 3]
                pool.set_stream(s)
                hd, hv, ht = A["bufs"][i % 3]
                pool.trace_batch_dev(origin, A["dirs"], hd, hv, ht)
            torch.cuda.synchronize()
            el = time.perf_counter() - t
            res[k]["pipelined_mrays_s"].append(round(n * a.launches / el / 1e6, 1))
            print(f"[probe] round {rnd} {k}: {res[k]['pipelined_mrays_s'][-1]} Mrays/s", file=sys.stderr, flush=True)
    pool.set_stream(stream)
    for k in res:
        res[k]["lone_ms_median"] = float(np.median(res[k]["lone_ms"]))
    print(json.dumps({"rays": n, "arms": res}))
    pool.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
