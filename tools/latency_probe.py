"""Serial latency of the longest rays: the frame time of the render kernel is
set by a handful of grazing rays (hundreds of PUSHes each), so this times
those rays alone on an idle GPU -- one ray, its 8x8 tile, and the full frame
-- per layout, and reports microseconds per ray and nanoseconds per PUSH.

python tools/latency_probe.py [--depth 12]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

WORST = {-0.6: [(657, 176), (663, 166)], 0.0: [(1064, 189), (1062, 192)]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--blocks", type=int, nargs="*", default=[64, 256])
    ap.add_argument("--out", default="gpurun_out/latency.json")
    ap.add_argument("--cache", default="/tmp/och_terrain_cache.npz", help="terrain cache shared by runs in one call")
    a = ap.parse_args()

    import torch
    import octree_ray_tracing_amd as ort

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    cache = Path(a.cache)
    if cache.exists() and int(np.load(cache)["depth"]) == a.depth:
        z = np.load(cache)
        nodes, root = z["nodes"], int(z["root"])
    else:
        tree = ort.build_terrain(a.depth, use_gpu=True)
        nodes, root = tree.nodes, tree.root
        np.savez(cache, nodes=nodes, root=root, depth=a.depth)
    pool = ort.HOctree(nodes, root, a.depth, device=0)
    pool.set_palette(ort.VoxelData().get_colours())
    stream = torch.cuda.current_stream()
    pool.set_stream(stream)
    o = torch.tensor([1.5, 1.5, 1.5], dtype=torch.float32, device=dev)
    res = {}

    def timed(fn):
        fn()
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        return float(np.median(ms))

    cams2 = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, 1920, 1080) for p in WORST]
    both = torch.empty(2 * 1920 * 1080, dtype=torch.int32, device=dev)
    for layout in (0, 1):
        pool.set_option("layout", layout)
        for block in a.blocks:
            pool.set_option("block", block)
            res[f"render2_layout{layout}_block{block}_us"] = round(timed(lambda: pool.render_views_dev(cams2, both)) * 1e3, 1)
    print(json.dumps({k: v for k, v in res.items()}), flush=True)
    for pitch, pix in WORST.items():
        cam = ort.camera((1.5, 1.5, 1.5), 0.3, pitch, 1.25, 1920, 1080)
        rays_dev = torch.empty(1920 * 1080 * 3, dtype=torch.float32, device=dev)
        pool.raygen_dev(cam, rays_dev)           # the reference's raygen, bit-exact (och_gpu_raygen_dev)
        rays = rays_dev.cpu().numpy().reshape(-1, 3)
        frame = torch.empty(1920 * 1080, dtype=torch.int32, device=dev)
        for layout in (0, 1):
            pool.set_option("layout", layout)
            for block in a.blocks:
                pool.set_option("block", block)
                row = {}
                for (y, x) in pix:
                    d = torch.from_numpy(rays[y * 1920 + x].copy()).to(dev)
                    hd = torch.empty(1, dtype=torch.int32, device=dev)
                    hv = torch.empty(1, dtype=torch.int32, device=dev)
                    ht = torch.empty(1, dtype=torch.float32, device=dev)
                    hp = torch.empty(1, dtype=torch.int32, device=dev)
                    pool.trace_batch_dev(o, d, hd, hv, ht, hp, n=1)
                    torch.cuda.synchronize()
                    push = int(hp.item())
                    ms = timed(lambda: pool.trace_batch_dev(o, d, hd, hv, ht, n=1))
                    row[f"ray_{y}_{x}"] = {"push": push, "us": round(ms * 1e3, 1),
                                           "ns_per_push": round(ms * 1e6 / push, 1)}
                    # the same ray in every lane of one wave, and in 8 waves (one per XCD: warm L2s)
                    for copies in (64, 512):
                        dc = d.repeat(copies)
                        hc = [torch.empty(copies, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.float32)]
                        row[f"ray_{y}_{x}_x{copies}_us"] = round(timed(lambda: pool.trace_batch_dev(o, dc, *hc, n=copies)) * 1e3, 1)
                    # its 8x8 tile alone (64 rays)
                    ty, tx = y // 8 * 8, x // 8 * 8
                    tile = np.ascontiguousarray(rays.reshape(1080, 1920, 3)[ty:ty + 8, tx:tx + 8].reshape(-1, 3))
                    dt = torch.from_numpy(tile).to(dev)
                    h64 = [torch.empty(64, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.float32)]
                    row[f"tile_{ty}_{tx}_us"] = round(timed(lambda: pool.trace_batch_dev(o, dt, *h64, n=64)) * 1e3, 1)
                row["frame_render_us"] = round(timed(lambda: pool.render_dev(cam, frame)) * 1e3, 1)
                key = f"pitch{pitch}_layout{layout}_block{block}"
                res[key] = row
                print(key, json.dumps(row), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))
    pool.close()


if __name__ == "__main__":
    main()
