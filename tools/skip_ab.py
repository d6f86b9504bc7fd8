"""Interleaved A/B of the per-node voxel-box skip (OCH_OPT_SKIP) by ray set.

DESIGN.md §4c measures the skip on the bench's frames (slower).  This times
och_gpu_trace_batch_tiled_dev / och_gpu_trace_batch_dev launches, skip off and
on in alternation, over ray sets whose walks differ: the bench's two camera
views at depth 12, rays from random interior origins in random directions, and
a sparse scene at depth 14 -- a few hundred solid blobs floating in empty
space (an asteroid field), where most occupied nodes hold a small box of voxels.
Deeper terrains do not fit the packed layout's 24-bit ids, and the skip needs
it.  Records are compared between the arms (the skip is exact;
tests/test_gpu_skip.py checks both against the oracle).

python tools/skip_ab.py [--reps 20] [--out gpurun_out/skip_ab.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

ORIGIN = (1.5, 1.5, 1.5)
YAW, FOV, PITCHES = 0.3, 1.25, (0.0, -0.6)
W, H = 1920, 1080


def blob_scene(depth: int, n_blobs: int = 600, radius: int = 8, seed: int = 7):
    """A 1-based hash-consed pool of n_blobs solid balls (voxel id 1..4) at
    random centres; child index x | y << 1 | z << 2."""
    rng = np.random.default_rng(seed)
    size = 1 << depth
    r = np.arange(-radius, radius + 1)
    dx, dy, dz = np.meshgrid(r, r, r, indexing="ij")
    ball = np.stack([dx, dy, dz], -1)[dx * dx + dy * dy + dz * dz <= radius * radius]
    centres = rng.integers(radius, size - radius, (n_blobs, 3))
    vox = {}
    for b, c in enumerate(centres):
        for x, y, z in (ball + c):
            vox[(int(x), int(y), int(z))] = 1 + b % 4
    table, nodes = {}, []

    def intern(children, lvl):
        key = (lvl, tuple(children))
        if key not in table:
            nodes.append(children)
            table[key] = len(nodes)
        return table[key]

    cells = {}
    for (x, y, z), v in vox.items():
        cells.setdefault((x >> 1, y >> 1, z >> 1), [0] * 8)[(x & 1) | (y & 1) << 1 | (z & 1) << 2] = v
    ids = {k: intern(c, 0) for k, c in cells.items()}
    for lvl in range(1, depth):
        up = {}
        for (x, y, z), i in ids.items():
            up.setdefault((x >> 1, y >> 1, z >> 1), [0] * 8)[(x & 1) | (y & 1) << 1 | (z & 1) << 2] = i
        ids = {k: intern(c, lvl) for k, c in up.items()}
    return np.array(nodes, np.uint32), ids[(0, 0, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/skip_ab.json")
    a = ap.parse_args()

    import torch
    import octree_ray_tracing_amd as ort

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    out = []
    for scene, depth in (("terrain", 12), ("blobs", 14)):
        if scene == "terrain":
            tree = ort.build_terrain(depth, use_gpu=True)
            nodes, root = tree.nodes, tree.root
        else:
            nodes, root = blob_scene(depth)
        pool = ort.HOctree(nodes, root, depth, device=0)
        assert pool.get_option("layout") == 1, "the skip needs the packed layout"
        pool.set_stream(stream)
        n_px = W * H
        cams = torch.empty(2 * n_px * 3, dtype=torch.float32, device=dev)
        for v, p in enumerate(PITCHES):
            pool.raygen_dev(ort.camera(ORIGIN, YAW, p, FOV, W, H), cams[v * n_px * 3:(v + 1) * n_px * 3])
        o_cam = torch.tensor(ORIGIN, dtype=torch.float32, device=dev)
        g = torch.Generator(device="cpu").manual_seed(depth)
        n_rand = 2 * n_px
        o_rand = (1.01 + 0.98 * torch.rand(n_rand, 3, generator=g)).to(dev).reshape(-1).contiguous()
        d_rand = torch.rand(n_rand, 3, generator=g) * 2 - 1
        d_rand = (d_rand / d_rand.norm(dim=1, keepdim=True)).to(dev).reshape(-1).contiguous()
        sets = [("camera_tiled", o_cam, cams, True), ("random", o_rand, d_rand, False)]
        for name, o, d, tiled in sets:
            n = d.numel() // 3
            bufs = {s: (torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
                        torch.empty(n, dtype=torch.float32, device=dev)) for s in (0, 1)}

            def launch(skip):
                pool.set_option("skip", skip)
                hd, hv, ht = bufs[skip]
                if tiled:
                    pool.trace_batch_tiled_dev(o, d, W, hd, hv, ht, n=n)
                else:
                    pool.trace_batch_dev(o, d, hd, hv, ht)

            for skip in (0, 1, 0, 1):          # warm-up, boxes built on first use
                launch(skip)
            torch.cuda.synchronize()
            ms = {0: [], 1: []}
            for _ in range(a.reps):
                for skip in (0, 1):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    launch(skip)
                    e1.record(stream)
                    ms[skip].append((e0, e1))
            torch.cuda.synchronize()
            med = {s: float(np.median([x.elapsed_time(y) for x, y in ms[s]])) for s in (0, 1)}
            same = all(torch.equal(bufs[0][i], bufs[1][i]) for i in range(3))
            row = {"scene": scene, "depth": depth, "rays": name, "n": n, "ms_off": round(med[0], 4), "ms_on": round(med[1], 4),
                   "grays_off": round(n / med[0] / 1e6, 2), "grays_on": round(n / med[1] / 1e6, 2),
                   "on_over_off": round(med[1] / med[0], 3), "records_equal": bool(same)}
            print(json.dumps(row), flush=True)
            out.append(row)
        pool.close()
        del cams, o_rand, d_rand
        torch.cuda.empty_cache()
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
