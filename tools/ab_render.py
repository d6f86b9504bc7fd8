"""A/B timing of the two-view render launch (the bench's dominant kernel)
under option sets, interleaved round-robin so clock drift hits every arm
alike; every arm's frames must equal the first arm's bit for bit.

python tools/ab_render.py --depth 12 --arm '{}' --arm '{"tile_order": 1}'
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--arm", action="append", default=[])
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cache", default="/tmp/och_terrain_cache.npz")
    ap.add_argument("--out", default="gpurun_out/ab.json")
    ap.add_argument("--bounce", action="store_true",
                    help="time config 5 instead (codes render with one secondary ray per hit pixel)")
    ap.add_argument("--pipelined", type=int, default=0,
                    help="also time this many bench-style steps per arm and round (codes render + shade over 3 "
                         "streams in flight, as bench.py), reporting wall-clock Mrays/s")
    a = ap.parse_args()
    arms = [json.loads(x) for x in (a.arm or ["{}"])]

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
    W, H = a.width, a.height
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in (0.0, -0.6)]
    if a.bounce:
        frames = [torch.empty(2 * W * H, dtype=torch.uint8, device=dev) for _ in arms]
    else:
        frames = [torch.empty(2 * W * H, dtype=torch.int32, device=dev) for _ in arms]
    defaults = {k: pool.get_option(k) for k in pool.OPTIONS}

    def apply(arm):
        for k, v in defaults.items():
            pool.set_option(k, arm.get(k, v))

    def plan_for(arm):
        # the launch order of tile_order=2 (same geometry as below); the plan is
        # keyed by the block size and the bounce compaction, so each arm plans its own
        if arm.get("tile_order") == 2:
            pool.plan_views(cams, 8, 0, 1)

    times = [[] for _ in arms]
    for r in range(a.rounds + 1):
        for i, arm in enumerate(arms):
            apply(arm)
            plan_for(arm)
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                if a.bounce:
                    pool.render_codes_views_dev(cams, frames[i], 8, 0, 1, True)
                else:
                    pool.render_views_dev(cams, frames[i], 8, 0, 1)
                e1.record(stream)
                torch.cuda.synchronize()
                if r:
                    times[i].append(e0.elapsed_time(e1))
    import time
    from octree_ray_tracing_amd.frame import ShardedFrame
    walls = [[] for _ in arms]
    if a.pipelined:
        streams = [stream] + [torch.cuda.Stream() for _ in range(2)]
        sfs = []
        for s_ in streams:
            with torch.cuda.stream(s_):
                sfs.append(ShardedFrame(pool, W, H, 8, n_views=2, indexed=True))
        shaded = [None] * len(arms)
        for r in range(a.rounds + 1):
            for i, arm in enumerate(arms):
                apply(arm)
                plan_for(arm)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(a.pipelined):
                    pool.set_stream(streams[k % 3])
                    with torch.cuda.stream(streams[k % 3]):
                        sfs[k % 3].render(cams, a.bounce)
                torch.cuda.synchronize()
                if r:
                    walls[i].append(time.perf_counter() - t0)
                shaded[i] = sfs[(a.pipelined - 1) % 3].frames.clone()
        pool.set_stream(stream)
    res = []
    for i, arm in enumerate(arms):
        t = np.array(times[i])
        row = {"arm": arm, "median_us": round(float(np.median(t)) * 1e3, 1), "min_us": round(float(t.min()) * 1e3, 1),
               "mrays_s": round(2 * W * H / float(np.median(t)) / 1e3, 1),
               "bit_exact_vs_arm0": bool(torch.equal(frames[i], frames[0]))}
        if a.pipelined:
            w = np.array(walls[i])
            row["pipelined_mrays_s"] = round(2 * W * H * a.pipelined / float(np.median(w)) / 1e6, 1)
            row["pipelined_ms_per_step"] = round(float(np.median(w)) / a.pipelined * 1e3, 4)
            row["pipelined_bit_exact_vs_arm0"] = bool(torch.equal(shaded[i], shaded[0]))
        res.append(row)
        print(json.dumps(row), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))
    pool.close()


if __name__ == "__main__":
    main()
