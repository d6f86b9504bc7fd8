"""Timeline of bench.py's timed window (GPU box): the same 20 pipelined steps
(codes render + shade over `inflight` streams), with HIP events at each
step's render start / render end / shade end on the step's own stream and
the host time of each launch, all relative to the window's start, so the
window's fill and drain are visible next to the steady state.

    python tools/window_probe.py --steps 20 --inflight 3 --out gpurun_out/window.json
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--inflight", type=int, action="append", default=[])
    ap.add_argument("--repeat", type=int, default=5)
    ap.add_argument("--prio", action="append", default=[],
                    help="per-stream priorities for one arm, e.g. -1,0,0 (torch/HIP: lower = higher priority)")
    ap.add_argument("--split-post", action="store_true",
                    help="also time the split arm: renders over 3 streams, every exchange + shade on one "
                         "post stream, 6 frame buffer sets (a render waits only for the shade that last "
                         "read its buffers)")
    ap.add_argument("--fresh", action="store_true",
                    help="every in-flight stream a new torch stream (none is the current/null stream)")
    ap.add_argument("--cache", default="/tmp/och_terrain_cache.npz")
    ap.add_argument("--out", default="gpurun_out/window.json")
    a = ap.parse_args()

    import torch
    import octree_ray_tracing_amd as ort
    from octree_ray_tracing_amd.frame import ShardedFrame

    torch.cuda.set_device(0)
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
    pool.plan_views(cams, 8, 0, 1)
    pool.set_option("tile_order", 2)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    print("stream priority range", torch.cuda.Stream.priority_range(), flush=True)
    arms = [(n, None) for n in (a.inflight or [3])] + [(len(p.split(",")), [int(x) for x in p.split(",")])
                                                       for p in a.prio]
    if a.split_post:
        arms.append((3, "split"))
    results = []
    for inflight, prio in arms:
        split = prio == "split"
        if prio is None or split:
            streams = ([] if a.fresh else [stream]) + [torch.cuda.Stream() for _ in range(inflight - (not a.fresh))]
        else:
            streams = [torch.cuda.Stream(priority=q) for q in prio]
        post = torch.cuda.Stream() if split else None
        n_sets = 2 * inflight if split else inflight
        sfs = []
        for i in range(n_sets):
            with torch.cuda.stream(streams[i % inflight]):
                sfs.append(ShardedFrame(pool, W, H, 8, n_views=2, indexed=True))
        pool.set_stream(stream)
        freed = [None] * n_sets      # split: event after the shade that last read set i

        def step(k, marks=None):
            s_, f_ = streams[k % inflight], sfs[k % n_sets]
            pool.set_stream(s_)
            with torch.cuda.stream(s_):
                if marks is not None:
                    e = [ev(), ev(), ev()]
                    e[0].record(s_)
                if split and freed[k % n_sets] is not None:
                    s_.wait_event(freed[k % n_sets])
                f_.render_local(cams)
                if marks is not None:
                    e[1].record(s_)
                if not split:
                    f_.exchange()
                    if marks is not None:
                        e[2].record(s_)
                        marks.append(e)
                    return
                done = ev()
                done.record(s_)
            pool.set_stream(post)
            with torch.cuda.stream(post):
                post.wait_event(done)
                f_.exchange()
                fe = ev()
                fe.record(post)
                freed[k % n_sets] = fe
                if marks is not None:
                    e[2] = fe
                    marks.append(e)

        for k in range(6):
            step(k)
        torch.cuda.synchronize()
        runs = []
        for _ in range(a.repeat):
            for k in range(3):
                step(k)
            torch.cuda.synchronize()
            marks, host = [], []
            g0 = ev()
            t0 = time.perf_counter()
            g0.record(stream)
            for k in range(a.steps):
                host.append((time.perf_counter() - t0) * 1e3)
                step(k, marks)
            t_issue = (time.perf_counter() - t0) * 1e3
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3
            rows = [[round(h, 4)] + [round(g0.elapsed_time(x), 4) for x in e] for h, e in zip(host, marks)]
            runs.append({"wall_ms": round(wall, 4), "host_issue_ms": round(t_issue, 4),
                         "gpu_last_ms": max(r[3] for r in rows), "steps": rows})
        pool.set_stream(stream)
        walls = [r["wall_ms"] for r in runs]
        best = runs[int(np.argsort(walls)[len(walls) // 2])]
        res = {"inflight": inflight, "prio": prio, "steps": a.steps, "wall_ms_median": float(np.median(walls)),
               "mrays_s_median": round(2 * W * H * a.steps / float(np.median(walls)) / 1e3, 1),
               "median_run": best,
               "columns": ["host_launch_ms", "render_start_ms", "render_end_ms", "shade_end_ms"]}
        results.append(res)
        print(json.dumps({k: v for k, v in res.items() if k != "median_run"}), flush=True)
        print(" host issue %.3f ms, gpu last %.3f ms, wall %.3f ms" %
              (best["host_issue_ms"], best["gpu_last_ms"], best["wall_ms"]), flush=True)
        for i, r in enumerate(best["steps"]):
            print("  step %2d  host %.3f  render %.3f -> %.3f  shade -> %.3f" % (i, *r), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(results, indent=1))
    pool.close()


if __name__ == "__main__":
    main()
