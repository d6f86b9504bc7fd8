"""Every rank's share of an N-rank bench step, on this one GPU (no collective).

At N > 1 bench.py renders configs[3] (3840x2160, two views) split over the
ranks; each rank renders its row chunks, all-gathers the 1-byte codes, and
the display rank (or, with --shade all, every rank) shades the whole frame.
This tool times exactly that per-rank GPU work -- the render of shard s of N
and the shade of the full frame where that rank shades, with the gathered
buffer written on the device instead of over xGMI -- for every shard s
(--shards all) and several frames-in-flight settings, so the N = 2/4/8
per-rank steps, and their maximum (the driver's value takes the max over
ranks), can be measured on a 1-GPU box.  The xGMI receive time is not in it
(estimated separately in DESIGN.md §5).

python tools/proxy_rank.py --worlds 8 --inflight 3

Run one (world, inflight) arm per process: HIP maps streams onto its hardware
queues in creation order, and which streams share a queue moves the result by
20 %, so every arm must create its streams as bench.py does --
the current stream plus inflight - 1 new ones -- in a fresh process.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--inflight", default="2,3,4,6")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--windows", type=int, default=7, help="20-step windows per arm (median)")
    ap.add_argument("--sustain-steps", type=int, default=400)
    ap.add_argument("--cache", default="/tmp/och_terrain_cache.npz")
    ap.add_argument("--out", default="gpurun_out/proxy_rank.json")
    ap.add_argument("--no-exchange", action="store_true", help="render only: no gather copy, no shade")
    ap.add_argument("--events", action="store_true",
                    help="timing events on every render, recorded by its dispatch (as bench.py)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE", help="pool option, e.g. chain=1")
    ap.add_argument("--shards", default="0", help="'all', or a comma list of shards to time")
    ap.add_argument("--shade", choices=("display", "all"), default="display",
                    help="as bench.py: 'display' = only rank 0 shades the gathered frame")
    ap.add_argument("--deal", choices=("cost", "count", "rr"), default="count", help="as bench.py")
    ap.add_argument("--display-weight", type=float, default=None, help="as bench.py (default 1 - 0.05 N)")
    ap.add_argument("--shade-stream", action="store_true", help="as bench.py: the display rank shades on its own stream")
    ap.add_argument("--exchange", choices=("all_gather", "gather"), default="all_gather",
                    help="as bench.py --exchange: 'gather' = only rank 0 receives the slices, so the other ranks' "
                         "step has no receive (no gathered-buffer write)")
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
    base = torch.cuda.current_stream()
    pool.set_stream(base)
    pool.set_option("tile_order", 2)
    opts = dict(kv.split("=") for kv in a.opt)
    for k, v in opts.items():
        pool.set_option(k, int(v))
    res = []
    for world in [int(x) for x in a.worlds.split(",")]:
        W, H = (1920, 1080) if world == 1 else (3840, 2160)     # configs[2] / configs[3]
        cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in (0.0, -0.6)]
        shards = list(range(world)) if a.shards == "all" else [int(x) for x in a.shards.split(",") if int(x) < world]
        deal = None
        w0 = max(0.5, 1.0 - 0.05 * world) if a.display_weight is None else a.display_weight
        if world > 1 and a.deal != "rr":            # as bench.py: chunks dealt by cost (or count) per weight
            w = [w0 if a.shade == "display" else 1.0] + [1.0] * (world - 1)
            costs = pool.chunk_costs(cams, 8) if a.deal == "cost" else np.ones(-(-H // 8), np.float32)
            deal = ort.deal_chunks(costs, world, w)
        if world > 1:
            pool.set_row_deal(H, 8, world, deal)
        for nf in [int(x) for x in a.inflight.split(",")]:
            streams = [base] + [torch.cuda.Stream() for _ in range(nf - 1)]
            shade_stream = torch.cuda.Stream() if a.shade_stream else None
            per_shard = []
            for shard in shards:
                pool.set_stream(base)
                pool.plan_views(cams, 8, shard, world)
                row = arm(a, torch, pool, streams, cams, W, H, world, shard, nf, opts, deal, shade_stream)
                row["display_weight"] = w0
                print(json.dumps(row), flush=True)
                res.append(row)
                per_shard.append(row)
            if len(per_shard) > 1:
                summ = {"world": world, "inflight": nf, "summary": True, "shade": a.shade,
                        "shards": len(per_shard)}
                for k in ("mrays_s_rank_20", "mrays_s_rank_sustained"):
                    v = [r[k] for r in per_shard]
                    summ[k.replace("mrays_s_rank", "min")] = min(v)
                    summ[k.replace("mrays_s_rank", "max")] = max(v)
                for k in ("ms_per_step_20", "ms_per_step_sustained"):
                    v = [r[k] for r in per_shard]
                    summ["slowest_" + k] = max(v)
                    summ["spread_" + k] = round(max(v) / min(v) - 1, 4)
                # the driver's value takes the max over ranks of the step time: the whole
                # job's rays over the slowest rank's step
                rays_all = sum(r["rays_per_step_rank"] for r in per_shard)
                summ["job_mrays_s_20"] = round(rays_all / (summ["slowest_ms_per_step_20"] * 1e-3) / 1e6, 1)
                summ["job_mrays_s_sustained"] = round(rays_all / (summ["slowest_ms_per_step_sustained"] * 1e-3) / 1e6, 1)
                print(json.dumps(summ), flush=True)
                res.append(summ)
            pool.set_stream(base)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))
    pool.close()


def arm(a, torch, pool, streams, cams, W, H, world, shard, nf, opts, deal=None, shade_stream=None):
    """One shard's pipelined steps: 20-step windows (median) and sustained runs."""
    from octree_ray_tracing_amd.frame import ShardedFrame, slice_row_map
    sfs = []
    for s_ in streams:
        with torch.cuda.stream(s_):
            sfs.append(ShardedFrame(pool, W, H, 8, n_views=2, indexed=True, shard=(shard, world),
                                    shade=a.shade, deal=deal, shade_stream=shade_stream))
    rows = sfs[0].rows
    rays_rank = int((slice_row_map(H, 8, world, shard, deal) >= 0).sum()) * W * 2

    from bench import FenceFreeEvent
    evs = [(FenceFreeEvent(), FenceFreeEvent()) for _ in range(64)] if a.events else None

    def drain():
        # as bench.py: poll the streams idle, then synchronize (no interrupt wake-up)
        while not all(s_.query() for s_ in streams):
            pass
        torch.cuda.synchronize()

    def run(n):
        drain()
        t0 = time.perf_counter()
        for k in range(n):
            s_, f_ = streams[k % nf], sfs[k % nf]
            pool.set_stream(s_)
            with torch.cuda.stream(s_):
                if evs is not None:                 # as bench.py: recorded by the render's own dispatch
                    pool.set_launch_events(*evs[k % len(evs)])
                f_.render_local(cams)
                if not a.no_exchange and (a.exchange == "all_gather" or shard == 0):
                    f_.exchange()
        drain()
        return time.perf_counter() - t0

    run(5)
    wins = [run(a.steps) for _ in range(a.windows)]
    sus = [run(a.sustain_steps) for _ in range(3)]
    row = {"world": world, "shard": shard, "frame": f"{W}x{H}", "inflight": nf, "opts": opts,
           "exchange": (a.exchange if not a.no_exchange else None), "shade": a.shade, "shades": a.shade == "all" or shard == 0,
           "deal": a.deal, "shade_stream": a.shade_stream,
           "events": a.events, "rays_per_step_rank": rays_rank, "slice_rows": rows,
           "ms_per_step_20": round(statistics.median(wins) / a.steps * 1e3, 4),
           "mrays_s_rank_20": round(rays_rank * a.steps / statistics.median(wins) / 1e6, 1),
           "ms_per_step_sustained": round(statistics.median(sus) / a.sustain_steps * 1e3, 4),
           "mrays_s_rank_sustained": round(rays_rank * a.sustain_steps / statistics.median(sus) / 1e6, 1)}
    del sfs
    return row


if __name__ == "__main__":
    main()
