"""What a lone two-view render launch ends on (design tool, not product).

One render of the bench's two views (depth 12, 1920x1080, pitch 0 / -0.6) with
per-wave stamps, in natural tile order (dispatch index = tile) and in the
planned order the bench uses, plus the walked PUSH count of every ray (the
product kernel's own count, OCH_OPT_CULL = 2).  Prints, per order: the span,
when the bulk of the waves has ended, and the longest waves with their
tile's longest lane; and over all tiles the wave lifetime against that lane's
PUSH count (ns per PUSH of the longest lane).

python tools/tail_probe.py [--out gpurun_out/tail_probe.npz]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

W, H = 1920, 1080


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/tail_probe.npz")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE")
    a = ap.parse_args()
    import torch
    import octree_ray_tracing_amd as ort

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    tree = ort.build_terrain(12, use_gpu=True)
    pool = ort.HOctree(tree.nodes, tree.root, 12, device=0)
    pool.set_palette(ort.VoxelData().get_colours())
    pool.set_stream(torch.cuda.current_stream())
    for kv in a.opt:
        k, v = kv.split("=")
        pool.set_option(k, int(v))
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in (0.0, -0.6)]
    # walked PUSHes per ray, tile-major: [view][tile][lane]
    o = torch.tensor([1.5, 1.5, 1.5], dtype=torch.float32, device=dev)
    d = torch.empty(W * H * 3, dtype=torch.float32, device=dev)
    hd, hv, hp = (torch.empty(W * H, dtype=torch.int32, device=dev) for _ in range(3))
    ht = torch.empty(W * H, dtype=torch.float32, device=dev)
    cull = pool.get_option("cull")
    push = []
    for cam in cams:
        pool.raygen_dev(cam, d)
        pool.set_option("cull", 2)
        pool.trace_batch_dev(o, d, hd, hv, ht, hp)
        torch.cuda.synchronize()
        push.append(hp.cpu().numpy().reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64))
    pool.set_option("cull", cull)
    push = np.concatenate(push)                        # tiles of view 0, then view 1: the render's tile order
    tile_max = push.max(1)
    frames = torch.empty(2 * W * H, dtype=torch.int32, device=dev)
    cap = 1 << 17
    stamps = torch.zeros(cap * 4, dtype=torch.int64, device=dev)
    out, saved = {}, {"push": push.astype(np.int16)}
    for label, order in (("natural", 0), ("planned", 2)):
        pool.set_option("tile_order", order)
        if order == 2:
            pool.plan_views(cams, 8, 0, 1)
        for _ in range(3):
            pool.render_views_dev(cams, frames, 8)
        kms = []
        for _ in range(5):
            pool.render_views_dev(cams, frames, 8)
            kms.append(pool.last_kernel_ms())
        stamps.zero_()
        pool.set_stamp_buffer(stamps, cap)
        pool.render_views_dev(cams, frames, 8)
        ms = pool.last_kernel_ms()
        pool.set_stamp_buffer(None, 0)
        st = stamps.cpu().numpy().reshape(-1, 4)[: len(tile_max)].astype(np.int64)
        t0 = st[:, 0].min()
        start, end = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0     # us (100 MHz)
        life = end - start
        res = {"kernel_ms_median_of_5": round(float(np.median(kms)), 4), "kernel_ms_stamped": round(ms, 4),
               "span_us": round(float(end.max()), 1),
               "waves_ended_by_us": {q: round(float(np.percentile(end, q)), 1) for q in (50, 90, 99, 99.9, 100)}}
        if order == 0:
            # natural order: the stamp of dispatch index i is tile i
            lm = tile_max
            slow = np.argsort(-life)[:12]
            res["longest_waves"] = [{"tile": int(i), "start_us": round(float(start[i]), 1),
                                     "life_us": round(float(life[i]), 1), "tile_max_push": int(lm[i])}
                                    for i in slow]
            big = lm >= 100
            res["ns_per_push_of_longest_lane"] = {
                "tiles_max_ge_100": int(big.sum()),
                "median": round(float(np.median(life[big] * 1e3 / lm[big])), 1),
                "p10_p90": [round(float(x), 1) for x in np.percentile(life[big] * 1e3 / lm[big], [10, 90])]}
            late = end > np.percentile(end, 99)
            res["last_1pct_waves_tile_max_push_median"] = int(np.median(lm[late]))
            saved["life_natural"] = life.astype(np.float32)
            saved["start_natural"] = start.astype(np.float32)
        else:
            saved["life_planned"] = life.astype(np.float32)
            saved["start_planned"] = start.astype(np.float32)
        out[label] = res
    s = np.sort(tile_max)[::-1]
    out["tile_max_push"] = {"top": s[:10].tolist(), "p99.9": int(s[len(s) // 1000]), "p99": int(s[len(s) // 100]),
                            "tiles_over_300": int((s > 300).sum()), "tiles_over_200": int((s > 200).sum())}
    print(json.dumps(out), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(a.out, **saved)
    pool.close()


if __name__ == "__main__":
    main()
