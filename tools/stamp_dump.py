"""Dump raw per-wave stamps {start, end, hw ids, rays} of the bench's
two-view render launch (block 64: one wave per 8x8 tile) and print a
timeline summary: bulk finish, tail length, the longest waves.

python tools/stamp_dump.py [depth] [extra option json]
"""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def summary(st):
    s = st[st[:, 1] > 0].astype(np.int64)
    t0 = s[:, 0].min()
    start, end = (s[:, 0] - t0) / 100.0, (s[:, 1] - t0) / 100.0
    life = end - start
    order = np.argsort(-life)[:8]
    return {"waves": int(len(s)), "span_us": round(float(end.max()), 1),
            "end_p50_p90_p99_p999_us": [round(float(x), 1) for x in np.percentile(end, [50, 90, 99, 99.9])],
            "start_p50_p99_max_us": [round(float(x), 1) for x in np.percentile(start, [50, 99, 100])],
            "life_p50_p99_max_us": [round(float(x), 1) for x in np.percentile(life, [50, 99, 100])],
            "longest": [[int(i), round(float(start[i]), 1), round(float(life[i]), 1)] for i in order]}


def main():
    import torch
    import octree_ray_tracing_amd as ort
    torch.cuda.set_device(0)
    depth = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    opts = json.loads(sys.argv[2]) if len(sys.argv) > 2 else {}
    cache = Path("/tmp/och_terrain_cache.npz")
    if cache.exists() and int(np.load(cache)["depth"]) == depth:
        z = np.load(cache)
        nodes, root = z["nodes"], int(z["root"])
    else:
        tree = ort.build_terrain(depth, use_gpu=True)
        nodes, root = tree.nodes, tree.root
        np.savez(cache, nodes=nodes, root=root, depth=depth)
    pool = ort.HOctree(nodes, root, depth, device=0)
    pool.set_palette(ort.VoxelData().get_colours())
    pool.set_stream(torch.cuda.current_stream())
    for k, v in opts.items():
        pool.set_option(k, v)
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, 1920, 1080) for p in (0.0, -0.6)]
    frames = torch.empty(2 * 1920 * 1080, dtype=torch.int32, device="cuda")
    cap = 1 << 17
    stamps = torch.zeros(cap * 4, dtype=torch.int64, device="cuda")
    for _ in range(3):
        pool.render_views_dev(cams, frames)
    stamps.zero_()
    pool.set_stamp_buffer(stamps, cap)
    pool.render_views_dev(cams, frames)
    ms = pool.last_kernel_ms()
    pool.set_stamp_buffer(None, 0)
    st = stamps.cpu().numpy().reshape(-1, 4)
    out = {"kernel_ms": ms, "opts": opts, **summary(st)}
    print(json.dumps(out), flush=True)
    np.savez_compressed("gpurun_out/stamps_d%d.npz" % depth, stamps=st[:70000])


if __name__ == "__main__":
    main()
