"""Render launches whose rays are all culled (the camera looking up, every
ray proven to miss the voxels' box) next to the bench's two views, for a PMC
pass: the VALU per wave of a wave that only sets up and culls its rays is the
most any skip of whole sky waves could save.

rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU -d gpurun_out/sky -o run -- python tools/sky_cost.py
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import torch
    import octree_ray_tracing_amd as ort

    torch.cuda.set_device(0)
    cache = Path("/tmp/och_terrain_cache.npz")
    if cache.exists() and int(np.load(cache)["depth"]) == 12:
        z = np.load(cache)
        nodes, root = z["nodes"], int(z["root"])
    else:
        tree = ort.build_terrain(12, use_gpu=True)
        nodes, root = tree.nodes, tree.root
        np.savez(cache, nodes=nodes, root=root, depth=12)
    pool = ort.HOctree(nodes, root, 12, device=0)
    pool.set_palette(ort.VoxelData().get_colours())
    pool.set_stream(torch.cuda.current_stream())
    W, H = 1920, 1080
    codes = torch.empty(2 * W * H, dtype=torch.uint8, device="cuda")
    for pitches in ((1.2, 1.2), (0.0, -0.6)):          # all sky, then the bench's views
        cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in pitches]
        for _ in range(3):
            pool.render_codes_views_dev(cams, codes, 8, 0, 1)
        torch.cuda.synchronize()
        print(pitches, "codes", np.bincount(codes.cpu().numpy(), minlength=256)[-3:].tolist(), flush=True)
    pool.close()


if __name__ == "__main__":
    main()
