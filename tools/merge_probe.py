"""One small k_trace_grid_merge launch (depth 8, 256x144, block 256, K = 2)
against the oracle: run with a short timeout before anything larger."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import torch
    import octree_ray_tracing_amd as ort
    from oracle import oracle as O
    torch.cuda.set_device(0)
    t = ort.build_terrain(8)
    pal = ort.VoxelData().get_colours()
    pool = ort.HOctree(t.nodes, t.root, 8, device=0)
    pool.set_palette(pal)
    pool.set_option("block", 256)
    pool.set_option("merge", 2)
    cam = ort.camera((1.5, 1.5, 1.5), 0.3, -0.6, 1.25, 256, 144)
    got = pool.render(cam)
    r = O.trace_batch(O.OraclePool(t.nodes, t.root, 8, 1), O.Rcp(None), np.array([1.5, 1.5, 1.5], np.float32),
                      O.raygen(0.3, -0.6, 1.25, 256, 144))
    want = O.shade(r["dir"], r["voxel"], pal).reshape(144, 256)
    print("merge probe:", "ok" if np.array_equal(got, want) else f"{int((got != want).sum())} pixels differ")


if __name__ == "__main__":
    main()
