"""Dump raw per-wave stamps of the render kernel (block 64: wave index = tile
index) for later analysis against per-ray iteration counts."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import torch
    import octree_ray_tracing_amd as ort
    torch.cuda.set_device(0)
    depth = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    tree = ort.build_terrain(depth)
    pool = ort.HOctree(tree.nodes, tree.root, depth, device=0)
    pool.set_palette(ort.VoxelData().get_colours())
    pool.set_stream(torch.cuda.current_stream())
    pool.set_option("block", 64)
    out = {}
    frame = torch.empty(1920 * 1080, dtype=torch.int32, device="cuda")
    stamps = torch.zeros((1 << 16) * 4, dtype=torch.int64, device="cuda")
    for pitch in (0.0, -0.6):
        cam = ort.camera((1.5, 1.5, 1.5), 0.3, pitch, 1.25, 1920, 1080)
        for layout in (0, 1):
            pool.set_option("layout", layout)
            for _ in range(3):
                pool.render_dev(cam, frame)
            stamps.zero_()
            pool.set_stamp_buffer(stamps, 1 << 16)
            pool.render_dev(cam, frame)
            ms = pool.last_kernel_ms()
            pool.set_stamp_buffer(None, 0)
            out[f"p{pitch}_l{layout}"] = stamps.cpu().numpy().reshape(-1, 4)[:32400 + 240]
            out[f"ms_p{pitch}_l{layout}"] = np.array([ms])
            print(pitch, layout, ms, flush=True)
    np.savez_compressed("gpurun_out/stamps_d%d.npz" % depth, **out)


if __name__ == "__main__":
    main()
