"""Residency probe: HIP occupancy answers and measured per-CU concurrency
(from per-wave stamps) of the render kernel at several pool depths / blocks."""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def concurrency(st):
    st = st[st[:, 1] > 0]
    xcc = (st[:, 2] >> 32) & 0xF
    hw = st[:, 2] & 0xFFFFFFFF
    key = xcc * 100000 + ((hw >> 13) & 7) * 1000 + ((hw >> 12) & 1) * 100 + ((hw >> 8) & 0xF)
    peaks = []
    for k in np.unique(key):
        s = st[key == k]
        ev = np.concatenate([np.stack([s[:, 0], np.ones(len(s))], 1), np.stack([s[:, 1], -np.ones(len(s))], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        peaks.append(np.cumsum(ev[:, 1]).max())
    simd = (hw >> 4) & 3
    return {"cus": int(len(peaks)), "peak_waves_per_cu_max": int(max(peaks)), "peak_waves_per_cu_median": float(np.median(peaks)),
            "simd_ids_seen": sorted(set(simd.tolist())),
            "wave_slot_ids_seen": int(len(set((hw & 0xF).tolist())))}


def main():
    import torch
    import octree_ray_tracing_amd as ort
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    out = {}
    stamps = torch.zeros((1 << 17) * 4, dtype=torch.int64, device=dev)
    frame = torch.empty(1920 * 1080, dtype=torch.int32, device=dev)
    for depth in (4, 8, 12):
        tree = ort.build_terrain(depth, use_gpu=True)
        pool = ort.HOctree(tree.nodes, tree.root, depth, device=0)
        pool.set_palette(ort.VoxelData().get_colours())
        pool.set_stream(torch.cuda.current_stream())
        cam = ort.camera((1.5, 1.5, 1.5), 0.3, -0.6, 1.25, 1920, 1080)
        for block in (64, 256, 1024):
            pool.set_option("block", block)
            for sched, w in ((0, 0), (1, 32)):
                pool.set_option("schedule", sched)
                if sched:
                    pool.set_option("waves_per_cu", w)
                    pool.set_option("refill", 64)
                occ = pool.occupancy(1 if sched else 0)
                stamps.zero_()
                pool.set_stamp_buffer(stamps, 1 << 17)
                pool.render_dev(cam, frame)
                ms = pool.last_kernel_ms()
                pool.set_stamp_buffer(None, 0)
                st = stamps.cpu().numpy().reshape(-1, 4).astype(np.uint64)
                r = {"hip_blocks_per_cu": occ, "hip_waves_per_cu": occ * block // 64, "ms": round(ms, 4), **concurrency(st)}
                key = f"d{depth}_b{block}_{'pers' if sched else 'grid'}"
                out[key] = r
                print(key, json.dumps(r), flush=True)
        pool.close()
    Path("gpurun_out/occupancy.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
