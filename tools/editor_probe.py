"""Editor cost probe (GPU box): adoption, first flush, windowed flushes, and
the frame time of the editor's slot-numbered pool vs the builder's
breadth-first pool on the same depth-12 tree (1920x1080, two views).

    python tools/editor_probe.py [--depth 12] [--edits 1000] --out gpurun_out/editor.json
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import octree_ray_tracing_amd as ort  # noqa: E402


def frame_ms(pool, cams, out, iters=20):
    s = torch.cuda.current_stream()
    pool.set_stream(s)
    for _ in range(100):   # warm clocks and caches
        for c, o in zip(cams, out):
            pool.render_dev(c, o)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(iters):
        for c, o in zip(cams, out):
            pool.render_dev(c, o)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--edits", type=int, default=1000)
    ap.add_argument("--out", default="gpurun_out/editor.json")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    res = {"depth": a.depth}
    t = time.perf_counter()
    tree = ort.build_terrain(a.depth, use_gpu=True)
    res["build_s"] = time.perf_counter() - t
    res["dag_nodes"] = int(tree.nodes.shape[0])
    print("built", res, flush=True)
    pal = ort.VoxelData().get_colours()
    W, H = 1920, 1080
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in (0.0, -0.6)]
    out = [torch.empty((H, W), dtype=torch.int32, device="cuda") for _ in cams]

    bfs = ort.HOctree(tree.nodes, tree.root, a.depth, device=0)
    bfs.set_palette(pal)
    res["bfs_frame_ms"] = frame_ms(bfs, cams, out)
    ref_frames = [o.cpu().numpy().copy() for o in out]

    t = time.perf_counter()
    ed = ort.Editor(tree.nodes, tree.root, a.depth, capacity=tree.nodes.shape[0] + (1 << 20))
    res["adopt_s"] = time.perf_counter() - t
    t = time.perf_counter()
    pool = ed.make_pool(device=0)
    res["make_pool_and_first_flush_s"] = time.perf_counter() - t
    pool.set_palette(pal)
    res["editor_frame_ms"] = frame_ms(pool, cams, out)
    res["frames_equal"] = all(np.array_equal(r, o.cpu().numpy()) for r, o in zip(ref_frames, out))
    print("adopted", res, flush=True)

    # edits near the camera's view of the surface: dig and place blocks
    dim = 1 << a.depth
    rng = np.random.default_rng(1)
    pts = rng.integers(dim // 4, 3 * dim // 4, (a.edits, 3))
    t = time.perf_counter()
    for i, (x, y, z) in enumerate(pts.tolist()):
        ed.set(x, y, z, 0 if i % 2 else 3)
    res["set_us_per_edit"] = (time.perf_counter() - t) / a.edits * 1e6
    st = ed.stats()
    res["dirty_slots"] = st["dirty_count"]
    t = time.perf_counter()
    ed.flush(pool)
    torch.cuda.synchronize()
    res["flush_ms"] = (time.perf_counter() - t) * 1e3
    # one edit then flush: the interactive case
    t = time.perf_counter()
    ed.set(int(pts[0, 0]), int(pts[0, 1]), int(pts[0, 2]), 2)
    ed.flush(pool)
    torch.cuda.synchronize()
    res["single_edit_flush_ms"] = (time.perf_counter() - t) * 1e3
    res["editor_frame_ms_after_edits"] = frame_ms(pool, cams, out)
    res["live_nodes"] = ed.stats()["live_nodes"]
    # measured again, interleaved, once both pools have run
    res["bfs_frame_ms_again"] = frame_ms(bfs, cams, out)
    res["editor_frame_ms_again"] = frame_ms(pool, cams, out)
    print(json.dumps(res), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
