"""A/B of the DAG's node order in HBM (the kernel unchanged): the builder's
breadth-first numbering against depth-first preorder (each subtree's first
visit contiguous, so a ray's path down one subtree stays in fewer cache lines)
-- view-independent orders only.  Frames must be identical (leaf slots hold
voxel ids, which are not renumbered).  Interleaved rounds: serial two-view
launch and bench-style pipelined steps (3 streams), as tools/ab_render.py.

python tools/reorder_ab.py --depth 12 --rounds 4 --pipelined 400
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def node_levels(nodes: np.ndarray, root: int, depth: int) -> np.ndarray:
    """Level (1 = root) of every node of a level-structured 1-based DAG; 0 = unreachable."""
    lvl = np.zeros(nodes.shape[0] + 1, np.int32)
    front = np.array([root], np.int64)
    for L in range(1, depth + 1):
        lvl[front] = L
        if L == depth:
            break
        ch = nodes[front - 1].reshape(-1)
        ch = np.unique(ch[ch != 0]).astype(np.int64)
        front = ch
    return lvl


def dfs_order(nodes: np.ndarray, root: int, depth: int) -> np.ndarray:
    """new_id[old] (1-based) in depth-first preorder, children in slot order."""
    lvl = node_levels(nodes, root, depth)
    n = nodes.shape[0]
    new_id = np.zeros(n + 1, np.uint32)
    nxt = 1
    stack = [root]
    nl = nodes.tolist()
    lv = lvl.tolist()
    while stack:
        v = stack.pop()
        if new_id[v]:
            continue
        new_id[v] = nxt
        nxt += 1
        if lv[v] < depth:
            for c in reversed(nl[v - 1]):
                if c and not new_id[c]:
                    stack.append(c)
    return new_id, lvl


def renumber(nodes, root, depth, new_id, lvl):
    n = nodes.shape[0]
    out = np.zeros_like(nodes)
    olds = np.nonzero(new_id[1:])[0] + 1
    interior = lvl[olds] < depth
    src = nodes[olds - 1]
    src_ren = np.where(src != 0, new_id[src.astype(np.int64)], 0).astype(np.uint32)
    out[new_id[olds] - 1] = np.where(interior[:, None], src_ren, src)
    return out[: int(new_id.max())], int(new_id[root])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pipelined", type=int, default=400)
    ap.add_argument("--cache", default="/tmp/och_terrain_cache.npz")
    ap.add_argument("--out", default="gpurun_out/reorder_ab.json")
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
        t = ort.build_terrain(a.depth, use_gpu=True)
        nodes, root = t.nodes, t.root
        np.savez(cache, nodes=nodes, root=root, depth=a.depth)
    t0 = time.time()
    new_id, lvl = dfs_order(nodes, root, a.depth)
    dnodes, droot = renumber(nodes, root, a.depth, new_id, lvl)
    print(json.dumps({"reorder_s": round(time.time() - t0, 1), "nodes": int(nodes.shape[0]),
                      "dfs_nodes": int(dnodes.shape[0])}), flush=True)
    pal = ort.VoxelData().get_colours()
    W, H = 1920, 1080
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in (0.0, -0.6)]
    arms = {"bfs": (nodes, root), "dfs": (dnodes, droot)}
    pools, frames = {}, {}
    stream = torch.cuda.current_stream()
    for k, (nd, rt) in arms.items():
        p = ort.HOctree(nd, rt, a.depth, device=0)
        p.set_palette(pal)
        p.set_stream(stream)
        p.set_option("tile_order", 2)
        p.plan_views(cams, 8, 0, 1)
        pools[k] = p
        frames[k] = torch.zeros((2, H, W), dtype=torch.int32, device="cuda")
    streams = [stream] + [torch.cuda.Stream() for _ in range(2)]
    sfs = {}
    for k, p in pools.items():
        sfs[k] = []
        for s_ in streams:
            with torch.cuda.stream(s_):
                sfs[k].append(ShardedFrame(p, W, H, 8, n_views=2, direct=True))
        p.set_stream(stream)
    lat = {k: [] for k in arms}
    wall = {k: [] for k in arms}
    for r in range(a.rounds + 1):
        for k, p in pools.items():
            p.set_stream(stream)
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                p.render_views_dev(cams, frames[k], 8, 0, 1)
                e1.record(stream)
                torch.cuda.synchronize()
                if r:
                    lat[k].append(e0.elapsed_time(e1))
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for i in range(a.pipelined):
                p.set_stream(streams[i % 3])
                with torch.cuda.stream(streams[i % 3]):
                    sfs[k][i % 3].render(cams)
            torch.cuda.synchronize()
            if r:
                wall[k].append(time.perf_counter() - t1)
            p.set_stream(stream)
    same = bool(torch.equal(frames["bfs"], frames["dfs"]))
    res = []
    for k in arms:
        row = {"order": k, "serial_us_median": round(float(np.median(lat[k])) * 1e3, 1),
               "pipelined_mrays_s": round(2 * W * H * a.pipelined / float(np.median(wall[k])) / 1e6, 1),
               "frames_identical": same}
        print(json.dumps(row), flush=True)
        res.append(row)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))
    for p in pools.values():
        p.close()


if __name__ == "__main__":
    main()
