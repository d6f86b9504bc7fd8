"""Per-node voxel bounding boxes of the packed DAG, and tools/skip_sim.c over them
(an exact per-node skip, priced before building).

python tools/skip_model.py --nodes nodes.npy --root 1 --depth 12 [--q 16]
(raw 1-based nodes; e.g. np.save of ort.build_terrain(12).nodes)
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def node_levels(pk, proot, depth):
    level = np.zeros(pk.shape[0], np.uint8)
    frontier = np.array([proot & 0xFFFFFF])
    level[frontier] = 1
    for lv in range(2, depth + 1):
        ch = pk[frontier]
        frontier = np.unique((ch & 0xFFFFFF)[ch != 0])
        level[frontier] = lv
    return level


def node_boxes(pk, level, depth):
    """[lo, hi) of the voxels under each node, voxel units relative to the node's corner."""
    n = pk.shape[0]
    lo = np.full((n, 3), 1 << 30, np.int64)
    hi = np.full((n, 3), -1, np.int64)
    off = np.array([[c & 1, (c >> 1) & 1, (c >> 2) & 1] for c in range(8)], np.int64)
    for lv in range(depth, 0, -1):
        ids = np.nonzero(level == lv)[0]
        half = 1 << (depth - lv)                      # child size in voxels
        for c in range(8):
            w = pk[ids, c]
            present = w != 0
            if lv == depth:
                clo = np.zeros((ids.size, 3), np.int64) + off[c]
                chi = clo + 1
            else:
                cid = (w & 0xFFFFFF).astype(np.int64)
                clo = lo[cid] + off[c] * half
                chi = hi[cid] + off[c] * half
            sel = ids[present]
            lo[sel] = np.minimum(lo[sel], clo[present])
            hi[sel] = np.maximum(hi[sel], chi[present])
    return lo, hi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", required=True)
    ap.add_argument("--root", type=int, default=1)
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--q", type=int, default=16)
    ap.add_argument("--qxy", type=int, default=None, help="coarser x / y quantisation (a multiple of --q's divisor); "
                    "1 = the whole cell (z-only boxes)")
    ap.add_argument("--min-level", type=int, default=2)
    ap.add_argument("--work", default="/tmp/skip_model")
    a = ap.parse_args()
    import octree_ray_tracing_amd as ort
    nodes = np.load(a.nodes)
    pk, proot = ort.pack_pool(nodes, a.root, a.depth)
    level = node_levels(pk, proot, a.depth)
    lo, hi = node_boxes(pk, level, a.depth)
    size = (1 << (a.depth - level.astype(np.int64) + 1))[:, None]          # node cell size in voxels
    qlo = np.floor(lo * a.q / size).clip(0, a.q).astype(np.int64)
    qhi = np.ceil(hi * a.q / size).clip(0, a.q).astype(np.int64)
    if a.qxy:                                   # x and y at a coarser grid, expressed in 1/q units
        f = a.q // a.qxy
        qlo[:, :2] = (qlo[:, :2] // f) * f
        qhi[:, :2] = -((-qhi[:, :2]) // f) * f
    qlo, qhi = qlo.astype(np.uint8), qhi.astype(np.uint8)
    qlo[level == 0] = 0
    qhi[level == 0] = a.q
    w = Path(a.work)
    w.mkdir(parents=True, exist_ok=True)
    pk.astype(np.uint32).tofile(w / "packed.bin")
    level.tofile(w / "levels.bin")
    np.concatenate([qlo, qhi], axis=1).astype(np.uint8).tofile(w / "boxes.bin")
    full = ((qlo == 0).all(1) & (qhi == a.q).all(1) & (level > 0)).mean()
    print(json.dumps({"nodes": int((level > 0).sum()), "boxes_full_cell_frac": round(float(full), 4)}), flush=True)
    exe = "/tmp/skip_sim"
    subprocess.run(["gcc", "-O2", "-msse2", "-o", exe, str(ROOT / "tools" / "skip_sim.c"), "-lm", "-lpthread"],
                   check=True)
    for pitch in (0.0, -0.6, 99.0):        # 99 = 2 M random rays (origins inside, any direction)
        subprocess.run([exe, str(w / "packed.bin"), str(w / "levels.bin"), str(w / "boxes.bin"), str(a.depth),
                        str(proot & 0xFFFFFF), str(a.q), str(pitch), str(a.min_level)], check=True)


if __name__ == "__main__":
    main()
