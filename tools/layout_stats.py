"""Footprint of the packed node layout per level, and what a sparse child-list
layout would save.  Writes the table of
profiles/r04/layout_d12.txt.

python tools/layout_stats.py --depth 12 [--nodes nodes.npy --root R]
(without --nodes the terrain is built: on the GPU when one is visible)
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--nodes", default=None, help="raw 1-based nodes (.npy), e.g. a saved build")
    ap.add_argument("--root", type=int, default=1)
    a = ap.parse_args()
    import octree_ray_tracing_amd as ort
    if a.nodes:
        nodes, root = np.load(a.nodes), a.root
    else:
        import torch
        tree = ort.build_terrain(a.depth, use_gpu=torch.cuda.is_available())
        nodes, root = tree.nodes, tree.root
    pk, proot = ort.pack_pool(nodes, root, a.depth)
    level = np.zeros(pk.shape[0], np.int8)
    frontier = np.array([proot & 0xFFFFFF])
    level[frontier] = 1
    for lv in range(2, a.depth + 1):
        ch = pk[frontier]
        frontier = np.unique((ch & 0xFFFFFF)[ch != 0])
        level[frontier] = lv
    pres = (pk != 0).sum(1)
    print(f"depth-{a.depth} terrain DAG (packed layout, och_pool_pack): present child slots per node, per level")
    print("level nodes avg_present")
    for lv in range(1, a.depth + 1):
        m = level == lv
        print(lv, int(m.sum()), round(float(pres[m].mean()), 3))
    live = level > 0
    print("present slots", int(pres[live].sum()), "dense slots", int(8 * live.sum()),
          "ratio", round(float(pres[live].sum() / (8 * live.sum())), 4))
    print("24-bit word offset limit", 1 << 24)


if __name__ == "__main__":
    main()
