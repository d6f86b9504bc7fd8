"""Prices a two-pass walk with an iteration budget (design tool, not product).

Pass 1 walks every ray for at most B PUSHes; the rays left over are saved and
resumed in pass 2, packed 64 to a wave.  The cost model is the walk's lockstep:
a wave costs its longest lane.  Per-ray PUSH counts are the product
kernel's own (tools/push_counts.py on the GPU box: the PUSHes the default
launch walks over the bench's two views at depth 12, rays the occupied-box cull
proves to miss at 0).  Prints the PUSH-level lane utilisation of 8x8 tiles and,
per budget B, pass 1 + pass 2 against one pass, with the leftovers grouped in
tile order or (best case, before any sorting cost) by length.  DESIGN.md §9 has
the numbers.

python tools/tail_model.py profiles/r04/r04q/push_d12.npz
"""
import sys

import numpy as np


def main(path: str) -> None:
    z = np.load(path)
    H, W = z["walked_p0"].shape
    tiles = [z[k].astype(np.int64).reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
             for k in ("walked_p0", "walked_p6")]
    t = np.concatenate(tiles)
    mx, mean = t.max(1), t.mean(1)
    print("tiles", len(t), "walked PUSH per ray", round(float(t.mean()), 3),
          "utilisation (sum mean / sum max)", round(float(mean.sum() / mx.sum()), 4))
    print("longest tile, percentiles 50/90/99/99.9/100:", np.percentile(mx, [50, 90, 99, 99.9, 100]).tolist())
    base = mx.sum()
    for B in (32, 48, 64, 96, 128):
        p1 = np.minimum(mx, B).sum()
        left = t[t > B] - B
        n = left.size
        pad = np.zeros((-n) % 64, left.dtype)
        p2 = np.concatenate([left, pad]).reshape(-1, 64).max(1).sum() if n else 0
        p2s = np.concatenate([np.sort(left)[::-1], pad]).reshape(-1, 64).max(1).sum() if n else 0
        print(f"B={B}: leftover rays {n} ({n / t.size:.4f}); two passes / one: {(p1 + p2) / base:.3f} in tile "
              f"order, {(p1 + p2s) / base:.3f} sorted by length")


if __name__ == "__main__":
    main(sys.argv[1])
