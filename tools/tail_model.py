"""Prices a two-pass walk with an iteration budget (design tool, not product).

Pass 1 walks every ray for at most B PUSHes; the rays left over are saved and
resumed in pass 2, packed 64 to a wave.  The cost model is the walk's lockstep:
a wave costs its longest lane.  Per-ray PUSH counts come from the oracle
(oracle/och_oracle.c via oracle.py) over the bench's two views at depth 12, with
the rays the occupied-box cull proves to miss set to 0 (a float64 slab test
against och_pool_occupied_box).  Prints the PUSH-level lane utilisation of 8x8
tiles and, per budget B, pass 1 + pass 2 against one pass, with the leftovers
grouped in tile order or (best case, before any sorting cost) by length.

Needs /tmp/d12.npz (nodes, root of build_terrain(12)) and /tmp/push_d12.npz
(per-ray PUSH counts, p0 / p6) -- see DESIGN.md §9 for the numbers.
"""
import sys, numpy as np
sys.path.insert(0, '/root/repo')
import octree_ray_tracing_amd as ort
from oracle import oracle as O
z = np.load('/tmp/d12.npz'); nodes, root = z['nodes'], int(z['root'])
lo, hi = ort.occupied_box(nodes, root, 12)
lo = 1 + np.array(lo) / 4096.0; hi = 1 + np.array(hi) / 4096.0
P = np.load('/tmp/push_d12.npz')
W, H = 1920, 1080
o = np.array([1.5, 1.5, 1.5])
def culled(pitch):
    d = O.raygen(0.3, pitch, 1.25, W, H).reshape(-1, 3).astype(np.float64)
    with np.errstate(divide='ignore', invalid='ignore'):
        inv = 1.0 / d
        t0 = (lo - o) * inv; t1 = (hi - o) * inv
    tmin = np.nanmax(np.minimum(t0, t1), axis=1); tmax = np.nanmin(np.maximum(t0, t1), axis=1)
    return (tmax < np.maximum(tmin, 0)).reshape(H, W)
tot = {}
for key, pitch in (('p0', 0.0), ('p6', -0.6)):
    p = P[key].copy(); c = culled(pitch); p[c] = 0
    print(key, 'culled frac', c.mean(), 'walked mean', p.mean())
    t = p.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
    tot[key] = t
t = np.concatenate([tot['p0'], tot['p6']])
mx = t.max(1); mean = t.mean(1)
print('tiles', len(t), 'util (sum mean / sum max)', mean.sum() / mx.sum())
print('max-per-tile percentiles', np.percentile(mx, [50, 90, 99, 99.9, 100]))
base = mx.sum()
for B in (32, 48, 64, 96, 128):
    p1 = np.minimum(mx, B).sum()
    left = t[t > B] - B
    n = left.size
    g = np.concatenate([left, np.zeros((-n) % 64, left.dtype)]).reshape(-1, 64)
    p2 = g.max(1).sum() if n else 0
    # sorted-by-length grouping of leftovers (best case)
    gs = np.concatenate([np.sort(left)[::-1], np.zeros((-n) % 64, left.dtype)]).reshape(-1, 64)
    p2s = gs.max(1).sum() if n else 0
    print(f'B={B}: leftover rays {n} ({n/t.size:.4f}), cost {(p1+p2)/base:.3f} (tile-order groups), {(p1+p2s)/base:.3f} (sorted)')
