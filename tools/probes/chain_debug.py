import sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import octree_ray_tracing_amd as ort
from oracle import oracle as O
from conftest import sparse_dag
from test_cull import _box_feature_targets
from test_gpu_parity import gpu_trace_dev
depth = 8
rng = np.random.default_rng(7)
vox = [(int(x), int(y), int(z), int(rng.integers(1, 7))) for x, y, z in rng.integers((100, 50, 200), (110, 53, 230), (120, 3))]
nodes, root = sparse_dag(depth, vox)
blo, bhi = ort.occupied_box(nodes, root, depth)
lo = 1 + np.array(blo) / 2.0 ** depth; hi = 1 + np.array(bhi) / 2.0 ** depth
pool = ort.HOctree(nodes, root, depth, device=0)
ref_pool = O.OraclePool(nodes, root, depth, 1)
n = 150000
o = rng.uniform(1.001, 1.999, (n, 3)).astype(np.float32)
tgt = _box_feature_targets(rng, lo, hi, n)
d = (tgt - o).astype(np.float32)
d[: n // 2] /= np.linalg.norm(d[: n // 2], axis=1, keepdims=True)
k = n // 3
d[:k, 0] *= rng.choice(np.array([0.0, 1e-30, 1e-41, 1.0], np.float32), k)
sets = [(o, d)]
with np.errstate(divide="ignore", invalid="ignore"):
    pass
rng.uniform(size=0)
oo = rng.uniform(0.95, 2.05, (n, 3)).astype(np.float32)
oo[: n // 4, 0] = np.float32(1.0)
oo[n // 4: n // 2, 2] = np.float32(2.0)
d2 = (_box_feature_targets(rng, lo, hi, n) - oo).astype(np.float32)
ORIGIN = np.array([1.5, 1.5, 1.5], np.float32)
sets += [(oo, d2), (np.tile(ORIGIN, (n, 1)), (tgt - ORIGIN).astype(np.float32))]
for si, (o, d) in enumerate(sets):
  ref = O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16, want_push=True)
  for layout in (1, 0):
    pool.set_option("layout", layout)
    for cull in (1, 0):
        pool.set_option("cull", cull)
        for push in (True, False):
            g = gpu_trace_dev(pool, o, d, want_push=push)
            bad = np.nonzero(g["dir"] != ref["dir"])[0]
            print(si, layout, cull, push, "mismatches", bad.size, bad[:8])
            if bad.size and layout == 1:
                np.savez(f"gpurun_out/chain_bad{si}.npz", o=o[bad[:200]], d=d[bad[:200]], gdir=g["dir"][bad[:200]], rdir=ref["dir"][bad[:200]],
                         gpush=g["push"][bad[:200]] if push else 0, rpush=ref["push"][bad[:200]], nodes=nodes, root=root)
                for i in bad[:3]:
                    print("  o", o[i].tolist(), "d", d[i].tolist(), "gpu", g["dir"][i], g["voxel"][i], "ref", ref["dir"][i], ref["voxel"][i], ref["push"][i], g.get("push", [0]*n)[i] if push else "")
