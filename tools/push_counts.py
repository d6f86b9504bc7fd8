"""Per-ray PUSH counts of the bench's two views at depth 12, from the product
kernel (och_gpu_trace_batch_dev with counts): `push` = the reference walk's
count (cull off, as sse_trace walks), `walked` = the count the default launch
walks (OCH_OPT_CULL = 2: rays the occupied-box cull proves to miss walk 0).
Input of tools/tail_model.py.

python tools/push_counts.py [--out gpurun_out/push_d12.npz]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/push_d12.npz")
    a = ap.parse_args()

    import torch
    import octree_ray_tracing_amd as ort

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    tree = ort.build_terrain(12, use_gpu=True)
    pool = ort.HOctree(tree.nodes, tree.root, 12, device=0)
    pool.set_stream(torch.cuda.current_stream())
    W, H = 1920, 1080
    o = torch.tensor([1.5, 1.5, 1.5], dtype=torch.float32, device=dev)
    d = torch.empty(W * H * 3, dtype=torch.float32, device=dev)
    hd, hv = (torch.empty(W * H, dtype=torch.int32, device=dev) for _ in range(2))
    ht = torch.empty(W * H, dtype=torch.float32, device=dev)
    hp = torch.empty(W * H, dtype=torch.int32, device=dev)
    out = {}
    for key, pitch in (("p0", 0.0), ("p6", -0.6)):
        pool.raygen_dev(ort.camera((1.5, 1.5, 1.5), 0.3, pitch, 1.25, W, H), d)
        for name, cull in (("push", 0), ("walked", 2)):
            pool.set_option("cull", cull)
            pool.trace_batch_dev(o, d, hd, hv, ht, hp)
            torch.cuda.synchronize()
            out[f"{name}_{key}"] = hp.cpu().numpy().reshape(H, W).astype(np.int16)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(a.out, **out)
    print({k: float(v.mean()) for k, v in out.items()})
    pool.close()


if __name__ == "__main__":
    main()
