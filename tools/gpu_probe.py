"""Quick GPU probe: trace one camera frame on a terrain DAG, time it, check parity.

python tools/gpu_probe.py --depth 10 --width 1920 --height 1080
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--pitch", type=float, nargs="*", default=[0.0, -0.6])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--check", type=int, default=1)
    a = ap.parse_args()

    import torch
    import octree_ray_tracing_amd as ort
    from oracle import oracle as O

    t0 = time.time()
    tree = ort.build_terrain(a.depth, use_gpu=True)
    print(f"build depth {a.depth}: {tree.n_nodes} nodes, {tree.build_seconds:.2f}s", flush=True)
    pool = ort.HOctree(tree.nodes, tree.root, tree.depth, device=0)
    stream = torch.cuda.current_stream()
    pool.set_stream(stream)
    W, H = a.width, a.height
    n = W * H
    dev = torch.device("cuda", 0)
    origin = torch.tensor([1.5, 1.5, 1.5], dtype=torch.float32, device=dev)
    dirs = torch.empty(n * 3, dtype=torch.float32, device=dev)
    hd = torch.empty(n, dtype=torch.int32, device=dev)
    hv = torch.empty(n, dtype=torch.int32, device=dev)
    ht = torch.empty(n, dtype=torch.float32, device=dev)
    push = torch.empty(n, dtype=torch.int32, device=dev)
    for pitch in a.pitch:
        cam = ort.camera((1.5, 1.5, 1.5), 0.3, pitch, 1.25, W, H)
        pool.raygen_dev(cam, dirs)
        pool.trace_batch_dev(origin, dirs, hd, hv, ht, push)
        torch.cuda.synchronize()
        P = push.cpu().numpy().astype(np.uint64).sum()
        ms = []
        for _ in range(a.iters):
            pool.trace_batch_dev(origin, dirs, hd, hv, ht)
            ms.append(pool.last_kernel_ms())
        ms = np.array(ms)
        med = float(np.median(ms))
        print(f"pitch {pitch}: trace median {med:.3f} ms  min {ms.min():.3f}  -> {n / med / 1e3:.1f} Mrays/s;"
              f" PUSH/ray {P / n:.2f}; alg GB/s {(n * 24 + 4 * P) / med / 1e6:.1f}", flush=True)
        slice_ = torch.empty(n, dtype=torch.int32, device=dev)
        pool.set_palette(ort.VoxelData().get_colours())
        rms = []
        for _ in range(a.iters):
            pool.render_dev(cam, slice_)
            rms.append(pool.last_kernel_ms())
        print(f"   render (raygen+trace+shade fused) median {np.median(rms):.3f} ms -> {n / np.median(rms) / 1e3:.1f} Mrays/s", flush=True)
        if a.check:
            rays_gpu = dirs.cpu().numpy().reshape(-1, 3)
            rays_ref = O.raygen(0.3, pitch, 1.25, W, H)
            assert np.array_equal(rays_gpu.view(np.uint32), rays_ref.view(np.uint32)), "raygen mismatch"
            ref_pool = O.OraclePool(tree.nodes, tree.root, tree.depth, 1)
            t1 = time.time()
            r = O.trace_batch(ref_pool, O.Rcp(ort.host_rcp_lut()), np.array([1.5, 1.5, 1.5], np.float32), rays_ref,
                              nthreads=16)
            cpu_s = time.time() - t1
            ok = (np.array_equal(hd.cpu().numpy(), r["dir"]) and np.array_equal(hv.cpu().numpy().view(np.uint32), r["voxel"])
                  and np.array_equal(ht.cpu().numpy().view(np.uint32), r["t"].view(np.uint32)))
            frame = slice_.cpu().numpy().view(np.uint32)
            want = np.where(r["dir"] == 6, 0xFFFEBF00, 0)
            print(f"   parity vs oracle: {'OK' if ok else 'MISMATCH'} (oracle 16 thr {n / cpu_s / 1e6:.1f} Mrays/s);"
                  f" frame sky pixels match: {bool(np.array_equal(frame == 0xFFFEBF00, r['dir'] == 6))}", flush=True)
            if not ok:
                bad = np.nonzero((hd.cpu().numpy() != r["dir"]) | (hv.cpu().numpy().view(np.uint32) != r["voxel"]))[0]
                print("   first bad", bad[:10], hd.cpu().numpy()[bad[:5]], r["dir"][bad[:5]])
    pool.close()
    print(f"total {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
