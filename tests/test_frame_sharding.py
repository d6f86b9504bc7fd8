"""Row-chunk sharding and the framebuffer all-gather (world size 2, gloo, CPU)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def test_slice_maps_cover_every_row_once(ort):
    from octree_ray_tracing_amd.frame import slice_row_map
    for H, chunk, n in [(1080, 8, 2), (2160, 8, 8), (10, 4, 3), (7, 16, 4), (1080, 1080, 1)]:
        rows = np.concatenate([slice_row_map(H, chunk, n, s) for s in range(n)])
        rows = rows[rows >= 0]
        assert np.array_equal(np.sort(rows), np.arange(H))


def test_unshard_host_roundtrip(ort):
    from octree_ray_tracing_amd.frame import slice_row_map, unshard_host
    H, W, chunk, n = 37, 5, 4, 3
    frame = np.arange(H * W, dtype=np.int32).reshape(H, W)
    slices = []
    for s in range(n):
        m = slice_row_map(H, chunk, n, s)
        sl = np.full((len(m), W), -7, np.int32)
        sl[m >= 0] = frame[m[m >= 0]]
        slices.append(sl)
    assert np.array_equal(unshard_host(np.stack(slices), H, chunk), frame)


def _worker(rank, world, port, H, W, chunk, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from octree_ray_tracing_amd.frame import slice_row_map, unshard_host
    m = slice_row_map(H, chunk, world, rank)
    sl = torch.from_numpy(np.where(m[:, None] >= 0, m[:, None] * 1000 + np.arange(W)[None, :], -1).astype(np.int32))
    out = [torch.empty_like(sl) for _ in range(world)]
    dist.all_gather(out, sl)
    frame = unshard_host(torch.stack(out).numpy(), H, chunk)
    q.put((rank, frame))
    dist.destroy_process_group()


def test_gloo_world2_frame_exchange():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    H, W, chunk, world = 45, 6, 4, 2
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, world, port, H, W, chunk, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.arange(H)[:, None] * 1000 + np.arange(W)[None, :]
    for r in range(world):
        assert np.array_equal(got[r], want)
