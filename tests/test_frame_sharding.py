"""Row-chunk sharding and the framebuffer all-gather (world sizes 2 and 8, gloo, CPU)."""
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


# ------------------------------------------------------------ row deal (och_deal_chunks)

def test_deal_chunks_balances_cost(ort):
    """och_deal_chunks: longest first onto the least loaded shard per weight,
    bounded chunk counts, deterministic."""
    rng = np.random.default_rng(3)
    costs = (rng.random(270) ** 4 * 100).astype(np.float32)       # a few expensive chunks, as a horizon
    for n, w in [(8, None), (8, [0.9] + [1.0] * 7), (3, [1.0, 2.0, 1.0]), (1, None)]:
        d = ort.deal_chunks(costs, n, w)
        assert d.shape == (270,) and d.min() >= 0 and d.max() < n
        assert np.array_equal(d, ort.deal_chunks(costs, n, w))        # same costs, same deal
        ww = np.ones(n) if w is None else np.asarray(w)
        per = np.array([costs[d == s].sum() for s in range(n)]) / ww
        assert per.max() - per.min() <= costs.max() / ww.min() + 1e-3
        cap = int(np.ceil(270 * ww.max() / ww.sum())) + 2
        assert np.bincount(d, minlength=n).max() <= cap
    # round-robin costs (all equal) still spread evenly
    d = ort.deal_chunks(np.ones(270, np.float32), 8)
    assert np.bincount(d).max() - np.bincount(d).min() <= 1
    with pytest.raises(ort.OchError):
        ort.deal_chunks(costs, 4, [1.0, 0.0, 1.0, 1.0])


def test_dealt_slice_maps_cover_every_row_once(ort):
    from octree_ray_tracing_amd.frame import deal_slice_rows, slice_row_map, unshard_host
    rng = np.random.default_rng(5)
    for H, chunk, n in [(2160, 8, 8), (37, 4, 3), (1080, 8, 2)]:
        n_chunks = -(-H // chunk)
        deal = ort.deal_chunks(rng.random(n_chunks).astype(np.float32), n, [0.8] + [1.0] * (n - 1))
        maps = [slice_row_map(H, chunk, n, s, deal) for s in range(n)]
        assert all(len(m) == deal_slice_rows(H, chunk, n, deal) for m in maps)
        rows = np.concatenate(maps)
        assert np.array_equal(np.sort(rows[rows >= 0]), np.arange(H))
        # each shard's chunks in order, its own rows only
        for s, m in enumerate(maps):
            g = m[m >= 0] // chunk
            assert np.all(deal[g] == s) and np.all(np.diff(g) >= 0)
        W = 3
        frame = np.arange(H * W, dtype=np.int32).reshape(H, W)
        sl = np.full((n, len(maps[0]), W), -7, np.int32)
        for s, m in enumerate(maps):
            sl[s][m >= 0] = frame[m[m >= 0]]
        assert np.array_equal(unshard_host(sl, H, chunk, deal), frame)


def _deal_worker(rank, world, port, H, W, chunk, deal, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from octree_ray_tracing_amd.frame import slice_row_map, unshard_host
    # rank 0's table reaches every rank, as bench.py broadcasts it
    t = torch.from_numpy(np.asarray(deal, np.int32)) if rank == 0 else torch.zeros(len(deal), dtype=torch.int32)
    dist.broadcast(t, 0)
    d = t.numpy()
    m = slice_row_map(H, chunk, world, rank, d)
    sl = torch.from_numpy(np.where(m[:, None] >= 0, m[:, None] * 1000 + np.arange(W)[None, :], -1).astype(np.int32))
    out = [torch.empty_like(sl) for _ in range(world)]
    dist.all_gather(out, sl)
    q.put((rank, unshard_host(torch.stack(out).numpy(), H, chunk, d)))
    dist.destroy_process_group()


def test_gloo_world2_dealt_exchange(ort):
    """The N > 1 path with a cost deal: equal (padded) slices all-gathered,
    every rank reassembles the whole frame."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    H, W, chunk, world = 45, 6, 4, 2
    deal = ort.deal_chunks(np.array([5, 1, 1, 9, 9, 9, 1, 1, 2, 3, 4, 1], np.float32), world, [0.7, 1.0])
    assert np.bincount(deal).tolist() != [6, 6]                  # uneven: slices are padded
    port = 30600 + os.getpid() % 1000
    procs = [ctx.Process(target=_deal_worker, args=(r, world, port, H, W, chunk, deal, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.arange(H)[:, None] * 1000 + np.arange(W)[None, :]
    for r in range(world):
        assert np.array_equal(got[r], want)


def test_gloo_world8_bench_deal_exchange(ort):
    """The deal the driver's 8-GPU run uses (configs[3]: 2160 rows in 8-row
    chunks, dealt by count with the display rank at display_weight(8) =
    0.5, the all-gather's weight, as bench.py does over RCCL), broadcast from rank 0 and
    exchanged by 8 gloo ranks: the padded slices all-gather into the whole
    frame on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    H, W, chunk, world = 2160, 4, 8, 8
    n_chunks = -(-H // chunk)
    assert ort.display_weight(world, "gather") == 0.5 and ort.display_weight(world) == 0.5
    deal = ort.deal_chunks(np.ones(n_chunks, np.float32), world, [ort.display_weight(world)] + [1.0] * (world - 1))
    counts = np.bincount(deal, minlength=world)
    assert counts[0] < counts[1:].min()                           # the display rank renders fewer rows
    assert counts.sum() == n_chunks and counts[1:].max() - counts[1:].min() <= 1
    port = 31700 + os.getpid() % 1000
    procs = [ctx.Process(target=_deal_worker, args=(r, world, port, H, W, chunk, deal, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.arange(H)[:, None] * 1000 + np.arange(W)[None, :]
    for r in range(world):
        assert np.array_equal(got[r], want)
