"""The N > 1 frame path on the GPU: two ranks (one process each, both on
device 0, gloo collectives through the host) run ShardedFrame's real render
-> all-gather -> shade + unshard, and both end with the oracle's frames.

This is bench.py's multi-GPU step (frame.py) with the process group the
driver's 8-GPU run uses swapped for gloo, since this box has one GPU."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, DEPTH, CHUNK = 640, 360, 9, 8
PITCHES = (0.0, -0.6)


def _rank(rank, world, port, root_dir, bounce, q, mode="rr"):
    import sys
    sys.path.insert(0, root_dir)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import octree_ray_tracing_amd as ort
    from octree_ray_tracing_amd.frame import ShardedFrame
    tree = ort.build_terrain(DEPTH)
    pool = ort.HOctree(tree.nodes, tree.root, DEPTH, device=0)
    pool.set_palette(ort.VoxelData().get_colours())
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in PITCHES]
    deal, shade = None, "all"
    if mode == "deal":
        # bench.py's N > 1 default: rank 0 deals the chunks by cost (rank 0 at
        # weight 0.7) and broadcasts the table; only rank 0 shades (display)
        t = torch.zeros(-(-H // CHUNK), dtype=torch.int32)
        if rank == 0:
            t.copy_(torch.from_numpy(ort.deal_chunks(pool.chunk_costs(cams, CHUNK), world, [0.7, 1.0])))
        dist.broadcast(t, 0)
        deal, shade = t.numpy(), "display"
    out = {}
    for indexed in (True, False):
        sf = ShardedFrame(pool, W, H, CHUNK, n_views=2, indexed=indexed, deal=deal, shade=shade)
        frames = sf.render(cams, bounce=bounce)
        torch.cuda.synchronize()
        out[indexed] = (None if frames is None else frames.cpu().numpy().view(np.uint32), sf.rows,
                        None if deal is None else deal.copy())
    pool.close()
    dist.destroy_process_group()
    q.put((rank, out))


@pytest.mark.parametrize("bounce,mode", [(False, "rr"), (True, "rr"), (False, "deal"), (True, "deal")])
def test_sharded_frame_two_ranks(ort, O, gpu_device, bounce, mode):
    import torch.multiprocessing as mp
    from conftest import ROOT
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + (os.getpid() + int(bounce) + 2 * (mode == "deal")) % 1000
    procs = [ctx.Process(target=_rank, args=(r, 2, port, str(ROOT), bounce, q, mode)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=110) for _ in range(2))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    tree = ort.build_terrain(DEPTH)
    ref_pool = O.OraclePool(tree.nodes, tree.root, DEPTH, 1)
    pal = ort.VoxelData().get_colours()
    o = np.array([1.5, 1.5, 1.5], np.float32)
    want = []
    for p in PITCHES:
        rays = O.raygen(0.3, p, 1.25, W, H)
        if bounce:
            r = O.trace_bounce_batch(ref_pool, O.Rcp(None), o, rays, nthreads=16)
            want.append(O.shade_bounce(r["dir"], r["voxel"], r["dir2"], pal).reshape(H, W))
        else:
            r = O.trace_batch(ref_pool, O.Rcp(None), o, rays, nthreads=16)
            want.append(O.shade_fast(r["dir"], r["voxel"], pal).reshape(H, W))
    for rank in (0, 1):
        for indexed in (True, False):
            frames, rows, deal = got[rank][indexed]
            if mode == "rr":
                assert rows == ort.shard_rows(H, CHUNK, 2)
            else:
                assert np.array_equal(deal, got[0][indexed][2])            # one table on every rank
                assert rows == int(np.bincount(deal, minlength=2).max()) * CHUNK
                if rank != 0:
                    assert frames is None                                   # shade="display": rank 0 only
                    continue
            for v in range(2):
                assert np.array_equal(frames[v], want[v]), (rank, indexed, v)
