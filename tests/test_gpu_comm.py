"""The N > 1 exchange on the GPU, at the world size a one-GPU box allows (1).

bench.py's sharded step -- this rank's rows rendered as colour codes, one
RCCL exchange, the display rank's shade -- runs here exactly as the driver's
8-GPU run issues it, only with one rank, so the exchange is the collective's
own copy of the one slice:
  * on the library's communicator (och_comm_*, ncclCommInitRank from an id),
    issued natively by och_gpu_render_sharded_steps_dev, for every exchange
    mode, primary and config 5, several frames in flight;
  * on torch.distributed's RCCL process group (dist.all_gather_into_tensor),
    with the library communicator's id broadcast through that group, as
    bench.py does at N > 1;
  * through the one-process device group's worker threads (och_frame_group_render_steps).
Every frame must equal the oracle's bit for bit (ORT/test_och_h_octree.cpp:437-457
update_image + trace_pixel, restated by oracle/och_oracle.c)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ORIGIN = np.array([1.5, 1.5, 1.5], np.float32)
PITCHES = (0.0, -0.6)
DEPTH, W, H, CHUNK = 10, 1280, 720, 8


@pytest.fixture(scope="module")
def scene(ort, O):
    tree = ort.build_terrain(DEPTH, use_gpu=True)
    pal = ort.VoxelData().get_colours()
    ref_pool = O.OraclePool(tree.nodes, tree.root, DEPTH, 1)
    want = {}
    for bounce in (False, True):
        frames = []
        for p in PITCHES:
            rays = O.raygen(0.3, p, 1.25, W, H)
            if bounce:
                r = O.trace_bounce_batch(ref_pool, O.Rcp(None), ORIGIN, rays, nthreads=16)
                frames.append(O.shade_bounce(r["dir"], r["voxel"], r["dir2"], pal).reshape(H, W))
            else:
                r = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, rays, nthreads=16)
                frames.append(O.shade_fast(r["dir"], r["voxel"], pal).reshape(H, W))
        want[bounce] = np.stack(frames)
    return tree, pal, want


def test_comm_local_collectives(ort, gpu_device):
    """och_comm_all_gather / och_comm_gather at one rank: the slice lands in recv[0]."""
    import torch
    comm = ort.RcclComm.local(0)
    assert (comm.n_ranks, comm.rank) == (1, 0)
    send = torch.randint(0, 256, (3, 17, 641), dtype=torch.uint8, device="cuda")
    recv = torch.zeros((1,) + tuple(send.shape), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    comm.all_gather(send, recv, s)
    torch.cuda.synchronize()
    assert torch.equal(recv[0], send)
    recv.zero_()
    comm.gather(send, recv, s)
    torch.cuda.synchronize()
    assert torch.equal(recv[0], send)
    comm.close()


@pytest.mark.parametrize("exchange", ["all_gather", "display", "gather"])
@pytest.mark.parametrize("bounce", [False, True])
def test_sharded_steps_native_world1(ort, gpu_device, scene, exchange, bounce):
    """och_gpu_render_sharded_steps_dev: 7 frames over 3 streams and buffer
    sets; every set's frames equal the oracle's."""
    import torch
    from octree_ray_tracing_amd.frame import ShardedFrame, ShardedSteps
    tree, pal, want = scene
    pool = ort.HOctree(tree.nodes, tree.root, DEPTH, device=0)
    pool.set_palette(pal)
    cams = [ort.camera(tuple(ORIGIN), 0.3, p, 1.25, W, H) for p in PITCHES]
    comm = ort.RcclComm.local(0)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(2)]
    shade = "all" if exchange == "all_gather" else "display"
    mode = "gather" if exchange == "gather" else "all_gather"
    sfs = []
    for s in streams:
        with torch.cuda.stream(s):
            sfs.append(ShardedFrame(pool, W, H, CHUNK, n_views=2, indexed=True, shade=shade, comm=comm,
                                    sharded=True, exchange=mode))
    pool.set_option("tile_order", 2)
    pool.plan_views(cams, CHUNK, 0, 1)
    steps = ShardedSteps(sfs, streams, comm, cams, bounce=bounce)
    assert steps.exchange == ort._lib.EXCHANGE[exchange]
    for f in sfs:
        f.frames.zero_()
    steps.run(7)
    torch.cuda.synchronize()
    for b, f in enumerate(sfs):
        got = f.frames.cpu().numpy().view(np.uint32)
        assert np.array_equal(got, want[bounce]), (exchange, bounce, b)
    # the same frames issued from Python through ShardedFrame.exchange on this comm
    for f in sfs:
        f.frames.zero_()
    with torch.cuda.stream(streams[1]):
        pool.set_stream(streams[1])
        sfs[1].render(cams, bounce=bounce)
    torch.cuda.synchronize()
    assert np.array_equal(sfs[1].frames.cpu().numpy().view(np.uint32), want[bounce])
    comm.close()
    pool.close()


def test_sharded_steps_argument_checks(ort, gpu_device, scene):
    import torch
    from octree_ray_tracing_amd.frame import ShardedFrame
    tree, pal, _ = scene
    pool = ort.HOctree(tree.nodes, tree.root, DEPTH, device=0)
    pool.set_palette(pal)
    with pytest.raises(ValueError):
        ShardedFrame(pool, W, H, CHUNK, n_views=2, indexed=True, shade="all", sharded=True, exchange="gather")
    lib = ort.load()
    comm = ort.RcclComm.local(0)
    cams = [ort.camera(tuple(ORIGIN), 0.3, 0.0, 1.25, W, H)]
    import ctypes as C
    arr = (ort._lib.Camera * 1)(*cams)
    sl = torch.empty(H * W, dtype=torch.uint8, device="cuda")
    st = (C.c_void_p * 1)(torch.cuda.current_stream().cuda_stream)
    sp = (C.c_void_p * 1)(sl.data_ptr())
    # rank 0 shades: frames are required
    rc = lib.och_gpu_render_sharded_steps_dev(pool._h, comm.handle, C.cast(arr, C.c_void_p), 1, 1, st, sp, sp, None,
                                               1, None, None, CHUNK, 0, 0)
    assert rc == -1 and b"frames" in lib.och_last_error()
    rc = lib.och_gpu_render_sharded_steps_dev(pool._h, comm.handle, C.cast(arr, C.c_void_p), 1, 1, st, sp, sp, None,
                                               1, None, None, CHUNK, 0, 7)
    assert rc == -1
    comm.close()
    pool.close()


def _torch_world1(root_dir, port, q):
    """A world-size-1 torch.distributed RCCL group: the exchange through torch
    (all_gather_into_tensor) and through the library communicator whose id
    torch broadcasts -- bench.py's N > 1 setup, one rank."""
    import sys
    sys.path.insert(0, root_dir)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    import octree_ray_tracing_amd as ort
    from octree_ray_tracing_amd.frame import ShardedFrame, ShardedSteps
    tree = ort.build_terrain(DEPTH, use_gpu=True)
    pool = ort.HOctree(tree.nodes, tree.root, DEPTH, device=0)
    pool.set_palette(ort.VoxelData().get_colours())
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in PITCHES]
    out = {}
    pool.set_stream(torch.cuda.current_stream())
    for bounce in (False, True):
        sf = ShardedFrame(pool, W, H, CHUNK, n_views=2, indexed=True, shade="display", sharded=True)
        assert sf.comm is None and not sf.direct
        frames = sf.render(cams, bounce=bounce)
        torch.cuda.synchronize()
        out[("torch", bounce)] = frames.cpu().numpy().view(np.uint32).copy()
    comm = ort.RcclComm.from_process_group()
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    sfs = []
    for s in streams:
        with torch.cuda.stream(s):
            sfs.append(ShardedFrame(pool, W, H, CHUNK, n_views=2, indexed=True, shade="display", comm=comm))
    for bounce in (False, True):
        f = ShardedSteps(sfs, streams, comm, cams, bounce=bounce).run(4)
        torch.cuda.synchronize()
        out[("rccl", bounce)] = f.frames.cpu().numpy().view(np.uint32).copy()
    comm.close()
    pool.close()
    dist.destroy_process_group()
    q.put(out)


def test_torch_process_group_world1(ort, gpu_device, scene):
    import torch.multiprocessing as mp
    from conftest import ROOT
    _, _, want = scene
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_torch_world1, args=(str(ROOT), 29700 + os.getpid() % 500, q))
    p.start()
    got = q.get(timeout=110)
    p.join(timeout=30)
    assert p.exitcode == 0
    for (kind, bounce), frames in got.items():
        assert np.array_equal(frames, want[bounce]), (kind, bounce)


def test_group_render_steps(ort, gpu_device, scene):
    """The one-process group's worker threads: 5 frames over 3 buffer sets."""
    tree, pal, want = scene
    g = ort.FrameGroup(tree.nodes, tree.root, DEPTH, devices=[0])
    g.set_palette(pal)
    cams = [ort.camera(tuple(ORIGIN), 0.3, p, 1.25, W, H) for p in PITCHES]
    for bounce in (False, True):
        g.render_steps(cams, 5, n_buffers=3, row_chunk=CHUNK, bounce=bounce)
        assert np.array_equal(g.download(0), want[bounce]), bounce
    g.plan(cams, row_chunk=CHUNK)
    g.render_steps(cams, 4, n_buffers=2, row_chunk=CHUNK)
    assert np.array_equal(g.download(0), want[False])
    g.close()


def test_row_deal_rejected_keeps_old_deal(ort, gpu_device, scene):
    """A bad och_gpu_set_row_deal leaves the pool's deal as it was."""
    tree, pal, _ = scene
    pool = ort.HOctree(tree.nodes, tree.root, DEPTH, device=0)
    n_chunks = -(-H // CHUNK)
    deal = (np.arange(n_chunks) % 3 == 0).astype(np.int32)           # shard 1 gets a third
    pool.set_row_deal(H, CHUNK, 2, deal)
    rows = pool.slice_rows(H, CHUNK, 2)
    bad = deal.copy()
    bad[5] = 9                                                         # shard 9 of 2
    with pytest.raises(ort.OchError):
        pool.set_row_deal(H, CHUNK, 2, bad)
    assert pool.slice_rows(H, CHUNK, 2) == rows != ort.shard_rows(H, CHUNK, 2)
    pool.set_row_deal(H, CHUNK, 2, None)
    assert pool.slice_rows(H, CHUNK, 2) == ort.shard_rows(H, CHUNK, 2)
    pool.close()
