"""och_gpu_trace_batch_tiled_dev: the drop-in batch path (ORT/test_och_h_octree.cpp:74,
per pixel) over resident rays laid out as a row-major image, one 8x8 tile of
neighbouring rays per wavefront, optionally in a planned launch order.
Records and PUSH counts in the caller's order, bit for bit against the oracle
and against the untiled batch, for both layouts and every cull setting,
ragged widths and sizes, shared and per-ray origins."""
import numpy as np
import pytest

from test_gpu_parity import assert_same, gpu_trace_dev

pytestmark = pytest.mark.gpu

ORIGIN = np.array([1.5, 1.5, 1.5], np.float32)


def tiled_dev(pool, origins, dirs, width, want_push=True, n=None):
    import torch
    dev = torch.device("cuda", 0)
    dirs = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
    n = dirs.shape[0] if n is None else n
    o = torch.from_numpy(np.ascontiguousarray(origins, np.float32).reshape(-1)).to(dev)
    d = torch.from_numpy(dirs.reshape(-1)).to(dev)
    bufs = [torch.full((max(n, 1),), -7, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.float32)]
    hp = torch.full((max(n, 1),), -7, dtype=torch.int32, device=dev) if want_push else None
    pool.set_stream(torch.cuda.current_stream())
    pool.trace_batch_tiled_dev(o, d, width, *bufs, hp, n=n)
    torch.cuda.synchronize()
    out = {"dir": bufs[0].cpu().numpy()[:n], "voxel": bufs[1].cpu().numpy().view(np.uint32)[:n],
           "t": bufs[2].cpu().numpy().view(np.uint32)[:n]}
    if want_push:
        out["push"] = hp.cpu().numpy().view(np.uint32)[:n]
    return out


@pytest.mark.parametrize("depth", [10, 12])
def test_tiled_camera_rays(ort, O, gpu_device, depth):
    """A 1920x1080 camera frame's rays, both survey pitches, width 1920 (the
    frame), 1000 and 37 (tiles straddling rows), both layouts."""
    tree = ort.build_terrain(depth, use_gpu=True)
    pool = ort.HOctree(tree.nodes, tree.root, depth, device=0)
    ref_pool = O.OraclePool(tree.nodes, tree.root, depth, 1)
    for pitch in (0.0, -0.6):
        rays = O.raygen(0.3, pitch, 1.25, 1920, 1080)
        ref = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, rays, nthreads=16, want_push=True)
        for layout in (1, 0):
            pool.set_option("layout", layout)
            for width in (1920, 1000, 37):
                assert_same(tiled_dev(pool, ORIGIN, rays, width), ref)
                # no PUSH counts: the exact cull runs
                assert_same(tiled_dev(pool, ORIGIN, rays, width, want_push=False), ref, push=False)
    pool.close()


def test_tiled_sizes_and_origins(ort, O, gpu_device):
    """Ragged sizes (0, 1, 63, 65, 4097 rays; widths 1, 5, 64, 100, 5000 --
    wider than the batch), per-ray origins, unnormalised and axis-aligned rays."""
    tree = ort.build_terrain(9)
    pool = ort.HOctree(tree.nodes, tree.root, 9, device=0)
    ref_pool = O.OraclePool(tree.nodes, tree.root, 9, 1)
    rng = np.random.default_rng(21)
    for n in (1, 63, 65, 4097, 30011):
        o = rng.uniform(1.01, 1.99, (n, 3)).astype(np.float32)
        d = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
        d[: n // 5, rng.integers(0, 3)] = 0.0
        d[n // 5: n // 3] *= np.float32(1e-20)
        ref = O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16, want_push=True)
        for width in (1, 5, 64, 100, 5000):
            for layout in (1, 0):
                pool.set_option("layout", layout)
                assert_same(tiled_dev(pool, o, d, width), ref)
                assert_same(tiled_dev(pool, o, d, width, want_push=False), ref, push=False)
    # an empty batch launches nothing and succeeds
    import torch
    z = torch.zeros(3, dtype=torch.float32, device="cuda")
    e = torch.zeros(1, dtype=torch.int32, device="cuda")
    pool.trace_batch_tiled_dev(z, z, 8, e, e, e, None, n=0)
    with pytest.raises(ort.OchError):
        pool.trace_batch_tiled_dev(z, z, 0, e, e, e, None, n=1)
    pool.close()


def test_tiled_planned_order(ort, O, gpu_device):
    """och_gpu_plan_batch_tiled from one camera's rays; batches of that
    geometry (another camera: the plan orders dispatch only) and of another
    geometry (natural order) are the oracle's."""
    tree = ort.build_terrain(10, use_gpu=True)
    pool = ort.HOctree(tree.nodes, tree.root, 10, device=0)
    ref_pool = O.OraclePool(tree.nodes, tree.root, 10, 1)
    import torch
    rays0 = O.raygen(0.3, 0.0, 1.25, 1920, 1080)
    pool.set_stream(torch.cuda.current_stream())
    pool.plan_batch_tiled(torch.from_numpy(ORIGIN).cuda(), torch.from_numpy(rays0.reshape(-1)).cuda(), 1920)
    pool.set_option("tile_order", 2)
    for pitch, width in ((-0.6, 1920), (0.0, 1920), (-0.6, 960)):
        rays = O.raygen(0.3, pitch, 1.25, 1920, 1080)
        ref = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, rays, nthreads=16, want_push=True)
        assert_same(tiled_dev(pool, ORIGIN, rays, width), ref)
        assert_same(tiled_dev(pool, ORIGIN, rays, width, want_push=False), ref, push=False)
        assert_same(gpu_trace_dev(pool, ORIGIN, rays), ref)
    pool.close()


def test_trace_batch_image_host_entry(ort, O, gpu_device):
    """och_gpu_trace_batch_image: host rays in the reference's camera layout
    (x + y * W, ORT/test_och_h_octree.cpp:135), host records out, traced as
    8x8 tiles -- the oracle's records, and och_gpu_trace_batch's, bit for bit;
    per-ray origins and a width that does not divide the batch too."""
    tree = ort.build_terrain(10, use_gpu=True)
    pool = ort.HOctree(tree.nodes, tree.root, 10, device=0)
    ref_pool = O.OraclePool(tree.nodes, tree.root, 10, 1)
    for pitch in (0.0, -0.6):
        rays = O.raygen(0.3, pitch, 1.25, 1920, 1080)
        ref = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, rays, nthreads=16)
        for width in (1920, 333):
            hd, hv, ht = pool.trace_batch(ORIGIN, rays, width=width)
            assert_same({"dir": hd, "voxel": hv, "t": ht.view(np.uint32)}, ref, push=False)
        hd, hv, ht = pool.trace_batch(ORIGIN, rays)
        assert_same({"dir": hd, "voxel": hv, "t": ht.view(np.uint32)}, ref, push=False)
    rng = np.random.default_rng(5)
    o = rng.uniform(1.01, 1.99, (5001, 3)).astype(np.float32)
    d = rng.uniform(-1, 1, (5001, 3)).astype(np.float32)
    ref = O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16)
    hd, hv, ht = pool.trace_batch(o, d, width=70)
    assert_same({"dir": hd, "voxel": hv, "t": ht.view(np.uint32)}, ref, push=False)
    from octree_ray_tracing_amd._lib import call
    with pytest.raises(ort.OchError, match="width"):            # width 0 is refused, not traced untiled
        call("och_gpu_trace_batch_image", pool._h, None, 0, None, 1, 0, None, None, None)
    pool.close()
