"""In-block wave merging (OCH_OPT_MERGE, k_trace_grid_merge): rays move between
the waves of a block mid-walk, each keeping its LDS stack column, and the
emptied waves exit.  Records and frames must stay the oracle's for every
merge interval (1 = after every iteration), block size, ragged block and
layout of the rays: camera frames (RGBA8 and codes, planned order), resident
ray batches (random origins, zero and tiny direction components)."""
import numpy as np
import pytest

from test_gpu_parity import assert_same, gpu_trace_dev

pytestmark = pytest.mark.gpu

ORIGIN = np.array([1.5, 1.5, 1.5], np.float32)


@pytest.mark.parametrize("depth", [10, 12])
def test_merge_frames_and_batches(ort, O, gpu_device, depth):
    import torch
    tree = ort.build_terrain(depth, use_gpu=True)
    pal = ort.VoxelData().get_colours()
    pool = ort.HOctree(tree.nodes, tree.root, depth, device=0)
    pool.set_palette(pal)
    pool.set_stream(torch.cuda.current_stream())
    ref_pool = O.OraclePool(tree.nodes, tree.root, depth, 1)
    W, H = (1920, 1080) if depth == 12 else (803, 451)
    cams = [ort.camera(tuple(ORIGIN), 0.3, p, 1.25, W, H) for p in (0.0, -0.6)]
    want = []
    for p in (0.0, -0.6):
        r = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, O.raygen(0.3, p, 1.25, W, H), nthreads=16)
        want.append(O.shade_fast(r["dir"], r["voxel"], pal).reshape(H, W))
    rng = np.random.default_rng(depth)
    o = rng.uniform(1.01, 1.99, (70001, 3)).astype(np.float32)
    d = rng.uniform(-1, 1, (70001, 3)).astype(np.float32)
    d[:5000, 0] = 0.0
    d[5000:8000] *= np.float32(1e-30)
    ref = O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16)
    blocks = (128, 256) if depth == 12 else (128, 256, 512)
    for block in blocks:
        pool.set_option("block", block)
        for k in ((1, 8) if depth == 12 else (1, 4, 8, 32)):
            pool.set_option("merge", k)
            for order in (0, 2):
                if order == 2:
                    pool.plan_views(cams, H, 0, 1)
                pool.set_option("tile_order", order)
                frames = torch.zeros((2, H, W), dtype=torch.int32, device="cuda")
                pool.render_views_dev(cams, frames)
                codes = torch.full((2, H, W), 255, dtype=torch.uint8, device="cuda")
                pool.render_codes_views_dev(cams, codes)
                full = torch.empty((2, H, W), dtype=torch.int32, device="cuda")
                pool.shade_unshard_dev(codes, full, W, H, H, 1, 2)
                torch.cuda.synchronize()
                for v in range(2):
                    assert np.array_equal(frames[v].cpu().numpy().view(np.uint32), want[v]), (block, k, order, v)
                    assert np.array_equal(full[v].cpu().numpy().view(np.uint32), want[v]), (block, k, order, v)
            pool.set_option("tile_order", 0)
            got = gpu_trace_dev(pool, o, d, want_push=False)        # no PUSH counts: the merging kernel
            assert_same(got, ref, push=False)
    pool.set_option("merge", 0)
    pool.set_option("block", 64)
    pool.close()
