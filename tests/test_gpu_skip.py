"""The per-node voxel-box skip (OCH_OPT_SKIP) against the oracle.

The skip is off by default (measured slower on the bench's terrain) and runs
as its own kernel instantiation (layout argument kPackedSkip), so every test
here switches it on.  Launches that count PUSHes keep the reference's walk
unless OCH_OPT_SKIP = 2, so every comparison uses launches WITHOUT PUSH counts
-- the product's -- on the bench's depth-12 terrain and on deep sparse trees:
camera rays of both views, random rays from inside the tree, rays with zero and
denormal components (where the skip must stand aside), config 5's secondary
rays, the tiled batch, the bench's frame kernels (fused RGBA8, indexed codes,
the merge schedule), and the pointer octree with empty nodes.  Records
(direction, voxel id, t bits) and frames must equal the reference's walk
(oracle/och_oracle.c), bit for bit, with the skip on and off.  The diagnostic
OCH_OPT_SKIP = 2 shows what the skip saves: the same records with fewer PUSHes."""
import numpy as np
import pytest

from test_gpu_parity import assert_same, assert_same_bounce, gpu_trace_bounce_dev, gpu_trace_dev

pytestmark = pytest.mark.gpu

ORIGIN = np.array([1.5, 1.5, 1.5], np.float32)
PITCHES = (0.0, -0.6)


@pytest.fixture(scope="module")
def d12(ort):
    return ort.build_terrain(12, use_gpu=True)


@pytest.fixture(scope="module")
def d12_ref(O, d12):
    return O.OraclePool(d12.nodes, d12.root, 12, 1)


def ray_sets(O, n=200000, seed=4):
    rng = np.random.default_rng(seed)
    ro = rng.uniform(1.01, 1.99, (n, 3)).astype(np.float32)
    rd = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    # edge rays: zero / denormal / tiny components, origins on mid planes
    m = 4000
    eo = rng.uniform(1.01, 1.99, (m, 3)).astype(np.float32)
    eo[: m // 4, 0] = 1.5
    eo[m // 4: m // 2, 2] = 1.25
    ed = rng.uniform(-1, 1, (m, 3)).astype(np.float32)
    ed[::3, 0] = 0.0
    ed[1::3, 2] = np.float32(1e-40)
    ed[2::5, 1] = np.float32(1e-30)
    sets = [(ORIGIN, O.raygen(0.3, p, 1.25, 1920, 1080)) for p in PITCHES]
    return sets + [(ro, rd), (eo, ed)]


@pytest.mark.parametrize("skip", [1, 0])
def test_d12_records_without_counts(ort, O, gpu_device, d12, d12_ref, skip):
    pool = ort.HOctree(d12.nodes, d12.root, 12, device=0)
    assert pool.get_option("skip") == 0, "the skip is off by default"
    pool.set_option("skip", skip)
    for origins, dirs in ray_sets(O):
        ref = O.trace_batch(d12_ref, O.Rcp(None), origins, dirs, nthreads=16)
        for cull in (1, 0):
            pool.set_option("cull", cull)
            assert_same(gpu_trace_dev(pool, origins, dirs, want_push=False), ref, push=False)
    pool.close()


def test_d12_skip_saves_pushes(ort, O, gpu_device, d12, d12_ref):
    """OCH_OPT_SKIP = 2: counting launches skip too; same records, fewer PUSHes."""
    pool = ort.HOctree(d12.nodes, d12.root, 12, device=0)
    pool.set_option("cull", 0)
    saved = []
    for origins, dirs in ray_sets(O)[:3]:
        ref = O.trace_batch(d12_ref, O.Rcp(None), origins, dirs, nthreads=16, want_push=True)
        pool.set_option("skip", 2)
        got = gpu_trace_dev(pool, origins, dirs, want_push=True)
        assert_same(got, ref, push=False)
        # the skip walks the same ray in at most as many PUSHes, plus one per node
        # it backs out of (that descent is counted); the totals drop
        saved.append(1.0 - got["push"].sum() / ref["push"].sum())
    assert min(saved) > 0.15, saved
    pool.close()


@pytest.mark.parametrize("compact", [1, 0])
def test_d12_bounce_records_without_counts(ort, O, gpu_device, d12, d12_ref, compact):
    pool = ort.HOctree(d12.nodes, d12.root, 12, device=0)
    pool.set_option("skip", 1)
    pool.set_option("bounce_compact", compact)
    for origins, dirs in ray_sets(O, n=100000)[:3]:
        ref = O.trace_bounce_batch(d12_ref, O.Rcp(None), origins, dirs, nthreads=16)
        assert_same_bounce(gpu_trace_bounce_dev(pool, origins, dirs, want_push=False), ref)
    pool.close()


def test_d12_tiled_batch_without_counts(ort, O, gpu_device, d12, d12_ref):
    import torch
    pool = ort.HOctree(d12.nodes, d12.root, 12, device=0)
    pool.set_option("skip", 1)
    W, H = 1920, 1080
    rays = O.raygen(0.3, -0.6, 1.25, W, H)
    ref = O.trace_batch(d12_ref, O.Rcp(None), ORIGIN, rays, nthreads=16)
    dev = torch.device("cuda", 0)
    o = torch.from_numpy(ORIGIN).to(dev)
    d = torch.from_numpy(rays.reshape(-1)).to(dev)
    n = W * H
    hd = torch.empty(n, dtype=torch.int32, device=dev)
    hv = torch.empty(n, dtype=torch.int32, device=dev)
    ht = torch.empty(n, dtype=torch.float32, device=dev)
    pool.set_stream(torch.cuda.current_stream())
    pool.trace_batch_tiled_dev(o, d, W, hd, hv, ht, n=n)
    torch.cuda.synchronize()
    got = {"dir": hd.cpu().numpy(), "voxel": hv.cpu().numpy().view(np.uint32), "t": ht.cpu().numpy().view(np.uint32)}
    assert_same(got, ref, push=False)
    pool.close()


@pytest.mark.parametrize("depth", [16, 20, 22])
def test_deep_sparse_trees_without_counts(ort, O, gpu_device, depth):
    """Deep stacks and node cells down to a few mantissa bits; depth 22 carries
    no boxes (a sixteenth of the leaf-parent cell would be below one bit)."""
    from conftest import sparse_dag
    rng = np.random.default_rng(depth + 100)
    c = 1 << (depth - 1)
    vox = []
    for k in range(2, depth - 1):
        base = c + rng.integers(-(1 << k), 1 << k, 3)
        for off in rng.integers(-2, 3, (40, 3)):
            x, y, z = (int(v) for v in np.clip(base + off, 0, (1 << depth) - 1))
            vox.append((x, y, z, int(1 + (x + y + z) % 4)))
    nodes, root = sparse_dag(depth, vox)
    ref_pool = O.OraclePool(nodes, root, depth, 1)
    n = 20000
    o = np.tile(ORIGIN.astype(np.float64), (n, 1))
    o[n // 2:] = rng.uniform(1.25, 1.75, (n - n // 2, 3))
    tgt = np.array([v[:3] for v in vox], np.float64)[rng.integers(0, len(vox), n)]
    tgt += np.where(rng.random((n, 1)) < 0.5, 0.5, rng.integers(0, 2, (n, 3)))
    d = (1.0 + tgt / (1 << depth)) - o
    d[::4] = rng.uniform(-1, 1, (d[::4].shape[0], 3))
    norm = np.linalg.norm(d, axis=1, keepdims=True)
    d = np.where(norm > 0, d / np.where(norm > 0, norm, 1), [[0.6, 0.0, -0.8]]).astype(np.float32)
    o = o.astype(np.float32)
    ref = O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16)
    pool = ort.HOctree(nodes, root, depth, device=0)
    pool.set_option("skip", 1)
    assert_same(gpu_trace_dev(pool, o, d, want_push=False), ref, push=False)
    refb = O.trace_bounce_batch(ref_pool, O.Rcp(None), o, d, nthreads=16)
    assert_same_bounce(gpu_trace_bounce_dev(pool, o, d, want_push=False), refb)
    pool.close()


def test_octree_table_with_empty_nodes(ort, O, gpu_device):
    """och::octree's own table after set(..., 0) (reachable empty nodes, A6):
    an empty node's box is empty, so the skip backs out of it at once."""
    t = O.ORef(8, 1 << 20)
    t.fill_terrain("set0")
    nodes = t.nodes()
    ref_pool = t.pool()
    rays = O.raygen(0.3, -0.6, 1.25, 512, 512)
    ref = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, rays, nthreads=16)
    pool = ort.Octree(nodes, 8, device=0)
    pool.set_option("skip", 1)
    assert_same(gpu_trace_dev(pool, ORIGIN, rays, want_push=False), ref, push=False)
    pool.close()


def test_d12_frames_with_skip(ort, O, gpu_device, d12, d12_ref):
    """The bench's frame kernels in the skip instantiation: the fused RGBA8
    launch, indexed codes + shade, and the merge schedule; config 5's frames."""
    import torch
    from octree_ray_tracing_amd.frame import ShardedFrame
    from test_gpu_configs import FOV, YAW, assert_frames, oracle_frames
    W, H = 1920, 1080
    pal = ort.VoxelData().get_colours()
    pool = ort.HOctree(d12.nodes, d12.root, 12, device=0)
    pool.set_palette(pal)
    pool.set_option("skip", 1)
    cams = [ort.camera(tuple(ORIGIN), YAW, p, FOV, W, H) for p in PITCHES]
    want = oracle_frames(O, d12_ref, pal, W, H)
    for direct, merge in ((True, 0), (False, 0), (False, 4)):
        pool.set_option("merge", merge)
        sf = ShardedFrame(pool, W, H, 8, n_views=2, indexed=True, direct=direct)
        sf.render(cams)
        torch.cuda.synchronize()
        assert_frames(sf.frames, want)
    pool.set_option("merge", 0)
    sf = ShardedFrame(pool, W, H, 8, n_views=2, indexed=True)
    sf.render(cams, bounce=True)
    torch.cuda.synchronize()
    assert_frames(sf.frames, oracle_frames(O, d12_ref, pal, W, H, bounce=True))
    pool.close()
