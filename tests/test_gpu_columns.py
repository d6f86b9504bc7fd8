"""The column cull (OCH_OPT_COLUMNS) against the oracle.

The cull is off by default (measured slower, §4d); here it is switched on
and off explicitly over the ray sets where it acts -- the bench's camera views
at depth 12 (row-major and tiled), random rays from inside the world, rays with
zero and denormal components (where it must stand aside), a depth-14 field of
small solid balls -- and over the bench's frame paths.  Records (direction, voxel id, t bits) and frames must equal the
reference's walk (oracle/och_oracle.c) bit for bit.  The cull diagnostic
(OCH_OPT_CULL = 2, counting launches cull too) shows that it acts: more rays
end with 0 PUSHes than under the occupied-box cull alone."""
import numpy as np
import pytest

from test_gpu_parity import assert_same, gpu_trace_dev
from test_gpu_skip import ORIGIN, PITCHES, ray_sets

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def d12(ort):
    return ort.build_terrain(12, use_gpu=True)


@pytest.fixture(scope="module")
def d12_ref(O, d12):
    return O.OraclePool(d12.nodes, d12.root, 12, 1)


def blob_scene(depth, n_blobs=300, radius=6, seed=7):
    from conftest import sparse_dag
    rng = np.random.default_rng(seed)
    r = np.arange(-radius, radius + 1)
    dx, dy, dz = np.meshgrid(r, r, r, indexing="ij")
    ball = np.stack([dx, dy, dz], -1)[dx * dx + dy * dy + dz * dz <= radius * radius]
    vox = {}
    for b, c in enumerate(rng.integers(radius, (1 << depth) - radius, (n_blobs, 3))):
        for x, y, z in ball + c:
            vox[(int(x), int(y), int(z))] = 1 + b % 4
    return sparse_dag(depth, [(x, y, z, v) for (x, y, z), v in vox.items()])


@pytest.mark.parametrize("columns", [6, 0, 3])
def test_d12_records(ort, O, gpu_device, d12, d12_ref, columns):
    pool = ort.HOctree(d12.nodes, d12.root, 12, device=0)
    assert pool.get_option("columns") == 0, "the column cull is off by default"
    pool.set_option("columns", columns)
    for origins, dirs in ray_sets(O):
        ref = O.trace_batch(d12_ref, O.Rcp(None), origins, dirs, nthreads=16)
        assert_same(gpu_trace_dev(pool, origins, dirs, want_push=False), ref, push=False)
    pool.close()


def test_d12_tiled_and_culled_counts(ort, O, gpu_device, d12, d12_ref):
    """The bench's views as a tiled batch, cull diagnostic on: records equal,
    and the column cull ends more rays at 0 PUSHes than the box cull alone."""
    import torch
    W, H = 1920, 1080
    dev = torch.device("cuda", 0)
    pool = ort.HOctree(d12.nodes, d12.root, 12, device=0)
    pool.set_stream(torch.cuda.current_stream())
    pool.set_option("cull", 2)
    o = torch.from_numpy(ORIGIN).to(dev)
    zero = {}
    for pitch in PITCHES:
        rays = O.raygen(0.3, pitch, 1.25, W, H)
        ref = O.trace_batch(d12_ref, O.Rcp(None), ORIGIN, rays, nthreads=16)
        d = torch.from_numpy(rays.reshape(-1)).to(dev)
        for columns in (0, 6):
            pool.set_option("columns", columns)
            out = [torch.empty(W * H, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.float32, torch.int32)]
            pool.trace_batch_tiled_dev(o, d, W, *out, n=W * H)
            torch.cuda.synchronize()
            got = {"dir": out[0].cpu().numpy(), "voxel": out[1].cpu().numpy().view(np.uint32),
                   "t": out[2].cpu().numpy().view(np.uint32)}
            assert_same(got, ref, push=False)
            zero[(pitch, columns)] = int((out[3] == 0).sum().item())
    for pitch in PITCHES:
        assert zero[(pitch, 6)] >= zero[(pitch, 0)]
    assert zero[(0.0, 6)] > 1.05 * zero[(0.0, 0)], zero
    pool.close()


def test_blob_field(ort, O, gpu_device):
    depth = 14
    nodes, root = blob_scene(depth)
    ref_pool = O.OraclePool(nodes, root, depth, 1)
    pool = ort.HOctree(nodes, root, depth, device=0)
    rng = np.random.default_rng(3)
    n = 100000
    o = rng.uniform(1.01, 1.99, (n, 3)).astype(np.float32)
    d = rng.uniform(-1, 1, (n, 3))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    sets = [(ORIGIN, O.raygen(0.3, p, 1.25, 640, 360)) for p in PITCHES] + [(o, d)]
    for columns in (6, 7, 0):
        pool.set_option("columns", columns)
        for origins, dirs in sets:
            ref = O.trace_batch(ref_pool, O.Rcp(None), origins, dirs, nthreads=16)
            assert_same(gpu_trace_dev(pool, origins, dirs, want_push=False), ref, push=False)
    pool.close()


def test_frames_with_and_without(ort, O, gpu_device, d12, d12_ref):
    import torch
    from octree_ray_tracing_amd.frame import ShardedFrame
    from test_gpu_configs import FOV, YAW, assert_frames, oracle_frames
    W, H = 1920, 1080
    pal = ort.VoxelData().get_colours()
    pool = ort.HOctree(d12.nodes, d12.root, 12, device=0)
    pool.set_palette(pal)
    cams = [ort.camera(tuple(ORIGIN), YAW, p, FOV, W, H) for p in PITCHES]
    want = oracle_frames(O, d12_ref, pal, W, H)
    for columns in (6, 0):
        pool.set_option("columns", columns)
        for direct, merge in ((True, 0), (False, 0), (False, 4)):
            pool.set_option("merge", merge)
            sf = ShardedFrame(pool, W, H, 8, n_views=2, indexed=True, direct=direct)
            sf.render(cams)
            torch.cuda.synchronize()
            assert_frames(sf.frames, want)
    pool.close()
