"""GPU parity: the gfx950 kernels (through the C ABI) vs the CPU oracle, bit for bit.

Hit records (direction, voxel id, t bit pattern) and PUSH counts must be
identical.  Two RCPPS regimes: the committed Intel table (golden vectors made
in the build container) and this host's own RCPPS (oracle in native mode vs
GPU with the table captured from the same host)."""
import math

import numpy as np
import pytest

from conftest import GOLD, sparse_dag

pytestmark = pytest.mark.gpu

ORIGIN = np.array([1.5, 1.5, 1.5], np.float32)


def gpu_trace_dev(pool, origins, dirs, want_push=True):
    import torch
    dev = torch.device("cuda", 0)
    dirs = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
    n = dirs.shape[0]
    o = torch.from_numpy(np.ascontiguousarray(origins, np.float32).reshape(-1)).to(dev)
    d = torch.from_numpy(dirs.reshape(-1)).to(dev)
    hd = torch.empty(n, dtype=torch.int32, device=dev)
    hv = torch.empty(n, dtype=torch.int32, device=dev)
    ht = torch.empty(n, dtype=torch.float32, device=dev)
    hp = torch.empty(n, dtype=torch.int32, device=dev) if want_push else None
    pool.set_stream(torch.cuda.current_stream())
    pool.trace_batch_dev(o, d, hd, hv, ht, hp, n=n)
    torch.cuda.synchronize()
    out = {"dir": hd.cpu().numpy(), "voxel": hv.cpu().numpy().view(np.uint32),
           "t": ht.cpu().numpy().view(np.uint32)}
    if want_push:
        out["push"] = hp.cpu().numpy().view(np.uint32)
    return out


def assert_same(gpu, ref, push=True):
    assert np.array_equal(gpu["dir"], ref["dir"]), _first_diff(gpu["dir"], ref["dir"])
    assert np.array_equal(gpu["voxel"], ref["voxel"].view(np.uint32))
    assert np.array_equal(np.asarray(gpu["t"]).view(np.uint32), np.asarray(ref["t"]).view(np.uint32))
    if push and "push" in gpu and ref.get("push") is not None:
        assert np.array_equal(gpu["push"], ref["push"])


def _first_diff(a, b):
    i = np.nonzero(a != b)[0]
    return f"{i.size} mismatches, first at {i[:5]}: {a[i[:5]]} vs {b[i[:5]]}"


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLD / "trace_d6.npz")


@pytest.mark.parametrize("layout", [0, 1])
def test_golden_vectors_intel_table(ort, gpu_device, golden, intel_lut, layout):
    pool = ort.HOctree(golden["nodes"], int(golden["root"]), int(golden["depth"]), device=0)
    pool.set_rcp_lut(intel_lut)
    pool.set_option("layout", layout)
    for name in ("cam", "rnd", "edge"):
        want = {"dir": golden[f"{name}_dir"], "voxel": golden[f"{name}_vox"], "t": golden[f"{name}_t"],
                "push": golden[f"{name}_push"]}
        assert_same(gpu_trace_dev(pool, golden[f"{name}_o"], golden[f"{name}_d"]), want)
        hd, hv, ht = pool.trace_batch(golden[f"{name}_o"], golden[f"{name}_d"])
        assert_same({"dir": hd, "voxel": hv, "t": ht}, want, push=False)
    pool.close()


def test_zero_direction_quirk_reference_table(ort, O, gpu_device, known, intel_lut):
    """SURVEY §7 known answer, traced on the reference's own hash-table layout."""
    k = known["zero_direction_quirk"]
    T = O.HRef(k["depth"], 10)
    for x, y, z, v in k["voxels"]:
        T.set(x, y, z, v)
    pool = ort.HOctree(T.nodes(), T.root, k["depth"], device=0)
    pool.set_rcp_lut(intel_lut)
    for case in k["cases"]:
        d, v, t = pool.sse_trace(*k["origin"], *case["dir"])
        assert (int(d), v) == (case["direction"], case["voxel"])
        assert float(np.float32(t)) == float.fromhex(case["t_hex"])
    pool.close()


@pytest.mark.parametrize("depth", [8, 10])
def test_camera_frames_host_rcpps(ort, O, gpu_device, depth):
    """Full 1920x1080 frames, both survey pitches, vs the oracle using this host's RCPPS."""
    tree = ort.build_terrain(depth)
    pool = ort.HOctree(tree.nodes, tree.root, depth, device=0)
    ref_pool = O.OraclePool(tree.nodes, tree.root, depth, 1)
    for pitch in (0.0, -0.6):
        rays = O.raygen(0.3, pitch, 1.25, 1920, 1080)
        ref = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, rays, nthreads=16, want_push=True)
        for layout in (0, 1):
            pool.set_option("layout", layout)
            assert_same(gpu_trace_dev(pool, ORIGIN, rays), ref)
    pool.close()


def test_reference_hash_table_layout(ort, O, gpu_device):
    """The reference's table->nodes (1-based, hash-scattered, gravestones) uploaded as-is."""
    T = O.HRef(8, 19)
    T.fill_terrain()
    nodes = T.nodes()
    pool = ort.HOctree(nodes, T.root, 8, device=0)
    rng = np.random.default_rng(9)
    o = rng.uniform(1.01, 1.99, (100000, 3)).astype(np.float32)
    d = rng.uniform(-1, 1, (100000, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    ref = O.trace_batch(T.pool(), O.Rcp(None), o, d, nthreads=16, want_push=True)
    for layout in (0, 1):
        pool.set_option("layout", layout)
        assert_same(gpu_trace_dev(pool, o, d), ref)
    rays = O.raygen(0.3, -0.6, 1.25, 640, 360)
    assert_same(gpu_trace_dev(pool, ORIGIN, rays), O.trace_batch(T.pool(), O.Rcp(None), ORIGIN, rays, want_push=True))
    pool.close()


@pytest.mark.parametrize("depth", [16, 20, 22])
def test_deep_sparse_trees(ort, O, gpu_device, depth):
    """Depths beyond the terrain's, up to the ABI's 22: a sparse DAG of voxel
    clusters at every scale around the cube's centre, traced from the centre
    and from random origins, most rays aimed at voxel centres and corners.
    Exercises deep LDS stacks, child sizes down to the float mantissa's last
    bits and long POP chains; both layouts against the oracle."""
    rng = np.random.default_rng(depth)
    c = 1 << (depth - 1)
    vox = []
    for k in range(2, depth - 1):                      # clusters 2^k voxels away, k = 2 .. depth - 2
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
    tgt += np.where(rng.random((n, 1)) < 0.5, 0.5, rng.integers(0, 2, (n, 3)))   # voxel centres or corners
    d = (1.0 + tgt / (1 << depth)) - o
    d[::4] = rng.uniform(-1, 1, (d[::4].shape[0], 3))                            # and some random rays
    norm = np.linalg.norm(d, axis=1, keepdims=True)
    d = np.where(norm > 0, d / np.where(norm > 0, norm, 1), [[0.6, 0.0, -0.8]]).astype(np.float32)
    o = o.astype(np.float32)
    ref = O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16, want_push=True)
    assert (ref["dir"] < 6).sum() > n // 10, "most aimed rays should hit the clusters"
    pool = ort.HOctree(nodes, root, depth, device=0)
    for layout in (0, 1):
        pool.set_option("layout", layout)
        assert_same(gpu_trace_dev(pool, o, d), ref)
    # config 5's secondary rays at these depths, every compaction mode
    refb = O.trace_bounce_batch(ref_pool, O.Rcp(None), o, d, nthreads=16, want_push=True)
    pool.set_option("layout", 1)
    for compact in (0, 1, 2):
        pool.set_option("bounce_compact", compact)
        assert_same_bounce(gpu_trace_bounce_dev(pool, o, d), refb)
    pool.close()


def test_octree_variant(ort, O, gpu_device):
    """och::octree: 0-based pool, root 0, miss t = 0.0F (ORT/och_octree.cpp:302)."""
    tree = ort.build_terrain(8, dedup=False)
    pool = ort.Octree(tree.nodes, 8, device=0)
    ref_pool = O.OraclePool(tree.nodes, 0, 8, 0)
    rays = O.raygen(0.3, 0.0, 1.25, 512, 512)
    ref = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, rays, want_push=True)
    got = gpu_trace_dev(pool, ORIGIN, rays)
    assert_same(got, ref)
    assert np.all(got["t"][got["dir"] == 6] == 0)
    pool.close()


def test_random_and_edge_rays_d10(ort, O, gpu_device):
    import sys
    sys.path.insert(0, str(GOLD.parent))
    from make_golden import edge_rays
    tree = ort.build_terrain(10)
    pool = ort.HOctree(tree.nodes, tree.root, 10, device=0)
    ref_pool = O.OraclePool(tree.nodes, tree.root, 10, 1)
    rng = np.random.default_rng(1)
    o = rng.uniform(1.01, 1.99, (200000, 3)).astype(np.float32)
    d = rng.uniform(-1, 1, (200000, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    assert_same(gpu_trace_dev(pool, o, d), O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16, want_push=True))
    eo, ed = edge_rays()
    assert_same(gpu_trace_dev(pool, eo, ed), O.trace_batch(ref_pool, O.Rcp(None), eo, ed, want_push=True))
    # unnormalised and tiny / huge directions
    d2 = d[:50000] * rng.choice(np.array([1e-20, 1e-5, 3.0, 1e20], np.float32), (50000, 1))
    assert_same(gpu_trace_dev(pool, o[:50000], d2), O.trace_batch(ref_pool, O.Rcp(None), o[:50000], d2, want_push=True))
    # origins on and just past the cube's faces (a bounce origin can sit half a
    # voxel outside): setup's root idx (p == 1.5, :324) then disagrees with the
    # POP's bit formula (:440-444), which the kernel must reproduce
    oo = rng.uniform(0.9, 2.1, (50000, 3)).astype(np.float32)
    oo[:10000, rng.integers(0, 3)] = np.float32(2.0000768)
    for layout in (1, 0):
        pool.set_option("layout", layout)
        assert_same(gpu_trace_dev(pool, oo, d[:50000]),
                    O.trace_batch(ref_pool, O.Rcp(None), oo, d[:50000], nthreads=16, want_push=True))
    pool.set_option("layout", 0)
    assert_same(gpu_trace_dev(pool, eo, ed), O.trace_batch(ref_pool, O.Rcp(None), eo, ed, want_push=True))
    pool.close()


def test_idx_plane_and_rebuild_waves(ort, O, gpu_device):
    """The walk's two loops (och_kernels.hip ray_trace): a wave whose rays all
    start inside the root reads each POP's child index from the stack's byte
    plane; a wave holding one ray from outside rebuilds it from the position
    bits, as :440-444 does.  Alternate the two kinds wave by wave (64 rays per
    wave in the trace kernel), with origins on the mid-planes (the default
    camera's 1.5, and 1.25 / 1.75) and just outside the cube's faces."""
    tree = ort.build_terrain(8)
    pool = ort.HOctree(tree.nodes, tree.root, 8, device=0)
    ref_pool = O.OraclePool(tree.nodes, tree.root, 8, 1)
    rng = np.random.default_rng(7)
    n_waves = 400
    o = rng.uniform(1.01, 1.99, (n_waves, 64, 3)).astype(np.float32)
    planes = np.array([1.25, 1.5, 1.75], np.float32)
    on_plane = rng.random((n_waves, 64, 3)) < 0.3
    o[on_plane] = rng.choice(planes, on_plane.sum())
    outside = np.array([2.0000768, 0.95, 2.5, 3.5], np.float32)
    for w in range(1, n_waves, 2):                       # odd waves: one ray from outside the root
        lane, axis = rng.integers(0, 64), rng.integers(0, 3)
        o[w, lane, axis] = outside[w % outside.size]
    d = rng.uniform(-1, 1, (n_waves, 64, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=2, keepdims=True)
    o, d = o.reshape(-1, 3), d.reshape(-1, 3)
    for layout in (1, 0):
        pool.set_option("layout", layout)
        assert_same(gpu_trace_dev(pool, o, d), O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16, want_push=True))
    pool.close()


def test_stale_hip_error_is_not_a_launch_failure(ort, O, gpu_device):
    """A launch reports hipGetLastError(), which also returns an error an earlier
    HIP call of the thread left behind (another library's: RCCL's communicator
    init, say).  The library clears it before each launch, so a failed HIP call
    made by someone else does not fail the next render or trace."""
    import ctypes
    import torch
    tree = ort.build_terrain(6)
    pool = ort.HOctree(tree.nodes, tree.root, 6, device=0)
    pool.set_stream(torch.cuda.current_stream())
    # every HIP runtime loaded in this process (torch's, and the one the library
    # resolved, if another): set the thread's last error in each
    paths = sorted({line.split()[-1] for line in open("/proc/self/maps") if "libamdhip64" in line})
    hips = [ctypes.CDLL(x) for x in paths]
    assert hips
    for h in hips:
        h.hipSetDevice.argtypes = [ctypes.c_int]

    def spoil():
        codes = {h.hipSetDevice(1 << 20) for h in hips}  # an invalid ordinal: the thread's last error is set
        assert 0 not in codes
        return codes
    from octree_ray_tracing_amd._lib import discarded_error
    cam = ort.camera((1.5, 1.5, 1.5), 0.3, -0.3, 1.25, 64, 36)
    want = pool.render(cam)
    discarded_error(reset=True)
    assert discarded_error() is None
    for k in range(2):
        codes = spoil()
        assert np.array_equal(pool.render(cam), want)
        # the cleared error is kept as evidence: its code, the C-ABI entry that found it
        got = discarded_error()
        assert got is not None and got["hip_error"] in codes and got["count"] == k + 1
        assert "och_gpu_render" in got["what"] and "launch" in got["what"]
    o = np.tile(ORIGIN, (256, 1))
    d = np.random.default_rng(3).uniform(-1, 1, (256, 3)).astype(np.float32)
    ref = gpu_trace_dev(pool, o, d)
    dev = torch.device("cuda", 0)
    o_t = torch.from_numpy(np.ascontiguousarray(o, np.float32).reshape(-1)).to(dev)
    d_t = torch.from_numpy(d.reshape(-1)).to(dev)
    out = [torch.empty(256, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.float32)]
    torch.cuda.synchronize()
    discarded_error(reset=True)
    spoil()
    pool.trace_batch_dev(o_t, d_t, *out, n=256)          # the launch right after the failed call
    torch.cuda.synchronize()
    assert np.array_equal(out[0].cpu().numpy(), ref["dir"])
    assert np.array_equal(out[1].cpu().numpy().view(np.uint32), ref["voxel"])
    assert np.array_equal(out[2].cpu().numpy().view(np.uint32), ref["t"].view(np.uint32))
    got = discarded_error(reset=True)
    assert got is not None and "och_gpu_trace_batch_dev" in got["what"]
    assert discarded_error() is None
    pool.close()


@pytest.mark.parametrize("W,H,pitch", [(1920, 1080, 0.0), (1920, 1080, -0.6), (641, 359, 0.4), (64, 36, -1.2)])
def test_raygen_bit_exact(ort, O, gpu_device, W, H, pitch):
    import torch
    tree = ort.build_terrain(4)
    pool = ort.HOctree(tree.nodes, tree.root, 4, device=0)
    pool.set_stream(torch.cuda.current_stream())
    cam = ort.camera((1.5, 1.5, 1.5), 0.3, pitch, 1.25, W, H)
    dirs = torch.empty(W * H * 3, dtype=torch.float32, device="cuda")
    pool.raygen_dev(cam, dirs)
    torch.cuda.synchronize()
    got = dirs.cpu().numpy().reshape(-1, 3)
    want = O.raygen(0.3, pitch, 1.25, W, H)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    pool.close()


def test_edge_sizes(ort, O, gpu_device):
    """Batches of 0, 1, 63, 64, 65 and 4097 rays (empty, lone, ragged waves and
    blocks) and frames of 1x1, 7x9, 8x8, 9x7 and 65x3 pixels (partial tiles,
    single rows), both layouts, against the oracle."""
    tree = ort.build_terrain(8)
    pal = ort.VoxelData().get_colours()
    pool = ort.HOctree(tree.nodes, tree.root, 8, device=0)
    pool.set_palette(pal)
    ref_pool = O.OraclePool(tree.nodes, tree.root, 8, 1)
    rng = np.random.default_rng(17)
    for layout in (0, 1):
        pool.set_option("layout", layout)
        for n in (0, 1, 63, 64, 65, 4097):
            o = rng.uniform(1.05, 1.95, (n, 3)).astype(np.float32)
            d = rng.uniform(-1, 1, (n, 3))
            d = (d / np.maximum(np.linalg.norm(d, axis=1, keepdims=True), 1e-6)).astype(np.float32)
            hd, hv, ht = pool.trace_batch(o, d)
            assert hd.shape == (n,)
            if n:
                want = O.trace_batch(ref_pool, O.Rcp(None), o, d)
                assert_same({"dir": hd, "voxel": hv, "t": ht}, want, push=False)
        for W, H in ((1, 1), (7, 9), (8, 8), (9, 7), (65, 3)):
            cam = ort.camera((1.5, 1.5, 1.5), 0.3, -0.6, 1.25, W, H)
            r = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, O.raygen(0.3, -0.6, 1.25, W, H))
            assert np.array_equal(pool.render(cam), O.shade(r["dir"], r["voxel"], pal).reshape(H, W)), (W, H)
    pool.close()


def test_render_frame_and_shards(ort, O, gpu_device):
    import torch
    tree = ort.build_terrain(9)
    pal = ort.VoxelData().get_colours()
    pool = ort.HOctree(tree.nodes, tree.root, 9, device=0)
    pool.set_palette(pal)
    W, H = 800, 450
    cam = ort.camera((1.5, 1.5, 1.5), 0.3, -0.6, 1.25, W, H)
    frame = pool.render(cam)
    rays = O.raygen(0.3, -0.6, 1.25, W, H)
    r = O.trace_batch(O.OraclePool(tree.nodes, tree.root, 9, 1), O.Rcp(None), ORIGIN, rays, nthreads=16)
    want = O.shade(r["dir"], r["voxel"], pal).reshape(H, W)
    assert np.array_equal(frame, want)
    # sharded: 3 shards of 8-row chunks, gathered and unsharded on the device
    pool.set_stream(torch.cuda.current_stream())
    n, chunk = 3, 8
    rows = ort.shard_rows(H, chunk, n)
    gathered = torch.zeros((n, rows, W), dtype=torch.int32, device="cuda")
    for s in range(n):
        pool.render_dev(cam, gathered[s], chunk, s, n)
    full = torch.empty((H, W), dtype=torch.int32, device="cuda")
    pool.unshard_dev(gathered, full, W, H, chunk, n)
    torch.cuda.synchronize()
    assert np.array_equal(full.cpu().numpy().view(np.uint32), want)
    pool.close()


def test_multi_view_render_and_unshard(ort, O, gpu_device):
    """Several cameras in one launch == one launch per camera; sharded multi-view
    slices reassemble exactly."""
    import torch
    tree = ort.build_terrain(9)
    pool = ort.HOctree(tree.nodes, tree.root, 9, device=0)
    pool.set_palette(ort.VoxelData().get_colours())
    pool.set_stream(torch.cuda.current_stream())
    W, H = 320, 200
    cams = [ort.camera((1.5, 1.5, 1.5), y, p, 1.25, W, H) for y, p in ((0.3, 0.0), (0.3, -0.6), (1.9, -0.2))]
    single = [torch.from_numpy(pool.render(c).view(np.int32)) for c in cams]
    out = torch.zeros((3, H, W), dtype=torch.int32, device="cuda")
    pool.render_views_dev(cams, out)
    torch.cuda.synchronize()
    for v in range(3):
        assert torch.equal(out[v].cpu(), single[v])
    n, chunk = 4, 8
    rows = ort.shard_rows(H, chunk, n)
    gathered = torch.zeros((n, 3, rows, W), dtype=torch.int32, device="cuda")
    for s_ in range(n):
        pool.render_views_dev(cams, gathered[s_], chunk, s_, n)
    frames = torch.empty((3, H, W), dtype=torch.int32, device="cuda")
    pool.unshard_dev(gathered, frames, W, H, chunk, n, 3)
    torch.cuda.synchronize()
    for v in range(3):
        assert torch.equal(frames[v].cpu(), single[v])
    pool.close()


def test_empty_tree_renders_sky(ort, gpu_device):
    pool = ort.HOctree(np.zeros((4, 8), np.uint32), 0, 5, device=0)
    pool.set_palette(ort.VoxelData().get_colours())
    frame = pool.render(ort.camera(width=32, height=16))
    assert np.all(frame == 0xFFFEBF00)
    d, v, t = pool.sse_trace(1.5, 1.5, 1.5, 0.3, 0.2, -0.9)
    assert (int(d), v) == (6, 0) and math.isinf(t)
    pool.close()


def test_pool_update_after_edits(ort, O, gpu_device):
    """h_octree::set path copies (ORT/och_h_octree.h:176-237) uploaded incrementally."""
    T = O.HRef(7, 16)
    T.fill_terrain()
    before = T.nodes()
    pool = ort.HOctree(before, T.root, 7, device=0)
    rng = np.random.default_rng(4)
    for x, y, z in rng.integers(30, 90, (300, 3)).tolist():      # dig and build
        T.set(x, y, z, 0 if (x + y) % 2 else 3)
    after = T.nodes()
    changed = np.nonzero(np.any(before != after, axis=1))[0]
    lo, hi = int(changed.min()), int(changed.max())
    pool.update(lo + 1, after[lo:hi + 1], T.root)
    rays = O.raygen(0.1, -0.3, 1.25, 320, 180)
    ref = O.trace_batch(T.pool(), O.Rcp(None), ORIGIN, rays, want_push=True)
    for layout in (1, 0):
        pool.set_option("layout", layout)
        assert_same(gpu_trace_dev(pool, ORIGIN, rays), ref)
    # an edit that would make a kernel read outside the pool is refused: the
    # root is an interior node, so its slots must name nodes of the pool
    bad = after[T.root - 1:T.root].copy()
    bad[0, :] = before.shape[0] + 50
    with pytest.raises(ort.OchError):
        pool.update(T.root, bad, T.root)
    assert_same(gpu_trace_dev(pool, ORIGIN, rays), ref)
    pool.close()


def test_error_paths(ort, gpu_device):
    tree = ort.build_terrain(4)
    pool = ort.HOctree(tree.nodes, tree.root, 4, device=0)
    with pytest.raises(ValueError):
        pool.set_rcp_lut(np.zeros(3, np.uint32))
    with pytest.raises(ort.OchError):
        pool.set_option("block", 100)
    with pytest.raises(ValueError):
        pool.set_palette(np.zeros(5, np.uint32))
    import ctypes as C
    from octree_ray_tracing_amd._lib import call
    with pytest.raises(ort.OchError):
        call("och_gpu_trace_batch", pool._h, None, 2, None, 1, None, None, None)
    pool.close()


@pytest.mark.slow
def test_depth12_camera_frame(ort, O, gpu_device):
    """BASELINE config 3: depth-12 terrain, 1920x1080, both pitches, full-frame parity."""
    tree = ort.build_terrain(12)
    pool = ort.HOctree(tree.nodes, tree.root, 12, device=0)
    ref_pool = O.OraclePool(tree.nodes, tree.root, 12, 1)
    for pitch in (0.0, -0.6):
        rays = O.raygen(0.3, pitch, 1.25, 1920, 1080)
        ref = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, rays, nthreads=16, want_push=True)
        assert_same(gpu_trace_dev(pool, ORIGIN, rays), ref)
    pool.close()


def gpu_trace_bounce_dev(pool, origins, dirs, want_push=True):
    import torch
    dev = torch.device("cuda", 0)
    dirs = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
    n = dirs.shape[0]
    o = torch.from_numpy(np.ascontiguousarray(origins, np.float32).reshape(-1)).to(dev)
    d = torch.from_numpy(dirs.reshape(-1)).to(dev)
    bufs = [torch.empty(n, dtype=t, device=dev) for t in
            (torch.int32, torch.int32, torch.float32, torch.int32, torch.int32, torch.float32, torch.int32)]
    pool.set_stream(torch.cuda.current_stream())
    pool.trace_bounce_batch_dev(o, d, *bufs[:6], push=bufs[6] if want_push else None, n=n)
    torch.cuda.synchronize()
    hd, hv, ht, hd2, hv2, ht2, hp = (b.cpu().numpy() for b in bufs)
    out = {"dir": hd, "voxel": hv.view(np.uint32), "t": ht.view(np.uint32), "dir2": hd2,
           "voxel2": hv2.view(np.uint32), "t2": ht2.view(np.uint32)}
    if want_push:
        out["push"] = hp.view(np.uint32)
    return out


def assert_same_bounce(gpu, ref):
    for k in ("dir", "voxel", "dir2", "voxel2", "push"):
        if k not in gpu:
            continue
        assert np.array_equal(gpu[k], np.asarray(ref[k]).view(gpu[k].dtype)), (k, _first_diff(gpu[k], np.asarray(ref[k])))
    for k in ("t", "t2"):
        assert np.array_equal(gpu[k], np.asarray(ref[k]).view(np.uint32)), k


@pytest.mark.parametrize("depth", [8, 10])
def test_bounce_records(ort, O, gpu_device, depth):
    """Config 5: primary and secondary hit records, bit for bit, camera frame and random rays."""
    tree = ort.build_terrain(depth)
    pool = ort.HOctree(tree.nodes, tree.root, depth, device=0)
    ref_pool = O.OraclePool(tree.nodes, tree.root, depth, 1)
    rays = O.raygen(0.3, -0.6, 1.25, 1920, 1080)
    rng = np.random.default_rng(5)
    ro = rng.uniform(1.01, 1.99, (100000, 3)).astype(np.float32)
    rd = rng.uniform(-1, 1, (100000, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    # the secondary walk: in place on the primary's stack (0), through the
    # block's queue from the root (1), per block (2); every mode, both layouts
    for origins, dirs in ((ORIGIN, rays), (ro, rd)):
        ref = O.trace_bounce_batch(ref_pool, O.Rcp(None), origins, dirs, nthreads=16, want_push=True)
        for layout in (1, 0):
            pool.set_option("layout", layout)
            for compact in (0, 1, 2):
                pool.set_option("bounce_compact", compact)
                assert_same_bounce(gpu_trace_bounce_dev(pool, origins, dirs), ref)
    pool.close()


def test_render_bounce_frames(ort, O, gpu_device):
    """Config 5 frames (two views, one launch), whole and row-sharded, vs the oracle's shading."""
    import torch
    tree = ort.build_terrain(9)
    pal = ort.VoxelData().get_colours()
    pool = ort.HOctree(tree.nodes, tree.root, 9, device=0)
    pool.set_palette(pal)
    pool.set_stream(torch.cuda.current_stream())
    ref_pool = O.OraclePool(tree.nodes, tree.root, 9, 1)
    W, H = 800, 450
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in (0.0, -0.6)]
    want = []
    for p in (0.0, -0.6):
        r = O.trace_bounce_batch(ref_pool, O.Rcp(None), ORIGIN, O.raygen(0.3, p, 1.25, W, H), nthreads=16)
        want.append(O.shade_bounce(r["dir"], r["voxel"], r["dir2"], pal).reshape(H, W))
    frames = torch.zeros((2, H, W), dtype=torch.int32, device="cuda")
    pool.render_bounce_views_dev(cams, frames)
    torch.cuda.synchronize()
    for v in range(2):
        assert np.array_equal(frames[v].cpu().numpy().view(np.uint32), want[v])
    n, chunk = 3, 8
    rows = ort.shard_rows(H, chunk, n)
    gathered = torch.zeros((n, 2, rows, W), dtype=torch.int32, device="cuda")
    for s_ in range(n):
        pool.render_bounce_views_dev(cams, gathered[s_], chunk, s_, n)
    full = torch.empty((2, H, W), dtype=torch.int32, device="cuda")
    pool.unshard_dev(gathered, full, W, H, chunk, n, 2)
    torch.cuda.synchronize()
    for v in range(2):
        assert np.array_equal(full[v].cpu().numpy().view(np.uint32), want[v])
    pool.close()


@pytest.mark.parametrize("bounce,W", [(False, 803), (True, 803), (False, 804)])
def test_indexed_colour_frames(ort, O, gpu_device, bounce, W):
    """The multi-GPU exchange format: 1-byte colour codes per pixel, gathered
    and shaded on the device, give the oracle's RGBA8 frames bit for bit
    (primary and config-5 shading), whole and row-sharded over 3 shards.
    W = 804 takes the four-pixels-per-thread shading kernel."""
    import torch
    tree = ort.build_terrain(9)
    pal = ort.VoxelData().get_colours()
    pool = ort.HOctree(tree.nodes, tree.root, 9, device=0)
    pool.set_palette(pal)
    pool.set_stream(torch.cuda.current_stream())
    ref_pool = O.OraclePool(tree.nodes, tree.root, 9, 1)
    H = 451
    pitches = (0.0, -0.6)
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in pitches]
    want = []
    for p in pitches:
        rays = O.raygen(0.3, p, 1.25, W, H)
        if bounce:
            r = O.trace_bounce_batch(ref_pool, O.Rcp(None), ORIGIN, rays, nthreads=16)
            want.append(O.shade_bounce(r["dir"], r["voxel"], r["dir2"], pal).reshape(H, W))
        else:
            r = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, rays, nthreads=16)
            want.append(O.shade(r["dir"], r["voxel"], pal).reshape(H, W))
    for n, chunk in ((1, H), (3, 8), (2, 5)):
        rows = ort.shard_rows(H, chunk, n)
        gathered = torch.full((n, 2, rows, W), 255, dtype=torch.uint8, device="cuda")
        for s_ in range(n):
            pool.render_codes_views_dev(cams, gathered[s_], chunk, s_, n, bounce)
        full = torch.empty((2, H, W), dtype=torch.int32, device="cuda")
        pool.shade_unshard_dev(gathered, full, W, H, chunk, n, 2)
        torch.cuda.synchronize()
        for v in range(2):
            assert np.array_equal(full[v].cpu().numpy().view(np.uint32), want[v]), (n, chunk, v)
    # a palette too large for one-byte codes is refused
    big = np.resize(np.asarray(pal, np.uint32).reshape(-1), 6 * 21)
    pool.set_palette(big)
    with pytest.raises(ort.OchError):
        pool.render_codes_views_dev(cams, gathered[0], chunk, 0, n, bounce)
    pool.close()


@pytest.mark.parametrize("order,shape", [(2, 10), (3, 10), (2, 0), (2, 100)])
def test_planned_launch_order(ort, O, gpu_device, order, shape):
    """OCH_OPT_TILE_ORDER = 2: the costliest tiles of a planning frame go first
    (och_gpu_plan_views); 3: the same, 64x64-pixel supertiles dealt over the XCDs.  Dispatch order only: frames of the planned geometry,
    of another geometry (natural order) and after the camera moved are all
    the oracle's."""
    import torch
    tree = ort.build_terrain(9)
    pal = ort.VoxelData().get_colours()
    pool = ort.HOctree(tree.nodes, tree.root, 9, device=0)
    pool.set_palette(pal)
    pool.set_stream(torch.cuda.current_stream())
    ref_pool = O.OraclePool(tree.nodes, tree.root, 9, 1)
    W, H = 803, 451
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in (0.0, -0.6)]
    assert pool.get_option("plan") == 10                 # default shape: costliest 10 % first
    pool.set_option("plan", shape)                       # OCH_OPT_PLAN: 0 all costliest first, 100 alternating
    pool.plan_views(cams, 8, 0, 1)
    pool.set_option("tile_order", order)
    for yaw in (0.3, 0.9):                   # the planned views, then a moved camera
        cams = [ort.camera((1.5, 1.5, 1.5), yaw, p, 1.25, W, H) for p in (0.0, -0.6)]
        want = []
        for p in (0.0, -0.6):
            r = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, O.raygen(yaw, p, 1.25, W, H), nthreads=16)
            want.append(O.shade(r["dir"], r["voxel"], pal).reshape(H, W))
        for n, rc in ((1, 8), (3, 8), (1, H)):    # planned geometry, then two others
            rows = ort.shard_rows(H, rc, n)
            gathered = torch.full((n, 2, rows, W), 255, dtype=torch.uint8, device="cuda")
            for s_ in range(n):
                pool.render_codes_views_dev(cams, gathered[s_], rc, s_, n)
            full = torch.empty((2, H, W), dtype=torch.int32, device="cuda")
            pool.shade_unshard_dev(gathered, full, W, H, rc, n, 2)
            torch.cuda.synchronize()
            for v in range(2):
                assert np.array_equal(full[v].cpu().numpy().view(np.uint32), want[v]), (yaw, n, rc, v)
    # config 5 frames in their planned order (the bounce kernel's own plan)
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in (0.0, -0.6)]
    gathered = torch.full((1, 2, ort.shard_rows(H, 8, 1), W), 255, dtype=torch.uint8, device="cuda")
    pool.render_codes_views_dev(cams, gathered[0], 8, 0, 1, bounce=True)
    full = torch.empty((2, H, W), dtype=torch.int32, device="cuda")
    pool.shade_unshard_dev(gathered, full, W, H, 8, 1, 2)
    torch.cuda.synchronize()
    for v, p in enumerate((0.0, -0.6)):
        r = O.trace_bounce_batch(ref_pool, O.Rcp(None), ORIGIN, O.raygen(0.3, p, 1.25, W, H), nthreads=16)
        want = O.shade_bounce(r["dir"], r["voxel"], r["dir2"], pal).reshape(H, W)
        assert np.array_equal(full[v].cpu().numpy().view(np.uint32), want), ("bounce", v)
    pool.close()


def test_eight_views_per_launch(ort, O, gpu_device):
    """OCH_MAX_VIEWS cameras of one size in one launch, each with its own
    position, yaw, pitch and fov: RGBA8 frames and colour codes (sharded over
    3 ranks, shaded after) equal the oracle's per view; a ninth view, or views
    of different sizes, are refused."""
    import torch
    tree = ort.build_terrain(9)
    pal = ort.VoxelData().get_colours()
    pool = ort.HOctree(tree.nodes, tree.root, 9, device=0)
    pool.set_palette(pal)
    pool.set_stream(torch.cuda.current_stream())
    ref_pool = O.OraclePool(tree.nodes, tree.root, 9, 1)
    rng = np.random.default_rng(8)
    W, H = 333, 187
    specs = [(tuple(float(x) for x in rng.uniform(1.05, 1.95, 3)), float(rng.uniform(-3, 3)),
              float(rng.uniform(-1.2, 1.2)), float((0.9, 1.25, 1.6)[k % 3])) for k in range(8)]
    cams = [ort.camera(pos, yaw, pitch, fov, W, H) for pos, yaw, pitch, fov in specs]
    want = []
    for pos, yaw, pitch, fov in specs:
        r = O.trace_batch(ref_pool, O.Rcp(None), np.array(pos, np.float32), O.raygen(yaw, pitch, fov, W, H),
                          nthreads=16)
        want.append(O.shade(r["dir"], r["voxel"], pal).reshape(H, W))
    frames = torch.zeros((8, H, W), dtype=torch.int32, device="cuda")
    pool.render_views_dev(cams, frames)
    n, rc = 3, 8
    rows = ort.shard_rows(H, rc, n)
    gathered = torch.full((n, 8, rows, W), 255, dtype=torch.uint8, device="cuda")
    for s_ in range(n):
        pool.render_codes_views_dev(cams, gathered[s_], rc, s_, n)
    full = torch.empty((8, H, W), dtype=torch.int32, device="cuda")
    pool.shade_unshard_dev(gathered, full, W, H, rc, n, 8)
    torch.cuda.synchronize()
    for v in range(8):
        assert np.array_equal(frames[v].cpu().numpy().view(np.uint32), want[v]), v
        assert np.array_equal(full[v].cpu().numpy().view(np.uint32), want[v]), v
    nine = torch.zeros((9, H, W), dtype=torch.int32, device="cuda")
    with pytest.raises(ort.OchError):
        pool.render_views_dev(cams + cams[:1], nine)
    with pytest.raises(ort.OchError):
        pool.render_views_dev([cams[0], ort.camera((1.5, 1.5, 1.5), 0.3, 0.0, 1.25, W + 1, H)], frames)
    pool.close()


def test_retired_options_refused(ort, gpu_device):
    """The option ids of the arms retired in round 5 (persistent / refill
    schedules, wave merging, the per-node skip, the column cull) fail loudly
    instead of being stored and ignored; the supported options round-trip."""
    import ctypes as C
    from octree_ray_tracing_amd._lib import load
    tree = ort.build_terrain(5)
    pool = ort.HOctree(tree.nodes, tree.root, 5, device=0)
    lib = load()
    v = C.c_int()
    for opt in (0, 2, 3, 7, 9, 12, 13):
        assert lib.och_gpu_set_option(pool._h, opt, 0) != 0
        assert "retired" in lib.och_last_error().decode()
        assert lib.och_gpu_get_option(pool._h, opt, C.byref(v)) != 0
    for name, value in (("block", 128), ("layout", 0), ("tile_order", 1), ("bounce_compact", 2), ("cull", 0),
                        ("timing", 2), ("plan", 0), ("split", 60), ("split_segs", 8), ("split_level", 5)):
        pool.set_option(name, value)
        assert pool.get_option(name) == value
    assert set(pool.OPTIONS) == {"block", "layout", "tile_order", "bounce_compact", "cull", "timing", "plan",
                                 "split", "split_segs", "split_level"}
    assert pool.get_option("split_tiles") == 0                # read only: no plan made
    pool.close()


def test_rcpps_every_exponent(ort, O, gpu_device):
    """The kernels' RCPPS takes one subtraction from the device table (entries
    + 127 << 23) where the model's result exponent stays in range, and the
    model itself elsewhere.  Directions with one component at every exponent
    (zero, denormals, 2^-126 .. 2^127, inf, NaN) walk the same records as the
    oracle, under this host's table, the Intel table, and a table with one
    non-negative entry (every x through the model)."""
    tree = ort.build_terrain(7)
    pool = ort.HOctree(tree.nodes, tree.root, 7, device=0)
    ref_pool = O.OraclePool(tree.nodes, tree.root, 7, 1)
    rng = np.random.default_rng(31)
    base = rng.uniform(-1, 1, (256 * 24, 3)).astype(np.float32)
    base /= np.linalg.norm(base, axis=1, keepdims=True)
    exps = np.repeat(np.arange(256, dtype=np.uint32), 24)
    mant = rng.integers(0, 1 << 23, exps.size, dtype=np.uint32)
    mant[::6] = 0                                                       # powers of two, inf
    bits = (exps << 23) | mant | (rng.integers(0, 2, exps.size, dtype=np.uint32) << 31)
    axis = rng.integers(0, 3, exps.size)
    base[np.arange(exps.size), axis] = bits.view(np.float32)
    o = rng.uniform(1.01, 1.99, (exps.size, 3)).astype(np.float32)
    intel = np.fromfile(GOLD / "rcp_lut_intel.bin", dtype=np.uint32)
    odd = intel.copy()
    odd[5] &= 0x7FFFFFFF
    for lut in (None, intel, odd):
        if lut is not None:
            pool.set_rcp_lut(lut)
        ref = O.trace_batch(ref_pool, O.Rcp(lut), o, base, nthreads=16, want_push=True)
        for layout in (1, 0):
            pool.set_option("layout", layout)
            assert_same(gpu_trace_dev(pool, o, base), ref)
    pool.close()
