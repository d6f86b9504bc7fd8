"""Product terrain builder (och_build_terrain) vs the oracle's exact
restatement of the reference's fill (h_octree table + set edits,
ORT/test_och_h_octree.cpp:651-787) and the survey's counts."""
import numpy as np
import pytest


@pytest.mark.parametrize("depth", [1, 2, 3, 4, 5, 6])
def test_content_equals_reference_fill(O, ort, depth):
    tree = ort.build_terrain(depth)
    T = O.HRef(depth, 16)
    T.fill_terrain()
    dim = 1 << depth
    for z in range(dim):
        for y in range(dim):
            for x in range(dim):
                assert tree.at(x, y, z) == T.at(x, y, z), (x, y, z)
    assert tree.n_nodes == T.fillcnt
    assert tree.tree_nodes == T.nodecnt


def test_d8_counts(ort, known):
    tree = ort.build_terrain(8)
    k = known["terrain_d8"]
    assert tree.n_nodes == k["unique_nodes"]
    assert tree.tree_nodes == k["tree_nodes"]
    assert tree.solid_voxels == k["solid_voxels"]
    assert {str(i): tree.voxel_hist[i] for i in range(1, 5)} == k["voxel_hist"]


def test_d8_sampled_content(O, ort):
    tree = ort.build_terrain(8)
    T = O.HRef(8, 19)
    T.fill_terrain()
    rng = np.random.default_rng(5)
    for x, y, z in rng.integers(0, 256, (20000, 3)).tolist():
        assert tree.at(x, y, z) == T.at(x, y, z)


@pytest.mark.slow
def test_d10_counts(ort, known):
    tree = ort.build_terrain(10)
    assert tree.n_nodes == known["terrain_d10"]["unique_nodes"]
    assert tree.tree_nodes == known["terrain_d10"]["tree_nodes"]


def test_octree_layout(ort, O, known):
    """dedup=0 gives the expanded och::octree (0-based, root 0)."""
    tree = ort.build_terrain(8, dedup=False)
    assert tree.index_base == 0 and tree.root == 0
    assert tree.n_nodes == known["terrain_d8"]["tree_nodes"]
    dag = ort.build_terrain(8)
    rng = np.random.default_rng(6)
    for x, y, z in rng.integers(0, 256, (5000, 3)).tolist():
        assert tree.at(x, y, z) == dag.at(x, y, z)


def test_breadth_first_layout(ort):
    """Root first; every interior child points forward; levels are contiguous."""
    tree = ort.build_terrain(7)
    assert tree.root == 1
    level_of = {1: 1}
    for i in range(1, tree.n_nodes + 1):
        lv = level_of[i]
        if lv == tree.depth:
            continue
        for c in tree.nodes[i - 1]:
            c = int(c)
            if c:
                assert c > i
                assert level_of.setdefault(c, lv + 1) == lv + 1
    levels = [level_of[i] for i in range(1, tree.n_nodes + 1)]
    assert levels == sorted(levels)


def test_rand_kinds(ort, O):
    """glibc rand() emulation == this platform's rand(); MSVC LCG differs."""
    g = ort.build_terrain(6, rand_kind="glibc")
    tops = O.column_tops(64)
    heights = np.array([[O.height(x, y, 64) for x in range(64)] for y in range(64)])
    for y in range(64):
        for x in range(64):
            z = heights[y, x]
            if not O.is_tunnel(x, y, z):
                assert g.at(x, y, z) == tops[y, x]
    m = ort.build_terrain(6, rand_kind="msvc")
    assert m.n_nodes > 0 and not np.array_equal(g.nodes, m.nodes)


def test_no_tunnels(ort, O):
    tree = ort.build_terrain(6, tunnels=False)
    T = O.HRef(6, 14)
    T.fill_terrain(tunnels=False)
    assert tree.n_nodes == T.fillcnt
    for x, y, z in np.random.default_rng(2).integers(0, 64, (3000, 3)).tolist():
        assert tree.at(x, y, z) == T.at(x, y, z)


def test_bad_params(ort):
    with pytest.raises(ort.OchError):
        ort.build_terrain(13)
    with pytest.raises(ort.OchError):
        ort.build_terrain(11, dedup=False)


def test_pool_file_round_trip_and_corruption(ort, tmp_path):
    """Linearised node-pool file (NodePool.save / load)."""
    tree = ort.build_terrain(6)
    p = tmp_path / "d6.ochpool"
    tree.save(p)
    assert p.stat().st_size == 64 + tree.nodes.nbytes
    for mm in (False, True):
        back = ort.NodePool.load(p, mmap=mm)
        assert (back.root, back.depth, back.index_base) == (tree.root, tree.depth, tree.index_base)
        assert np.array_equal(back.nodes, tree.nodes)
        assert back.at(10, 20, 5) == tree.at(10, 20, 5)
    octree = ort.build_terrain(4, dedup=False)
    octree.save(p)
    back = ort.NodePool.load(p)
    assert back.index_base == 0 and np.array_equal(back.nodes, octree.nodes)
    raw = bytearray(p.read_bytes())
    raw[70] ^= 1                                  # flip one bit of a slot
    p.write_bytes(bytes(raw))
    with pytest.raises(ValueError, match="checksum"):
        ort.NodePool.load(p)
    ort.NodePool.load(p, verify=False)
    p.write_bytes(bytes(raw[:-4]))
    with pytest.raises(ValueError, match="bytes"):
        ort.NodePool.load(p)
    p.write_bytes(b"NOTAPOOL" + bytes(raw[8:]))
    with pytest.raises(ValueError, match="node-pool"):
        ort.NodePool.load(p)
    p.write_bytes(bytes(raw[:10]))
    with pytest.raises(ValueError, match="truncated"):
        ort.NodePool.load(p)


def test_pool_file_header_corruption(ort, tmp_path):
    """the checksum covers depth / index base / root / count, and a
    root outside the pool is refused even when the checksum is skipped."""
    import struct
    tree = ort.build_terrain(5)
    p = tmp_path / "d5.ochpool"
    tree.save(p)
    good = p.read_bytes()
    # field offsets in the header: magic 0, version 8, depth 12, index_base 16, root 20, n 24, crc 32
    for off, val in ((12, 6), (20, 2), (16, 1)):
        raw = bytearray(good)
        raw[off:off + 4] = struct.pack("<i", val)
        if off == 16:                                   # index base 1 -> 0 makes root 1 invalid too
            raw[off:off + 4] = struct.pack("<i", 0)
        p.write_bytes(bytes(raw))
        with pytest.raises(ValueError):
            ort.NodePool.load(p)
    raw = bytearray(good)
    raw[20:24] = struct.pack("<I", tree.n_nodes + 1)    # root past the end
    p.write_bytes(bytes(raw))
    with pytest.raises(ValueError, match="root"):
        ort.NodePool.load(p, verify=False)
    # a version-1 file (checksum of the slots only) still loads
    v1 = bytearray(good)
    v1[8:12] = struct.pack("<I", 1)
    import zlib
    v1[32:36] = struct.pack("<I", zlib.crc32(good[64:]))
    p.write_bytes(bytes(v1))
    back = ort.NodePool.load(p)
    assert np.array_equal(back.nodes, tree.nodes) and back.root == tree.root


def pool_at_many(nodes, root, depth, xyz):
    """h_octree::at (ORT/och_h_octree.h:239-258) at many points, vectorised over a 1-based pool."""
    xyz = np.asarray(xyz, np.int64)
    cur = np.full(xyz.shape[0], root, np.int64)
    out = np.zeros(xyz.shape[0], np.uint32)
    live = np.ones(xyz.shape[0], bool)
    for level in range(depth - 1, -1, -1):
        c = ((xyz[:, 0] >> level) & 1) | (((xyz[:, 1] >> level) & 1) << 1) | (((xyz[:, 2] >> level) & 1) << 2)
        nxt = np.where(live, nodes[np.maximum(cur - 1, 0), c], 0).astype(np.int64)
        if level == 0:
            out = nxt.astype(np.uint32)
        live &= nxt != 0
        cur = nxt
    return np.where(live | (out != 0), out, 0).astype(np.uint32)


@pytest.mark.slow
def test_d12_tree_pinned(ort, O, known):
    """The headline workload's tree (depth 12, 4096^3), built in parallel by
    och_build_terrain, against the oracle's closed-form voxel function
    (ORT/test_och_h_octree.cpp:561-787, ORT/och_noise.h:73-366): 10^6 random
    voxels, every column's top voxel, and +-2 voxels around tunnel boundaries
    found along 2 000 random columns.  Node counts and the pool checksum are
    pinned (SURVEY §6.1 has no depth-12 figures: pinned by this build, and
    every GPU depth-12 parity test runs on this exact pool)."""
    import zlib
    depth, dim = 12, 4096
    tree = ort.build_terrain(depth)
    k = known["terrain_d12"]
    assert tree.n_nodes == k["unique_nodes"] and tree.tree_nodes == k["tree_nodes"]
    assert tree.solid_voxels == k["solid_voxels"]
    assert zlib.crc32(tree.nodes.astype("<u4").tobytes()) == k["pool_crc32"]
    tops = O.column_tops(dim)
    hmap = O.height_map(dim)
    rng = np.random.default_rng(12)
    # 10^6 random voxels, half of them in the band the surface and tunnels cross
    pts = rng.integers(0, dim, (1_000_000, 3)).astype(np.int32)
    pts[:500_000, 2] = rng.integers(0, int(hmap.max()) + 3, 500_000)
    assert np.array_equal(pool_at_many(tree.nodes, tree.root, depth, pts), O.voxels_at(dim, pts, tops))
    # every column's top voxel (x, y, h(x, y)) and the two under it
    ys, xs = np.mgrid[0:dim, 0:dim]
    for dz in (0, -1, -2):
        xyz = np.stack([xs.ravel(), ys.ravel(), hmap.ravel() + dz], 1).astype(np.int32)
        xyz = xyz[xyz[:, 2] >= 0]
        for part in np.array_split(xyz, 8):
            assert np.array_equal(pool_at_many(tree.nodes, tree.root, depth, part), O.voxels_at(dim, part, tops))
    # 2 000 random columns in full (z = 0 .. h + 2): every tunnel boundary along
    # them, with the voxels around it, and the column tops
    n_bound = 0
    for x, y in rng.integers(0, dim, (2000, 2)).tolist():
        h = int(hmap[y, x])
        z = np.arange(0, h + 3, dtype=np.int32)
        xyz = np.stack([np.full_like(z, x), np.full_like(z, y), z], 1)
        want = O.voxels_at(dim, xyz, tops)
        n_bound += int(np.count_nonzero((want[1:] == 0) != (want[:-1] == 0)))
        assert np.array_equal(pool_at_many(tree.nodes, tree.root, depth, xyz), want), (x, y)
    assert n_bound > 1000          # the columns do cross tunnels


@pytest.mark.gpu
@pytest.mark.parametrize("depth,dedup", [(5, True), (8, True), (8, False), (10, True), (12, True)])
def test_gpu_voxelisation_same_pool(ort, gpu_device, depth, dedup):
    """use_gpu=1 (k_brick_codes + host hash-consing) builds the host builder's
    pool slot for slot, with the same statistics; depth 12 is the bench's tree."""
    import time
    t0 = time.perf_counter()
    g = ort.build_terrain(depth, dedup=dedup, use_gpu=True)
    t_gpu = time.perf_counter() - t0
    h = ort.build_terrain(depth, dedup=dedup, use_gpu=False)
    assert (g.root, g.depth, g.index_base) == (h.root, h.depth, h.index_base)
    assert np.array_equal(g.nodes, h.nodes)
    assert (g.tree_nodes, g.solid_voxels) == (h.tree_nodes, h.solid_voxels)
    assert list(g.voxel_hist) == list(h.voxel_hist)
    print(f"depth {depth}: GPU voxelisation {t_gpu:.2f} s ({g.build_seconds:.2f} s in och_build_terrain), "
          f"host {h.build_seconds:.2f} s")


def test_gpu_voxelisation_needs_a_gpu(ort):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(ort.OchError, match="NODEV"):
        ort.build_terrain(6, use_gpu=True)
    assert ort.build_terrain(4, use_gpu=True).n_nodes > 0     # below depth 5: host, as documented
