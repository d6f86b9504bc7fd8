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
