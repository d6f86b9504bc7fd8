"""The column cull's quadtree (och_pool_columns, OCH_OPT_COLUMNS; DESIGN.md
§4d): for every level l, the 2^l x 2^l blocks of the world's x-y columns in
Morton order, each the inclusive z range of the voxels above it.  Checked here
against the voxels themselves -- the listed voxels of sparse trees, and every
voxel of a depth-6 terrain read back through och_pool_at.  The cull is exact
by §4d and checked against the oracle by tests/test_gpu_columns.py."""
import numpy as np
import pytest

from conftest import sparse_dag


def morton(x, y, levels):
    m = 0
    for i in range(levels):
        m |= ((x >> i) & 1) << (2 * i) | ((y >> i) & 1) << (2 * i + 1)
    return m


def expected(vox, depth, levels):
    """One array per level: zlo | zmax << 16 per Morton block, 0xFFFF when empty."""
    vox = np.asarray(vox, np.int64).reshape(-1, 3)
    out = []
    for lv in range(1, levels + 1):
        shift = depth - lv
        words = np.full(1 << (2 * lv), 0xFFFF, np.uint32)
        bx, by = vox[:, 0] >> shift, vox[:, 1] >> shift
        for x, y in set(zip(bx.tolist(), by.tolist())):
            z = vox[(bx == x) & (by == y), 2]
            words[morton(x, y, lv)] = int(z.min()) | int(z.max()) << 16
        out.append(words)
    return out


@pytest.mark.parametrize("depth,levels", [(8, 4), (10, 7), (12, 6)])
def test_columns_of_sparse_trees(ort, depth, levels):
    rng = np.random.default_rng(depth)
    n = 1 << depth
    centres = rng.integers(2, n - 2, (12, 3))
    vox = [(int(x), int(y), int(z), 1 + i % 4) for i, c in enumerate(centres)
           for x, y, z in c + rng.integers(-2, 3, (20, 3))]
    nodes, root = sparse_dag(depth, vox)
    pk, proot = ort.pack_pool(nodes, root, depth)
    got = ort.columns(pk, proot, depth, levels)
    want = expected([v[:3] for v in vox], depth, levels)
    for lv, (g, w) in enumerate(zip(got, want), 1):
        assert np.array_equal(g, w), lv


def test_columns_of_terrain(ort):
    depth, levels = 6, 5
    tree = ort.build_terrain(depth)
    n = 1 << depth
    solid = []
    for x in range(n):
        for y in range(n):
            for z in range(n):
                if ort._lib.call("och_pool_at", tree.nodes.ctypes.data, tree.root, depth, 1, x, y, z):
                    solid.append((x, y, z))
    pk, proot = ort.pack_pool(tree.nodes, tree.root, depth)
    got = ort.columns(pk, proot, depth, levels)
    for lv, (g, w) in enumerate(zip(got, expected(solid, depth, levels)), 1):
        assert np.array_equal(g, w), lv
    # the terrain's air: the blocks' tops differ
    assert len(set((got[-1] >> 16).tolist())) > 4


def test_columns_refuse_bad_levels(ort):
    nodes, root = sparse_dag(6, [(1, 2, 3, 1)])
    pk, proot = ort.pack_pool(nodes, root, 6)
    for levels in (0, 6, 8):
        with pytest.raises(ort.OchError):
            ort.columns(pk, proot, 6, levels)
    nodes, root = sparse_dag(17, [(1, 2, 3, 1)])
    pk, proot = ort.pack_pool(nodes, root, 17)
    with pytest.raises(ort.OchError):
        ort.columns(pk, proot, 17, 4)
