"""The packed device layout (och_pool_pack, OCH_OPT_LAYOUT 1): ids per level,
child masks consistent with the child's slots, and a pool that -- masks
stripped -- traces exactly like the caller's pool."""
import numpy as np
import pytest


def unpack(packed, proot, depth):
    """Strip masks: an ordinary 0-based pool (slot 0 padding) with the same content."""
    nodes = packed.copy()
    level = {proot & 0xFFFFFF: 1}
    order = [proot & 0xFFFFFF]
    for v in order:
        if level[v] == depth:
            continue
        for k in range(8):
            s = int(packed[v, k])
            if s:
                c, m = s & 0xFFFFFF, s >> 24
                child = packed[c]
                assert m == sum(1 << j for j in range(8) if child[j]), "mask disagrees with the child's slots"
                assert level.setdefault(c, level[v] + 1) == level[v] + 1, "id shared between levels"
                if c not in order:
                    order.append(c)
                nodes[v, k] = c
    return nodes


@pytest.mark.parametrize("depth", [3, 6, 8])
def test_packed_pool_traces_like_raw(ort, O, depth):
    tree = ort.build_terrain(depth)
    packed, proot = ort.pack_pool(tree.nodes, tree.root, depth, 1)
    assert packed.shape[0] == tree.n_nodes + 1                 # one id per node: no sharing across levels
    assert proot >> 24 == sum(1 << k for k in range(8) if tree.nodes[0][k])
    flat = unpack(packed, proot, depth)
    rng = np.random.default_rng(depth)
    o = rng.uniform(1.01, 1.99, (20000, 3)).astype(np.float32)
    d = rng.uniform(-1, 1, (20000, 3)).astype(np.float32)
    a = O.trace_batch(O.OraclePool(tree.nodes, tree.root, depth, 1), O.Rcp(None), o, d, want_push=True)
    b = O.trace_batch(O.OraclePool(flat, proot & 0xFFFFFF, depth, 0, miss_t=float("inf")), O.Rcp(None), o, d,
                      want_push=True)
    for k in ("dir", "voxel", "push"):
        assert np.array_equal(a[k], b[k])
    assert np.array_equal(a["t"].view(np.uint32), b["t"].view(np.uint32))


def test_node_shared_between_levels(ort, O):
    """The reference's table keys nodes by content alone, so one slot can be an
    interior node at one level and a leaf-level node at the next (here node 2:
    at level 2 its slots name node 2, at level 3 they are voxel id 2).
    Packing emits it once per level."""
    raw = np.array([[2, 0, 0, 0, 0, 0, 0, 0], [2] * 8], np.uint32)
    packed, proot = ort.pack_pool(raw, 1, 3, 1)
    assert packed.shape[0] == 4                                   # padding + root + node 2 at two levels
    flat = unpack(packed, proot, 3)
    want = ort.NodePool(raw, 1, 3, 1)
    got = ort.NodePool(flat, proot & 0xFFFFFF, 3, 0)
    for x in range(8):
        for y in range(8):
            for z in range(8):
                assert got.at(x, y, z) == want.at(x, y, z) == (2 if max(x, y, z) < 4 else 0)
    rng = np.random.default_rng(1)
    o = rng.uniform(1.01, 1.99, (5000, 3)).astype(np.float32)
    d = rng.uniform(-1, 1, (5000, 3)).astype(np.float32)
    a = O.trace_batch(O.OraclePool(raw, 1, 3, 1), O.Rcp(None), o, d)
    b = O.trace_batch(O.OraclePool(flat, proot & 0xFFFFFF, 3, 0, miss_t=float("inf")), O.Rcp(None), o, d)
    assert np.array_equal(a["dir"], b["dir"]) and np.array_equal(a["voxel"], b["voxel"])


def test_empty_pool_packs_to_padding(ort):
    packed, proot = ort.pack_pool(np.zeros((3, 8), np.uint32), 0, 5, 1)
    assert packed.shape == (1, 8) and proot == 0
