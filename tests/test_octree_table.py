"""och::octree's own table (BASELINE configs[0]): the oracle's
ORef restates create_table / alloc / dealloc / set / unset / at
(ORT/och_octree.cpp:14-160) slot for slot.  CPU checks of the restatement
against the reference's published counts and against hand-derived tables;
the GPU traces of these tables are in tests/test_gpu_octree_table.py."""
import numpy as np
import pytest

ORIGIN = np.array([1.5, 1.5, 1.5], np.float32)


def free_chain(nodes, head):
    """The free list from head through children[0] (ORT/och_octree.cpp:58, :69)."""
    out = []
    while head:
        out.append(int(head))
        head = nodes[head, 0]
        assert len(out) <= nodes.shape[0], "free list has a cycle"
    return out


@pytest.fixture(scope="module")
def tables(O):
    t_unset = O.ORef(8, 1 << 20)
    t_unset.fill_terrain("unset")
    t_set0 = O.ORef(8, 1 << 20)
    t_set0.fill_terrain("set0")
    return {"unset": t_unset, "set0": t_set0}


def test_create_table_free_list(O):
    """create_table (:21-34): all zero, node i's children[0] = i + 1 for
    i = 1 .. cap - 2, the last 0; head = 1; the root (0) is not on the list."""
    T = O.ORef(4, 10)
    n = T.nodes()
    assert T.head == 1 and T.node_cnt == 1
    assert np.array_equal(n[:, 0], [0, 2, 3, 4, 5, 6, 7, 8, 9, 0])
    assert not n[:, 1:].any()
    assert free_chain(n, T.head) == list(range(1, 10))


def test_unset_fill_matches_survey_node_count(O, tables):
    """Config 1 filled the reference's way: non-zero set(), then unset() of the
    tunnel voxels, gives the survey's pointer-octree node count at depth 8
    (548 325) and a free list holding every other slot."""
    T = tables["unset"]
    n = T.nodes()
    assert T.node_cnt == 548325
    assert len(free_chain(n, T.head)) == T.capacity - T.node_cnt


def test_tables_hold_the_terrain(O, tables):
    """at() (:141-160) equals the closed-form voxel function on
    random voxels and on every column's top three voxels, for both fills."""
    dim = 256
    h = O.height_map(dim)
    tops = O.column_tops(dim)
    rng = np.random.default_rng(3)
    xyz = rng.integers(0, dim, (20000, 3)).astype(np.int32)
    ys, xs = np.mgrid[0:dim, 0:dim]
    cols = np.stack([xs.ravel(), ys.ravel(), h.ravel()], 1).astype(np.int32)
    for dz in (0, -1, -2, 1):
        c = cols.copy()
        c[:, 2] += dz
        xyz = np.concatenate([xyz, c[(c[:, 2] >= 0) & (c[:, 2] < dim)]])
    want = O.voxels_at(dim, xyz, tops)
    for name, T in tables.items():
        got = np.array([T.at(*p) for p in xyz.tolist()], np.uint32)
        assert np.array_equal(got, want), name


def test_set0_leaves_reachable_empty_nodes(O, tables):
    """remove()'s set(..., 0) (:74-91) allocates the paths of tunnel voxels,
    air included, and leaves them allocated: reachable nodes with no child."""
    n = tables["set0"].nodes()
    seen, cur, empty = set(), [0], 0
    for _ in range(8):
        nxt = []
        for v in cur:
            c = n[v]
            if not c.any():
                empty += 1
            for k in range(8):
                if c[k] and _ < 7 and int(c[k]) not in seen:
                    seen.add(int(c[k]))
                    nxt.append(int(c[k]))
        cur = nxt
    assert empty > 1000
    assert tables["set0"].node_cnt > tables["unset"].node_cnt


@pytest.mark.parametrize("pitch", [0.0, -0.6])
def test_tables_trace_like_the_compact_octree(O, tables, pitch):
    """Config 1's rays (512x512, yaw 0.3) on the reference's own tables: the
    unset() table is the compact octree node for node, so records and PUSH
    counts equal the builder-shaped octree's; the set(..., 0) table walks its
    empty nodes (more PUSHes) to the same records."""
    compact = O.build_terrain(8, dedup=False)
    rays = O.raygen(0.3, pitch, 1.25, 512, 512)
    want = O.trace_batch(compact, O.Rcp(None), ORIGIN, rays, nthreads=8, want_push=True)
    for name, T in tables.items():
        got = O.trace_batch(T.pool(), O.Rcp(None), ORIGIN, rays, nthreads=8, want_push=True)
        for k in ("dir", "voxel"):
            assert np.array_equal(got[k], want[k]), (name, k)
        assert np.array_equal(got["t"].view(np.uint32), want["t"].view(np.uint32)), name
        assert np.all(got["t"][got["dir"] == 6] == 0)                  # miss t = 0.0F (:302)
        if name == "unset":
            assert np.array_equal(got["push"], want["push"])
        else:
            assert np.all(got["push"] >= want["push"]) and np.any(got["push"] > want["push"])


def root_emptied_table(O):
    """Hand-derived from ORT/och_octree.cpp:46-139, capacity 16, depth 3:
    set(0,0,0,5) allocates 1, 2; set(7,7,7,6) allocates 3, 4; unset(0,0,0)
    frees 2 then 1 (head 1); unset(7,7,7) frees 4 (its children[0] = 1), then
    3 (children[0] = 4), then empties the root: dealloc(0) writes head (3)
    into root.children[0] and sets head = 0.  The root now reaches the free
    list: root -> 3 -> 4, whose children[0] = 1 sits at the leaf level -- the
    reference traces "voxel 1" in the corner voxel (0, 0, 0)."""
    T = O.ORef(3, 16)
    T.set(0, 0, 0, 5)
    T.set(7, 7, 7, 6)
    T.unset(0, 0, 0)
    T.unset(7, 7, 7)
    return T


def test_root_emptied_quirk(O):
    T = root_emptied_table(O)
    n = T.nodes()
    assert T.head == 0
    assert n[0].tolist() == [3, 0, 0, 0, 0, 0, 0, 0]
    assert n[3].tolist() == [4, 0, 0, 0, 0, 0, 0, 0]
    assert n[4].tolist() == [1, 0, 0, 0, 0, 0, 0, 0]
    assert n[1].tolist() == [2, 0, 0, 0, 0, 0, 0, 0]
    assert n[2].tolist() == [5, 0, 0, 0, 0, 0, 0, 0]
    assert T.at(0, 0, 0) == 1 and T.at(7, 7, 7) == 0 and T.at(1, 0, 0) == 0
    # the trace sees the same: a ray at voxel (0,0,0)'s centre hits "voxel 1"
    d = np.array([1.06 - 1.5, 1.07 - 1.5, 1.065 - 1.5], np.float32)
    d /= np.linalg.norm(d)
    dr, vx, t, _ = O.trace(T.pool(), O.Rcp(None), ORIGIN, d)
    assert vx == 1 and dr in (3, 4, 5) and t > 0
    dr, vx, t, _ = O.trace(T.pool(), O.Rcp(None), ORIGIN, -d)
    assert (dr, vx, t) == (6, 0, 0.0)
    # the next allocation finds head == 0: the reference exit(0)s
    with pytest.raises(RuntimeError):
        T.set(5, 5, 5, 2)


def test_unset_of_absent_voxel_is_a_no_op(O):
    T = O.ORef(4, 64)
    T.set(3, 4, 5, 2)
    before = T.nodes()
    T.unset(9, 9, 9)              # path missing: returns before touching anything (:109-110)
    T.unset(3, 4, 4)              # same leaf node, another voxel: cleared, node not empty
    assert np.array_equal(T.nodes(), before)
    assert T.at(3, 4, 5) == 2
