"""Native editor (och_editor_*, h_octree::set / at, ORT/och_h_octree.h:176-258)
against the oracle's exact restatement of the reference's hash table (HRef).

The editor numbers slots its own way, so parity is on what a user observes:
at() for every voxel, and traced hit records (direction, voxel, t bits, PUSH
count) over the edited trees.  CPU tests trace both pools with the CPU oracle
(the checker); the GPU test traces the editor's device mirror after flushes."""
import numpy as np
import pytest

ORIGIN = np.array([1.5, 1.5, 1.5], np.float32)


def _edits(seed, n, lo, hi):
    rng = np.random.default_rng(seed)
    out = []
    for x, y, z in rng.integers(lo, hi, (n, 3)).tolist():
        out.append((x, y, z, 0 if (x + y + z) % 3 == 0 else int(1 + (x * 7 + z) % 4)))
    return out


def _traces_equal(O, pool_a, pool_b, rays):
    rcp = O.Rcp(None)
    a = O.trace_batch(pool_a, rcp, ORIGIN, rays, want_push=True)
    b = O.trace_batch(pool_b, rcp, ORIGIN, rays, want_push=True)
    for k in ("dir", "voxel", "push"):
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a["t"].view(np.uint32), b["t"].view(np.uint32))
    return a


def _all_voxels(depth):
    d = 1 << depth
    return [(x, y, z) for z in range(d) for y in range(d) for x in range(d)]


def test_adopt_and_edit_matches_reference_table(ort, O):
    depth = 5
    T = O.HRef(depth, 14)
    T.fill_terrain()
    ed = ort.Editor(T.nodes(), T.root, depth)
    for x, y, z in _all_voxels(depth):
        assert ed.at(x, y, z) == T.at(x, y, z)
    for x, y, z, v in _edits(1, 400, 0, 32):
        T.set(x, y, z, v)
        ed.set(x, y, z, v)
    for x, y, z in _all_voxels(depth):
        assert ed.at(x, y, z) == T.at(x, y, z), (x, y, z)
    rays = O.raygen(0.3, -0.6, 1.25, 96, 54)
    r = _traces_equal(O, T.pool(), O.OraclePool(ed.nodes(), ed.root, depth), rays)
    assert (r["dir"] < 6).any() and (r["dir"] == 6).any()


def test_no_leaked_nodes(ort, O):
    """Exact refcounts: after edits the live count equals that of a fresh
    adoption of the same tree; clearing every voxel frees every slot."""
    depth = 4
    T = O.HRef(depth, 12)
    T.fill_terrain()
    ed = ort.Editor(T.nodes(), T.root, depth, capacity=4096)
    for x, y, z, v in _edits(2, 300, 0, 16):
        ed.set(x, y, z, v)
    fresh = ort.Editor(ed.nodes(), ed.root, depth, capacity=4096)
    assert ed.stats()["live_nodes"] == fresh.stats()["live_nodes"]
    for x, y, z in _all_voxels(depth):
        ed.set(x, y, z, 0)
    st = ed.stats()
    assert st["root"] == 0 and st["live_nodes"] == 0
    assert not ed.nodes().any()          # dead slots are zeroed
    ed.set(3, 4, 5, 2)                   # regrow from an empty tree
    assert ed.at(3, 4, 5) == 2 and ed.stats()["live_nodes"] == depth


def test_empty_tree_and_out_of_range(ort):
    ed = ort.Editor(np.zeros((0, 8), np.uint32), 0, 6, capacity=64)
    assert ed.root == 0 and ed.at(1, 2, 3) == 0
    ed.set(64, 0, 0, 1)                  # outside [0, 2^depth): ignored, as the reference
    ed.set(-1, 0, 0, 1)
    assert ed.root == 0
    ed.set(0, 0, 0, 0)                   # removing from an empty tree is a no-op
    assert ed.root == 0
    ed.set(63, 0, 17, 5)
    assert ed.at(63, 0, 17) == 5 and ed.at(62, 0, 17) == 0


def test_capacity_is_reported_before_the_edit(ort):
    depth = 6
    ed = ort.Editor(np.zeros((0, 8), np.uint32), 0, depth, capacity=2 * depth)
    ed.set(1, 1, 1, 1)                   # uses depth slots
    before = (ed.nodes(), ed.root)
    with pytest.raises(ort.OchError) as e:
        ed.set(60, 60, 60, 2)            # needs depth more; only depth free -> ok
        ed.set(30, 2, 40, 3)             # now fewer than depth free
    assert e.value.status == -6
    assert ed.at(60, 60, 60) == 2 and ed.at(30, 2, 40) == 0
    assert ed.at(1, 1, 1) == 1 and before[1] != 0


def test_bad_pools_are_refused(ort):
    nodes = np.zeros((2, 8), np.uint32)
    nodes[0, 0] = 7                      # child outside the pool
    with pytest.raises(ort.OchError):
        ort.Editor(nodes, 1, 2)
    nodes[0, 0] = 2                      # child is an empty interior node
    with pytest.raises(ort.OchError):
        ort.Editor(nodes, 1, 2)
    with pytest.raises(ort.OchError):
        ort.Editor(nodes, 1, 2, capacity=0)


def test_adopts_builder_pool(ort, O):
    """The parallel builder's DAG (och_build_terrain) adopted as is."""
    tree = ort.build_terrain(6)
    ed = ort.Editor(tree.nodes, tree.root, 6)
    ref = O.OraclePool(tree.nodes, tree.root, 6)
    rng = np.random.default_rng(3)
    for x, y, z in rng.integers(0, 64, (2000, 3)).tolist():
        assert ed.at(x, y, z) == ref.at(x, y, z)
    # adoption renumbers breadth-first: the builder's canonical pool comes back as is
    assert ed.root == tree.root and ed.stats()["live_nodes"] == tree.nodes.shape[0]
    assert np.array_equal(ed.nodes()[:tree.nodes.shape[0]], tree.nodes)


def _levels(nodes, root, depth):
    """Height above the voxels of every node reachable from root (1-based ids)."""
    lvl, order = {root: depth - 1}, [root]
    for v in order:
        if lvl[v]:
            for c in nodes[v - 1].tolist():
                if c and c not in lvl:
                    lvl[c] = lvl[v] - 1
                    order.append(c)
    return lvl


def test_canonical_adoption_matches_general_path(ort):
    """och_editor_create adopts a canonical DAG (a builder pool) in O(n),
    renumbering it breadth-first when it is numbered otherwise (here: ids
    reversed).  A pool holding a reachable duplicate node is not canonical and
    takes the general recursive adoption, which merges the duplicate.  All give
    the same slots, refcounts (the same slots again after the same edits) and
    statistics."""
    depth = 6
    tree = ort.build_terrain(depth)
    nodes, n = tree.nodes, tree.nodes.shape[0]
    lvl = _levels(nodes, tree.root, depth)
    # a node referenced from two slots; one reference is redirected to a copy
    seen, shared = {}, None
    for pid, h in lvl.items():
        if h:
            for k, c in enumerate(nodes[pid - 1].tolist()):
                if c and c in seen and shared is None:
                    shared = (c, pid, k)
                seen.setdefault(c, (pid, k))
    assert shared is not None
    c, pid, k = shared
    dup = np.vstack([nodes, nodes[c - 1][None, :]])
    dup[pid - 1, k] = n + 1
    # the same DAG with ids reversed (old id i -> n + 1 - i)
    rev = np.zeros_like(nodes)
    for i in range(1, n + 1):
        rev[n - i] = [n + 1 - c if (c and lvl.get(i, 0) > 0) else c for c in nodes[i - 1].tolist()]

    eds = [ort.Editor(nodes, tree.root, depth, capacity=1 << 16),
           ort.Editor(dup, tree.root, depth, capacity=1 << 16),
           ort.Editor(rev, n + 1 - tree.root, depth, capacity=1 << 16)]
    for e in eds[1:]:
        assert e.root == eds[0].root and e.stats() == eds[0].stats()
        assert np.array_equal(e.nodes(), eds[0].nodes())
    for x, y, z, v in _edits(5, 600, 0, 64):
        for e in eds:
            e.set(x, y, z, v)
    for e in eds[1:]:
        assert e.stats() == eds[0].stats()
        assert np.array_equal(e.nodes(), eds[0].nodes())


@pytest.mark.gpu
def test_gpu_mirror_after_flushes(ort, O, gpu_device):
    """Edits flushed to the device pool in small windows trace bit-identically
    to the reference table after the same edits."""
    from test_gpu_parity import assert_same, gpu_trace_dev
    depth = 7
    T = O.HRef(depth, 16)
    T.fill_terrain()
    ed = ort.Editor(T.nodes(), T.root, depth)
    pool = ed.make_pool(device=0)
    assert ed.stats()["dirty_count"] == 0
    rays = O.raygen(0.1, -0.3, 1.25, 320, 180)
    for batch in range(3):
        for x, y, z, v in _edits(10 + batch, 150, 30, 90):
            T.set(x, y, z, v)
            ed.set(x, y, z, v)
        st = ed.stats()
        assert 0 < st["dirty_count"] < st["capacity"]
        ed.flush(pool)
        assert ed.stats()["dirty_count"] == 0 and pool.get_root() == ed.root
        ref = O.trace_batch(T.pool(), O.Rcp(None), ORIGIN, rays, want_push=True)
        for layout in (1, 0):
            pool.set_option("layout", layout)
            assert_same(gpu_trace_dev(pool, ORIGIN, rays), ref)
            # launches without PUSH counts cull by the editor's voxel box, grown by
            # the edits above the terrain (OCH_OPT_CULL)
            assert_same(gpu_trace_dev(pool, ORIGIN, rays, want_push=False), ref, push=False)
    pool.close()
    ed.close()


@pytest.mark.gpu
def test_gpu_mirror_cleared_and_regrown(ort, O, gpu_device):
    """Root -> 0 (every voxel removed) and back, flushed each time."""
    from test_gpu_parity import gpu_trace_dev
    depth = 4
    T = O.HRef(depth, 12)
    T.fill_terrain()
    ed = ort.Editor(T.nodes(), T.root, depth, capacity=1024)
    pool = ed.make_pool(device=0)
    rays = O.raygen(0.3, -0.6, 1.25, 64, 36)
    for x, y, z in _all_voxels(depth):
        ed.set(x, y, z, 0)
    ed.flush(pool)
    assert pool.get_root() == 0
    for layout in (1, 0):
        pool.set_option("layout", layout)
        assert (gpu_trace_dev(pool, ORIGIN, rays)["dir"] == 6).all()
    R = O.HRef(depth, 12)
    for x, y, z, v in _edits(5, 200, 0, 16):
        ed.set(x, y, z, v)
        R.set(x, y, z, v)
    ed.flush(pool)
    ref = O.trace_batch(R.pool(), O.Rcp(None), ORIGIN, rays, want_push=True)
    for layout in (1, 0):
        pool.set_option("layout", layout)
        got = gpu_trace_dev(pool, ORIGIN, rays)
        assert np.array_equal(got["dir"], ref["dir"]) and np.array_equal(got["voxel"], ref["voxel"])
        nc = gpu_trace_dev(pool, ORIGIN, rays, want_push=False)
        assert np.array_equal(nc["dir"], ref["dir"]) and np.array_equal(nc["t"], ref["t"].view(np.uint32))
        assert np.array_equal(got["t"], ref["t"].view(np.uint32)) and np.array_equal(got["push"], ref["push"])
    pool.close()


def test_churn_reuses_slots_and_tombstones(ort):
    """Thousands of place/remove cycles in a small pool: freed slots are
    reused and the hash index's tombstones are swept (no capacity error)."""
    depth = 4
    ed = ort.Editor(np.zeros((0, 8), np.uint32), 0, depth, capacity=3 * depth)
    ed.set(0, 0, 0, 1)
    for i in range(3000):
        x, y, z = i % 16, (i * 7) % 16, (i * 3) % 16
        if (x, y, z) == (0, 0, 0):
            continue
        ed.set(x, y, z, 2)
        assert ed.at(x, y, z) == 2 and ed.at(0, 0, 0) == 1
        ed.set(x, y, z, 0)
        assert ed.at(x, y, z) == 0
    st = ed.stats()
    assert st["live_nodes"] == depth and st["high_water"] <= 3 * depth


@pytest.mark.gpu
def test_gpu_flush_pool_identity(ort, O, gpu_device):
    """pools are told apart by serial, not address.  A pool closed
    and replaced by a new one (likely at the same address), one editor flushed
    to two pools in turn, a pool rewritten by och_gpu_pool_update in between,
    and a second editor flushing the same pool: every flush leaves the device
    tracing exactly the reference table after the same edits."""
    from test_gpu_parity import assert_same, gpu_trace_dev
    depth = 6
    T = O.HRef(depth, 14)
    T.fill_terrain()
    ed = ort.Editor(T.nodes(), T.root, depth)
    rays = O.raygen(0.3, -0.6, 1.25, 160, 90)

    def check(pool):
        ref = O.trace_batch(T.pool(), O.Rcp(None), ORIGIN, rays, want_push=True)
        for layout in (1, 0):
            pool.set_option("layout", layout)
            assert_same(gpu_trace_dev(pool, ORIGIN, rays), ref)
        pool.set_option("layout", 1)

    def edit(seed):
        for x, y, z, v in _edits(seed, 60, 10, 50):
            T.set(x, y, z, v)
            ed.set(x, y, z, v)

    a = ed.make_pool(device=0)
    edit(1)
    ed.flush(a)
    check(a)
    a.close()                                   # its address is free for the next pool
    for k in range(3):
        b = ed.make_pool(device=0)
        edit(2 + k)
        ed.flush(b)
        check(b)
        b.close()
    p, q = ed.make_pool(device=0), ed.make_pool(device=0)
    for k in range(3):                          # alternate flushes: each pool misses the other's window
        edit(10 + k)
        ed.flush(p)
        check(p)
        edit(20 + k)
        ed.flush(q)
        check(q)
    # och_gpu_pool_update rewrites p (same content, caller-managed) -> next flush is whole
    nodes = ed.nodes()
    p.update(1, nodes, ed.root)
    edit(30)
    ed.flush(p)
    check(p)
    # a second editor with the same slot count writes q; the first editor's next flush is whole
    ed2 = ort.Editor(T.nodes(), T.root, depth, capacity=ed.stats()["capacity"])
    ed2.flush(q)
    edit(40)
    ed.flush(q)
    check(q)
    for x in (p, q):
        x.close()
    ed2.close()
    ed.close()
