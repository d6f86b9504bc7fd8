"""GPU parity on och::octree's own table (BASELINE configs[0]).

The capacity-sized _table that ORT/och_octree.cpp:14-160 leaves behind --
free list threaded through children[0], empty nodes from set(..., 0), the
root-emptied quirk -- uploaded unchanged (index_base 0, root 0, miss t 0,
ORT/och_octree.cpp:207, :302) and traced through the C ABI, every layout,
cull setting, against the oracle on the same table: direction,
voxel, t bits and PUSH count per ray.  The tables come from the oracle's ORef
restatement (tests/test_octree_table.py pins it)."""
import numpy as np
import pytest

from test_gpu_parity import assert_same, gpu_trace_dev
from test_octree_table import root_emptied_table

pytestmark = pytest.mark.gpu

ORIGIN = np.array([1.5, 1.5, 1.5], np.float32)


def _rays():
    rng = np.random.default_rng(11)
    o = rng.uniform(1.01, 1.99, (100000, 3)).astype(np.float32)
    d = rng.uniform(-1, 1, (100000, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d


@pytest.mark.parametrize("fill", ["unset", "set0"])
def test_reference_octree_table(ort, O, gpu_device, fill):
    """Config 1: depth-8 terrain in the reference's och::octree, filled with
    non-zero set() and then unset() ("unset") or set(..., 0) ("set0": allocated
    empty nodes stay reachable, child mask 0 in the packed layout)."""
    T = O.ORef(8, 1 << 20)
    T.fill_terrain(fill)
    nodes = T.nodes()
    ref_pool = T.pool()
    pool = ort.Octree(nodes, 8, device=0)
    assert pool.info()["n_nodes"] == nodes.shape[0]              # uploaded capacity-sized, as it lies
    cams = [(ORIGIN, O.raygen(0.3, p, 1.25, 512, 512)) for p in (0.0, -0.6)]
    ro, rd = _rays()
    cases = cams + [(ro, rd)]
    refs = [O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16, want_push=True) for o, d in cases]
    for layout in (0, 1):
        pool.set_option("layout", layout)
        for cull in (0, 1, 2):
            pool.set_option("cull", cull)
            for (o, d), ref in zip(cases, refs):
                got = gpu_trace_dev(pool, o, d)
                # PUSH counts are the reference's unless the diagnostic cull 2 is on
                assert_same(got, ref, push=cull != 2)
                hd, hv, ht = pool.trace_batch(o, d)            # no counts: culled when cull > 0
                assert_same({"dir": hd, "voxel": hv, "t": ht}, ref, push=False)
    pool.close()


def test_reference_octree_frames(ort, O, gpu_device):
    """The render path (raygen + trace + shade, camera shortcut and cull on)
    on the unset()-filled table: config 1's 512x512 frames, both pitches."""
    T = O.ORef(8, 1 << 20)
    T.fill_terrain("unset")
    pal = ort.VoxelData().get_colours()
    pool = ort.Octree(T.nodes(), 8, device=0)
    pool.set_palette(pal)
    for layout in (0, 1):
        pool.set_option("layout", layout)
        for p in (0.0, -0.6):
            r = O.trace_batch(T.pool(), O.Rcp(None), ORIGIN, O.raygen(0.3, p, 1.25, 512, 512), nthreads=16)
            want = O.shade(r["dir"], r["voxel"], pal).reshape(512, 512)
            assert np.array_equal(pool.render(ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, 512, 512)), want)
    pool.close()


def test_root_emptied_table_reproduced(ort, O, gpu_device):
    """unset() that empties the root deallocates index 0 (ORT/och_octree.cpp:
    126-135, :65-72): the root's children[0] then names the free list's head.
    The GPU reproduces the reference bit for bit rather than refusing: it
    traces the table as it lies, the corner voxel included ("voxel 1")."""
    T = root_emptied_table(O)
    rng = np.random.default_rng(2)
    o = rng.uniform(1.01, 1.99, (20000, 3)).astype(np.float32)
    tgt = rng.uniform(1.0, 1.125, (20000, 3)).astype(np.float32)    # aimed at the corner voxel
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    ref = O.trace_batch(T.pool(), O.Rcp(None), o, d, want_push=True)
    assert (ref["voxel"] == 1).sum() > 1000
    pool = ort.Octree(T.nodes(), 3, device=0)
    for layout in (0, 1):
        pool.set_option("layout", layout)
        for cull in (0, 1):
            pool.set_option("cull", cull)
            assert_same(gpu_trace_dev(pool, o, d), ref)
            hd, hv, ht = pool.trace_batch(o, d)
            assert_same({"dir": hd, "voxel": hv, "t": ht}, ref, push=False)
    pool.close()
