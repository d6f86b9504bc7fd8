"""Batches walked in coherence order (OCH_OPT_SORT, och_sort.hip): the rays of
och_gpu_trace_batch_dev and the config-5 bounce batch are sorted on the device
by origin cell and direction, the kernel walks ray perm[i] as its i-th ray and
writes its record at perm[i].  Records, PUSH counts and their order must be the
oracle's for every batch shape: shared and per-ray origins, camera rays in
row-major order, random rays, zero and denormal direction components, sizes on
either side of the sorting threshold (16384 rays) and ragged sizes."""
import numpy as np
import pytest

from test_gpu_parity import assert_same, assert_same_bounce, gpu_trace_bounce_dev, gpu_trace_dev

pytestmark = pytest.mark.gpu

ORIGIN = np.array([1.5, 1.5, 1.5], np.float32)


def _random(n, seed):
    rng = np.random.default_rng(seed)
    o = rng.uniform(1.01, 1.99, (n, 3)).astype(np.float32)
    d = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    d[: n // 20, 1] = 0.0                       # zero components (NaN t at every STEP)
    d[n // 20: n // 10] *= np.float32(1e-39)    # denormal directions
    return o, d


@pytest.mark.parametrize("depth", [8, 10])
def test_sorted_batches(ort, O, gpu_device, depth):
    tree = ort.build_terrain(depth)
    pool = ort.HOctree(tree.nodes, tree.root, depth, device=0)
    ref_pool = O.OraclePool(tree.nodes, tree.root, depth, 1)
    assert pool.get_option("sort") == 0
    cam = O.raygen(0.3, -0.6, 1.25, 1920, 1080)
    ro, rd = _random(100001, depth)
    cases = [(ORIGIN, cam), (ro, rd), (ro[:16383], rd[:16383]), (ro[:16384], rd[:16384]), (ORIGIN, rd[:40000])]
    refs = [O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16, want_push=True) for o, d in cases]
    pool.set_option("sort", 1)
    for layout in (1, 0):
        pool.set_option("layout", layout)
        for cull in (0, 1):
            pool.set_option("cull", cull)
            for (o, d), ref in zip(cases, refs):
                assert_same(gpu_trace_dev(pool, o, d), ref)                          # PUSH counts too (cull 1: not culled)
                assert_same(gpu_trace_dev(pool, o, d, want_push=False), ref, push=False)
    pool.set_option("cull", 1)
    pool.set_option("layout", 1)
    # host batches go through the same path
    hd, hv, ht = pool.trace_batch(ro, rd)
    assert_same({"dir": hd, "voxel": hv, "t": ht}, refs[1], push=False)
    # config 5: primary and secondary records
    for o, d in ((ORIGIN, cam), (ro, rd)):
        ref = O.trace_bounce_batch(ref_pool, O.Rcp(None), o, d, nthreads=16, want_push=True)
        assert_same_bounce(gpu_trace_bounce_dev(pool, o, d), ref)
    with pytest.raises(ort.OchError):
        pool.set_option("sort", 2)
    pool.close()
