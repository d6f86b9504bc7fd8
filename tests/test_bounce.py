"""Config 5 (BASELINE configs[4]) on the CPU oracle: the secondary ray of a
hit and the shading of a bounced pixel.  Build-defined -- the reference
renders primary rays only -- so the secondary records are pinned to the
oracle's primary tracer (itself pinned) and to the reference's
get_directional_hit_offset (ORT/test_och_h_octree.cpp:487-502)."""
import numpy as np


def test_bounce_ray_is_the_placement_point_mirrored(O):
    """o2 = (o + d*t) - offset(dir) in float32, d2 = d with the hit axis negated."""
    rng = np.random.default_rng(3)
    f = np.float32
    for depth in (3, 8, 12):
        half = f(f(1.0) / f(1 << depth)) / f(2)
        for _ in range(300):
            o = rng.uniform(1.01, 1.99, 3).astype(f)
            d = rng.uniform(-1, 1, 3).astype(f)
            direction = int(rng.integers(0, 6))
            t = f(rng.uniform(0, 1))
            o2, d2 = O.bounce_ray(o, d, direction, t, depth)
            axis = direction % 3
            off = np.zeros(3, f)
            off[axis] = half if direction < 3 else -half
            want_o = (o + d * t) - off
            want_d = d.copy()
            want_d[axis] = -want_d[axis]
            assert np.array_equal(o2.view(np.uint32), want_o.view(np.uint32))
            assert np.array_equal(d2.view(np.uint32), want_d.view(np.uint32))


def _floor_tree(O, roof: bool):
    """Depth-3 tree: a floor of voxel 1 at z = 0, optionally a roof of voxel 2 at z = 7."""
    T = O.HRef(3, 10)
    for x in range(8):
        for y in range(8):
            T.set(x, y, 0, 1)
            if roof:
                T.set(x, y, 7, 2)
    return T


def test_bounce_known_answers(O):
    """A ray falling on the floor hits its top face travelling -z (z_neg); the
    mirrored ray escapes (exit) without a roof and hits the roof's underside
    (z_pos, voxel 2) with one."""
    o = np.array([1.5, 1.5, 1.6], np.float32)
    d = np.array([0.3, 0.2, -0.9], np.float32)
    d /= np.linalg.norm(d)
    for roof, want2 in ((False, (6, 0)), (True, (2, 2))):
        T = _floor_tree(O, roof)
        r = O.trace_bounce_batch(T.pool(), O.Rcp(None), o, d[None, :])
        assert (int(r["dir"][0]), int(r["voxel"][0])) == (5, 1)
        assert (int(r["dir2"][0]), int(r["voxel2"][0])) == want2
        # the secondary origin sits half a voxel above the floor face z = 1 + 1/8
        o2, d2 = O.bounce_ray(o, d, 5, float(r["t"][0]), 3)
        assert abs(float(o2[2]) - (1.0 + 1.0 / 8 + 1.0 / 16)) < 1e-3 and d2[2] > 0


def test_no_bounce_records(O, ort):
    """Misses and inside-origin rays carry no secondary ray: direction -1."""
    tree = ort.build_terrain(6)
    pool = O.OraclePool(tree.nodes, tree.root, 6, 1)
    rays = O.raygen(0.3, 0.0, 1.25, 64, 36)
    r = O.trace_bounce_batch(pool, O.Rcp(None), np.array([1.5] * 3, np.float32), rays, want_push=True)
    miss = r["dir"] >= 6
    assert miss.any() and (~miss).any()
    assert np.all(r["dir2"][miss] == -1) and np.all(r["voxel2"][miss] == 0)
    assert np.all(r["dir2"][~miss] >= 0)
    # push counts cover both rays: never fewer than the primary ray's alone
    p1 = O.trace_batch(pool, O.Rcp(None), np.array([1.5] * 3, np.float32), rays, want_push=True)["push"]
    assert np.all(r["push"] >= p1) and np.all(r["push"][miss] == p1[miss])


def test_shade_bounce_matches_c(O, ort):
    pal = ort.VoxelData().get_colours()
    rng = np.random.default_rng(0)
    d = rng.integers(-1, 8, 4000)
    v = rng.integers(0, 6, 4000).astype(np.uint32)
    d2 = rng.integers(-1, 8, 4000)
    want = np.array([O.lib().ora_shade_bounce(int(a), int(b), int(c), pal.ctypes.data, pal.size // 6)
                     for a, b, c in zip(d, v, d2)], np.uint32)
    assert np.array_equal(O.shade_bounce(d, v, d2, pal), want)
    # blocked bounce halves RGB and keeps alpha; escaped bounce keeps the face colour
    c = int(pal[6 * 1 + 5])
    assert O.lib().ora_shade_bounce(5, 2, 6, pal.ctypes.data, pal.size // 6) == c
    assert O.lib().ora_shade_bounce(5, 2, 2, pal.ctypes.data, pal.size // 6) == ((c >> 1) & 0x7F7F7F) | (c & 0xFF000000)
