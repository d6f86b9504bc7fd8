"""The CPU oracle against everything that pins it:
the reference's own noise / z-order code (golden vectors made by
oracle/_ref/ref_harness from ORT/och_noise.h and ORT/och_z_order.cpp), the
known-answer values SURVEY.md records from the reference run in this
container, and the host's RCPPS instruction."""
import hashlib
import math

import numpy as np
import pytest

from conftest import GOLD


def test_noise_matches_reference_golden(O):
    g = np.load(GOLD / "noise_ref.npz")
    n2 = np.array([O.noise2(0.5, *p) for p in g["n2_in"].tolist()], np.float32)
    n3 = np.array([O.noise3(0.5, *p) for p in g["n3_in"].tolist()], np.float32)
    assert np.array_equal(n2.view(np.uint32), g["n2_out"].view(np.uint32))
    assert np.array_equal(n3.view(np.uint32), g["n3_out"].view(np.uint32))


def test_noise_matches_live_reference(O):
    if not O.ref_harness_available():
        pytest.skip("oracle/_ref/ref_harness not built (no /root/reference)")
    rng = np.random.default_rng(11)
    pts = rng.uniform(0, 512, (5000, 3)).astype(np.float32)
    ref = np.frombuffer(O.ref_run("noise3", pts, 0.5), np.float32)
    mine = np.array([O.noise3(0.5, *p) for p in pts.tolist()], np.float32)
    assert np.array_equal(ref.view(np.uint32), mine.view(np.uint32))


def test_child_index_convention_matches_z_encode(O):
    """Child slot c = x | y << 1 | z << 2 per level == the reference's z_encode_16 digits."""
    g = np.load(GOLD / "zorder_ref.npz")
    zin, zout = g["zin"].astype(np.int64), g["zout"]
    mine = np.zeros(len(zin), np.uint64)
    for lvl in range(16):
        digit = ((zin[:, 0] >> lvl) & 1) | (((zin[:, 1] >> lvl) & 1) << 1) | (((zin[:, 2] >> lvl) & 1) << 2)
        mine |= digit.astype(np.uint64) << np.uint64(3 * lvl)
    assert np.array_equal(mine, zout)


def test_intel_rcp_table_is_the_surveyed_one(intel_lut, known):
    k = known["rcp_lut_intel"]
    assert hashlib.sha256(intel_lut.tobytes()).hexdigest() == k["sha256"]
    assert intel_lut.size == 1 << k["log2_entries"]
    assert intel_lut[0] == int(k["entry0"], 16) and intel_lut[-1] == int(k["entry2047"], 16)


def test_rcp_table_model_matches_host_instruction(O, ort):
    """On this host the native RCPPS and the table model agree on sampled inputs."""
    lut = ort.host_rcp_lut()
    rng = np.random.default_rng(3)
    xs = (rng.integers(0, 1 << 31, 20000, dtype=np.uint64) | (1 << 31)).astype(np.uint32)
    for x in xs.tolist():
        if (x >> 23) & 0xFF == 0xFF:
            continue
        assert O.rcpps_native(x) == O.rcp_lut(x, lut), hex(x)


def _kat_tree(O, known):
    k = known["zero_direction_quirk"]
    T = O.HRef(k["depth"], 10)
    for x, y, z, v in k["voxels"]:
        T.set(x, y, z, v)
    return T, k


def test_zero_direction_quirk(O, known, intel_lut):
    T, k = _kat_tree(O, known)
    P = T.pool()
    for case in k["cases"]:
        d, v, t, _ = O.trace(P, O.Rcp(intel_lut), k["origin"], case["dir"])
        assert (d, v) == (case["direction"], case["voxel"])
        assert float(np.float32(t)) == float.fromhex(case["t_hex"])


def test_h_octree_table_counts_d8(O, known):
    T = O.HRef(8, 19)
    T.fill_terrain()
    assert T.fillcnt == known["terrain_d8"]["unique_nodes"]
    assert T.nodecnt == known["terrain_d8"]["tree_nodes"]


def _hist_quantiles(push, qs):
    """The survey's quantile: smallest k with cumulative count >= q * N."""
    cnt = np.bincount(np.minimum(push, 63))
    acc = np.cumsum(cnt)
    return [int(np.argmax(acc >= q * len(push))) for q in qs]


def test_traversal_statistics_d8(O, ort, known):
    k = known["traversal_d8_1080p"]
    tree = ort.build_terrain(8)
    pool = O.OraclePool(tree.nodes, tree.root, 8, 1)
    for i, pitch in enumerate(k["pitch"]):
        rays = O.raygen(0.3, pitch, 1.25, 1920, 1080)
        r = O.trace_batch(pool, O.Rcp(None), np.array([1.5] * 3, np.float32), rays, nthreads=8, want_push=True)
        n = len(rays)
        push, step, pop = (c / n for c in r["counts"])
        assert round(push, 1) == k["push_per_ray"][i]
        assert round(step, 1) == k["step_per_ray"][i]
        assert round(pop, 1) == k["pop_per_ray"][i]
        p = r["push"]
        hit, miss = r["dir"] < 6, r["dir"] == 6
        assert round(float(p[hit].mean()), 1) == k["push_hit_mean"][i]
        assert round(float(p[miss].mean()), 1) == k["push_miss_mean"][i]
        assert int(p.max()) == k["push_max"][i]
        assert _hist_quantiles(p, (0.5, 0.9, 0.99)) == k["push_p50_p90_p99"][i]


@pytest.mark.slow
def test_traversal_statistics_d10(O, ort, known):
    k = known["traversal_d10_1080p"]
    tree = ort.build_terrain(10)
    pool = O.OraclePool(tree.nodes, tree.root, 10, 1)
    for i, pitch in enumerate(k["pitch"]):
        rays = O.raygen(0.3, pitch, 1.25, 1920, 1080)
        r = O.trace_batch(pool, O.Rcp(None), np.array([1.5] * 3, np.float32), rays, nthreads=8)
        n = len(rays)
        assert round(100 * float(np.mean(r["dir"] < 6)), 1) == k["hit_percent"][i]
        assert [round(c / n, 1) for c in r["counts"]] == [k["push_per_ray"][i], k["step_per_ray"][i], k["pop_per_ray"][i]]


def test_h_octree_and_octree_tracers_agree(O, ort):
    """both reference tracers agree on 200k random rays (miss t excluded)."""
    dag = ort.build_terrain(7)
    tree = ort.build_terrain(7, dedup=False)
    pd = O.OraclePool(dag.nodes, dag.root, 7, 1)
    pt = O.OraclePool(tree.nodes, tree.root, 7, 0)
    rng = np.random.default_rng(1)
    o = rng.uniform(1.01, 1.99, (200000, 3)).astype(np.float32)
    d = rng.uniform(-1, 1, (200000, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    a = O.trace_batch(pd, O.Rcp(None), o, d, nthreads=8)
    b = O.trace_batch(pt, O.Rcp(None), o, d, nthreads=8)
    assert np.array_equal(a["dir"], b["dir"]) and np.array_equal(a["voxel"], b["voxel"])
    hit = a["dir"] != 6
    assert np.array_equal(a["t"][hit].view(np.uint32), b["t"][hit].view(np.uint32))
    assert np.all(np.isinf(a["t"][~hit])) and np.all(b["t"][~hit] == 0.0)


def test_golden_trace_vectors(O, intel_lut):
    g = np.load(GOLD / "trace_d6.npz")
    pool = O.OraclePool(g["nodes"], int(g["root"]), int(g["depth"]), 1)
    for name in ("cam", "rnd", "edge"):
        r = O.trace_batch(pool, O.Rcp(intel_lut), g[f"{name}_o"], g[f"{name}_d"], want_push=True)
        assert np.array_equal(r["dir"], g[f"{name}_dir"])
        assert np.array_equal(r["voxel"], g[f"{name}_vox"])
        assert np.array_equal(r["t"].view(np.uint32), g[f"{name}_t"])
        assert np.array_equal(r["push"], g[f"{name}_push"])


def test_sparse_dag_matches_reference_set(O):
    """tests/conftest.py's sparse_dag (the deep-tree GPU tests' pool builder)
    against the reference's own h_octree::set (HRef) at depth 16, the deepest
    its z_encode_16 coordinates reach: the same records, PUSH counts included."""
    from conftest import sparse_dag
    depth = 16
    rng = np.random.default_rng(16)
    c = 1 << (depth - 1)
    vox = []
    for k in range(2, depth - 1):
        base = c + rng.integers(-(1 << k), 1 << k, 3)
        for off in rng.integers(-2, 3, (40, 3)):
            x, y, z = (int(v) for v in np.clip(base + off, 0, (1 << depth) - 1))
            vox.append((x, y, z, int(1 + (x + y + z) % 4)))
    nodes, root = sparse_dag(depth, vox)
    T = O.HRef(depth, 17)
    for x, y, z, v in vox:
        T.set(x, y, z, v)
    o = np.tile(np.float32(1.5), (4000, 3)).astype(np.float32)
    d = rng.uniform(-1, 1, (4000, 3))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    tgt = np.array([v[:3] for v in vox], np.float64)[rng.integers(0, len(vox), 2000)] + 0.5
    aimed = (1.0 + tgt / (1 << depth)) - 1.5
    d[:2000] = (aimed / np.linalg.norm(aimed, axis=1, keepdims=True)).astype(np.float32)
    a = O.trace_batch(O.OraclePool(nodes, root, depth, 1), O.Rcp(None), o, d, want_push=True)
    b = O.trace_batch(T.pool(), O.Rcp(None), o, d, want_push=True)
    assert (a["dir"] < 6).sum() > 500
    for k in ("dir", "voxel", "push"):
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a["t"].view(np.uint32), b["t"].view(np.uint32))
    final = {(x, y, z): v for x, y, z, v in vox}      # a later set() of a voxel wins
    for (x, y, z), v in list(final.items())[::7]:
        assert T.at(x, y, z) == v
