"""The per-node skip's boxes (och_pool_slot_boxes, OCH_OPT_SKIP): for every
interior slot of a packed pool, the bounding box of the voxels under its child,
quantised outwards.  Checked here against an independent numpy restatement and
for being conservative: every voxel under a child lies inside its box.  The
skip itself is exact by DESIGN.md §4c and bit-exact against the oracle in the
GPU parity tests (every parity test runs with it on, its default)."""
import numpy as np
import pytest

Q = (4, 4, 16)


def levels_of(pk, proot, depth):
    level = np.zeros(pk.shape[0], np.int64)
    frontier = np.array([proot & 0xFFFFFF])
    level[frontier] = 1
    for lv in range(2, depth + 1):
        ch = pk[frontier]
        frontier = np.unique((ch & 0xFFFFFF)[ch != 0])
        level[frontier] = lv
    return level


def voxel_boxes(pk, level, depth):
    n = pk.shape[0]
    lo = np.full((n, 3), 1 << 40, np.int64)
    hi = np.full((n, 3), -1, np.int64)
    off = np.array([[c & 1, (c >> 1) & 1, (c >> 2) & 1] for c in range(8)], np.int64)
    for lv in range(depth, 0, -1):
        ids = np.nonzero(level == lv)[0]
        half = 1 << (depth - lv)
        for c in range(8):
            w = pk[ids, c].astype(np.int64)
            sel = ids[w != 0]
            if lv == depth:
                clo, chi = off[c], off[c] + 1
            else:
                cid = w[w != 0] & 0xFFFFFF
                ok = lo[cid, 0] <= hi[cid, 0]
                sel, cid = sel[ok], cid[ok]
                clo, chi = lo[cid] + off[c] * half, hi[cid] + off[c] * half
            lo[sel] = np.minimum(lo[sel], clo)
            hi[sel] = np.maximum(hi[sel], chi)
    return lo, hi


def expected_codes(pk, proot, depth):
    level = levels_of(pk, proot, depth)
    lo, hi = voxel_boxes(pk, level, depth)
    out = np.zeros(pk.shape, np.uint16)
    for v in np.nonzero((level > 0) & (level < depth))[0]:
        size = 1 << (depth - level[v])
        for k in range(8):
            w = int(pk[v, k])
            if not w:
                continue
            c = w & 0xFFFFFF
            if lo[c, 0] > hi[c, 0]:
                out[v, k] = 0xFFFF
                continue
            code = 0
            for a in range(3):
                bits = 2 if a < 2 else 4
                qlo = lo[c, a] * Q[a] // size
                qhi = -((-hi[c, a] * Q[a]) // size)
                code |= int(qlo) << (4 * a) | int(Q[a] - qhi) << (4 * a + bits)
            out[v, k] = code
    return out, level


@pytest.mark.parametrize("depth", [5, 7])
def test_slot_boxes_match_restatement(ort, depth):
    tree = ort.build_terrain(depth)
    pk, proot = ort.pack_pool(tree.nodes, tree.root, depth)
    got = ort.slot_boxes(pk, proot, depth)
    want, _ = expected_codes(pk, proot, depth)
    assert np.array_equal(got, want)
    assert (got != 0).any(), "the terrain's air leaves partial boxes"


def test_slot_boxes_are_conservative(ort):
    depth = 6
    tree = ort.build_terrain(depth)
    pk, proot = ort.pack_pool(tree.nodes, tree.root, depth)
    boxes = ort.slot_boxes(pk, proot, depth)
    level = levels_of(pk, proot, depth)
    n = 1 << depth
    # every voxel of the world, by walking the packed pool down from the root
    solid = np.zeros((n, n, n), bool)
    for x in range(n):
        for y in range(n):
            for z in range(n):
                solid[x, y, z] = ort._lib.call("och_pool_at", tree.nodes.ctypes.data, tree.root, depth, 1, x, y, z) != 0
    # the corner and size of every node on the paths, checked against its box
    stack = [(proot & 0xFFFFFF, 1, 0, 0, 0)]
    checked = 0
    while stack:
        v, lv, x0, y0, z0 = stack.pop()
        if lv == depth:
            continue
        half = 1 << (depth - lv)
        for k in range(8):
            w = int(pk[v, k])
            if not w:
                continue
            cx, cy, cz = x0 + (k & 1) * half, y0 + ((k >> 1) & 1) * half, z0 + ((k >> 2) & 1) * half
            sub = solid[cx:cx + half, cy:cy + half, cz:cz + half]
            b = int(boxes[v, k])
            if b == 0xFFFF:
                assert not sub.any()
            else:
                lo = [(b >> (4 * a)) & (3 if a < 2 else 15) for a in range(3)]
                hc = [(b >> (4 * a + (2 if a < 2 else 4))) & (3 if a < 2 else 15) for a in range(3)]
                inside = np.zeros_like(sub)
                s = [slice(lo[a] * half // Q[a], (Q[a] - hc[a]) * half // Q[a]) for a in range(3)]
                inside[s[0], s[1], s[2]] = True
                assert not (sub & ~inside).any(), (v, k, lv)
            checked += 1
            stack.append((w & 0xFFFFFF, lv + 1, cx, cy, cz))
    assert checked > 1000


def test_slot_boxes_refuse_deep_pools(ort):
    nodes = np.zeros((2, 8), np.uint32)
    nodes[0, 0] = 1
    pk = np.zeros((2, 8), np.uint32)
    with pytest.raises(ort.OchError):
        ort.slot_boxes(pk, 1, 21)
