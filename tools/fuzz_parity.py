"""Randomised parity campaign (GPU box): random scenes, rays and launch options
through the C ABI against the CPU oracle, bit for bit, for a fixed time.

Each case draws a depth (2..16), a voxel set (uniform scatter, solid boxes,
one-voxel slabs, checkerboards, clusters around dyadic corners), voxel ids up
to 2^32 - 1, and rays (origins inside the root, on dyadic planes of the
scene's depth, at the centre, outside the root; directions uniform, exactly
axis-aligned, with zero / denormal / tiny components, aimed at voxel centres,
corners and edges); then one launch path with random options:
  trace     och_gpu_trace_batch_dev, layout 0/1, cull 0/1/2, block 64/128/256
            (PUSH counts compared where the launch counts: cull 0 and 1)
  tiled     och_gpu_trace_batch_tiled_dev (rays as an image of random width)
  bounce    och_gpu_trace_bounce_batch_dev, compaction 0/1/2
  octree    the same scene as och::octree (0-based, miss t = 0.0F)
  render    camera frames (RGBA8) of 1-8 views of one random size, each with its
            own position, field of view, yaw and pitch; random palettes;
            natural or planned order (sometimes planned on other cameras); the
            heavy-tile split at random thresholds / segment counts / levels
  codes     every shard's indexed-colour slice (1-8 shards, round-robin or
            weighted row deals, primary or config 5; each shard planned, with
            the split, as each rank of the N = 8 bench) + shade_unshard
  bounce_frames  config 5 RGBA8 frames, every compaction mode
  image     och_gpu_trace_batch_image (host rays, x + y * W, 8x8 tiles)
  editor    h_octree::set edits flushed to the device pool in 1-3 windows
  steps     the N = 1 frame loop issued by the library (och_gpu_render_steps_dev)
  sharded_steps  the N > 1 window at world size 1: codes, RCCL exchange, shade
and compares direction, voxel id, t bits (and secondary records), or every
frame's pixels, with oracle/och_oracle.c.  The oracle is the checker here, as
in tests/.  --terrain P puts a fraction P of the cases on the reference's
terrain DAG at depth 10 or 12 (the bench's); --paths and --force-split narrow a
campaign (the split's own: --paths render,codes,sharded_steps --force-split).

Writes one JSON line per case and a summary to --out; exit 1 on any mismatch.
Usage: python tools/fuzz_parity.py --seconds 300 --out gpurun_out/fuzz.jsonl
(or --cases N; tests/test_gpu_fuzz.py runs a fixed-seed slice of it)"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def voxels_for(rng, depth):
    """A random voxel set (x, y, z, id) at this depth and its kind."""
    side = 1 << depth
    kind = rng.choice(["scatter", "boxes", "slab", "checker", "corners"])
    pts = []
    if kind == "scatter":
        k = int(rng.integers(1, min(side ** 3, 30000) + 1))
        pts = rng.integers(0, side, (k, 3))
    elif kind == "boxes":
        for _ in range(int(rng.integers(1, 4))):
            lo = rng.integers(0, side, 3)
            ext = np.minimum(rng.integers(1, max(2, min(side, 48)), 3), side - lo)
            g = np.stack(np.meshgrid(*[np.arange(lo[a], lo[a] + ext[a]) for a in range(3)], indexing="ij"), -1)
            pts.append(g.reshape(-1, 3))
        pts = np.concatenate(pts)
    elif kind == "slab":
        a = int(rng.integers(0, 3))
        q = int(rng.integers(0, side))
        n = min(side, 64)
        u, v = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
        u, v = u.ravel() * (side // n), v.ravel() * (side // n)
        pts = np.zeros((u.size, 3), np.int64)
        pts[:, a], pts[:, (a + 1) % 3], pts[:, (a + 2) % 3] = q, u, v
    elif kind == "checker":
        n = min(side, 24)
        lo = rng.integers(0, side - n + 1, 3)
        g = np.stack(np.meshgrid(*[np.arange(n)] * 3, indexing="ij"), -1).reshape(-1, 3)
        g = g[(g.sum(1) % 2) == 0]
        pts = g + lo
    else:
        for k in range(1, depth):
            c = (rng.integers(0, 1 << k, 3) * (side >> k))
            off = rng.integers(-2, 3, (12, 3))
            pts.append(np.clip(c + off, 0, side - 1))
        pts = np.concatenate(pts) if pts else rng.integers(0, side, (1, 3))
    pts = np.unique(np.asarray(pts, np.int64).reshape(-1, 3), axis=0)
    big = rng.random() < 0.3
    ids = rng.integers(1, 2 ** 32 if big else 256, pts.shape[0], dtype=np.uint64)
    return kind, [(int(x), int(y), int(z), int(i)) for (x, y, z), i in zip(pts, ids)]


def rays_for(rng, depth, vox, n):
    side = 1 << depth
    o = rng.uniform(1.0, 2.0, (n, 3))
    kinds = rng.integers(0, 4, n)
    dy = (rng.integers(0, side + 1, (n, 3)) / side) + 1.0            # dyadic planes of this depth
    pick = rng.random((n, 3)) < 0.5
    o = np.where((kinds == 1)[:, None] & pick, dy, o)
    o[kinds == 2] = 1.5
    out = kinds == 3
    o[out] = rng.uniform(0.5, 2.5, (out.sum(), 3))
    tgt = np.array([v[:3] for v in vox], np.float64)[rng.integers(0, len(vox), n)]
    tgt = tgt + rng.choice([0.0, 0.5, 1.0], (n, 3))                   # corners, centres, edges
    d = (1.0 + tgt / side) - o
    r = rng.random(n)
    d[r < 0.25] = rng.normal(size=((r < 0.25).sum(), 3))
    ax = (r >= 0.25) & (r < 0.32)
    d[ax] = 0.0
    d[ax, rng.integers(0, 3, ax.sum())] = rng.choice([-1.0, 1.0], ax.sum())
    zc = (r >= 0.32) & (r < 0.40)
    d[zc, rng.integers(0, 3, zc.sum())] = rng.choice([0.0, 1e-40, -1e-30, 1e-12], zc.sum())
    norm = np.linalg.norm(d, axis=1, keepdims=True)
    scale = np.where(rng.random((n, 1)) < 0.8, norm, 1.0)             # most normalised, some not
    d = np.where(norm > 0, d / np.where(scale > 0, scale, 1.0), [[0.6, 0.0, -0.8]])
    return o.astype(np.float32), d.astype(np.float32)


TERRAIN = {}


def terrain_rays(rng, n):
    """Rays for the terrain DAG: origins inside the cube (the camera's 1.5 among
    them), on its mid-planes, outside it; directions mostly downward (the
    ground fills z < 1.31), some axis-aligned or with zero components."""
    o = rng.uniform(1.0, 2.0, (n, 3))
    o[rng.random(n) < 0.2] = 1.5
    mid = rng.random((n, 3)) < 0.1
    o[mid] = rng.choice([1.25, 1.5, 1.75], mid.sum())
    out = rng.random(n) < 0.1
    o[out] = rng.uniform(0.6, 2.4, (out.sum(), 3))
    d = rng.normal(size=(n, 3))
    d[:, 2] -= np.abs(rng.normal(1.0, 0.5, n))
    zc = rng.random(n) < 0.08
    d[zc, rng.integers(0, 3, zc.sum())] = 0.0
    d /= np.maximum(np.linalg.norm(d, axis=1, keepdims=True), 1e-30)
    return o.astype(np.float32), d.astype(np.float32)


def to_octree(nodes, root, depth):
    """The 1-based DAG as och::octree's 0-based table: root first, 0 = empty."""
    n = nodes.shape[0]
    order = [root] + [i for i in range(1, n + 1) if i != root]
    new = {old: k for k, old in enumerate(order)}
    out = np.zeros_like(nodes)
    # interior levels hold node indices, the last level voxel ids: tell them apart by level
    level = {root: 0}
    stack = [root]
    while stack:
        i = stack.pop()
        if level[i] == depth - 1:
            continue
        for c in nodes[i - 1]:
            if c and int(c) not in level:
                level[int(c)] = level[i] + 1
                stack.append(int(c))
    for old, k in new.items():
        row = nodes[old - 1]
        if level.get(old, depth - 1) == depth - 1:
            out[k] = row
        else:
            out[k] = [new[int(c)] if c else 0 for c in row]
    return out


def render_case(rng, ort, O, torch, dev, pool, ref_pool, depth, opts, scene, o, d):
    """Camera frames (och_gpu_render_views_dev, RGBA8) of random views, sizes and
    palettes, in natural or planned launch order, with the heavy-tile split at
    random thresholds, segment counts and levels; against the oracle's raygen,
    trace and trace_pixel shading.  Returns (mismatching pixels, rays, hits)."""
    W, H = int(rng.integers(1, 321)), int(rng.integers(1, 201))
    nv = int(rng.integers(1, 3)) if rng.random() < 0.7 else int(rng.integers(3, 9))
    views, cams = random_views(rng, ort, depth, W, H, nv)
    pal = rng.integers(0, 2 ** 32, 6 * int(rng.integers(1, 300)), dtype=np.uint64).astype(np.uint32)
    pool.set_palette(pal)
    row_chunk = int(rng.choice([1, 2, 4, 8, 16]))
    plan = FORCE_SPLIT[0] or rng.random() < 0.6
    pool.set_option("tile_order", 2 if plan else 0)
    random_split(rng, pool, opts, depth, plan)
    moved = plan and rng.random() < 0.3           # planned on other cameras (bench.py's moving camera)
    opts.update({"W": W, "H": H, "views": nv, "row_chunk": row_chunk, "plan": plan, "moved": moved})
    if plan:
        pool.plan_views(random_views(rng, ort, depth, W, H, nv)[1] if moved else cams, row_chunk)
        opts["split_tiles"] = pool.get_option("split_tiles")
    rows = pool.slice_rows(H, row_chunk, 1)                            # a view's slice: whole row chunks
    out = torch.full((nv * rows * W,), 7, dtype=torch.int32, device=dev)
    pool.set_stream(torch.cuda.current_stream())
    pool.render_views_dev(cams, out, row_chunk)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32).reshape(nv, rows * W)[:, :H * W]
    return compare_frames(O, ref_pool, got, views, W, H, pal, False)


def random_views(rng, ort, depth, W, H, nv):
    """nv views of one size, each with its own position (outside the root now
    and then), field of view, yaw and pitch: views = [(pos, fov, yaw, pitch)]."""
    views = []
    for _ in range(nv):
        pos = rng.uniform(1.0, 2.0, 3) if rng.random() < 0.85 else rng.uniform(0.6, 2.4, 3)
        if rng.random() < 0.3:                                         # on dyadic planes of the scene
            pos = np.where(rng.random(3) < 0.5, 1.0 + rng.integers(0, (1 << depth) + 1, 3) / (1 << depth), pos)
        views.append((tuple(float(np.float32(v)) for v in pos), float(rng.choice([1.25, float(rng.uniform(0.2, 2.5))])),
                      float(rng.uniform(-3.2, 3.2)), float(rng.uniform(-1.5, 1.5))))
    return views, [ort.camera(pos, y, p, fov, W, H) for pos, fov, y, p in views]


def codes_case(rng, ort, O, torch, dev, pool, ref_pool, depth, opts, scene, o, d):
    """The multi-GPU frame path on one device: every shard's indexed-colour slice
    (och_gpu_render_codes_views_dev, primary or config 5) under a round-robin or
    weighted row deal, then och_gpu_shade_unshard_views_dev into RGBA8 frames."""
    W, H, nv = int(rng.integers(1, 193)), int(rng.integers(1, 121)), int(rng.integers(1, 9))
    n, rc = int(rng.integers(1, 9)), int(rng.choice([1, 2, 5, 8, 16]))
    bounce = bool(rng.random() < 0.4)
    views, cams = random_views(rng, ort, depth, W, H, nv)
    pal = rng.integers(0, 2 ** 32, 6 * int(rng.integers(1, 21)), dtype=np.uint64).astype(np.uint32)
    pool.set_palette(pal)
    chunks = -(-H // rc)
    if rng.random() < 0.5:
        deal = ort.deal_chunks(rng.uniform(0.1, 2.0, chunks), n, rng.uniform(0.3, 1.0, n))
        pool.set_row_deal(H, rc, n, deal)
    else:
        pool.set_row_deal(H, rc, n, None)
    plan = not bounce and (FORCE_SPLIT[0] or rng.random() < 0.5)
    pool.set_option("tile_order", 2 if plan else 0)
    random_split(rng, pool, opts, depth, plan)
    opts.update({"W": W, "H": H, "views": nv, "n_shards": n, "row_chunk": rc, "bounce": bounce, "plan": plan})
    rows = pool.slice_rows(H, rc, n)
    gathered = torch.full((n, nv, rows, W), 255, dtype=torch.uint8, device=dev)
    pool.set_stream(torch.cuda.current_stream())
    for s_ in range(n):
        if plan:                                   # each shard's own plan, as each rank makes it
            pool.plan_views(cams, rc, s_, n)
        pool.render_codes_views_dev(cams, gathered[s_], rc, s_, n, bounce)
    full = torch.empty((nv, H, W), dtype=torch.int32, device=dev)
    pool.shade_unshard_dev(gathered, full, W, H, rc, n, nv)
    torch.cuda.synchronize()
    got = full.cpu().numpy().view(np.uint32).reshape(nv, H * W)
    return compare_frames(O, ref_pool, got, views, W, H, pal, bounce)


def bounce_frames_case(rng, ort, O, torch, dev, pool, ref_pool, depth, opts, scene, o, d):
    """Config 5 RGBA8 frames (och_gpu_render_bounce_views_dev), every compaction mode."""
    W, H, nv = int(rng.integers(1, 193)), int(rng.integers(1, 121)), int(rng.integers(1, 9))
    rc = int(rng.choice([1, 4, 8, 16]))
    views, cams = random_views(rng, ort, depth, W, H, nv)
    pal = rng.integers(0, 2 ** 32, 6 * int(rng.integers(1, 300)), dtype=np.uint64).astype(np.uint32)
    pool.set_palette(pal)
    pool.set_option("bounce_compact", int(rng.integers(0, 3)))
    plan = rng.random() < 0.5
    pool.set_option("tile_order", 2 if plan else 0)
    if plan:
        pool.plan_views(cams, rc)
    opts.update({"W": W, "H": H, "views": nv, "row_chunk": rc, "plan": plan})
    rows = pool.slice_rows(H, rc, 1)
    out = torch.full((nv * rows * W,), 7, dtype=torch.int32, device=dev)
    pool.set_stream(torch.cuda.current_stream())
    pool.render_bounce_views_dev(cams, out, rc)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32).reshape(nv, rows * W)[:, :H * W]
    return compare_frames(O, ref_pool, got, views, W, H, pal, True)


FORCE_SPLIT = [False]


def random_split(rng, pool, opts, depth, plan):
    """The heavy-tile split's options where a launch can take it (planned order,
    block 64, the packed layout), at random thresholds, segment counts, levels."""
    if plan and opts["block"] == 64 and opts["layout"] == 1 and depth > 1 and (FORCE_SPLIT[0] or rng.random() < 0.6):
        split = {"split": int(rng.integers(1, 101)), "split_segs": int(rng.choice([2, 4, 8, 16])),
                 "split_level": int(rng.integers(1, depth))}
    else:
        split = {"split": 0}
    for k, v in split.items():
        pool.set_option(k, v)
    opts.update(split)


def steps_case(rng, ort, O, torch, dev, pool, ref_pool, depth, opts, scene, o, d):
    """The N = 1 frame loop issued by the library (och_gpu_render_steps_dev):
    n frames round-robin over B streams and frame buffers, primary or config 5."""
    W, H, nv = int(rng.integers(1, 193)), int(rng.integers(1, 121)), int(rng.integers(1, 9))
    rc, B, n = int(rng.choice([1, 4, 8, 16])), int(rng.integers(1, 4)), int(rng.integers(1, 7))
    bounce = bool(rng.random() < 0.4)
    views, cams = random_views(rng, ort, depth, W, H, nv)
    pal = rng.integers(0, 2 ** 32, 6 * int(rng.integers(1, 300)), dtype=np.uint64).astype(np.uint32)
    pool.set_palette(pal)
    opts.update({"W": W, "H": H, "views": nv, "row_chunk": rc, "buffers": B, "steps": n, "bounce": bounce})
    rows = pool.slice_rows(H, rc, 1)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream(device=dev) for _ in range(B - 1)]
    frames = [torch.full((nv * rows * W,), 7, dtype=torch.int32, device=dev) for _ in range(B)]
    pool.render_steps_dev(cams, frames, streams, n, row_chunk=rc, bounce=bounce)
    torch.cuda.synchronize()
    miss = hits = 0
    for b in range(min(B, n)):                                         # buffers no frame reached stay 7
        got = frames[b].cpu().numpy().view(np.uint32).reshape(nv, rows * W)[:, :H * W]
        m, _, hits = compare_frames(O, ref_pool, got, views, W, H, pal, bounce)
        miss += m
    pool.set_stream(torch.cuda.current_stream())
    return miss, n * nv * W * H, hits


COMM = []


def sharded_steps_case(rng, ort, O, torch, dev, pool, ref_pool, depth, opts, scene, o, d):
    """The N > 1 window at world size 1 (och_gpu_render_sharded_steps_dev on the
    library's RCCL communicator): colour codes, the exchange (all-gather, display
    rank, gather), the shade; several frames over B streams and buffer sets."""
    from octree_ray_tracing_amd.frame import ShardedFrame, ShardedSteps
    if not COMM:
        COMM.append(ort.RcclComm.local(0))
    comm = COMM[0]
    W, H, nv = int(rng.integers(1, 193)), int(rng.integers(1, 121)), int(rng.integers(1, 9))
    rc, B, n = int(rng.choice([1, 2, 5, 8, 16])), int(rng.integers(1, 4)), int(rng.integers(1, 6))
    bounce = bool(rng.random() < 0.4)
    exchange = str(rng.choice(["all_gather", "display", "gather"]))
    views, cams = random_views(rng, ort, depth, W, H, nv)
    pal = rng.integers(0, 2 ** 32, 6 * int(rng.integers(1, 21)), dtype=np.uint64).astype(np.uint32)
    pool.set_palette(pal)
    plan = FORCE_SPLIT[0] or rng.random() < 0.5
    pool.set_option("tile_order", 2 if plan else 0)
    random_split(rng, pool, opts, depth, plan and not bounce)
    if plan:
        pool.plan_views(cams, rc, 0, 1)
    opts.update({"W": W, "H": H, "views": nv, "row_chunk": rc, "buffers": B, "steps": n, "bounce": bounce,
                 "exchange": exchange, "plan": plan})
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream(device=dev) for _ in range(B - 1)]
    shade = "all" if exchange == "all_gather" else "display"
    mode = "gather" if exchange == "gather" else "all_gather"
    sfs = []
    for s_ in streams:
        with torch.cuda.stream(s_):
            sfs.append(ShardedFrame(pool, W, H, rc, n_views=nv, indexed=True, shade=shade, comm=comm,
                                    sharded=True, exchange=mode))
    for f in sfs:
        f.frames.fill_(7)
    ShardedSteps(sfs, streams, comm, cams, bounce=bounce).run(n)
    torch.cuda.synchronize()
    miss = hits = 0
    for b in range(min(B, n)):
        got = sfs[b].frames.cpu().numpy().view(np.uint32).reshape(nv, H * W)
        m, _, hits = compare_frames(O, ref_pool, got, views, W, H, pal, bounce)
        miss += m
    pool.set_stream(torch.cuda.current_stream())
    return miss, n * nv * W * H, hits


def compare_frames(O, ref_pool, got, views, W, H, pal, bounce):
    miss = hits = 0
    for v, (pos, fov, y, p) in enumerate(views):
        rays = O.raygen(y, p, fov, W, H)
        if bounce:
            r = O.trace_bounce_batch(ref_pool, O.Rcp(None), np.array(pos, np.float32), rays, nthreads=16)
            want = O.shade_bounce(r["dir"], r["voxel"], r["dir2"], pal)
        else:
            r = O.trace_batch(ref_pool, O.Rcp(None), np.array(pos, np.float32), rays, nthreads=16)
            want = O.shade_fast(r["dir"], r["voxel"], pal)
        miss += int((got[v] != want).sum())
        hits += int((r["dir"] < 6).sum())
    return miss, len(views) * W * H, hits


def image_case(rng, ort, O, torch, dev, pool, ref_pool, depth, opts, scene, o, d):
    """och_gpu_trace_batch_image: host rays in x + y * W order, traced as 8x8 tiles."""
    width = int(rng.integers(1, 600))
    opts["width"] = width
    hd, hv, ht = pool.trace_batch(o, d, width=width)
    r = O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16)
    miss = int((hd != r["dir"]).sum() + (hv != r["voxel"].view(np.uint32)).sum()
               + (ht.view(np.uint32) != r["t"].view(np.uint32)).sum())
    return miss, o.shape[0], int((r["dir"] < 6).sum())


def editor_case(rng, ort, O, torch, dev, pool, ref_pool, depth, opts, scene, o, d):
    """h_octree::set edits through the editor (och_editor_*), flushed to the
    device pool in one to three windows, traced; against the oracle on a DAG
    built afresh from the edited voxel set."""
    from conftest import sparse_dag
    nodes, root, vox = scene
    if depth > 16:
        return 0, 0, 0
    ed = ort.Editor(nodes, root, depth, capacity=int(nodes.shape[0] + 700 * depth + 64))   # <= 597 edits
    pool = ed.make_pool(device=0)
    for k, v in (("layout", opts["layout"]), ("cull", opts["cull"]), ("block", opts["block"])):
        pool.set_option(k, v)
    cells = {(x, y, z): v for x, y, z, v in vox}
    side = 1 << depth
    flushes = int(rng.integers(1, 4))
    n_edits = 0
    for _ in range(flushes):
        for _ in range(int(rng.integers(1, 200))):
            if cells and rng.random() < 0.4:                      # remove or recolour an existing voxel
                x, y, z = list(cells)[int(rng.integers(0, len(cells)))]
            else:
                x, y, z = (int(c) for c in rng.integers(0, side, 3))
            v = 0 if rng.random() < 0.3 else int(rng.integers(1, 2 ** 32, dtype=np.uint64))
            ed.set(x, y, z, v)
            n_edits += 1
            if v:
                cells[(x, y, z)] = v
            else:
                cells.pop((x, y, z), None)
        ed.flush(pool)
    opts.update({"edits": n_edits, "flushes": flushes})
    if not cells:
        ed.close()
        pool.close()
        return 0, 0, 0
    ref_nodes, ref_root = sparse_dag(depth, [(x, y, z, v) for (x, y, z), v in cells.items()])
    ref_pool = O.OraclePool(ref_nodes, ref_root, depth, 1)
    n = o.shape[0]
    od = torch.from_numpy(np.ascontiguousarray(o.reshape(-1))).to(dev)
    dd = torch.from_numpy(np.ascontiguousarray(d.reshape(-1))).to(dev)
    hd, hv, ht = (torch.empty(n, dtype=torch.int32, device=dev) for _ in range(3))
    pool.set_stream(torch.cuda.current_stream())
    pool.trace_batch_dev(od, dd, hd, hv, ht, None, n=n)
    torch.cuda.synchronize()
    r = O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16)
    miss = int((hd.cpu().numpy() != r["dir"]).sum() + (hv.cpu().numpy().view(np.uint32) != r["voxel"].view(np.uint32)).sum()
               + (ht.cpu().numpy().view(np.uint32) != r["t"].view(np.uint32)).sum())
    ed.close()
    pool.close()
    return miss, n, int((r["dir"] < 6).sum())


CASES = {"render": render_case, "codes": codes_case, "bounce_frames": bounce_frames_case, "image": image_case,
         "editor": editor_case, "steps": steps_case, "sharded_steps": sharded_steps_case}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=300)
    ap.add_argument("--seed", type=int, default=2026)
    ap.add_argument("--rays", type=int, default=60000)
    ap.add_argument("--cases", type=int, default=0, help="stop after this many cases (0: run for --seconds)")
    ap.add_argument("--out", default="gpurun_out/fuzz.jsonl")
    ap.add_argument("--paths", default="", help="comma list: only these paths (default: all)")
    ap.add_argument("--terrain", type=float, default=0.0,
                    help="probability of a case on the reference's terrain at depth 10 or 12 (the bench's DAG) "
                         "instead of a random scene")
    ap.add_argument("--force-split", action="store_true",
                    help="frame paths always planned, block 64, packed layout and split (the split's own campaign)")
    a = ap.parse_args(argv)
    import torch
    import octree_ray_tracing_amd as ort
    import oracle.oracle as O
    from conftest import sparse_dag

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(a.seed)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    fout = open(a.out, "w")
    t_end = time.time() + a.seconds
    cases = bad = rays_total = 0
    by_path = {}

    def dt(x, dtype=torch.int32):
        return torch.from_numpy(np.ascontiguousarray(x)).to(dev) if x is not None else None

    paths = ["trace", "trace", "tiled", "bounce", "octree", "render", "render", "codes", "bounce_frames", "image",
             "editor", "steps", "sharded_steps"]
    if a.paths:
        paths = [p for p in a.paths.split(",") if p]
    FORCE_SPLIT[:] = [a.force_split]
    while time.time() < t_end and not (a.cases and cases >= a.cases):
        if a.terrain and rng.random() < a.terrain:
            depth, kind, vox = int(rng.choice([10, 12])), "terrain", []
            if depth not in TERRAIN:
                t = ort.build_terrain(depth, use_gpu=True)
                TERRAIN[depth] = (t.nodes, t.root)
            nodes, root = TERRAIN[depth]
            o, d = terrain_rays(rng, a.rays)
            path = str(rng.choice([p for p in paths if p not in ("editor", "octree")] or ["trace"]))
        else:
            depth = int(rng.choice(np.arange(2, 17), p=np.r_[[1, 2, 3, 4, 4, 4, 4, 4, 3, 2, 2, 1, 1, 1, 1]] / 37))
            kind, vox = voxels_for(rng, depth)
            nodes, root = sparse_dag(depth, vox)
            o, d = rays_for(rng, depth, vox, a.rays)
            path = str(rng.choice(paths))
        n = o.shape[0]
        opts = {"layout": int(rng.integers(0, 2)), "cull": int(rng.integers(0, 3)),
                "block": int(rng.choice([64, 128, 256]))}
        if a.force_split:
            opts.update({"layout": 1, "block": 64})
        if path == "octree":
            onodes = to_octree(nodes, root, depth)
            pool = ort.Octree(onodes, depth, device=0)
            ref_pool = O.OraclePool(onodes, 0, depth, 0)
        else:
            pool = ort.HOctree(nodes, root, depth, device=0)
            ref_pool = O.OraclePool(nodes, root, depth, 1)
        for k, v in opts.items():
            pool.set_option(k, v)
        pool.set_stream(torch.cuda.current_stream())
        if path in CASES:
            if path == "editor":                   # the editor makes its own pool
                pool.close()
                pool = None
            miss, n, hits = CASES[path](rng, ort, O, torch, dev, pool, ref_pool, depth, opts, (nodes, root, vox), o, d)
            if pool is not None:
                pool.close()
            cases += 1
            rays_total += n
            bad += miss != 0
            by_path[path] = by_path.get(path, 0) + 1
            rec = {"case": cases, "path": path, "depth": depth, "scene": kind, "voxels": len(vox),
                   "nodes": int(nodes.shape[0]), "rays": n, "hits": hits, "opts": opts, "mismatches": miss}
            fout.write(json.dumps(rec) + "\n")
            fout.flush()
            print(f"[fuzz] {cases} {path} d{depth} {kind} vox {len(vox)} hits {hits} opts {opts} -> {miss}",
                  file=sys.stderr, flush=True)
            continue
        od, dd = dt(o.reshape(-1)), dt(d.reshape(-1))
        hd, hv, ht, hp = (torch.empty(n, dtype=torch.int32, device=dev) for _ in range(4))
        counts = opts["cull"] != 2
        if path == "bounce":
            pool.set_option("bounce_compact", int(rng.integers(0, 3)))
            bd, bv, bt = (torch.empty(n, dtype=torch.int32, device=dev) for _ in range(3))
            pool.trace_bounce_batch_dev(od, dd, hd, hv, ht, bd, bv, bt, hp if counts else None, n=n)
            ref = O.trace_bounce_batch(ref_pool, O.Rcp(None), o, d, nthreads=16, want_push=True)
        elif path == "tiled":
            width = int(rng.integers(1, 700))
            pool.trace_batch_tiled_dev(od, dd, width, hd, hv, ht, hp if counts else None, n=n)
            ref = O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16, want_push=True)
            opts["width"] = width
        else:
            pool.trace_batch_dev(od, dd, hd, hv, ht, hp if counts else None, n=n)
            ref = O.trace_batch(ref_pool, O.Rcp(None), o, d, nthreads=16, want_push=True)
        torch.cuda.synchronize()
        got = {"dir": hd.cpu().numpy(), "voxel": hv.cpu().numpy().view(np.uint32), "t": ht.cpu().numpy().view(np.uint32)}
        miss = int((got["dir"] != ref["dir"]).sum() + (got["voxel"] != ref["voxel"].view(np.uint32)).sum()
                   + (got["t"] != ref["t"].view(np.uint32)).sum())
        # PUSH counts: launches that count cull only at cull 2 (a culled ray counts 0)
        if counts and path != "bounce":
            miss += int((hp.cpu().numpy().view(np.uint32) != ref["push"]).sum())
        if path == "bounce":
            for k, b in (("dir2", bd), ("voxel2", bv), ("t2", bt)):
                g = b.cpu().numpy()
                r = ref[k]
                if k == "t2":
                    g, r = g.view(np.uint32), r.view(np.uint32)
                elif k == "voxel2":
                    g, r = g.view(np.uint32), r.view(np.uint32)
                miss += int((g != r).sum())
        pool.close()
        cases += 1
        rays_total += n
        bad += miss != 0
        by_path[path] = by_path.get(path, 0) + 1
        hits = int((ref["dir"] < 6).sum())
        rec = {"case": cases, "path": path, "depth": depth, "scene": kind, "voxels": len(vox), "nodes": int(nodes.shape[0]),
               "rays": n, "hits": hits, "opts": opts, "mismatches": miss}
        fout.write(json.dumps(rec) + "\n")
        fout.flush()
        print(f"[fuzz] {cases} {path} d{depth} {kind} vox {len(vox)} hits {hits} opts {opts} -> {miss}",
              file=sys.stderr, flush=True)
    for c in COMM:
        c.close()
    COMM.clear()
    summary = {"summary": True, "cases": cases, "rays": rays_total, "cases_with_mismatches": bad, "by_path": by_path,
               "seed": a.seed, "seconds": a.seconds}
    fout.write(json.dumps(summary) + "\n")
    fout.close()
    print(json.dumps(summary))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
