"""bench.py -- primary-ray throughput of the MI355X SVO-DAG ray caster.

Workload (BASELINE.json configs[2] at N=1): the reference's terrain at depth 12
(4096^3, built in parallel by och_build_terrain), camera at (1.5,1.5,1.5),
yaw 0.3, fov 1.25.  One step = two frames, pitch 0 and pitch -0.6 (the two
views every BASELINE config is quoted at), each frame being the reference's
update_position + update_image (raygen, SVO-DAG traversal, palette shading)
as one fused gfx950 kernel writing the RGBA8 framebuffer.

N > 1 (weak scaling, configs[3]'s frame at N=4): the frame grows to
round(1920*sqrt(N)) x round(1080*sqrt(N)) so each rank keeps ~1920x1080 rays;
rows are dealt in 8-row chunks round-robin over ranks, and every frame ends
with an RCCL all-gather of the framebuffer slices plus an on-device unshard.
The node pool is built once on rank 0 and broadcast over RCCL.

Steps alternate over --inflight (default 3) HIP streams with their own frame
buffers, so one step's slowest rays (a few grazing tiles)
overlap the next step's bulk; every step is rendered in full.  The serial
frame latency is reported beside it (roofline.kernel_ms_idle_gpu).

value = rays of all frames of all ranks / (max over ranks of the timed wall
time), timed between barrier + synchronize on both sides.

The same line carries config 5 (BASELINE configs[4]) under "bounce": the same
frames with one mirrored secondary ray per hit pixel, in-block wavefront
compaction on, rays = primary + secondary.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
PITCHES = (0.0, -0.6)
YAW, FOV = 0.3, 1.25
ORIGIN = (1.5, 1.5, 1.5)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def frame_size(n_gpus: int, width: int | None, height: int | None):
    if width and height:
        return width, height
    s = math.sqrt(n_gpus)
    return int(round(1920 * s)), int(round(1080 * s))


def coll(fn, t, *args, **kw):
    """Run a collective on `t`.  RCCL takes device tensors; the gloo rehearsal
    backend (OCH_DIST_BACKEND=gloo, several ranks on one GPU) goes through the
    host."""
    import torch.distributed as dist

    if dist.get_backend() == "gloo" and t.is_cuda:
        h = t.cpu()
        fn(h, *args, **kw)
        t.copy_(h)
    else:
        fn(t, *args, **kw)


def build_pool_nodes(depth: int, rank: int, world: int, dev):
    """Rank 0 builds the DAG; the node array is broadcast to the other ranks."""
    import torch
    import torch.distributed as dist
    import octree_ray_tracing_amd as ort

    meta = torch.zeros(3, dtype=torch.int64, device=dev)
    nodes = None
    build_s = 0.0
    if rank == 0:
        # OCH_TREE_CACHE=<file.npz>: reuse a DAG built by an earlier run in the
        # same job (A/B tooling); off by default, every bench builds its tree.
        cache = os.environ.get("OCH_TREE_CACHE")
        if cache and os.path.exists(cache) and int(np.load(cache)["depth"]) == depth:
            z = np.load(cache)
            nodes, build_s = z["nodes"], float(z["build_s"])
            meta[:] = torch.tensor([nodes.shape[0], int(z["root"]), int(z["tree_nodes"])])
        else:
            tree = ort.build_terrain(depth)
            nodes, build_s = tree.nodes, tree.build_seconds
            meta[:] = torch.tensor([tree.n_nodes, tree.root, tree.tree_nodes])
            if cache:
                np.savez(cache, nodes=nodes, root=tree.root, depth=depth, tree_nodes=tree.tree_nodes,
                         build_s=build_s)
    if world > 1:
        coll(dist.broadcast, meta, 0)
    n, root, tree_nodes = (int(v) for v in meta.tolist())
    buf = torch.empty(n * 8, dtype=torch.int32, device=dev)
    if rank == 0:
        buf.copy_(torch.from_numpy(nodes.reshape(-1).view(np.int32)))
    if world > 1:
        coll(dist.broadcast, buf, 0)
    if rank != 0:
        nodes = buf.cpu().numpy().view(np.uint32).reshape(n, 8)
    return nodes, root, tree_nodes, build_s


def cpu_baseline(nodes, root, depth, width, height, budget_s: float = 8.0):
    """The CPU oracle (a C port of the reference tracer, native RCPPS) on this
    host, rank 0 only.  `value`: traversal of the two views' camera rays
    (generated once, outside the timed region) on every allowed thread for
    about budget_s; `value_1core`: the same two views once on one thread;
    `value_frame_path`: raygen + trace + numpy shading of two frames, the
    whole per-frame job as this harness runs it."""
    from oracle import oracle as O
    import octree_ray_tracing_amd as ort

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, 64))
    pool = O.OraclePool(nodes, root, depth, 1)
    rcp = O.Rcp(None)
    pal = ort.VoxelData().get_colours()
    origin = np.array(ORIGIN, np.float32)
    views = [O.raygen(YAW, p, FOV, width, height) for p in PITCHES]
    rays_done, t_total, frames = 0, 0.0, 0
    t_end = time.perf_counter() + budget_s
    while time.perf_counter() < t_end or frames < 2:
        rays = views[frames % 2]
        t0 = time.perf_counter()
        O.trace_batch(pool, rcp, origin, rays, nthreads=threads)
        t_total += time.perf_counter() - t0
        rays_done += rays.shape[0]
        frames += 1
    # One core (SURVEY 8d asks for 1 thread and all threads).
    t1 = time.perf_counter()
    for rays in views:
        O.trace_batch(pool, rcp, origin, rays, nthreads=1)
    t1 = time.perf_counter() - t1
    # The whole frame as this harness runs it (single-threaded raygen, numpy shading).
    tf = time.perf_counter()
    for p in PITCHES:
        r = O.trace_batch(pool, rcp, origin, O.raygen(YAW, p, FOV, width, height), nthreads=threads)
        O.shade_fast(r["dir"], r["voxel"], pal)
    tf = time.perf_counter() - tf
    try:
        cpu = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:
        cpu = "unknown"
    n2 = width * height * len(PITCHES)
    return {"value": rays_done / t_total / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{frames} traversals of full {width}x{height} camera frames (pitch 0 / -0.6 alternating, "
                      f"rays generated untimed), depth {depth}, {threads} threads on {cpu}, {t_total:.1f}s",
            "value_1core": n2 / t1 / 1e6,
            "sample_1core": f"the two views' traversal once on 1 thread, {t1:.1f}s",
            "value_frame_path": n2 / tf / 1e6,
            "sample_frame_path": f"raygen (1 thread) + traversal ({threads} threads) + numpy shading of the two views, {tf:.2f}s"}


# gfx950 VALU issue: a wave64 VALU instruction takes 2 cycles of its SIMD
# (MI355X_MICROARCH.md), 4 SIMDs per CU, 256 CUs, 2.4 GHz peak engine clock.
VALU_PEAK_GINST_S = 256 * 4 * 2.4 / 2


def valu_roofline(pmc, step_s: float):
    """The render kernel's real limiter: VALU wave-instructions per launch
    (rocprofv3 SQ_INSTS_VALU from profiles/pmc_summary.json, the same config)
    issued per second of the pipelined step, against the chip's issue peak."""
    if not pmc or "SQ_INSTS_VALU" not in pmc:
        return None
    insts = float(pmc["SQ_INSTS_VALU"])
    ach = insts / step_s / 1e9
    return {"bound": "valu-issue", "insts_per_launch": int(insts), "insts_per_wave": pmc.get("valu_insts_per_wave"),
            "achieved": round(ach, 1), "peak": VALU_PEAK_GINST_S, "unit": "G wave-instructions/s",
            "frac": round(ach / VALU_PEAK_GINST_S, 4),
            "source": "rocprofv3 --pmc SQ_INSTS_VALU (profiles/pmc_summary.json) / bench ms_per_step"}


def load_pmc(kernel: str, config_key: str):
    p = ROOT / "profiles" / "pmc_summary.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        return d.get(config_key, {}).get(kernel)
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--row-chunk", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=8.0)
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="pool launch option (och_gpu_set_option), e.g. tile_order=1")
    ap.add_argument("--no-bounce", action="store_true", help="skip the config-5 (secondary rays) measurement")
    ap.add_argument("--rgba-frames", action="store_true",
                    help="render and exchange RGBA8 slices instead of 1-byte indexed-colour codes")
    ap.add_argument("--inflight", type=int, default=3,
                    help="frames in flight: steps alternate over this many HIP streams, so one step's "
                         "slowest rays overlap the next step's bulk (1 = serialised)")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("OCH_DIST_BACKEND", "nccl")
    if backend == "gloo":
        # Rehearsal of the N > 1 path on a box with fewer GPUs than ranks:
        # ranks share devices round-robin and collectives go through the host.
        local %= max(1, torch.cuda.device_count())
    if world != a.gpus:
        log(f"warning: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    import octree_ray_tracing_amd as ort
    from octree_ray_tracing_amd.frame import ShardedFrame, slice_row_map

    W, H = frame_size(world, a.width, a.height)
    nodes, root, tree_nodes, build_s = build_pool_nodes(a.depth, rank, world, dev)
    pool = ort.HOctree(nodes, root, a.depth, device=local)
    pool.set_palette(ort.VoxelData().get_colours())
    for kv in a.opt:
        k, v = kv.split("=")
        pool.set_option(k, int(v))
    stream = torch.cuda.current_stream()
    pool.set_stream(stream)
    # Frames travel between ranks as 1-byte colour codes and are shaded after
    # the gather (same RGBA8 frames, a quarter of the bytes on xGMI).
    indexed = not a.rgba_frames and ort.VoxelData().get_colours().size // 6 <= pool.CODE_MAX_VOXELS
    cams = [ort.camera(ORIGIN, YAW, p, FOV, W, H) for p in PITCHES]
    # One frame buffer set and one HIP stream per frame in flight.
    streams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(max(1, a.inflight) - 1)]
    sfs = []
    for s_ in streams:
        with torch.cuda.stream(s_):
            sfs.append(ShardedFrame(pool, W, H, a.row_chunk, n_views=len(PITCHES), indexed=indexed))
    pool.set_stream(stream)
    sf = sfs[0]

    # PUSH counts of this rank's rays (for the algorithmic byte count): trace
    # the rank's own rows once with counting on; not part of the timed region.
    rows = torch.from_numpy(slice_row_map(H, a.row_chunk, world, rank))
    push_total, hits_total, rays_rank = 0, 0, 0
    dirs = torch.empty(W * H * 3, dtype=torch.float32, device=dev)
    o_t = torch.tensor(ORIGIN, dtype=torch.float32, device=dev)
    for cam in cams:
        pool.raygen_dev(cam, dirs)
        n = W * H
        hd = torch.empty(n, dtype=torch.int32, device=dev)
        hv = torch.empty(n, dtype=torch.int32, device=dev)
        ht = torch.empty(n, dtype=torch.float32, device=dev)
        hp = torch.empty(n, dtype=torch.int32, device=dev)
        pool.trace_batch_dev(o_t, dirs, hd, hv, ht, hp)
        mine = rows[rows >= 0].to(dev).long()
        hp2 = hp.view(H, W)[mine]
        push_total += int(hp2.sum().item())
        hits_total += int((hd.view(H, W)[mine] < 6).sum().item())
        rays_rank += int(mine.numel()) * W
    # trace-only throughput over resident rays (the och_gpu_trace_batch_dev path), N=1 only
    trace_only = None
    if world == 1:
        tms = []
        for cam in cams:
            pool.raygen_dev(cam, dirs)
            for _ in range(5):
                pool.trace_batch_dev(o_t, dirs, hd, hv, ht)
            for _ in range(10):
                s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s0.record(stream)
                pool.trace_batch_dev(o_t, dirs, hd, hv, ht)
                s1.record(stream)
                tms.append((s0, s1))
        torch.cuda.synchronize()
        ms = np.array([x.elapsed_time(y) for x, y in tms])
        trace_only = {"mrays_s": W * H * len(cams) * 10 / ms.sum() / 1e3, "ms_per_frame": float(ms.mean()),
                      "bytes_per_ray": 12 + 12 + 4 * push_total / (W * H * len(cams))}
        del hd, hv, ht, hp

    def step(k, ev=None, bounce=False):
        """One step: render both views of this rank's rows, all-gather, unshard --
        on stream k % inflight, into that stream's own frame buffers."""
        s_, f_ = streams[k % len(streams)], sfs[k % len(sfs)]
        pool.set_stream(s_)
        with torch.cuda.stream(s_):
            if ev is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s_)
            f_.render_local(cams, bounce)
            if ev is not None:
                e1.record(s_)
                ev.append((e0, e1))
            f_.exchange()

    # Frame latency: the render launch alone on an otherwise idle GPU.
    lat = []
    for k in range(max(a.warmup, 1) + 5):
        step(0, lat if k >= max(a.warmup, 1) else None)
        torch.cuda.synchronize()
    latency_ms = float(np.median([x.elapsed_time(y) for x, y in lat]))
    # warmup
    for k in range(a.warmup):
        step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = []
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(k, ev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    pool.set_stream(stream)
    kms = np.array([x.elapsed_time(y) for x, y in ev])
    t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        coll(dist.all_reduce, t_max, op=dist.ReduceOp.MAX)
    elapsed = float(t_max.item())

    # Config 5 (BASELINE configs[4]): the same frames with one mirrored
    # secondary ray per hit pixel, in-block wavefront compaction on; same
    # pipelining and timing discipline.  Rays = primary + secondary.
    bounce = None
    if not a.no_bounce:
        def timed_steps(n, bounce_on=True):
            for k in range(2):
                step(k, None, bounce_on)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            bev = []
            tb = time.perf_counter()
            for k in range(n):
                step(k, bev, bounce_on)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            el = torch.tensor([time.perf_counter() - tb], dtype=torch.float64, device=dev)
            if world > 1:
                coll(dist.all_reduce, el, op=dist.ReduceOp.MAX)
            return float(el.item()), float(np.mean([x.elapsed_time(y) for x, y in bev]))
        b_el, b_kms = timed_steps(a.steps)
        pool.set_option("bounce_compact", 0)
        nc_el, nc_kms = timed_steps(max(a.steps // 2, 3))
        pool.set_option("bounce_compact", 1)
        pool.set_stream(stream)
        hits = torch.tensor([hits_total], dtype=torch.int64, device=dev)
        if world > 1:
            coll(dist.all_reduce, hits)
        secondary = int(hits.item())
        primary = W * H * len(cams)
        bounce = {"workload": "configs[4]: depth-12, primary + 1-bounce secondary rays (divergent), "
                              "wavefront compaction on" + ("" if world == 1 else f", {world} GPUs"),
                  "value": round((primary + secondary) * a.steps / b_el / 1e6, 2), "unit": "Mrays/s",
                  "primary_mrays_s": round(primary * a.steps / b_el / 1e6, 2),
                  "ms_per_step": round(b_el / a.steps * 1e3, 4), "secondary_rays_per_step": secondary,
                  "kernel_ms": round(b_kms, 4),
                  "compaction_off_ms_per_step": round(nc_el / max(a.steps // 2, 3) * 1e3, 4),
                  "compaction_off_kernel_ms": round(nc_kms, 4)}

    frames = a.steps * len(cams)
    total_rays = W * H * frames
    value = total_rays / elapsed / 1e6
    # Algorithmic bytes of the dominant kernel (the render launch, both views)
    # on this rank: the pixel store per ray (1 B code, or 4 B RGBA8 + a 4 B
    # palette read per hit ray) + 4 B per child-slot read (PUSH).
    if indexed:
        bytes_per_launch = 1 * rays_rank + 4 * push_total
    else:
        bytes_per_launch = 4 * rays_rank + 4 * push_total + 4 * hits_total
    k_avg_ms = float(kms.mean())
    achieved = bytes_per_launch / (k_avg_ms * 1e-3) / 1e9
    pmc = load_pmc("k_render", f"d{a.depth}_{W}x{H}_n{world}")

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(nodes, root, a.depth, W, H, a.cpu_budget)

    if rank == 0:
        line = {
            "metric": "Mrays/sec primary traversal (depth-12 SVO-DAG, raygen+trace+shade per frame)",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: reference terrain fill (simplex heightmap + tunnels) at depth 12, built on the host",
            "config": {"workload": "configs[2]: 4096^3 depth-12 och_h_octree DAG, 1920x1080 primary rays, 1 MI355X"
                                   if world == 1 else
                                   f"configs[3]-style: depth-12 DAG, {W}x{H} frame row-sharded over {world} MI355X + RCCL all-gather",
                       "depth": a.depth, "width": W, "height": H, "frames_per_step": len(cams),
                       "pitches": list(PITCHES), "yaw": YAW, "fov": FOV, "row_chunk": a.row_chunk,
                       "dag_nodes": int(nodes.shape[0]), "tree_nodes": tree_nodes,
                       "pool_mb": round(nodes.nbytes / 2**20, 1), "build_s": round(build_s, 2),
                       "parallelism": f"rows{world}",
                       "frames": "indexed-colour codes, shaded after the exchange" if indexed else "rgba8",
                       "options": {k: pool.get_option(k) for k in pool.OPTIONS}},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": None if pmc is None else pmc.get("hbm_bytes_per_launch"),
                         "kernel": f"k_trace_grid<CameraSource,{'CodeSink' if indexed else 'FrameSink'}> (2 views per launch)",
                         "kernel_ms": round(k_avg_ms, 4),
                         "kernel_ms_idle_gpu": round(latency_ms, 4), "frames_in_flight": len(streams),
                         "bytes_per_launch": int(bytes_per_launch),
                         "push_per_ray": round(push_total / rays_rank, 3),
                         "valu": valu_roofline(pmc, elapsed / a.steps),
                         "note": "pointer-chase over an L2/MALL-resident DAG: latency/VALU-bound, not HBM-bound"},
            "cpu_baseline": cpu,
            "trace_batch": trace_only,
            "bounce": bounce,
        }
        print(json.dumps(line), flush=True)
    pool.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
