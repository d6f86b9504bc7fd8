"""bench.py -- primary-ray throughput of the MI355X SVO-DAG ray caster.

Workloads (BASELINE.json):
  N = 1  configs[2]: the reference's terrain at depth 12 (4096^3, built in
         parallel by och_build_terrain), 1920x1080, camera at (1.5,1.5,1.5),
         yaw 0.3, fov 1.25.
  N > 1  configs[3]: the same tree, one fixed 3840x2160 frame split over the
         N ranks (strong scaling; --scaling weak grows the frame with N
         instead).  Rows are dealt in 8-row chunks over ranks by their cost in one
         timed render on rank 0 (--deal rr: round-robin), and
         every frame ends with an RCCL all-gather of the slices (1-byte colour
         codes) plus an on-device shade + unshard.  Rank 0 builds the pool and
         broadcasts it over RCCL.
One step = two frames, pitch 0 and pitch -0.6 (the two views every BASELINE
config is quoted at), each being the reference's update_position +
update_image (raygen, SVO-DAG traversal, palette shading) as one fused gfx950
launch for both views, then the exchange.

Steps alternate over --inflight (default 3; 6 at N >= 8) HIP streams with their own frame
buffers, so one step's slowest rays (a few grazing tiles)
overlap the next step's bulk; every step is rendered in full.  The serial
frame latency is reported beside it (roofline.kernel_ms_serial).

value = rays of all frames of all ranks / (max over ranks of the timed wall
time), timed between barrier + synchronize on both sides.  `sustained`
repeats the measurement over >= --sustain seconds, three times (median).

The same line carries config 5 (BASELINE configs[4]) under "bounce": the same
frames with one mirrored secondary ray per hit pixel, in-block wavefront
compaction on, rays = primary + secondary.

The cpu leg (rank 0): the CPU oracle (test infrastructure) is timed on this
host's cores at N = 1 (`cpu_baseline`), and at every N it checks the frames
of the last timed step -- primary and config 5 -- pixel for pixel (`parity`).
"""
from __future__ import annotations

import argparse
import ctypes
import gc
import hashlib
import json
import math
import os
import statistics
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
# gfx950 VALU issue: a wave64 VALU instruction takes 2 cycles of its SIMD-32
# (MI355X_MICROARCH.md), 4 SIMDs per CU, 256 CUs, 2.4 GHz peak engine clock.
VALU_PEAK_GINST_S = 256 * 4 * 2.4 / 2
PITCHES = (0.0, -0.6)
YAW, FOV = 0.3, 1.25
ORIGIN = (1.5, 1.5, 1.5)
PMC_PATH = ROOT / "profiles" / "pmc_summary.json"
WINDOW_PATH = ROOT / "profiles" / "window_summary.json"


class FenceFreeEvent:
    """A HIP timing event created with hipEventDisableSystemFence, recorded on a
    torch stream.  torch.cuda.Event records with a system-scope release (an L2
    writeback and invalidate on every record): two per step put ~10 us of idle
    GPU between each lockstep group of frames in the bench window
    (profiles/r03/window/).  Timestamps need no such fence; the
    host reads them only after torch.cuda.synchronize().  The HIP runtime is
    torch's own (libamdhip64.so.7 is already loaded by soname)."""
    _hip = None

    def __init__(self):
        import ctypes
        if FenceFreeEvent._hip is None:
            hip = ctypes.CDLL("libamdhip64.so.7")
            hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
            hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
            FenceFreeEvent._hip = hip
        self._c = ctypes
        self.h = ctypes.c_void_p()
        rc = self._hip.hipEventCreateWithFlags(ctypes.byref(self.h), 0x20000000)    # hipEventDisableSystemFence
        if rc != 0:
            raise RuntimeError(f"hipEventCreateWithFlags failed ({rc})")

    def record(self, stream):
        rc = self._hip.hipEventRecord(self.h, self._c.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"hipEventRecord failed ({rc})")

    def elapsed_time(self, end) -> float:
        ms = self._c.c_float()
        rc = self._hip.hipEventElapsedTime(self._c.byref(ms), self.h, end.h)
        if rc != 0:
            raise RuntimeError(f"hipEventElapsedTime failed ({rc})")
        return float(ms.value)

    def __del__(self):
        if self._hip is not None and self.h:
            self._hip.hipEventDestroy(self.h)


def make_event(kind: str):
    return torch_event() if kind == "torch" else FenceFreeEvent()


def torch_event():
    import torch
    return torch.cuda.Event(enable_timing=True)


def pipeline_defaults(world: int, inflight=None, hw_queues=None):
    """Frames in flight and GPU_MAX_HW_QUEUES for a world size (DESIGN.md §5,
    tools/proxy_rank.py sweeps): 3 frames on the environment's queues below
    N = 8, 6 frames on 8 queues from N = 8.  Explicit values win."""
    if inflight is None:
        inflight = 6 if world >= 8 else 3
    if hw_queues is None and world >= 8:
        hw_queues = 8
    if inflight < 1:
        raise SystemExit("--inflight must be >= 1")
    if hw_queues is not None and not 1 <= hw_queues <= 32:
        raise SystemExit("--hw-queues must be in 1..32")
    return inflight, hw_queues


def plan_label(pool) -> str:
    """The render launches' workgroup order (OCH_OPT_TILE_ORDER, OCH_OPT_PLAN)."""
    if pool.get_option("tile_order") < 2:
        return "natural"
    p = pool.get_option("plan")
    shape = ("every workgroup costliest first" if p == 0 else "costliest and cheapest alternating" if p == 100
             else f"the costliest {p} % first, the rest in natural order")
    return f"planned from a timed planning frame: {shape}"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


METRIC = "Mrays/sec primary traversal (depth-12 SVO-DAG, raygen+trace+shade per frame)"


class Watchdog:
    """A deadline on every stage of a run, so a hang ends the run at once and
    says where.  A collective whose peer never comes (a rank that died, or never
    issued its side) blocks its stream and the host waiting on it; torch's own
    timeout does not cover the library's RCCL communicator or the spin-waits on
    the frame streams.  The stage names what this rank is doing; when its
    deadline passes, a thread of this process aborts the library's
    communicator(s) (ncclCommAbort, och_comm_abort), prints one JSON line
    naming the stage (rank 0 on stdout, the others on stderr) and ends the
    process with status 3 -- never by exec.  The launcher then stops the other
    ranks.  enter(stage, seconds) starts a stage; done() disarms."""

    EXIT = 3

    def __init__(self, rank: int, world: int, poll_s: float = 0.25, exit_fn=None, out=None):
        self.rank, self.world = rank, world
        self.stage, self.deadline, self.limit = "start", None, None
        self.aborts = []
        self.poll_s = poll_s
        self._exit = exit_fn or os._exit
        self._out = out
        self._lock = threading.Lock()
        self._t0 = time.monotonic()
        threading.Thread(target=self._run, name="bench-watchdog", daemon=True).start()

    def enter(self, stage: str, seconds: float):
        with self._lock:
            self.stage, self.limit = stage, float(seconds)
            self.deadline = time.monotonic() + float(seconds)

    def done(self):
        with self._lock:
            self.deadline = None

    def on_expiry(self, fn):
        """fn() runs (on the watchdog's thread, bounded) before the exit."""
        self.aborts.append(fn)

    def _run(self):
        while True:
            time.sleep(self.poll_s)
            with self._lock:
                late = self.deadline is not None and time.monotonic() > self.deadline
                stage, limit = self.stage, self.limit
            if late:
                self._expire(stage, limit)
                return

    def _expire(self, stage, limit):
        aborted = []

        def abort(fn):
            fn()
            aborted.append(fn)
        for fn in self.aborts:              # each abort on its own thread: a hung abort cannot hold the exit
            t = threading.Thread(target=abort, args=(fn,), daemon=True)
            t.start()
            t.join(timeout=10.0)
        line = {"metric": METRIC, "value": None, "unit": "Mrays/s", "n_gpus": self.world,
                "error": f"stage '{stage}' passed its {limit:g} s deadline on rank {self.rank}",
                "stage": stage, "rank": self.rank, "deadline_s": limit,
                "elapsed_s": round(time.monotonic() - self._t0, 1), "communicators_aborted": len(aborted)}
        out = self._out or (sys.stdout if self.rank == 0 else sys.stderr)
        try:
            print(json.dumps(line), file=out, flush=True)
            if out is not sys.stderr:
                log(f"bench watchdog: {line['error']}")
        finally:
            self._exit(self.EXIT)


# Deadlines per stage (seconds).  The driver gives a whole bench run 600 s;
# every stage of a healthy run takes a small part of its deadline (the
# slowest, the N > 1 parity check on the CPU, about 30 s), so only a hang
# reaches one.
DEADLINES = {"init": 120, "pool": 120, "comm": 120, "setup": 120, "exchange check": 60, "window": 60,
             "scaling base": 120, "cpu leg": 300, "other configs": 180, "teardown": 60}
# torch.distributed's timeout: rendezvous, and every torch collective (a rank
# waits in one at most through another rank's "pool" or "scaling base" stage).
PG_TIMEOUT_S = 150


def kernel_source_digest() -> str:
    """Identity of the kernel code a PMC profile was taken of."""
    h = hashlib.sha256()
    for f in ("och_kernels.hip", "och_internal.h", "Makefile"):
        h.update((ROOT / "octree_ray_tracing_amd" / "csrc" / f).read_bytes())
    return h.hexdigest()[:16]


def frame_size(n_gpus: int, width: int | None, height: int | None, scaling: str):
    if width and height:
        return width, height
    if n_gpus == 1:
        return 1920, 1080                                  # configs[2]
    if scaling == "strong":
        return 3840, 2160                                  # configs[3]
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
            # voxelised (k_brick_codes), hash-consed (k_intern) and renumbered on the GPU
            tree = ort.build_terrain(depth, use_gpu=True)
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


def cpu_leg(nodes, root, depth, width, height, frames, bounce_frames, time_it: bool, budget_s: float,
            moving=None):
    """The cpu leg, rank 0: the CPU oracle (a C port of the reference tracer
    with the host's native RCPPS; test infrastructure, used only here as the
    baseline and the checker).

    time_it (N = 1): `value` = traversal of the two views' camera rays
    (generated once, outside the timed region) on every allowed thread for
    about budget_s; `value_1core` = the same two views once on one thread;
    `value_frame_path` = raygen + trace + numpy shading of both frames.
    Always: the GPU frames of the last timed step (primary and config 5)
    against the oracle's, pixel for pixel."""
    from oracle import oracle as O
    import octree_ray_tracing_amd as ort

    allowed = len(os.sched_getaffinity(0))
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or allowed
    threads = max(1, min(threads, allowed, 64))
    hw_threads = os.cpu_count() or allowed
    pool = O.OraclePool(nodes, root, depth, 1)
    rcp = O.Rcp(None)
    pal = ort.VoxelData().get_colours()
    origin = np.array(ORIGIN, np.float32)
    t_ray = time.perf_counter()
    views = [O.raygen(YAW, p, FOV, width, height) for p in PITCHES]
    t_ray = time.perf_counter() - t_ray
    # parity of the bench's own frames (also the frame-path timing)
    tf = time.perf_counter()
    refs = [O.trace_batch(pool, rcp, origin, rays, nthreads=threads) for rays in views]
    want = [O.shade_fast(r["dir"], r["voxel"], pal).reshape(height, width) for r in refs]
    tf = time.perf_counter() - tf + t_ray
    parity = {"frames": len(want), "pixels": 0, "mismatches": 0}
    for v, w in enumerate(want):
        g = frames[v].view(np.uint32)
        parity["pixels"] += int(w.size)
        parity["mismatches"] += int(np.count_nonzero(g != w))
    if bounce_frames is not None:
        for v, rays in enumerate(views):
            r = O.trace_bounce_batch(pool, rcp, origin, rays, nthreads=threads)
            w = O.shade_bounce(r["dir"], r["voxel"], r["dir2"], pal).reshape(height, width)
            parity["frames"] += 1
            parity["pixels"] += int(w.size)
            parity["mismatches"] += int(np.count_nonzero(bounce_frames[v].view(np.uint32) != w))
    if moving is not None:                   # (yaw, frames) of the moving-camera window's last step
        yaw_m, frames_m = moving
        for v, p in enumerate(PITCHES):
            r = O.trace_batch(pool, rcp, origin, O.raygen(yaw_m, p, FOV, width, height), nthreads=threads)
            w = O.shade_fast(r["dir"], r["voxel"], pal).reshape(height, width)
            parity["frames"] += 1
            parity["pixels"] += int(w.size)
            parity["mismatches"] += int(np.count_nonzero(frames_m[v].view(np.uint32) != w))
    parity["checked"] = ("last timed step: both views, primary" + (" and config 5" if bounce_frames is not None else "")
                         + (" and the moving-camera window's last step" if moving is not None else "")
                         + ", GPU RGBA8 frames vs oracle trace + trace_pixel shading, native RCPPS on both sides")
    if not time_it:
        return None, parity
    rays_done, t_total, n = 0, 0.0, 0
    t_end = time.perf_counter() + budget_s
    while time.perf_counter() < t_end or n < 2:
        rays = views[n % 2]
        t0 = time.perf_counter()
        O.trace_batch(pool, rcp, origin, rays, nthreads=threads)
        t_total += time.perf_counter() - t0
        rays_done += rays.shape[0]
        n += 1
    # One core (SURVEY 8d asks for 1 thread and all threads).
    t1 = time.perf_counter()
    for rays in views:
        O.trace_batch(pool, rcp, origin, rays, nthreads=1)
    t1 = time.perf_counter() - t1
    try:
        cpu = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:
        cpu = "unknown"
    n2 = width * height * len(PITCHES)
    share = (f"{threads} of {hw_threads} hardware threads ({cpu}; this process's CPU affinity allows {allowed}, "
             f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')})")
    base = {"value": rays_done / t_total / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "cores_note": share, "hardware_threads": hw_threads, "affinity_threads": allowed, "cpu_model": cpu,
            "sample": f"{n} traversals of full {width}x{height} camera frames (pitch 0 / -0.6 alternating, "
                      f"rays generated untimed), depth {depth}, {share}, {t_total:.1f}s",
            "value_1core": n2 / t1 / 1e6,
            "sample_1core": f"the two views' traversal once on 1 thread, {t1:.1f}s",
            "value_frame_path": n2 / tf / 1e6,
            "sample_frame_path": f"raygen (1 thread) + traversal ({threads} threads) + numpy shading of the two views, "
                                 f"{tf:.2f}s"}
    return base, parity


def other_configs(a, dev, stream):
    """configs[1] (depth 10, 1920x1080, two views per pipelined step) and
    configs[0] (depth-8 och::octree, 512x512, trace batch + CPU oracle)."""
    import torch
    import octree_ray_tracing_amd as ort
    from octree_ray_tracing_amd.frame import ShardedFrame

    out = {}
    tree = ort.build_terrain(10, use_gpu=True)
    pool = ort.HOctree(tree.nodes, tree.root, 10, device=dev.index)
    pool.set_palette(ort.VoxelData().get_colours())
    pool.set_stream(stream)
    cams = [ort.camera(ORIGIN, YAW, p, FOV, 1920, 1080) for p in PITCHES]
    pool.plan_views(cams, a.row_chunk, 0, 1)
    pool.set_option("tile_order", 2)
    streams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(2)]
    sfs = []
    for s_ in streams:
        with torch.cuda.stream(s_):
            sfs.append(ShardedFrame(pool, 1920, 1080, a.row_chunk, n_views=2, indexed=True, direct=not a.no_direct))

    def run(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(n):
            pool.set_stream(streams[k % 3])
            with torch.cuda.stream(streams[k % 3]):
                sfs[k % 3].render(cams)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    run(5)
    el = run(a.steps)
    n_s = max(a.steps, int(1.0 / (el / a.steps)))
    sus = statistics.median([2 * 1920 * 1080 * n_s / run(n_s) / 1e6 for _ in range(3)])
    out["configs[1]"] = {"workload": "depth-10 och_h_octree DAG (334 025 nodes), 1920x1080, two views per step, 1 MI355X",
                         "value": round(2 * 1920 * 1080 * a.steps / el / 1e6, 2), "sustained": round(sus, 2),
                         "unit": "Mrays/s", "ms_per_step": round(el / a.steps * 1e3, 4)}
    pool.set_stream(stream)
    pool.close()
    # configs[0]: the pointer octree (index base 0, miss t = 0) at depth 8
    oct_ = ort.build_terrain(8, dedup=False, use_gpu=True)
    opool = ort.Octree(oct_.nodes, 8, device=dev.index)
    opool.set_stream(stream)
    cam = ort.camera(ORIGIN, YAW, 0.0, FOV, 512, 512)
    dirs = torch.empty(512 * 512 * 3, dtype=torch.float32, device=dev)
    opool.raygen_dev(cam, dirs)
    o_t = torch.tensor(ORIGIN, dtype=torch.float32, device=dev)
    bufs = [torch.empty(512 * 512, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.float32)]
    for _ in range(3):
        opool.trace_batch_dev(o_t, dirs, *bufs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        opool.trace_batch_dev(o_t, dirs, *bufs)
    torch.cuda.synchronize()
    g_el = (time.perf_counter() - t0) / 50
    gpu_rec = [b.cpu().numpy() for b in bufs]
    cpu_mrays, match = None, None
    if not a.no_parity:
        from oracle import oracle as O
        rays = O.raygen(YAW, 0.0, FOV, 512, 512)
        ref_pool = O.OraclePool(oct_.nodes, 0, 8, 0)
        t0 = time.perf_counter()
        ref = O.trace_batch(ref_pool, O.Rcp(None), np.array(ORIGIN, np.float32), rays, nthreads=1)
        cpu_mrays = 512 * 512 / (time.perf_counter() - t0) / 1e6
        match = bool(np.array_equal(gpu_rec[0], ref["dir"]) and np.array_equal(gpu_rec[1].view(np.uint32), ref["voxel"])
                     and np.array_equal(gpu_rec[2].view(np.uint32), ref["t"].view(np.uint32)))
    out["configs[0]"] = {"workload": "depth-8 och::octree (548 325 nodes, 0-based, miss t = 0), 512x512 primary rays",
                         "gpu_mrays_s": round(512 * 512 / g_el / 1e6, 2), "gpu_ms_per_frame": round(g_el * 1e3, 4),
                         "cpu_oracle_mrays_s_1core": None if cpu_mrays is None else round(cpu_mrays, 2),
                         "records_match_oracle": match}
    opool.close()
    return out


def single_gpu_base(a, nodes, root, W, H, cams, streams, dev, frames_ref):
    """scaling_base (N > 1, rank 0 alone): the same W x H two-view frame on one
    GPU, rendered the way the N = 1 bench renders configs[2] -- the fused RGBA8
    launch (raygen + traversal + trace_pixel shading) of both views, three
    frames in flight, the window issued by one och_gpu_render_steps_dev call,
    the launch order planned at the library's default -- while the other ranks
    wait at a barrier.  frames_ref: the sharded run's last RGBA8 frames on rank
    0, which this run's must equal (same cameras)."""
    import torch
    import octree_ray_tracing_amd as ort
    from octree_ray_tracing_amd._lib import Camera, load as load_lib

    lib = load_lib()
    B = min(3, len(streams))
    st = list(streams[:B])
    pool = ort.HOctree(nodes, root, a.depth, device=dev.index)
    try:
        pool.set_palette(ort.VoxelData().get_colours())
        for kv in a.opt:
            k, v = kv.split("=")
            pool.set_option(k, int(v))
        pool.set_stream(st[0])
        if not any(kv.startswith("tile_order=") for kv in a.opt):
            pool.set_option("tile_order", 2)
        if pool.get_option("tile_order") >= 2:
            pool.plan_views(cams, a.row_chunk, 0, 1)
        frames = [torch.empty((len(cams), H, W), dtype=torch.int32, device=dev) for _ in range(B)]
        arr = (Camera * len(cams))(*cams)
        sp = (ctypes.c_void_p * B)(*[s_.cuda_stream for s_ in st])
        fp = (ctypes.c_void_p * B)(*[f.data_ptr() for f in frames])

        def drain():
            while not all(s_.query() for s_ in st):
                pass
            torch.cuda.synchronize()

        def window(n):
            drain()
            t0 = time.perf_counter()
            if lib.och_gpu_render_steps_dev(pool._h, ctypes.cast(arr, ctypes.c_void_p), len(cams), n, sp, fp, B,
                                            None, None, a.row_chunk, 0):
                raise RuntimeError(f"scaling_base: {lib.och_last_error().decode()}")
            drain()
            return time.perf_counter() - t0

        window(max(a.warmup, 1))
        el = window(a.steps)
        last = frames[(a.steps - 1) % B].cpu().numpy()
        rays = W * H * len(cams)
        out = {"value": round(rays * a.steps / el / 1e6, 2), "unit": "Mrays/s",
               "ms_per_step": round(el / a.steps * 1e3, 4), "steps": a.steps, "frames_in_flight": B,
               "workload": f"the same {W}x{H} two-view frame on one MI355X (rank 0 alone): the N = 1 bench's path "
                           "(fused RGBA8 launch, och_gpu_render_steps_dev window)",
               "frames_equal_sharded": None if frames_ref is None else bool(np.array_equal(last, frames_ref))}
        if a.sustain > 0:
            n_s = max(a.steps, int(math.ceil(a.sustain / (el / a.steps))))
            out["sustained"] = round(statistics.median([rays * n_s / window(n_s) / 1e6 for _ in range(3)]), 2)
        return out
    finally:
        torch.cuda.synchronize()
        pool.close()


def group_bench(a):
    """`bench.py --gpus N --launch group`: one process drives N devices through
    the library's device group (och_frame_group_*, the form a C++ host of the
    reference would use): a pool replica per device, rows dealt by one timed
    render (och_frame_group_plan), per frame every device renders its slice
    as colour codes, RCCL all-gathers the slices (ncclCommInitAll
    communicators, one issuing thread per device) and shades the whole frame.
    A window is one och_frame_group_render_steps call; value = the frames'
    rays / the wall time between synchronisations of every device.  The
    last frame of every device is checked against the oracle (rank 0's) and
    against rank 0's copy."""
    import torch
    import octree_ray_tracing_amd as ort
    from octree_ray_tracing_amd.frame import FrameGroup

    n = a.gpus
    inflight, hw_queues = pipeline_defaults(n, a.inflight, a.hw_queues)
    if hw_queues is not None and os.environ.get("GPU_MAX_HW_QUEUES") != str(hw_queues):
        raise SystemExit("--launch group: GPU_MAX_HW_QUEUES must be set before HIP starts (main does)")
    wd = Watchdog(0, n)
    wd.enter("setup", DEADLINES["setup"])
    W, H = frame_size(n, a.width, a.height, a.scaling)
    torch.cuda.set_device(0)
    tree = ort.build_terrain(a.depth, use_gpu=True)
    cams = [ort.camera(ORIGIN, YAW, p, FOV, W, H) for p in PITCHES]
    g = FrameGroup(tree.nodes, tree.root, a.depth, devices=list(range(n)))
    try:
        g.set_palette(ort.VoxelData().get_colours())
        for kv in a.opt:
            k, v = kv.split("=")
            g.set_option(k, int(v))
        if not any(kv.startswith("split") for kv in a.opt):      # as the rank path: by world size
            for k, v in ort.split_defaults(n).items():
                g.set_option(k, v)
        g.plan(cams, a.row_chunk)

        def window(steps):
            wd.enter("window", DEADLINES["window"])
            g.synchronize()
            t0 = time.perf_counter()
            g.render_steps(cams, steps, inflight, a.row_chunk)
            g.synchronize()
            el_ = time.perf_counter() - t0
            wd.enter("setup", DEADLINES["setup"])
            return el_

        window(max(a.warmup, 1))
        el = window(a.steps)
        frames = [g.download(r) for r in range(n)]
        rays = W * H * len(cams)
        sustained = None
        if a.sustain > 0:
            n_s = max(a.steps, int(math.ceil(a.sustain / (el / a.steps))))
            vals = [rays * n_s / window(n_s) / 1e6 for _ in range(3)]
            sustained = {"value": round(statistics.median(vals), 2), "unit": "Mrays/s", "steps_per_run": n_s,
                         "values": [round(v, 2) for v in vals]}
    finally:
        g.close()
    parity = None
    wd.enter("cpu leg", DEADLINES["cpu leg"])
    if not a.no_parity:
        _, parity = cpu_leg(tree.nodes, tree.root, a.depth, W, H, frames[0], None, time_it=False, budget_s=0)
        parity["devices_equal_rank0"] = all(np.array_equal(f, frames[0]) for f in frames)
        if not parity["devices_equal_rank0"]:
            parity["mismatches"] += 1
    line = {
        "metric": METRIC,
        "value": round(rays * a.steps / el / 1e6, 2), "unit": "Mrays/s", "n_gpus": n, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: the reference's terrain fill at depth %d, built on the GPU (och_build_terrain)" % a.depth,
        "config": {"workload": (f"{W}x{H}, two views per step, depth-{a.depth} DAG over {n} MI355X from one process "
                                "(och_frame_group_*)"),
                   "launch": "one process, one issuing thread per device (och_frame_group_render_steps)",
                   "exchange": "RCCL all-gather (ncclCommInitAll communicators), every device shades the frame",
                   "row_deal": "och_frame_group_plan: chunks dealt by their cost in one timed render",
                   "frames_in_flight": inflight, "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                   "width": W, "height": H, "depth": a.depth,
                   "dag_nodes": int(tree.n_nodes), "parallelism": f"rows{n}"},
        "sustained": sustained, "parity": parity, "roofline": None, "cpu_baseline": None,
    }
    print(json.dumps(line), flush=True)
    wd.done()
    if parity is not None and parity["mismatches"]:
        raise SystemExit("group frames differ from the oracle")


def load_pmc(kernel: str, config_key: str):
    """The committed rocprofv3 PMC summary of this configuration, if it was
    taken of the kernel source in this tree (profiles/pmc_summary.json,
    written by tools/pmc_summary.py)."""
    if not PMC_PATH.exists():
        return None, "no profiles/pmc_summary.json"
    try:
        d = json.loads(PMC_PATH.read_text())
    except Exception as e:
        return None, f"unreadable PMC summary: {e}"
    if d.get("config") != config_key:
        return None, f"PMC summary is of {d.get('config')}, not {config_key}"
    if d.get("kernel_source_sha") != kernel_source_digest():
        return None, "PMC summary was taken of other kernel sources (stale profile)"
    return d.get("kernels", {}).get(kernel), "profiles/pmc_summary.json"


def load_window():
    """The committed rocprofv3 kernel-trace summary of the bench's pipelined
    window (profiles/window_summary.json, written by tools/window_trace.py),
    if it was taken of the kernel source in this tree."""
    if not WINDOW_PATH.exists():
        return None
    try:
        d = json.loads(WINDOW_PATH.read_text())
    except Exception:
        return None
    if d.get("kernel_source_sha") != kernel_source_digest():
        return {"source": "profiles/window_summary.json", "stale": True}
    keep = ("config", "steps", "ms_per_step_trace", "busy_union_ms_per_step", "kernel_ms_sum_per_step",
            "mean_concurrency", "concurrency_hist_ms", "render_mean_ms")
    return {"source": "profiles/window_summary.json", **{k: d.get(k) for k in keep}}


def resolve_launch(gpus: int, env, launch: str, n_devices: int) -> str:
    """How `bench.py --gpus N` runs, decided before HIP starts:
      "rank"  -- this process is one rank of a launcher's job (WORLD_SIZE set,
                 e.g. the driver's torch.distributed.run), or N = 1;
      "procs" -- no launcher and N > 1: start N ranks under
                 torch.distributed.run as child processes and exit with their
                 status (never exec: this process has not touched the GPU);
      "group" -- --launch group: this one process drives N devices through
                 och_frame_group_* (one issuing thread per device).
    Exits non-zero, instead of silently measuring fewer GPUs, when fewer than
    N devices are visible or when WORLD_SIZE disagrees with --gpus.
    n_devices: torch.cuda.device_count() (does not initialise HIP here)."""
    if gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    world = env.get("WORLD_SIZE")
    if world is not None:
        if launch == "group":
            raise SystemExit("--launch group drives every device from one process; run it without a launcher")
        if int(world) != gpus:
            raise SystemExit(f"--gpus {gpus} but WORLD_SIZE {world}: refusing to measure a different GPU count")
        # the gloo rehearsal runs several ranks per GPU on purpose
        if env.get("OCH_DIST_BACKEND", "nccl") != "gloo" and n_devices < int(world):
            raise SystemExit(f"WORLD_SIZE {world} ranks but {n_devices} GPU(s) visible")
        return "rank"
    if launch == "group":
        if n_devices < gpus:
            raise SystemExit(f"--gpus {gpus} asked, {n_devices} GPU(s) visible")
        return "group"
    if gpus == 1:
        return "rank"
    if n_devices < gpus:
        raise SystemExit(f"--gpus {gpus} asked, {n_devices} GPU(s) visible: refusing to run fewer ranks")
    return "procs"


def spawn_ranks(gpus: int, argv) -> int:
    """`bench.py --gpus N` without a launcher: the same N-rank job the driver
    starts (torch.distributed.run, one process per GPU, 127.0.0.1), run as a
    child process; returns its exit status."""
    import socket
    import subprocess

    with socket.socket() as s:                 # a free rendezvous port on the loopback
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve()), *argv]
    log(f"bench: no launcher in the environment; starting {gpus} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd).returncode


def slice_checksum(t):
    """Order-sensitive checksum of a device tensor's bytes (int64, on its device)."""
    import torch
    x = t.reshape(-1).view(torch.uint8).to(torch.int64)
    w = torch.arange(x.numel(), device=x.device, dtype=torch.int64) % 65521 + 1
    return (x * w).sum()


def check_exchange(frame, world: int, rank: int, receives: bool):
    """After one exchanged frame in `frame` (a ShardedFrame): every rank's
    checksum of its own slice goes to every rank over torch.distributed, and
    every rank that received the slices (all of them after an all-gather,
    rank 0 after a gather) compares them with its copies in `gathered`.
    Returns the total count of mismatching slices over all ranks."""
    import torch
    import torch.distributed as dist

    own = slice_checksum(frame.slice).reshape(1)
    every = torch.zeros(world, dtype=torch.int64, device=own.device)
    if dist.get_backend() == "gloo":
        outs = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(outs, own.cpu())
        every.copy_(torch.cat(outs))
    else:
        dist.all_gather_into_tensor(every, own)
    bad = torch.zeros(1, dtype=torch.int64, device=own.device)
    if receives:
        got = torch.stack([slice_checksum(frame.gathered[r]) for r in range(world)])
        bad += (got != every).sum()
    coll(dist.all_reduce, bad)
    return int(bad.item())


def agreed_comm(world: int, rank: int, dev, unique_id, available, create, log=print, id_bytes: int = 128):
    """The library's RCCL communicator, or None on every rank.  The ranks agree
    before each step that could leave one of them in a collective the others
    never join:
      1. rank 0 makes the id; whether it could travels in the same broadcast;
      2. every rank says whether it can join at all (RCCL loadable): MIN all-reduce;
      3. every rank joins (ncclCommInitRank returns once all of them have joined;
         a rank that fails inside it leaves its peers there -- the watchdog's
         'comm' deadline ends that);
      4. MIN all-reduce of the join's outcome: if any rank failed, the ranks
         that joined close theirs, and all fall back to torch.distributed's
         all-gather together.
    unique_id() -> bytes; available() -> bool; create(uid) -> communicator
    (each may raise)."""
    import torch
    import torch.distributed as dist

    def fell_back(what, e):
        log(f"bench: the library's RCCL communicator: {what} failed on this rank ({e}); "
            "falling back to torch.distributed all_gather_into_tensor")

    def agree(ok):
        if world == 1:
            return ok
        flag = torch.tensor([int(ok)], dtype=torch.int32, device=dev)
        coll(dist.all_reduce, flag, op=dist.ReduceOp.MIN)
        return int(flag.item())

    uid, ok = b"", 1
    if rank == 0:
        try:
            uid = unique_id()
        except Exception as e:                     # OchError: RCCL missing, or no id
            fell_back("ncclGetUniqueId", e)
            ok = 0
    if world > 1:                                  # step 1: the id and rank 0's flag, one broadcast
        buf = torch.zeros(id_bytes + 1, dtype=torch.uint8, device=dev)
        if rank == 0:
            ok = int(ok and len(uid) == id_bytes)
            buf[0] = ok
            if ok:
                buf[1:] = torch.frombuffer(bytearray(uid), dtype=torch.uint8)
        coll(dist.broadcast, buf, 0)
        h = buf.cpu()
        ok, uid = int(h[0]), bytes(h[1:].numpy().tobytes())
    if ok and rank != 0:                           # step 2
        try:
            ok = int(bool(available()))
        except Exception as e:
            fell_back("loading RCCL", e)
            ok = 0
    if not agree(ok):
        return None
    comm = None
    try:                                           # step 3
        comm = create(uid)
    except Exception as e:
        fell_back("ncclCommInitRank", e)
    if not agree(comm is not None):                # step 4
        if comm is not None:
            comm.close()
        return None
    return comm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--launch", choices=("procs", "group"), default="procs",
                    help="--gpus N > 1 without a launcher (no WORLD_SIZE): 'procs' (default) starts N ranks under "
                         "torch.distributed.run, one process per GPU, as the driver does; 'group' drives the N "
                         "devices from this one process through och_frame_group_* (ncclCommInitAll, one issuing "
                         "thread per device).  --launch group also runs at --gpus 1")
    ap.add_argument("--no-scaling-base", action="store_true",
                    help="N > 1: skip scaling_base (rank 0 alone rendering the same frame, as N = 1 would)")
    ap.add_argument("--no-exchange-check", action="store_true",
                    help="N > 1: skip the checksum check of one exchanged frame before the timed window")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--warm-issue", choices=("native", "step"), default="native",
                    help="how the W warmup steps are issued: as the window issues its steps (default), "
                         "or one C-ABI render call per step")
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="N > 1: strong = configs[3]'s fixed 3840x2160 frame; weak = ~1920x1080 rays per rank")
    ap.add_argument("--row-chunk", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip the CPU timing (parity is still checked)")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle check of the last step's frames")
    ap.add_argument("--cpu-budget", type=float, default=8.0)
    ap.add_argument("--sustain", type=float, default=1.0,
                    help="seconds per sustained-throughput run (three runs, median); 0 = off")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="pool launch option (och_gpu_set_option), e.g. tile_order=1")
    ap.add_argument("--no-bounce", action="store_true", help="skip the config-5 (secondary rays) measurement")
    ap.add_argument("--no-other-configs", action="store_true", help="skip the configs[0] / configs[1] side measurements")
    ap.add_argument("--rgba-frames", action="store_true",
                    help="render and exchange RGBA8 slices instead of 1-byte indexed-colour codes")
    ap.add_argument("--fresh-streams", action="store_true",
                    help="put every frame in flight on a new stream, none on the current stream")
    ap.add_argument("--no-step-events", action="store_true",
                    help="diagnostic: no per-step timing events in the headline window (no per-launch kernel_ms)")
    ap.add_argument("--step-events", choices=("dispatch", "nofence", "torch"), default="dispatch",
                    help="per-step timing events of the render launch: recorded by the launch's own dispatch "
                         "(och_gpu_set_launch_events, default), or hipEventRecord of fence-free events before "
                         "and after it, or torch.cuda.Event records (a system-scope release per record)")
    ap.add_argument("--wait", choices=("spin", "block"), default="spin",
                    help="end of a timed window: poll the frame streams (hipStreamQuery) until they are idle, then "
                         "synchronize (default), or synchronize at once (a wait of milliseconds sleeps on an "
                         "interrupt, whose wake-up lands inside the window)")
    ap.add_argument("--host-spin-us", type=int, default=0,
                    help="diagnostic: busy-loop the host this long after each synchronize around a window")
    ap.add_argument("--pool-timing", type=int, default=None,
                    help="diagnostic: the pool's OCH_OPT_TIMING for launches without step events (default 1)")
    ap.add_argument("--moving-steps", type=int, default=20,
                    help="N = 1: also time this many steps of a camera panning by --moving-dyaw per step, its "
                         "launch order planned once from the first step's cameras (and in natural order); 0 = off")
    ap.add_argument("--moving-dyaw", type=float, default=0.004,
                    help="yaw change per step of the moving-camera window (radians; 0.004 = 14 deg/s at 60 fps)")
    ap.add_argument("--issue", choices=("native", "python"), default="native",
                    help="N = 1 timed windows: 'native' = one och_gpu_render_steps_dev call issues the window's "
                         "frames from the library's own loop (as a C++ host's frame loop would); 'python' = one "
                         "prepared C-ABI render call per step from this interpreter")
    ap.add_argument("--no-fast-issue", action="store_true",
                    help="diagnostic: issue N = 1 steps through the Python wrappers and torch stream contexts")
    ap.add_argument("--isolate-main", action="store_true",
                    help="diagnostic, with --pin-core: move the process's other threads off the issuing CPU")
    ap.add_argument("--pin-core", action="store_true",
                    help="diagnostic: pin the issuing (main) thread to one of its allowed CPUs")
    ap.add_argument("--host-rehearse", action="store_true",
                    help="diagnostic: before a window, switch the pool and torch to each frame stream (no GPU work)")
    ap.add_argument("--host-stamps", action="store_true",
                    help="diagnostic: report the headline window's host clock readings (ns, CLOCK_MONOTONIC and "
                         "CLOCK_BOOTTIME) to line them up with a rocprofv3 kernel trace")
    ap.add_argument("--stream-priority", default="",
                    help="diagnostic: comma-separated HIP priorities of the new frame streams (lower = higher)")
    ap.add_argument("--extra-windows", type=int, default=0,
                    help="diagnostic: this many more warmup + timed windows after the first (reported, not value)")
    ap.add_argument("--shade", choices=("display", "all"), default="display",
                    help="N > 1: every rank all-gathers the frame's codes; 'display' = only rank 0 (the display) "
                         "expands them to RGBA8 frames, 'all' = every rank does")
    ap.add_argument("--no-cull-off", action="store_true", help="skip the cull-off window (value_cull_off)")
    ap.add_argument("--no-split-arm", action="store_true",
                    help="N = 1: skip the heavy-tile split arm (lone launch, window and sustained with the split on)")
    ap.add_argument("--deal", choices=("cost", "count", "rr"), default="count",
                    help="N > 1: row chunks dealt by their cost in one timed render on rank 0 (och_gpu_chunk_costs "
                         "+ och_deal_chunks), by count (rank 0 at --display-weight), or round-robin")
    ap.add_argument("--display-weight", type=float, default=None,
                    help="N > 1 with --shade display: rank 0's share of the row chunks relative to the other ranks "
                         "(it also shades the whole frame); default ort.display_weight(N, exchange): 0.9 / 0.8 / "
                         "0.5 at N = 2 / 4 / 8 with the all-gather, 0.9 / 0.7 / 0.5 with the gather, from "
                         "tools/proxy_rank.py sweeps (DESIGN.md §5)")
    ap.add_argument("--no-direct", action="store_true",
                    help="N = 1: render codes and shade them in a second pass, as ranks do at N > 1, instead of "
                         "the fused launch writing the RGBA8 frames directly")
    ap.add_argument("--inflight", type=int, default=None,
                    help="frames in flight: steps alternate over this many HIP streams, so one step's "
                         "slowest rays overlap the next step's bulk (1 = serialised); default 3, 6 at N >= 8")
    ap.add_argument("--sharded", action="store_true",
                    help="N = 1: the N > 1 step at world size 1 -- render colour codes, exchange them over RCCL "
                         "(--exchange) and shade -- instead of the fused launch writing RGBA8 frames")
    ap.add_argument("--exchange", choices=("rccl", "gather", "torch"), default="rccl",
                    help="sharded steps (N > 1, or --sharded): 'rccl' (default; configs[3]'s 'RCCL framebuffer "
                         "all-gather') = ncclAllGather of the slices on the library's own RCCL communicator "
                         "(och_comm_*, its id broadcast by torch.distributed), the window issued by one "
                         "och_gpu_render_sharded_steps_dev call per rank; 'gather' = only rank 0 (the display) "
                         "receives them (ncclSend / ncclRecv; also timed beside the all-gather as "
                         "exchange_gather); 'torch' = dist.all_gather_into_tensor per step from Python.  The gloo "
                         "rehearsal backend always exchanges through torch"),
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for this process (set before HIP starts); default the "
                         "environment's (4 on the box), 8 at N >= 8")
    a = ap.parse_args()

    # Frames in flight and hardware queues by world size (tools/proxy_rank.py,
    # every shard, profiles/r03/proxy/r03z*): at N = 8 a rank's launches are half
    # the size of N = 1's and end on the same ~0.2 ms grazing tiles, so more
    # frames must overlap -- 6 frames on 8 hardware queues: job 192 -> 211 G rays/s
    # over 20 steps, 215 -> 242 G sustained; at N = 1, 2, 4 the default 3 on 4
    # queues is best.  Set before anything can start HIP (torch.cuda.device_count
    # below does not on this image while amdsmi is importable, but may without it).
    world_env = int(os.environ.get("WORLD_SIZE", "0")) or (a.gpus if a.launch == "group" else 1)
    a.inflight, a.hw_queues = pipeline_defaults(world_env, a.inflight, a.hw_queues)
    if a.hw_queues is not None:
        os.environ["GPU_MAX_HW_QUEUES"] = str(a.hw_queues)

    # A plain `bench.py --gpus N` (no launcher) must measure N GPUs or fail;
    # the child ranks are started from here, never by exec.
    import torch
    launch = resolve_launch(a.gpus, os.environ, a.launch, torch.cuda.device_count())
    if launch == "procs":
        sys.exit(spawn_ranks(a.gpus, sys.argv[1:]))
    if launch == "group":
        return group_bench(a)

    import datetime
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("OCH_DIST_BACKEND", "nccl")
    wd = Watchdog(rank, world)
    wd.enter("init", DEADLINES["init"])
    if backend == "gloo":
        # Rehearsal of the N > 1 path on a box with fewer GPUs than ranks:
        # ranks share devices round-robin and collectives go through the host.
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    sharded = world > 1 or a.sharded
    if world > 1 or (a.sharded and a.exchange == "torch"):
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        # torch's own deadline (rendezvous and its collectives), well under the
        # driver's 600 s and past every stage deadline a rank can spend inside
        # a torch collective, so the watchdog names the stage first
        pg_timeout = datetime.timedelta(seconds=PG_TIMEOUT_S)
        if backend == "gloo":
            dist.init_process_group("gloo", rank=rank, world_size=world, timeout=pg_timeout)
        else:
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world, timeout=pg_timeout)

    import octree_ray_tracing_amd as ort
    from octree_ray_tracing_amd.frame import RcclComm, ShardedFrame, ShardedSteps, slice_row_map

    W, H = frame_size(world, a.width, a.height, a.scaling)
    wd.enter("pool", DEADLINES["pool"])
    nodes, root, tree_nodes, build_s = build_pool_nodes(a.depth, rank, world, dev)
    wd.enter("setup", DEADLINES["setup"])
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
    direct = world == 1 and not a.no_direct and not a.sharded
    # The library's own RCCL communicator for the exchange (N > 1 over nccl, or
    # --sharded): rank 0's id broadcast by torch.distributed, ncclCommInitRank
    # on every rank.  The gloo rehearsal (several ranks per GPU) keeps torch's.
    comm = None
    if sharded and indexed and backend == "nccl" and a.exchange in ("rccl", "gather"):
        wd.enter("comm", DEADLINES["comm"])
        comm = agreed_comm(world, rank, dev, RcclComm.unique_id, RcclComm.available,
                           lambda uid: RcclComm(uid, world, rank, local), log)
        if comm is not None:
            wd.on_expiry(comm.abort)
        wd.enter("setup", DEADLINES["setup"])
    exch_mode = "gather" if (comm is not None and a.exchange == "gather") else "all_gather"
    if exch_mode == "gather" and a.shade != "display":
        raise SystemExit("--exchange gather needs --shade display")

    def exchange_label():
        """What the sharded step's exchange is, as it runs now (config.exchange)."""
        if not sharded:
            return None
        if comm is not None:
            return ("RCCL " + ("gather to rank 0 (ncclSend / ncclRecv)" if exch_mode == "gather" else
                               "all-gather (ncclAllGather)") + " on the library's communicator (och_comm_*)")
        return ("torch.distributed all_gather_into_tensor" if backend == "nccl" else
                "torch.distributed gloo all_gather through the host (rehearsal)")
    cams = [ort.camera(ORIGIN, YAW, p, FOV, W, H) for p in PITCHES]
    # N > 1: which rank renders which row chunks.  Rank 0 times one render of
    # the whole frame per chunk and deals the chunks longest first onto the
    # least loaded rank (rank 0, which also shades for the display, counts its
    # share at --display-weight); every rank gets the same table.
    deal = None
    if a.display_weight is None:
        a.display_weight = ort.display_weight(world, exch_mode)
    if world > 1 and a.deal != "rr":
        n_chunks = -(-H // a.row_chunk)
        table = torch.zeros(n_chunks, dtype=torch.int32, device=dev)
        if rank == 0:
            w = [a.display_weight if a.shade == "display" else 1.0] + [1.0] * (world - 1)
            costs = pool.chunk_costs(cams, a.row_chunk) if a.deal == "cost" else np.ones(n_chunks, np.float32)
            table.copy_(torch.from_numpy(ort.deal_chunks(costs, world, w)))
        coll(dist.broadcast, table, 0)
        deal = table.cpu().numpy()
    # One frame buffer set and one HIP stream per frame in flight.
    if a.fresh_streams:      # every frame in flight on a new stream (none on the current one)
        streams = [torch.cuda.Stream(device=dev) for _ in range(max(1, a.inflight))]
    else:
        prio = [int(x) for x in a.stream_priority.split(",") if x.strip()]
        streams = [stream] + [torch.cuda.Stream(device=dev, priority=prio[i] if i < len(prio) else 0)
                              for i in range(max(1, a.inflight) - 1)]

    def make_frames():
        out = []
        for s_ in streams:
            with torch.cuda.stream(s_):
                out.append(ShardedFrame(pool, W, H, a.row_chunk, n_views=len(PITCHES), indexed=indexed,
                                        shade=a.shade, direct=direct, deal=deal, comm=comm, sharded=sharded,
                                        exchange=exch_mode))
        pool.set_stream(stream)
        return out
    sfs = make_frames()
    # Launch order: one planning render of these views times every tile, and
    # the costliest tiles go first (och_gpu_plan_views; dispatch order only,
    # frames identical), so no frame ends on a few late grazing tiles.
    if not any(kv.startswith("tile_order=") for kv in a.opt):
        pool.set_option("tile_order", 2)
    # The heavy-tile split by world size (ort.split_defaults, DESIGN.md §4d:
    # on where a rank's launches end on their tails), unless --opt sets it;
    # set before planning, which makes the split plan.
    if not any(kv.startswith("split") for kv in a.opt):
        for k, v in ort.split_defaults(world).items():
            pool.set_option(k, v)
    if world >= 8 and not any(kv.startswith("plan=") for kv in a.opt):
        # N = 8 (proxy, 6 frames on 8 queues, profiles/r03/ab/plan_n8/): costliest-first
        # 204-210 G over 20 steps against 200-202 G for the 10 % shape (sustained
        # 238-243 against 244-247 G); the driver times 20 steps
        pool.set_option("plan", 0)
    elif world == 1 and not any(kv.startswith("plan=") for kv in a.opt):
        # N = 1 (profiles/r06/r06x/, 9-12 interleaved runs per shape): the costliest
        # 3 % first gives 38.87 G over the driver's 20 steps against 38.61 G for the
        # library's 10 % (2 %: 39.01, 5 %: 39.06); sustained the same (45.8 G)
        pool.set_option("plan", 3)
    if a.pool_timing is not None:
        pool.set_option("timing", a.pool_timing)
    if pool.get_option("tile_order") >= 2:
        pool.plan_views(cams, a.row_chunk, rank, world)

    # PUSH counts of this rank's rays (for the algorithmic byte count): trace
    # the rank's own rows once with counting on; not part of the timed region.
    rows = torch.from_numpy(slice_row_map(H, a.row_chunk, world, rank, deal))
    push_total, walk_push, culled, hits_total, rays_rank = 0, 0, 0, 0, 0
    dirs = torch.empty(W * H * 3, dtype=torch.float32, device=dev)
    o_t = torch.tensor(ORIGIN, dtype=torch.float32, device=dev)
    n_px = W * H
    hd = torch.empty(n_px, dtype=torch.int32, device=dev)
    hv = torch.empty(n_px, dtype=torch.int32, device=dev)
    ht = torch.empty(n_px, dtype=torch.float32, device=dev)
    hp = torch.empty(n_px, dtype=torch.int32, device=dev)
    mine = rows[rows >= 0].to(dev).long()
    cull = pool.get_option("cull")
    for cam in cams:
        pool.raygen_dev(cam, dirs)
        pool.set_option("cull", 0)             # the reference's PUSH counts
        pool.trace_batch_dev(o_t, dirs, hd, hv, ht, hp)
        push_total += int(hp.view(H, W)[mine].sum().item())
        hits_total += int((hd.view(H, W)[mine] < 6).sum().item())
        rays_rank += int(mine.numel()) * W
        if cull:                               # the PUSHes the timed (culled) launches walk
            pool.set_option("cull", 2)
            pool.trace_batch_dev(o_t, dirs, hd, hv, ht, hp)
            walked = hp.view(H, W)[mine]
            walk_push += int(walked.sum().item())
            culled += int((walked == 0).sum().item())
    if not cull:
        walk_push = push_total
    pool.set_option("cull", cull)
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
        trace_only = {"mrays_s": n_px * len(cams) * 10 / ms.sum() / 1e3, "ms_per_frame": float(ms.mean()),
                      "bytes_per_ray": 12 + 12 + 4 * push_total / (n_px * len(cams)),
                      "path": "och_gpu_trace_batch_dev: resident rays, 64 consecutive rays per wave"}
        # the same rays through och_gpu_trace_batch_tiled_dev (8x8 tiles of the W-wide
        # ray image per wave): one launch per view, and both views' rays in one
        # launch (a W x 2H image, as the render launch takes both views), that
        # geometry's launch order planned (och_gpu_plan_batch_tiled)
        both = torch.empty(2 * n_px * 3, dtype=torch.float32, device=dev)
        bd = torch.empty(2 * n_px, dtype=torch.int32, device=dev)
        bv = torch.empty(2 * n_px, dtype=torch.int32, device=dev)
        bt = torch.empty(2 * n_px, dtype=torch.float32, device=dev)
        for v, cam in enumerate(cams):
            pool.raygen_dev(cam, both[v * n_px * 3:(v + 1) * n_px * 3])
        pool.plan_batch_tiled(o_t, both, W)      # the plan keys one geometry: the two-view batch
        tiled = {}
        for label, n_rays, buf in (("per_view", n_px, None), ("two_views", 2 * n_px, both)):
            tms = []
            for v in range(len(cams) if buf is None else 1):
                src = both[v * n_px * 3:(v + 1) * n_px * 3] if buf is None else buf
                for _ in range(5):
                    pool.trace_batch_tiled_dev(o_t, src, W, bd, bv, bt, n=n_rays)
                for _ in range(10):
                    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s0.record(stream)
                    pool.trace_batch_tiled_dev(o_t, src, W, bd, bv, bt, n=n_rays)
                    s1.record(stream)
                    tms.append((s0, s1))
            torch.cuda.synchronize()
            ms = np.array([x.elapsed_time(y) for x, y in tms])
            tiled[label] = {"mrays_s": n_rays * len(tms) / ms.sum() / 1e3, "ms_per_launch": float(ms.mean()),
                            "rays_per_launch": n_rays}
        tiled["path"] = (f"och_gpu_trace_batch_tiled_dev: the same resident rays as a {W}-wide image, one 8x8 tile "
                         "per wave; per_view = one launch per view, two_views = both views' rays in one launch "
                         "(W x 2H, planned with och_gpu_plan_batch_tiled)")
        trace_only["tiled"] = tiled
        # the reference-signature host entry over the reference's ray layout
        # (och_gpu_trace_batch_image: host rays x + y * W, host records): both
        # views' rays as one W x 2H image, as the two-view tiled launch above
        # (whose plan it uses); kernel time from the launch's own events, the
        # whole call (PCIe both ways) beside it.  Its records must equal the
        # device path's.
        host_rays = both.cpu().numpy().reshape(-1, 3)
        want = (bd.cpu().numpy(), bv.cpu().numpy().view(np.uint32), bt.cpu().numpy().view(np.uint32))
        img = pool.trace_batch(o_t.cpu().numpy(), host_rays, width=W)
        kms_img, call_s = [], []
        for _ in range(5):
            t0 = time.perf_counter()
            img = pool.trace_batch(o_t.cpu().numpy(), host_rays, width=W)
            call_s.append(time.perf_counter() - t0)
            kms_img.append(pool.last_kernel_ms())
        same = (np.array_equal(img[0], want[0]) and np.array_equal(img[1], want[1])
                and np.array_equal(img[2].view(np.uint32), want[2]))
        k_img = float(np.median(kms_img))
        trace_only["image"] = {"mrays_s": 2 * n_px / k_img / 1e3, "ms_per_launch": k_img, "rays_per_launch": 2 * n_px,
                               "call_ms": round(float(np.median(call_s)) * 1e3, 3),
                               "call_mrays_s": round(2 * n_px / float(np.median(call_s)) / 1e6, 1),
                               "records_equal_tiled_dev": bool(same),
                               "path": "och_gpu_trace_batch_image: host rays in the reference's layout (x + y * W), "
                                       f"both views as one {W}-wide image, traced as 8x8 tiles; ms_per_launch = the "
                                       "kernel (dispatch-recorded events), call_ms = the whole call including the "
                                       "host-device copies"}
        if not same:
            raise SystemExit("och_gpu_trace_batch_image records differ from och_gpu_trace_batch_tiled_dev's")
        # the arbitrary-order call with both views' rays in one launch: the same
        # launch size as the render's, so the per-ray comparison with it is not
        # set by one launch's latency floor (a lone launch ends on its grazing tiles)
        tms = []
        for _ in range(5):
            pool.trace_batch_dev(o_t, both, bd, bv, bt)
        for _ in range(10):
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record(stream)
            pool.trace_batch_dev(o_t, both, bd, bv, bt)
            s1.record(stream)
            tms.append((s0, s1))
        torch.cuda.synchronize()
        ms = np.array([x.elapsed_time(y) for x, y in tms])
        trace_only["two_views"] = {"mrays_s": 2 * n_px * len(tms) / ms.sum() / 1e3, "ms_per_launch": float(ms.mean()),
                                   "rays_per_launch": 2 * n_px,
                                   "path": "och_gpu_trace_batch_dev over both views' rays (row-major) in one launch"}
        del both, bd, bv, bt
    del hd, hv, ht, hp, dirs

    # timing events for every step of a window, created once, outside the timed region
    ev_pool = [(make_event(a.step_events), make_event(a.step_events)) for _ in range(max(a.steps, 1))]

    # N = 1 with direct RGBA8 frames: a step is the render launch alone, issued as
    # three prepared C-ABI calls (stream, events, render) with their arguments built
    # here -- no torch stream context or wrapper code per step.  The first step of a
    # window otherwise took ~0.1 ms longer to issue than the rest, while the GPU
    # waited (rocprofv3 --hip-trace, profiles/r03/window/).
    # N > 1 (colour codes): the render is issued the same way; the all-gather and
    # the display rank's shade stay in ShardedFrame.exchange, on the frame's stream.
    def make_fast():
        if not ((direct or (indexed and sharded)) and not a.no_fast_issue):
            return None
        from octree_ray_tracing_amd._lib import Camera, load as load_lib
        lib = load_lib()
        cam_arr = (Camera * len(cams))(*cams)
        h = pool._h
        cp = ctypes.cast(cam_arr, ctypes.c_void_p)
        if direct:
            args = [(h, cp, len(cams), ctypes.c_void_p(f_.frames.data_ptr()), a.row_chunk, 0, 1) for f_ in sfs]
        else:
            args = [(h, cp, len(cams), ctypes.c_void_p(f_.slice.data_ptr()), a.row_chunk, rank, world) for f_ in sfs]
        return {"lib": lib, "cams": cam_arr, "h": h, "direct": direct,
                "args": [[(h, ctypes.c_void_p(s_.cuda_stream)), ra] for s_, ra in zip(streams, args)]}
    fast = make_fast()

    def prepare_native(n, bounce, ev):
        """N = 1, direct frames: the window's n frames as ONE library call
        (och_gpu_render_steps_dev) that issues frame k on stream k % inflight into
        that stream's frames, its dispatch recording event pair k -- the same
        launches, streams, buffers and events as n step_fast calls, without the
        interpreter between them.  Arguments are built here, before the window."""
        lib = fast["lib"]
        B = len(streams)
        sp = (ctypes.c_void_p * B)(*[s_.cuda_stream for s_ in streams])
        fp = (ctypes.c_void_p * B)(*[f_.frames.data_ptr() for f_ in sfs])
        e0 = e1 = None
        pairs = []
        if ev is not None:
            pairs = [ev_pool[(len(ev) + k) % len(ev_pool)] for k in range(n)]
            e0 = (ctypes.c_void_p * n)(*[x.h.value for x, _ in pairs])
            e1 = (ctypes.c_void_p * n)(*[y.h.value for _, y in pairs])
        args = (fast["h"], fast["cams"], len(cams), n, sp, fp, B, e0, e1, a.row_chunk, int(bool(bounce)))
        fn = lib.och_gpu_render_steps_dev

        def issue():
            if fn(*args):
                raise RuntimeError(f"render steps: {lib.och_last_error().decode()}")
            if ev is not None:
                ev.extend(pairs)
        return issue

    native_issue = fast is not None and fast["direct"] and a.issue == "native" and a.step_events == "dispatch"
    # Sharded steps (N > 1, or --sharded) on the library's communicator: the
    # window's frames -- render codes, exchange, display-rank shade, per
    # frame on stream k % inflight -- issued by ONE och_gpu_render_sharded_steps_dev
    # call per rank, as prepare_native does at N = 1.
    sharded_steps = None
    if comm is not None and a.issue == "native" and a.step_events == "dispatch" and not a.no_fast_issue:
        sharded_steps = {b: ShardedSteps(sfs, streams, comm, cams, bounce=b) for b in (False, True)}
        native_issue = True
    arm_steps = None           # a timed arm with another exchange (exchange_gather): its ShardedSteps

    def prepare_sharded(n, bounce, ev):
        pairs = [ev_pool[(len(ev) + k) % len(ev_pool)] for k in range(n)] if ev is not None else []
        issue_ = (arm_steps or sharded_steps)[bool(bounce)].prepare(
            n, [x.h.value for x, _ in pairs] if ev is not None else None,
            [y.h.value for _, y in pairs] if ev is not None else None)

        def issue():
            issue_()
            if ev is not None:
                ev.extend(pairs)
        return issue

    def step_fast(k, ev, bounce):
        lib, (sa, ra) = fast["lib"], fast["args"][k % len(streams)]
        st = lib.och_gpu_set_stream(*sa)
        if ev is not None:
            e0, e1 = ev_pool[len(ev) % len(ev_pool)]
            st |= lib.och_gpu_set_launch_events(fast["h"], e0.h, e1.h)
            ev.append((e0, e1))
        if fast["direct"]:
            st |= (lib.och_gpu_render_bounce_views_dev if bounce else lib.och_gpu_render_views_dev)(*ra)
        else:
            st |= lib.och_gpu_render_codes_views_dev(*ra, int(bool(bounce)))
        if st:
            raise RuntimeError(f"step {k}: {lib.och_last_error().decode()}")
        if not fast["direct"]:
            s_ = streams[k % len(streams)]
            with torch.cuda.stream(s_):
                sfs[k % len(sfs)].exchange()

    def step(k, ev=None, bounce=False):
        """One step: render both views of this rank's rows, all-gather, unshard --
        on stream k % inflight, into that stream's own frame buffers."""
        if fast is not None and a.step_events == "dispatch":
            return step_fast(k, ev, bounce)
        s_, f_ = streams[k % len(streams)], sfs[k % len(sfs)]
        sub = stamps.setdefault("step_parts", []) if (trace_parts and k < 3) else None
        if sub is not None:
            sub.append(("begin", time.monotonic_ns()))
        pool.set_stream(s_)
        with torch.cuda.stream(s_):
            if sub is not None:
                sub.append(("stream", time.monotonic_ns()))
            if ev is not None:
                # event pairs are made before the timed region (ev_pool); the render
                # launch's dispatch records them (or a record before and after it)
                e0, e1 = ev_pool[len(ev) % len(ev_pool)]
                if a.step_events == "dispatch":
                    pool.set_launch_events(e0, e1)
                else:
                    e0.record(s_)
            if sub is not None:
                sub.append(("events", time.monotonic_ns()))
            f_.render_local(cams, bounce)
            if sub is not None:
                sub.append(("render", time.monotonic_ns()))
            if ev is not None:
                if a.step_events != "dispatch":
                    e1.record(s_)
                ev.append((e0, e1))
            f_.exchange()

    if a.pin_core:
        cpus = sorted(os.sched_getaffinity(0))
        main_tid = threading.get_native_id()
        os.sched_setaffinity(0, {cpus[0]})
        if a.isolate_main and len(cpus) > 1:   # every other thread of the process off the issuing CPU
            for tid in os.listdir("/proc/self/task"):
                if int(tid) != main_tid:
                    try:
                        os.sched_setaffinity(int(tid), set(cpus[1:]))
                    except OSError:
                        pass
    stamps = {}                            # --host-stamps
    trace_parts = False
    in_window = False
    issue_s = []                           # host time to issue each timed window's steps
    rank_s = []                            # every rank's wall time of each timed window
    marker = torch.zeros(1, dtype=torch.int64, device=dev)

    def mark():
        """A one-element bitwise_not kernel: brackets the headline window in a
        rocprofv3 kernel trace (tools/window_trace.py), outside the timed region."""
        torch.bitwise_not(marker, out=marker)

    def drain():
        """torch.cuda.synchronize(), after polling the streams (hipStreamQuery)
        until they are idle (--wait spin, default).  A blocking wait of
        milliseconds sleeps on an interrupt: the wake-up lands inside the window
        at its end, and at its start the woken core issued the first step ~5x
        slower than the next ones (~0.17 ms, profiles/r03/window/)."""
        if a.wait == "spin":
            watch = list(streams) + [torch.cuda.current_stream()]
            while not all(s_.query() for s_ in watch):
                pass
        torch.cuda.synchronize()
        if a.host_spin_us > 0 and not in_window:
            t_end = time.perf_counter_ns() + a.host_spin_us * 1000
            while time.perf_counter_ns() < t_end:
                pass
        if a.host_rehearse and not in_window:
            for s_ in streams:                 # the step's host calls, no GPU work
                pool.set_stream(s_)
                with torch.cuda.stream(s_):
                    pool.get_option("cull")
            pool.set_stream(stream)

    def warm(n, bounce=False, events=True):
        """The W untimed steps before a window, issued the way the window issues
        its steps (one library call for all of them when the window is issued
        natively, its dispatches recording event pairs as the window's do), so
        the window's first call is not the process's first of that path."""
        if native_issue and a.warm_issue == "native" and n > 0:
            (prepare_sharded if sharded_steps is not None else prepare_native)(n, bounce, [] if events else None)()
        else:
            for k in range(n):
                step(k, None, bounce)

    def timed(n, bounce=False, ev=None, marked=False, stage="window"):
        """n steps between barrier + synchronize; max over ranks of the wall time."""
        wd.enter(stage, DEADLINES["window"])
        try:
            return timed_(n, bounce, ev, marked)
        finally:
            wd.enter("setup", DEADLINES["setup"])

    def timed_(n, bounce, ev, marked):
        if marked:
            mark()
        drain()
        if world > 1:
            dist.barrier()
        drain()
        issue = None
        if native_issue and not (marked and a.host_stamps):
            issue = prepare_sharded(n, bounce, ev) if sharded_steps is not None else prepare_native(n, bounce, ev)
        gc_was = gc.isenabled()
        gc.disable()                       # no collector pause inside the timed region (as timeit)
        if marked and a.host_stamps:
            stamps["t0"] = (time.monotonic_ns(), time.clock_gettime_ns(time.CLOCK_BOOTTIME))
        t0 = time.perf_counter()
        nonlocal trace_parts, in_window
        trace_parts = marked and a.host_stamps
        if issue is not None:
            issue()                        # the n frames, issued by the library's own loop
        elif marked and a.host_stamps:
            issued = stamps.setdefault("issued", [])
            for k in range(n):
                step(k, ev, bounce)
                issued.append(time.monotonic_ns())
        else:
            for k in range(n):
                step(k, ev, bounce)
        issue_s.append(time.perf_counter() - t0)
        trace_parts = False
        in_window = True
        drain()
        if world > 1:                      # the ranks' barrier, then this rank's synchronize again
            dist.barrier()
            drain()
        in_window = False
        t1 = time.perf_counter()
        if marked and a.host_stamps:
            stamps["t1"] = (time.monotonic_ns(), time.clock_gettime_ns(time.CLOCK_BOOTTIME))
        el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
        if gc_was:
            gc.enable()
        if marked:
            mark()
        if world > 1:
            if dist.get_backend() == "gloo":               # the rehearsal backend: host tensors
                outs = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
                dist.all_gather(outs, el.cpu())
                every = [float(o.item()) for o in outs]
            else:
                buf = torch.zeros(world, dtype=torch.float64, device=dev)
                dist.all_gather_into_tensor(buf, el)
                every = buf.tolist()
            rank_s.append(every)
            return max(every)
        rank_s.append([float(el.item())])
        return float(el.item())

    # N > 1: one frame through the exchange the window will time, checked before
    # anything is timed -- every rank's checksum of its own slice against the
    # receiving ranks' copies.  A library-communicator exchange that delivers
    # wrong bytes falls back to torch.distributed's all-gather (checked again);
    # a second mismatch ends the run with a non-zero status.
    exchange_check = None
    if world > 1 and not a.no_exchange_check:
        def one_frame():
            if sharded_steps is not None:
                prepare_sharded(1, False, None)()
            else:
                step(0)
            drain()

        def checked(label):
            wd.enter("exchange check", DEADLINES["exchange check"])
            one_frame()
            bad = check_exchange(sfs[0], world, rank, exch_mode != "gather" or rank == 0)
            wd.enter("setup", DEADLINES["setup"])
            return {"exchange": label, "frames": 1, "slices": world, "mismatches": bad}
        exchange_check = checked(exchange_label())
        if exchange_check["mismatches"] and comm is not None:
            log(f"exchange check: {exchange_check['mismatches']} slice(s) differ after {exchange_label()}; "
                "falling back to torch.distributed all_gather_into_tensor")
            torch.cuda.synchronize()
            comm.close()
            comm, exch_mode, a.exchange = None, "all_gather", "torch"
            sfs = make_frames()
            fast = make_fast()
            sharded_steps, native_issue = None, False
            exchange_check["fallback"] = checked(exchange_label())
            if exchange_check["fallback"]["mismatches"]:
                raise SystemExit(f"exchange check failed twice: {exchange_check}")
        elif exchange_check["mismatches"]:
            raise SystemExit(f"exchange check failed: {exchange_check}")

    # Frame latency: the render launch alone on an otherwise idle GPU.
    def lone_latency():
        lat = []
        for k in range(max(a.warmup, 1) + 5):
            step(0, lat if k >= max(a.warmup, 1) else None)
            torch.cuda.synchronize()
        return float(np.median([x.elapsed_time(y) for x, y in lat]))
    latency_ms = lone_latency()
    if trace_only is not None:
        # per ray against a lone render launch (both views, raygen + trace + shade)
        lone = latency_ms / (W * H * len(cams))
        trace_only["vs_lone_render_per_ray"] = {
            "untiled_per_view": round(trace_only["ms_per_frame"] / n_px / lone, 3),
            "untiled_two_views": round(trace_only["two_views"]["ms_per_launch"] / (2 * n_px) / lone, 3),
            "tiled_two_views": round(trace_only["tiled"]["two_views"]["ms_per_launch"] / (2 * n_px) / lone, 3),
            "image_two_views": round(trace_only["image"]["ms_per_launch"] / (2 * n_px) / lone, 3)}
    # warmup, then the timed steps
    warm(a.warmup, events=not a.no_step_events)
    ev = None if a.no_step_events else []
    elapsed = timed(a.steps, ev=ev, marked=True, stage="window (headline)")
    ev = ev or []
    per_rank_ms = [round(t / a.steps * 1e3, 4) for t in rank_s[-1]]
    last = (a.steps - 1) % len(sfs)
    frames_host = sfs[last].frames.cpu().numpy() if rank == 0 else None
    pool.set_stream(stream)
    kms = np.array([x.elapsed_time(y) for x, y in ev])
    # the window's GPU span: the first launch's start to the last launch's end
    # (dispatch-recorded events); the rest of the host window is issue latency
    # before the first kernel and completion detection after the last
    gpu_span_ms = max(ev[0][0].elapsed_time(y) for _, y in ev) if ev else None
    frames = a.steps * len(cams)
    total_rays = W * H * frames
    value = total_rays / elapsed / 1e6
    host_issue_ms = round(issue_s[-1] * 1e3, 4)
    extra, extra_noev = [], []
    for _ in range(a.extra_windows):
        # alternately with and without the per-step timing events
        warm(a.warmup)
        extra.append(round(total_rays / timed(a.steps, ev=[]) / 1e6, 1))
        warm(a.warmup, events=False)
        extra_noev.append(round(total_rays / timed(a.steps) / 1e6, 1))

    # Sustained: >= a.sustain seconds of steps, three runs, median.
    sustained = None
    if a.sustain > 0:
        n_s = max(a.steps, int(math.ceil(a.sustain / (elapsed / a.steps))))
        runs = [timed(n_s, stage="window (sustained)") for _ in range(3)]
        vals = [W * H * len(cams) * n_s / r / 1e6 for r in runs]
        sustained = {"value": round(statistics.median(vals), 2), "unit": "Mrays/s", "steps_per_run": n_s,
                     "runs_s": [round(r, 4) for r in runs], "values": [round(v, 2) for v in vals]}

    # N > 1 with the all-gather: the same window with the other exchange the
    # library offers -- only the display rank receives the slices (ncclSend /
    # ncclRecv) -- beside it, on the same frames, deal and streams, after its
    # own one-frame check.  Not the line's value: configs[3] names the all-gather.
    exchange_gather = None
    if world > 1 and sharded_steps is not None and exch_mode == "all_gather" and a.shade == "display":
        arm_steps = {False: ShardedSteps(sfs, streams, comm, cams, exchange="gather")}
        wd.enter("exchange check (gather)", DEADLINES["exchange check"])
        prepare_sharded(1, False, None)()
        drain()
        bad = check_exchange(sfs[0], world, rank, rank == 0)
        wd.enter("setup", DEADLINES["setup"])
        exchange_gather = {"exchange": "RCCL gather to rank 0 (ncclSend / ncclRecv) on the library's communicator",
                           "check_mismatches": bad}
        if not bad:
            prepare_sharded(a.warmup, False, None)()
            el_g = timed(a.steps, stage="window (gather)")
            exchange_gather.update({"value": round(total_rays / el_g / 1e6, 2),
                                    "ms_per_step": round(el_g / a.steps * 1e3, 4),
                                    "per_rank_ms_per_step": [round(t / a.steps * 1e3, 4) for t in rank_s[-1]]})
            if sustained is not None:
                el_gs = timed(sustained["steps_per_run"])
                exchange_gather["sustained"] = round(W * H * len(cams) * sustained["steps_per_run"] / el_gs / 1e6, 2)
        exchange_gather["note"] = ("same frames, streams and row deal as the headline (rank 0 at the all-gather's "
                                   f"weight {a.display_weight}); only rank 0 receives and shades")
        arm_steps = None

    # The same window with the occupied-box cull off (every ray walks): the
    # traversal speed like-for-like with round 1 and with the CPU baseline.
    cull_off = None
    if not a.no_cull_off and pool.get_option("cull"):
        c_prev = pool.get_option("cull")
        pool.set_option("cull", 0)
        if pool.get_option("tile_order") >= 2:
            pool.plan_views(cams, a.row_chunk, rank, world)       # the plan is per cull setting
        warm(a.warmup, events=False)
        el_off = timed(a.steps, stage="window (cull off)")
        cull_off = {"value": round(total_rays / el_off / 1e6, 2), "ms_per_step": round(el_off / a.steps * 1e3, 4),
                    "note": "same warmup and window, OCH_OPT_CULL = 0: every ray walks from the root"}
        pool.set_option("cull", c_prev)
        if pool.get_option("tile_order") >= 2:
            pool.plan_views(cams, a.row_chunk, rank, world)
        pool.set_stream(stream)

    # The heavy-tile split against off at N = 1: with it a lone
    # frame no longer waits on its few longest rays, for a little throughput
    # (the split waves walk the coarse levels once per lane).  Same cameras,
    # the same window; its last frames must equal the headline's.
    split_arm = None
    if world == 1 and direct and not a.no_split_arm:
        # Interleaved, in the same state of the GPU: by now it has rendered for
        # seconds, and windows this late run faster than the headline's (the
        # warm-up ramp) -- compare the arms here, not with the
        # headline.  "on" is the headline's split, or the N = 8 default when the
        # headline ran without one.
        headline_split = {k: pool.get_option(k) for k in ("split", "split_segs", "split_level")}
        sopts = headline_split if headline_split["split"] else ort.split_defaults(8)
        arms = {"off": {"split": 0}, "on": sopts}
        res = {k: {"lone": [], "window": [], "sustained": []} for k in arms}
        last_s = None
        for rnd in range(2):
            for name, opts in arms.items():
                for k, v in opts.items():
                    pool.set_option(k, v)
                pool.plan_views(cams, a.row_chunk, 0, 1)
                res[name]["lone"].append(lone_latency())
                warm(a.warmup, events=False)
                res[name]["window"].append(total_rays / timed(a.steps, stage=f"window (split {name})") / 1e6)
                if name == "on":
                    res[name]["tiles"] = pool.get_option("split_tiles")
                    last_s = sfs[(a.steps - 1) % len(sfs)].frames.cpu().numpy()
                if sustained is not None and rnd == 0:
                    res[name]["sustained"].append(W * H * len(cams) * sustained["steps_per_run"] /
                                                  timed(sustained["steps_per_run"], stage=f"window (split {name})") / 1e6)
        for k, v in headline_split.items():        # back to the headline's options and plan
            pool.set_option(k, v)
        pool.plan_views(cams, a.row_chunk, 0, 1)
        pool.set_stream(stream)

        def summ(r):
            return {"kernel_ms_serial": [round(x, 4) for x in r["lone"]], "value": [round(x, 2) for x in r["window"]],
                    "sustained": [round(x, 2) for x in r["sustained"]] or None}
        split_arm = {"options": sopts, "tiles_split": res["on"].get("tiles"), "on": summ(res["on"]),
                     "off": summ(res["off"]),
                     "frames_equal_headline": None if frames_host is None else bool(np.array_equal(last_s, frames_host)),
                     "note": "heavy-tile split on (the headline's options, or the N >= 8 default when the headline "
                             "ran without) against off, interleaved twice in the same GPU state after the headline: "
                             "lone two-view launch (kernel_ms_serial), 20-step window (value) and one sustained run "
                             "each; the planned costliest tiles walk their long rays over 4 lanes each"}
        if split_arm["frames_equal_headline"] is False:
            raise SystemExit("split frames differ from the headline's")

    # A moving camera (N = 1): the bench's cameras pan by dyaw per step, so no
    # step's launch order was planned from its own cameras -- the plan is made
    # once from the first step's (as an interactive app would plan from an
    # earlier frame), and the same window runs in natural order for comparison.
    moving, moving_frames = None, None
    if direct and a.moving_steps > 0:
        from octree_ray_tracing_amd._lib import Camera, load as load_lib
        lib = load_lib()
        n_mv = a.moving_steps
        seq = [[ort.camera(ORIGIN, YAW + k * a.moving_dyaw, p, FOV, W, H) for p in PITCHES]
               for k in range(a.warmup + n_mv)]
        arrs = [(Camera * len(c))(*c) for c in seq]
        fr = [ctypes.c_void_p(f_.frames.data_ptr()) for f_ in sfs]
        sp = [ctypes.c_void_p(s_.cuda_stream) for s_ in streams]

        def mv_step(k):
            j = k % len(streams)
            st = lib.och_gpu_set_stream(pool._h, sp[j])
            st |= lib.och_gpu_render_views_dev(pool._h, ctypes.cast(arrs[k], ctypes.c_void_p), len(PITCHES), fr[j],
                                               a.row_chunk, 0, 1)
            if st:
                raise RuntimeError(lib.och_last_error().decode())

        def mv_window():
            for k in range(a.warmup):
                mv_step(k)
            drain()
            t0 = time.perf_counter()
            for k in range(a.warmup, a.warmup + n_mv):
                mv_step(k)
            drain()
            return time.perf_counter() - t0

        order_prev = pool.get_option("tile_order")
        rays_mv = W * H * len(PITCHES) * n_mv
        pool.set_option("tile_order", 2)
        pool.plan_views(seq[0], a.row_chunk, 0, 1)
        el_plan = mv_window()
        last = (a.warmup + n_mv - 1) % len(sfs)
        moving_frames = (YAW + (a.warmup + n_mv - 1) * a.moving_dyaw, sfs[last].frames.cpu().numpy())
        pool.set_option("tile_order", 0)
        el_nat = mv_window()
        pool.set_option("tile_order", order_prev)
        if order_prev >= 2:
            pool.plan_views(cams, a.row_chunk, rank, world)
        pool.set_stream(stream)
        moving = {"value": round(rays_mv / el_plan / 1e6, 2), "ms_per_step": round(el_plan / n_mv * 1e3, 4),
                  "value_natural_order": round(rays_mv / el_nat / 1e6, 2), "steps": n_mv, "warmup": a.warmup,
                  "dyaw_per_step": a.moving_dyaw,
                  "yaw_range": [YAW, round(YAW + (a.warmup + n_mv - 1) * a.moving_dyaw, 4)],
                  "note": "camera panning every step; launch order planned once from the first step's cameras "
                          "(value) or natural order (value_natural_order); the last step is checked in parity"}

    # Config 5 (BASELINE configs[4]): the same frames with one mirrored
    # secondary ray per hit pixel, in-block wavefront compaction on; same
    # pipelining and timing discipline.  Rays = primary + secondary.
    bounce = None
    bounce_host = None
    if not a.no_bounce:
        def bounce_run(n):
            # warmup as for the primary line, then the median of three timed runs
            # (one 20-step window alone swings by +-10 %)
            warm(max(a.warmup, 2), bounce=True)
            els, kms_ = [], []
            for _ in range(3):
                bev = []
                els.append(timed(n, bounce=True, ev=bev, stage="window (config 5)"))
                kms_.append(float(np.mean([x.elapsed_time(y) for x, y in bev])))
            return statistics.median(els), statistics.median(kms_)
        # the pool's compaction mode (OCH_OPT_BOUNCE_COMPACT, default or --opt)
        # is the line's value; the other two modes are timed beside it
        mode0 = pool.get_option("bounce_compact")
        b_el, b_kms = bounce_run(a.steps)
        if rank == 0:
            bounce_host = sfs[(a.steps - 1) % len(sfs)].frames.cpu().numpy()
        modes = {}
        for m in (0, 1, 2):
            if m == mode0:
                continue
            pool.set_option("bounce_compact", m)
            if pool.get_option("tile_order") >= 2:
                pool.plan_views(cams, a.row_chunk, rank, world)       # the plan is per compaction setting
            m_el, m_kms = bounce_run(max(a.steps // 2, 3))
            modes[m] = (m_el / max(a.steps // 2, 3), m_kms)
        pool.set_option("bounce_compact", mode0)
        if pool.get_option("tile_order") >= 2:
            pool.plan_views(cams, a.row_chunk, rank, world)
        pool.set_stream(stream)
        hits = torch.tensor([hits_total], dtype=torch.int64, device=dev)
        if world > 1:
            coll(dist.all_reduce, hits)
        secondary = int(hits.item())
        primary = W * H * len(cams)
        bounce = {"workload": "configs[4]: depth-12, primary + 1-bounce secondary rays (divergent), "
                              "wavefront compaction on" + ("" if world == 1 else f", {W}x{H} over {world} GPUs"),
                  "value": round((primary + secondary) * a.steps / b_el / 1e6, 2), "unit": "Mrays/s",
                  "primary_mrays_s": round(primary * a.steps / b_el / 1e6, 2),
                  "ms_per_step": round(b_el / a.steps * 1e3, 4), "secondary_rays_per_step": secondary,
                  "kernel_ms": round(b_kms, 4),
                  "compaction_mode": {0: "in place, secondary walk started on the primary's stack",
                                      1: "every block's secondary rays through its LDS queue",
                                      2: "per block: the queue when it frees a wave, else in place"}[mode0],
                  "other_modes": {("in_place", "queue", "per_block")[m]: {"ms_per_step": round(t * 1e3, 4),
                                                                          "kernel_ms": round(k, 4)}
                                  for m, (t, k) in modes.items()}}
        if 0 in modes:        # round 3's names: "compaction off" = in place
            bounce["compaction_off_ms_per_step"] = round(modes[0][0] * 1e3, 4)
            bounce["compaction_off_kernel_ms"] = round(modes[0][1], 4)

    # Roofline of the dominant kernel (the render launch, both views, this
    # rank's rows).  Binding limit: VALU issue -- VALU
    # wave-instructions per launch (rocprofv3 SQ_INSTS_VALU, the committed
    # profile of this configuration and kernel source) per second of the
    # pipelined step, against the chip's issue peak.  HBM: SURVEY §8(d)'s
    # canonical algorithmic bytes, 24 B in + 12 B out + 4 B per PUSH per ray.
    step_s = elapsed / a.steps
    k_avg_ms = float(kms.mean()) if kms.size else latency_ms    # --no-step-events: the lone launch instead
    # SURVEY §8(d)'s canonical count takes the reference's PUSHes of every ray
    # (the walk without the cull); the walked figure counts what the timed,
    # culled launch walks (proven misses read nothing).  Both per launch.
    canon_bytes = 36 * rays_rank + 4 * push_total
    walked_bytes = 36 * rays_rank + 4 * walk_push

    def gbs(nbytes, ms):
        return round(nbytes / (ms * 1e-3) / 1e9, 2) if ms else None

    hbm = {"bound": "hbm", "bytes_per_launch": int(canon_bytes),
           "bytes_model": "SURVEY 8(d) canonical: 24 B ray in + 12 B hit record out per ray + 4 B per PUSH of the "
                          "reference's walk (push_per_ray: every ray walks, as sse_trace does)",
           "achieved": gbs(canon_bytes, k_avg_ms), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(canon_bytes / (k_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
           "achieved_per_step": gbs(canon_bytes, step_s * 1e3),
           "frac_per_step": round(canon_bytes / step_s / 1e9 / HBM_PEAK_GBS, 5),
           "walked_bytes_per_launch": int(walked_bytes),
           "walked_bytes_model": "the same with the PUSHes the timed launch walks (walked_push_per_ray: rays the "
                                 "occupied-box cull proves to miss walk none)",
           "walked_achieved": gbs(walked_bytes, k_avg_ms),
           "walked_frac_per_step": round(walked_bytes / step_s / 1e9 / HBM_PEAK_GBS, 5),
           "note": "achieved / frac: per launch, over the launch's mean duration in the timed window (HIP events "
                   "recorded by its dispatch; three frames overlap, so a launch lasts longer than a step); "
                   "*_per_step: over the pipelined step time"}
    rgba_launch = direct or not indexed
    pmc, pmc_src = load_pmc("k_render_rgba" if rgba_launch else "k_render", f"d{a.depth}_{W}x{H}_n{world}")
    roof = {"kernel": f"k_trace_grid<CameraSource,{'FrameSink' if rgba_launch else 'CodeSink'}> (2 views per launch)",
            "kernel_ms": round(k_avg_ms, 4), "kernel_ms_serial": round(latency_ms, 4),
            "host_issue_ms": host_issue_ms,
            "window_gpu_span_ms": None if gpu_span_ms is None else round(gpu_span_ms, 4),
            "window_overhead_ms": None if gpu_span_ms is None else round(elapsed * 1e3 - gpu_span_ms, 4),
            "host_issue_ms_per_step": round(host_issue_ms / max(a.steps, 1), 5),
            "ms_per_step": round(step_s * 1e3, 4), "frames_in_flight": len(streams),
            "push_per_ray": round(push_total / rays_rank, 3), "rays_per_launch": rays_rank,
            "walked_push_per_ray": round(walk_push / rays_rank, 3), "culled_frac": round(culled / rays_rank, 4),
            "traffic": None if pmc is None else pmc.get("hbm_bytes_per_launch"),
            "traffic_note": "PMC 2*FETCH_SIZE + WRITE_SIZE per render launch (MI355X_MICROARCH.md HBM): bytes "
                            "leaving L2, Infinity-Cache hits included", "pmc_source": pmc_src, "hbm": hbm,
            "window_profile": load_window()}
    if pmc and "SQ_INSTS_VALU" in pmc:
        insts = float(pmc["SQ_INSTS_VALU"])
        ach = insts / step_s / 1e9
        # the PMC passes' own launch duration: rocprofv3 serialises the
        # dispatches of a counter pass, so this is one launch alone
        prof_ms = float(pmc.get("pmc_mean_ms") or 0.0)
        if prof_ms:
            hbm["achieved_pmc_launch"] = gbs(canon_bytes, prof_ms)
            hbm["frac_pmc_launch"] = round(canon_bytes / (prof_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
            hbm["walked_frac_pmc_launch"] = round(walked_bytes / (prof_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
        roof.update({"bound": "valu-issue", "achieved": round(ach, 1), "peak": VALU_PEAK_GINST_S,
                     "unit": "G VALU wave-instructions/s", "frac": round(ach / VALU_PEAK_GINST_S, 4),
                     "valu_insts_per_launch": int(insts), "valu_insts_per_wave": pmc.get("valu_insts_per_wave"),
                     "valu_lane_utilization": pmc.get("valu_lane_utilization"),
                     "achieved_per_launch": round(insts / (k_avg_ms * 1e-3) / 1e9, 1),
                     # per launch, from the profile alone: SQ_INSTS_VALU / the PMC passes' mean (serialised)
                     # launch duration, both in profiles/pmc_summary.json
                     "frac_profile": round(insts / (prof_ms * 1e-3) / 1e9 / VALU_PEAK_GINST_S, 4) if prof_ms else None,
                     "profile_mean_ms": prof_ms or None,
                     "profile_mean_ms_basis": "pmc_mean_ms: the PMC passes' mean launch duration (dispatches "
                                              "serialised by the profiler)",
                     "frac_serial_launch": round(insts / (latency_ms * 1e-3) / 1e9 / VALU_PEAK_GINST_S, 4),
                     "effective_clock_ghz": pmc.get("effective_clock_ghz"),
                     "note": "frac = issue rate over the pipelined step (three frames overlap, so a launch lasts "
                             "longer than a step: window_profile shows the overlap); frac_profile = the same "
                             "instructions over one serialised launch under the profiler (pmc_mean_ms); "
                             "frac_serial_launch = over kernel_ms_serial, one launch on an idle GPU timed here; "
                             "the DAG is L2/MALL-resident, so HBM is far from binding (see hbm)"})
    else:
        roof.update({k: hbm[k] for k in ("bound", "achieved", "peak", "unit", "frac")})

    # N > 1: the like-for-like one-GPU rate of this same frame (rank 0 alone,
    # the other ranks idle at a barrier), so a scaling curve compares frames
    # of one size: the driver's N = 1 line is configs[2]'s 1920x1080 frame.
    scaling_base = None
    if world > 1 and not a.no_scaling_base:
        wd.enter("scaling base", DEADLINES["scaling base"])
        drain()
        dist.barrier()
        if rank == 0:
            scaling_base = single_gpu_base(a, nodes, root, W, H, cams, streams, dev, frames_host)
        dist.barrier()

    # The other BASELINE configs on this GPU, N = 1 only (each a separate,
    # smaller workload; not the headline): configs[1] = depth-10 DAG at
    # 1920x1080 through the same pipelined two-view step; configs[0] = the
    # depth-8 och::octree (0-based pool) at 512x512, one trace batch of
    # resident rays, next to the CPU oracle on the same rays.
    others = None
    if world == 1 and not a.no_other_configs:
        wd.enter("other configs", DEADLINES["other configs"])
        others = other_configs(a, dev, stream)

    cpu, parity = None, None
    # the other ranks go on to the teardown while rank 0 checks parity
    wd.enter("cpu leg" if rank == 0 else "teardown",
             DEADLINES["cpu leg"] + (0 if rank == 0 else DEADLINES["teardown"]))
    if rank == 0 and not a.no_parity:
        cpu, parity = cpu_leg(nodes, root, a.depth, W, H, frames_host, bounce_host,
                              time_it=world == 1 and not a.no_cpu_baseline, budget_s=a.cpu_budget,
                              moving=moving_frames)

    # a HIP error some other call left pending, cleared by a launch (och_discarded_error):
    # reported once, with the entry that found it
    from octree_ray_tracing_amd._lib import discarded_error
    discarded = discarded_error(reset=True)
    if discarded is not None:
        log(f"bench rank {rank}: {discarded['count']} pending HIP error(s) cleared before launches; "
            f"the first: {discarded['what']}")
    if rank == 0:
        if world == 1:
            workload = "configs[2]: 4096^3 depth-12 och_h_octree DAG, 1920x1080 primary rays, 1 MI355X" + (
                " (the sharded N > 1 step at world size 1: codes, RCCL exchange, shade)" if sharded else "")
        else:
            how = ("RCCL framebuffer all-gather" if exch_mode == "all_gather" and backend == "nccl" else
                   "RCCL gather of the framebuffer to the display rank" if exch_mode == "gather" else
                   "a gloo all-gather through the host (rehearsal, not RCCL)")
            if a.scaling == "strong" and (W, H) == (3840, 2160) and a.depth == 12:
                workload = f"configs[3]: 4096^3 depth-12, 3840x2160 primary rays tiled across {world} MI355X with {how}"
            else:
                workload = f"depth-{a.depth} DAG, {W}x{H} frame row-sharded over {world} MI355X with {how}"
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(step_s * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak" if (world > 1 and a.scaling == "weak") else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: the reference's terrain fill (simplex heightmap + tunnels) at depth 12, voxelised, "
                    "hash-consed and renumbered on the GPU (och_build_terrain)",
            "config": {"workload": workload,
                       "depth": a.depth, "width": W, "height": H, "frames_per_step": len(cams),
                       "pitches": list(PITCHES), "yaw": YAW, "fov": FOV, "row_chunk": a.row_chunk,
                       "dag_nodes": int(nodes.shape[0]), "tree_nodes": tree_nodes,
                       "pool_mb": round(nodes.nbytes / 2**20, 1), "build_s": round(build_s, 2),
                       "build": "och_build_terrain, use_gpu=1: 32^3 bricks voxelised, hash-consed and renumbered on the GPU",
                       "parallelism": f"rows{world}",
                       "frames_in_flight": len(streams),
                       "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "launch_order": plan_label(pool),
                       "heavy_tile_split": ({k: pool.get_option(k) for k in ("split", "split_segs", "split_level")}
                                            if pool.get_option("split") else "off"),
                       "issue": ("one och_gpu_render_sharded_steps_dev call per timed window and rank (the "
                                 "library issues each step's render, RCCL exchange and shade)" if sharded_steps
                                 else "one och_gpu_render_steps_dev call per timed window (the library issues each "
                                 "step's launch)" if native_issue else "one C-ABI render call per step"
                                 if fast is not None else "Python wrappers per step"),
                       "exchange": exchange_label(),
                       "launch": ("one process per GPU (torch.distributed.run)" if world > 1 else "one process"),
                       "row_deal": (None if world == 1 else
                                    "round-robin 8-row chunks" if deal is None else
                                    f"row chunks dealt by {a.deal} (och_deal_chunks), rank 0 weight "
                                    f"{a.display_weight if a.shade == 'display' else 1.0}; chunks per rank "
                                    f"{np.bincount(deal, minlength=world).tolist()}"),
                       "shade": ("the render launch shades each pixel (trace_pixel) into the RGBA8 frames" if direct
                                 else ("rank 0 gathers" if exch_mode == "gather" else "every rank all-gathers")
                                 + " the frame's codes; " +
                                 ("rank 0 (the display) shades them to RGBA8" if a.shade == "display" and world > 1
                                  else "every rank shades them to RGBA8")),
                       "frames": ("rgba8 frames written by the fused launch (no exchange at N = 1)" if direct else
                                  "indexed-colour codes, shaded after the exchange" if indexed else "rgba8 slices"),
                       "options": {k: pool.get_option(k) for k in (*pool.OPTIONS, *pool.READ_ONLY)}},
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity": parity,
            "sustained": sustained,
            "value_cull_off": None if cull_off is None else cull_off["value"],
            "cull_off": cull_off,
            **({"split": split_arm} if split_arm else {}),
            **({"moving_camera": moving} if moving else {}),
            "walked_rays_per_s": round(value * (1 - culled / rays_rank), 2),
            "walked_rays_note": "Mrays/s of the rays that walk the DAG (value x (1 - culled_frac)); the "
                                "occupied-box cull ends the rest as proven misses",
            "per_rank_ms_per_step": per_rank_ms,
            **({"exchange_check": exchange_check} if exchange_check else {}),
            **({"exchange_gather": exchange_gather} if exchange_gather else {}),
            **({"scaling_base": scaling_base} if scaling_base else {}),
            **({"extra_windows": extra, "extra_windows_no_events": extra_noev} if extra else {}),
            **({"host_stamps_ns": stamps} if stamps else {}),
            "trace_batch": trace_only,
            **({"discarded_hip_error": discarded} if discarded else {}),
            "bounce": bounce,
            "other_configs": others,
        }
        print(json.dumps(line), flush=True)
        wd.enter("teardown", DEADLINES["teardown"])
    if comm is not None:
        torch.cuda.synchronize()
        comm.close()
    pool.close()
    if dist.is_initialized():
        dist.destroy_process_group()
    wd.done()


if __name__ == "__main__":
    main()
