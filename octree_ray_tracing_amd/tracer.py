"""Host-side mirror of the reference's tracer interface over the C ABI.

Reference (ORT/ = Octree_Ray_Tracing/):
  och::h_octree<L, D>::sse_trace(ox, oy, oz, dx, dy, dz, dir&, voxel&, t&)   ORT/och_h_octree.h:292-452
  och::octree::sse_trace(...)                                              ORT/och_octree.cpp:167-325
  tree_camera::update_position / trace_pixel                               ORT/test_och_h_octree.cpp:64-138
  tree_window::update_image                                                ORT/test_och_h_octree.cpp:437-457

`HOctree` / `Octree` wrap a device-resident node pool (`och_gpu_pool`).  Every
compute call runs the gfx950 kernels in liboch_gpu.so; nothing here computes
a hit on the CPU.
"""
from __future__ import annotations

import ctypes as C
import enum
import math

import numpy as np

from . import _lib
from ._lib import Camera, OchError, call


class Direction(enum.IntEnum):
    """och::direction (ORT/och_tree_helper.h:7-18)."""
    x_pos = 0
    y_pos = 1
    z_pos = 2
    x_neg = 3
    y_neg = 4
    z_neg = 5
    exit = 6
    inside = 7
    error = 8


def _np_ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _event_handle(e):
    """A hipEvent_t as an int: a raw handle, a ctypes c_void_p, or an object with ``h``."""
    if e is None:
        return None
    h = getattr(e, "h", e)
    return h.value if hasattr(h, "value") else int(h)


def _dev_ptr(t) -> int:
    """Device pointer of a torch tensor (or an int already)."""
    if isinstance(t, int):
        return t
    if not t.is_cuda:
        raise ValueError("expected a device tensor")
    if not t.is_contiguous():
        raise ValueError("expected a contiguous tensor")
    return t.data_ptr()


def _need(t, nbytes: int, what: str):
    """A device buffer passed as a tensor must hold what the launch writes or
    reads: the C ABI takes bare pointers (as the reference's interface takes
    references), so the sizes are checked here.  Raw pointers pass unchecked."""
    if hasattr(t, "numel") and hasattr(t, "element_size"):
        have = t.numel() * t.element_size()
        if have < nbytes:
            raise ValueError(f"{what}: the buffer holds {have} B, the launch needs {nbytes} B")


def host_rcp_lut() -> np.ndarray:
    """This host's RCPPS (_mm_rcp_ps, ORT/och_h_octree.h:316) as a 2^k table."""
    buf = np.empty(1 << 23, np.uint32)
    k = C.c_int()
    call("och_host_rcp_lut", _np_ptr(buf), C.byref(k))
    return buf[: 1 << k.value].copy()


def rcp_from_lut(xbits: int, lut: np.ndarray) -> int:
    lut = np.ascontiguousarray(lut, np.uint32)
    return call("och_rcp_from_lut", xbits, _np_ptr(lut), int(round(math.log2(lut.size))))


def rcp_lut_error(lut: np.ndarray) -> float:
    """Largest relative error of an RCPPS table over [-2, -1) (och_rcp_lut_error)."""
    lut = np.ascontiguousarray(lut, np.uint32)
    e = C.c_double()
    call("och_rcp_lut_error", _np_ptr(lut), int(round(math.log2(lut.size))), C.byref(e))
    return e.value


def device_list() -> list[int]:
    """HIP indices of the visible gfx950 devices (och_device_list)."""
    n = C.c_int()
    call("och_device_list", None, 0, C.byref(n))
    arr = (C.c_int * max(n.value, 1))()
    call("och_device_list", C.cast(arr, C.c_void_p), n.value, C.byref(n))
    return list(arr[:n.value])


def device_count() -> int:
    n = C.c_int()
    call("och_device_count", C.byref(n))
    return n.value


def camera(pos=(1.5, 1.5, 1.5), yaw: float = 0.0, pitch: float = 0.0, fov: float = 1.25,
           width: int = 640, height: int = 360) -> Camera:
    """tree_camera state -> per-frame uniforms (ORT/test_och_h_octree.cpp:53-55, :87-115).
    yaw = camera.dir.x, pitch = camera.dir.y."""
    cam = Camera()
    call("och_camera_setup", float(pos[0]), float(pos[1]), float(pos[2]), float(yaw), float(pitch),
         float(fov), int(width), int(height), C.byref(cam))
    return cam


class GpuPool:
    """A node pool resident in HBM on one device, traced by the gfx950 kernels."""

    def __init__(self, nodes: np.ndarray, root: int, depth: int, index_base: int = 1,
                 miss_t: float | None = None, device: int = -1):
        nodes = np.ascontiguousarray(nodes, dtype=np.uint32).reshape(-1, 8)
        if miss_t is None:
            miss_t = math.inf if index_base == 1 else 0.0
        self.depth, self.index_base, self.miss_t = int(depth), int(index_base), float(miss_t)
        self._h = C.c_void_p()
        call("och_gpu_pool_create", _np_ptr(nodes), nodes.shape[0], int(root), int(depth),
             int(index_base), float(miss_t), int(device), C.byref(self._h))
        self._palette_n = 0

    # -- lifetime
    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            call("och_gpu_pool_destroy", self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- configuration
    def info(self) -> dict:
        inf = _lib.PoolInfo()
        call("och_gpu_pool_info", self._h, C.byref(inf))
        return {f: getattr(inf, f) for f, _ in _lib.PoolInfo._fields_}

    def get_root(self) -> int:
        return self.info()["root"]

    def set_rcp_lut(self, lut: np.ndarray):
        lut = np.ascontiguousarray(lut, np.uint32).reshape(-1)
        if lut.size < 2 or lut.size & (lut.size - 1):
            raise ValueError("RCPPS table size must be a power of two")
        call("och_gpu_set_rcp_lut", self._h, _np_ptr(lut), int(round(math.log2(lut.size))))

    def set_palette(self, rgba: np.ndarray):
        rgba = np.ascontiguousarray(rgba, np.uint32).reshape(-1)
        if rgba.size % 6:
            raise ValueError("palette must hold 6 colours per voxel id")
        call("och_gpu_set_palette", self._h, _np_ptr(rgba), rgba.size // 6)
        self._palette_n = rgba.size // 6

    def set_stream(self, stream):
        """Enqueue _dev work on a caller stream (torch.cuda.Stream or raw handle)."""
        handle = getattr(stream, "cuda_stream", stream)
        call("och_gpu_set_stream", self._h, C.c_void_p(handle))

    def update(self, first: int, nodes: np.ndarray, root: int):
        nodes = np.ascontiguousarray(nodes, np.uint32).reshape(-1, 8)
        call("och_gpu_pool_update", self._h, int(first), nodes.shape[0], _np_ptr(nodes), int(root))

    # och_option (include/och_gpu.h); ids 0, 2, 3, 7, 9, 12, 13 were retired arms
    OPTIONS = {"block": 1, "layout": 4, "tile_order": 5, "bounce_compact": 6, "cull": 8, "timing": 10, "plan": 11,
               "split": 14, "split_segs": 15, "split_level": 16}
    READ_ONLY = {"split_tiles": 17}

    def set_option(self, name: str, value: int):
        """Launch options (och_gpu_set_option): block, layout, tile_order, bounce_compact, cull
        (1 = rays proven to miss the voxels' bounding box skip the walk; exact), timing, plan."""
        call("och_gpu_set_option", self._h, self.OPTIONS[name], int(value))

    def get_option(self, name: str) -> int:
        v = C.c_int()
        call("och_gpu_get_option", self._h, self.OPTIONS.get(name) or self.READ_ONLY[name], C.byref(v))
        return v.value

    def set_stamp_buffer(self, stamps, capacity_waves: int):
        """Per-wave residency records (diagnostics); stamps = device int64 tensor or None."""
        call("och_gpu_set_stamp_buffer", self._h, None if stamps is None else _dev_ptr(stamps), int(capacity_waves))

    def occupancy(self, kind: int = 0) -> int:
        """HIP's workgroups-per-CU answer: 0 render grid, 2 trace grid."""
        v = C.c_int()
        call("och_gpu_occupancy", self._h, int(kind), C.byref(v))
        return v.value

    def synchronize(self):
        call("och_gpu_synchronize", self._h)

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        call("och_gpu_last_kernel_ms", self._h, C.byref(ms))
        return ms.value

    def set_launch_events(self, start, stop):
        """The next trace/render launch records these HIP events (raw hipEvent_t
        handles, or objects with an ``h`` handle) through its own dispatch."""
        call("och_gpu_set_launch_events", self._h, _event_handle(start), _event_handle(stop))

    # -- tracing (reference signature)
    def sse_trace(self, ox, oy, oz, dx, dy, dz):
        """h_octree::sse_trace: returns (Direction, voxel, t)."""
        d, v, t = C.c_int32(), C.c_uint32(), C.c_float()
        call("och_gpu_trace", self._h, float(ox), float(oy), float(oz), float(dx), float(dy), float(dz),
             C.byref(d), C.byref(v), C.byref(t))
        return Direction(d.value), v.value, t.value

    def trace_batch(self, origins, dirs, width: int | None = None):
        """Host arrays in, host arrays out (synchronous).  origins (3,) or (n,3).
        width: the rays are a row-major image that many rays wide (a camera's
        rays, x + y * W): traced 8x8 tiles per wave (och_gpu_trace_batch_image)."""
        dirs = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        origins = np.ascontiguousarray(origins, np.float32)
        stride = 0 if origins.size == 3 else 3
        n = dirs.shape[0]
        hd, hv, ht = np.empty(n, np.int32), np.empty(n, np.uint32), np.empty(n, np.float32)
        if width:
            call("och_gpu_trace_batch_image", self._h, _np_ptr(origins), stride, _np_ptr(dirs), n, int(width),
                 _np_ptr(hd), _np_ptr(hv), _np_ptr(ht))
        else:
            call("och_gpu_trace_batch", self._h, _np_ptr(origins), stride, _np_ptr(dirs), n,
                 _np_ptr(hd), _np_ptr(hv), _np_ptr(ht))
        return hd, hv, ht

    def trace_batch_dev(self, origins, dirs, hit_dir, hit_voxel, hit_time, push=None, n=None):
        """Device buffers (torch tensors), asynchronous on the pool's stream."""
        if n is None:
            n = dirs.numel() // 3
        stride = 0 if origins.numel() == 3 else 3
        self._need_batch(origins, dirs, n, stride, (hit_dir, hit_voxel, hit_time, push))
        call("och_gpu_trace_batch_dev", self._h, _dev_ptr(origins), stride, _dev_ptr(dirs), int(n),
             _dev_ptr(hit_dir), _dev_ptr(hit_voxel), _dev_ptr(hit_time),
             None if push is None else _dev_ptr(push))

    def trace_batch_tiled_dev(self, origins, dirs, width: int, hit_dir, hit_voxel, hit_time, push=None, n=None):
        """trace_batch_dev for rays laid out as a row-major image `width` wide: one 8x8 tile of
        neighbouring rays per wavefront (och_gpu_trace_batch_tiled_dev); records in the caller's order."""
        if n is None:
            n = dirs.numel() // 3
        stride = 0 if origins.numel() == 3 else 3
        self._need_batch(origins, dirs, n, stride, (hit_dir, hit_voxel, hit_time, push))
        call("och_gpu_trace_batch_tiled_dev", self._h, _dev_ptr(origins), stride, _dev_ptr(dirs), int(n), int(width),
             _dev_ptr(hit_dir), _dev_ptr(hit_voxel), _dev_ptr(hit_time), None if push is None else _dev_ptr(push))

    def plan_batch_tiled(self, origins, dirs, width: int, n=None):
        """Plan the launch order of tiled batches of this geometry (och_gpu_plan_batch_tiled); used with
        set_option("tile_order", 2).  Synchronous."""
        if n is None:
            n = dirs.numel() // 3
        stride = 0 if origins.numel() == 3 else 3
        call("och_gpu_plan_batch_tiled", self._h, _dev_ptr(origins), stride, _dev_ptr(dirs), int(n), int(width))

    def trace_bounce_batch_dev(self, origins, dirs, hit_dir, hit_voxel, hit_time, bounce_dir, bounce_voxel,
                               bounce_time, push=None, n=None):
        """Config 5: primary + one mirrored secondary ray per hit (device tensors, async)."""
        if n is None:
            n = dirs.numel() // 3
        stride = 0 if origins.numel() == 3 else 3
        self._need_batch(origins, dirs, n, stride, (hit_dir, hit_voxel, hit_time, bounce_dir, bounce_voxel,
                                                    bounce_time, push))
        call("och_gpu_trace_bounce_batch_dev", self._h, _dev_ptr(origins), stride, _dev_ptr(dirs), int(n),
             _dev_ptr(hit_dir), _dev_ptr(hit_voxel), _dev_ptr(hit_time), _dev_ptr(bounce_dir),
             _dev_ptr(bounce_voxel), _dev_ptr(bounce_time), None if push is None else _dev_ptr(push))

    @staticmethod
    def _need_batch(origins, dirs, n, stride, outs):
        _need(origins, 12 * (int(n) if stride else 1), "origins")
        _need(dirs, 12 * int(n), "dirs")
        for o in outs:
            if o is not None:
                _need(o, 4 * int(n), "hit records")

    def _need_frames(self, buf, cams, row_chunk, shard, n_shards, bytes_per_pixel, what):
        cams = cams if isinstance(cams, (list, tuple)) else [cams]
        rows = self.slice_rows(cams[0].height, int(row_chunk), int(n_shards))
        _need(buf, len(cams) * rows * cams[0].width * bytes_per_pixel, what)

    # -- frame path
    def raygen_dev(self, cam: Camera, dirs):
        _need(dirs, 12 * cam.width * cam.height, "dirs")
        call("och_gpu_raygen_dev", self._h, C.byref(cam), _dev_ptr(dirs))

    def render(self, cam: Camera) -> np.ndarray:
        """update_position + update_image: RGBA8 (olc::Pixel) frame, H x W uint32."""
        out = np.empty((cam.height, cam.width), np.uint32)
        call("och_gpu_render", self._h, C.byref(cam), _np_ptr(out))
        return out

    def render_dev(self, cam: Camera, rgba_slice, row_chunk: int | None = None, shard: int = 0,
                   n_shards: int = 1):
        if row_chunk is None:
            row_chunk = cam.height
        self._need_frames(rgba_slice, cam, row_chunk, shard, n_shards, 4, "rgba_slice")
        call("och_gpu_render_dev", self._h, C.byref(cam), _dev_ptr(rgba_slice), int(row_chunk),
             int(shard), int(n_shards))

    def render_views_dev(self, cams, rgba_slices, row_chunk: int | None = None, shard: int = 0, n_shards: int = 1):
        """Several equal-size cameras in one launch; rgba_slices holds the views' slices back to back."""
        arr = (Camera * len(cams))(*cams)
        if row_chunk is None:
            row_chunk = cams[0].height
        self._need_frames(rgba_slices, cams, row_chunk, shard, n_shards, 4, "rgba_slices")
        call("och_gpu_render_views_dev", self._h, C.cast(arr, C.c_void_p), len(cams), _dev_ptr(rgba_slices),
             int(row_chunk), int(shard), int(n_shards))

    def render_steps_dev(self, cams, frames, streams, n_steps: int, events=None, row_chunk: int | None = None,
                         bounce: bool = False):
        """n_steps whole frames of these cameras issued by the library's own loop
        (och_gpu_render_steps_dev): frame k on streams[k % B] into frames[k % B],
        B = len(frames) = len(streams); events = n_steps (start, stop) pairs of HIP
        events (raw handles or objects with ``h``) recorded by each frame's dispatch."""
        if len(frames) != len(streams) or not frames:
            raise ValueError("one stream per frame buffer")
        arr = (Camera * len(cams))(*cams)
        if row_chunk is None:
            row_chunk = cams[0].height
        sp = (C.c_void_p * len(streams))(*[getattr(s_, "cuda_stream", s_) for s_ in streams])
        for f in frames:
            self._need_frames(f, list(cams), row_chunk, 0, 1, 4, "frames")
        fp = (C.c_void_p * len(frames))(*[_dev_ptr(f) for f in frames])
        e0 = e1 = None
        if events is not None:
            if len(events) != n_steps:
                raise ValueError("one event pair per step")
            e0 = (C.c_void_p * n_steps)(*[_event_handle(a) for a, _ in events])
            e1 = (C.c_void_p * n_steps)(*[_event_handle(b) for _, b in events])
        call("och_gpu_render_steps_dev", self._h, C.cast(arr, C.c_void_p), len(cams), int(n_steps), sp, fp,
             len(frames), e0, e1, int(row_chunk), int(bool(bounce)))

    def plan_views(self, cams, row_chunk: int | None = None, shard: int = 0, n_shards: int = 1):
        """Plan the launch order of frames of this geometry (och_gpu_plan_views); used with
        set_option("tile_order", 2).  Synchronous."""
        arr = (Camera * len(cams))(*cams)
        if row_chunk is None:
            row_chunk = cams[0].height
        call("och_gpu_plan_views", self._h, C.cast(arr, C.c_void_p), len(cams), int(row_chunk), int(shard),
             int(n_shards))

    def render_bounce_views_dev(self, cams, rgba_slices, row_chunk: int | None = None, shard: int = 0,
                                n_shards: int = 1):
        """Config 5 frames: one bounce per hit pixel, shaded (see och_gpu_render_bounce_views_dev)."""
        arr = (Camera * len(cams))(*cams)
        if row_chunk is None:
            row_chunk = cams[0].height
        self._need_frames(rgba_slices, cams, row_chunk, shard, n_shards, 4, "rgba_slices")
        call("och_gpu_render_bounce_views_dev", self._h, C.cast(arr, C.c_void_p), len(cams), _dev_ptr(rgba_slices),
             int(row_chunk), int(shard), int(n_shards))

    # Row deal (och_gpu_set_row_deal): which shard renders each row chunk.
    def set_row_deal(self, height: int, row_chunk: int, n_shards: int, chunk_shard=None):
        """chunk_shard[g] = shard of row chunk g (None = round-robin) for frames of this geometry."""
        if chunk_shard is None:
            call("och_gpu_set_row_deal", self._h, int(height), int(row_chunk), int(n_shards), None)
            return
        deal = np.ascontiguousarray(chunk_shard, np.int32).reshape(-1)
        if deal.size != -(-int(height) // int(row_chunk)):
            raise ValueError("one shard per row chunk expected")
        call("och_gpu_set_row_deal", self._h, int(height), int(row_chunk), int(n_shards), _np_ptr(deal))

    def slice_rows(self, height: int, row_chunk: int, n_shards: int) -> int:
        """Rows per slice for this geometry under the pool's deal (och_gpu_slice_rows)."""
        v = C.c_int()
        call("och_gpu_slice_rows", self._h, int(height), int(row_chunk), int(n_shards), C.byref(v))
        return v.value

    def chunk_costs(self, cams, row_chunk: int) -> np.ndarray:
        """Per-row-chunk cost of these views from one timed render (och_gpu_chunk_costs)."""
        cams = list(cams) if isinstance(cams, (list, tuple)) else [cams]
        arr = (Camera * len(cams))(*cams)
        out = np.empty(-(-cams[0].height // int(row_chunk)), np.float32)
        call("och_gpu_chunk_costs", self._h, C.cast(arr, C.c_void_p), len(cams), int(row_chunk), _np_ptr(out))
        return out

    def unshard_dev(self, gathered, frame, width: int, height: int, row_chunk: int, n_shards: int, n_views: int = 1):
        rows = self.slice_rows(height, row_chunk, n_shards)
        _need(gathered, 4 * n_shards * n_views * rows * width, "gathered")
        _need(frame, 4 * n_views * height * width, "frame")
        call("och_gpu_unshard_views_dev", self._h, _dev_ptr(gathered), _dev_ptr(frame), int(width), int(height),
             int(row_chunk), int(n_shards), int(n_views))

    # Indexed-colour frames (include/och_gpu.h OCH_CODE_*): one byte per pixel,
    # the multi-GPU exchange format; shade_unshard_dev yields the RGBA8 frames.
    CODE_MAX_VOXELS = 20

    def render_codes_views_dev(self, cams, code_slices, row_chunk: int | None = None, shard: int = 0,
                               n_shards: int = 1, bounce: bool = False):
        arr = (Camera * len(cams))(*cams)
        if row_chunk is None:
            row_chunk = cams[0].height
        self._need_frames(code_slices, cams, row_chunk, shard, n_shards, 1, "code_slices")
        call("och_gpu_render_codes_views_dev", self._h, C.cast(arr, C.c_void_p), len(cams), _dev_ptr(code_slices),
             int(row_chunk), int(shard), int(n_shards), int(bool(bounce)))

    def shade_unshard_dev(self, gathered_codes, frames, width: int, height: int, row_chunk: int, n_shards: int,
                          n_views: int = 1):
        rows = self.slice_rows(height, row_chunk, n_shards)
        _need(gathered_codes, n_shards * n_views * rows * width, "gathered_codes")
        _need(frames, 4 * n_views * height * width, "frames")
        call("och_gpu_shade_unshard_views_dev", self._h, _dev_ptr(gathered_codes), _dev_ptr(frames), int(width),
             int(height), int(row_chunk), int(n_shards), int(n_views))


def shard_rows(height: int, row_chunk: int, n_shards: int) -> int:
    return call("och_shard_rows", int(height), int(row_chunk), int(n_shards))


def deal_chunks(costs, n_shards: int, weights=None) -> np.ndarray:
    """och_deal_chunks: row chunks dealt longest-first onto the least loaded shard per weight."""
    costs = np.ascontiguousarray(costs, np.float32).reshape(-1)
    out = np.empty(costs.size, np.int32)
    w = None if weights is None else np.ascontiguousarray(weights, np.float32).reshape(-1)
    if w is not None and w.size != n_shards:
        raise ValueError("one weight per shard expected")
    call("och_deal_chunks", _np_ptr(costs), costs.size, int(n_shards), None if w is None else _np_ptr(w), _np_ptr(out))
    return out


# The display rank's share of the row chunks (it also shades the whole frame),
# per world size and exchange, from tools/proxy_rank.py sweeps of every shard
# (profiles/r04/r04e/, r04f/): with the gather to rank 0 the
# other ranks receive nothing, so the display rank takes a smaller share.
# rank 0's deal weight by exchange and world size (tools/proxy_rank.py sweeps,
# DESIGN.md §5); N = 8 all-gather 0.5 since round 5's faster kernel made the
# display rank's whole-frame shade a larger part of its step (profiles/r05/r05al/)
DISPLAY_WEIGHTS = {"gather": {2: 0.9, 4: 0.7, 8: 0.5}, "all_gather": {2: 0.9, 4: 0.8, 8: 0.5}}


def display_weight(world: int, exchange: str = "all_gather") -> float:
    """Default deal weight of rank 0 (the display rank) at this world size,
    for the exchange configs[3] names (the all-gather) unless told otherwise."""
    table = DISPLAY_WEIGHTS.get(exchange, DISPLAY_WEIGHTS["all_gather"])
    if world in table:
        return table[world]
    return max(0.5, 1.0 - (0.0625 if exchange == "gather" else 0.05) * world)


# The heavy-tile split (OCH_OPT_SPLIT) by world size: a lone
# launch no longer waits on its longest rays, but the split waves cost
# throughput, so it pays where a rank's launches are small and end on their
# tails (tools/split_sweep.sh, profiles/r06/).  World sizes not listed: off.
# The heavy-tile split by world size (bench.py sweeps): at N = 1
# the costliest tiles only (T 80: +1.2 % over the 20-step window, -0.4 %
# sustained, a lone frame 0.19 -> 0.16 ms; profiles/r06/r06ah/), off at N = 2 and
# 4 (a tie), T 60 from N = 8, whose half-size launches end on their tails.
SPLIT_DEFAULTS = {1: {"split": 80, "split_segs": 4, "split_level": 6}, 2: {"split": 0},
                  8: {"split": 60, "split_segs": 4, "split_level": 6}}


def split_defaults(world: int) -> dict:
    """Pool options of the heavy-tile split at this world size ({"split": 0} = off)."""
    best = {"split": 0}
    for w, opts in sorted(SPLIT_DEFAULTS.items()):
        if world >= w:
            best = dict(opts)
    return best


class HOctree(GpuPool):
    """och::h_octree's table on the GPU: 1-based, miss t = +INF (ORT/och_h_octree.h:429)."""

    def __init__(self, nodes, root, depth, device: int = -1):
        super().__init__(nodes, root, depth, index_base=1, miss_t=math.inf, device=device)


class Octree(GpuPool):
    """och::octree's table on the GPU: 0-based, root 0, miss t = 0 (ORT/och_octree.cpp:302)."""

    def __init__(self, nodes, depth, device: int = -1):
        super().__init__(nodes, 0, depth, index_base=0, miss_t=0.0, device=device)
