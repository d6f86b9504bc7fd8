"""Multi-GPU frames: row-chunk sharding + all-gather of the RGBA8 framebuffer.

The reference renders one frame on one core (ORT/test_och_h_octree.cpp:448-450).
Here each rank (one process per GPU, torch.distributed over RCCL/xGMI) renders
the rows dealt to it -- chunks of `row_chunk` rows round-robin over ranks, so
sky and terrain cost is balanced -- into a compact slice, then one all-gather
assembles the slices and a tiny device kernel restores row order.  The node
pool is replicated (read-only, uploaded once per rank); the only data-path
collective is the framebuffer exchange.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from ._lib import COMM_ID_BYTES, EXCHANGE, Camera, call, load
from .tracer import GpuPool, shard_rows


def deal_slice_rows(height: int, row_chunk: int, n_shards: int, deal=None) -> int:
    """Rows per slice: och_shard_rows, or the largest shard's chunks under a row deal."""
    if deal is None:
        return shard_rows(height, row_chunk, n_shards)
    deal = np.asarray(deal)
    return int(max(1, np.bincount(deal, minlength=n_shards).max())) * row_chunk


def slice_row_map(height: int, row_chunk: int, n_shards: int, shard: int, deal=None) -> np.ndarray:
    """Global row of each row of `shard`'s compact slice (-1 = padding).
    deal: chunk -> shard (och_gpu_set_row_deal), or None for round-robin."""
    rows = deal_slice_rows(height, row_chunk, n_shards, deal)
    local = np.arange(rows)
    if deal is None:
        gchunk = (local // row_chunk) * n_shards + shard
    else:
        mine = np.nonzero(np.asarray(deal) == shard)[0]
        lchunk = local // row_chunk
        gchunk = np.where(lchunk < mine.size, mine[np.minimum(lchunk, max(mine.size - 1, 0))] if mine.size else -1, -1)
    g = gchunk * row_chunk + local % row_chunk
    return np.where((gchunk >= 0) & (g < height), g, -1)


def unshard_host(gathered: np.ndarray, height: int, row_chunk: int, deal=None) -> np.ndarray:
    """Host restatement of the unshard kernel: (n, rows, W) slices -> (H, W) frame."""
    n, rows, width = gathered.shape
    frame = np.zeros((height, width), gathered.dtype)
    for s in range(n):
        m = slice_row_map(height, row_chunk, n, s, deal)
        ok = m >= 0
        frame[m[ok]] = gathered[s][ok]
    return frame


class RcclComm:
    """The library's own RCCL communicator (och_comm_*): one rank per process
    and GPU, as the driver's torch.distributed launch runs them.  Rank 0 makes
    the id, torch.distributed broadcasts it, every rank joins
    (ncclCommInitRank).  The sharded frame loop (och_gpu_render_sharded_steps_dev)
    exchanges its slices over it, so a frame's render, all-gather and shade
    are issued by one library call with no interpreter between them."""

    def __init__(self, uid: bytes, n_ranks: int, rank: int, device: int):
        if len(uid) != COMM_ID_BYTES:
            raise ValueError(f"an RCCL id has {COMM_ID_BYTES} bytes")
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        self._h = C.c_void_p()
        call("och_comm_create", C.cast(buf, C.c_void_p), int(n_ranks), int(rank), int(device), C.byref(self._h))
        self.n_ranks, self.rank, self.device = int(n_ranks), int(rank), int(device)

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * COMM_ID_BYTES)()
        call("och_comm_unique_id", C.cast(buf, C.c_void_p))
        return bytes(buf)

    @classmethod
    def local(cls, device: int):
        """A communicator of one rank (world size 1): the exchange is RCCL's
        copy of the one slice."""
        return cls(cls.unique_id(), 1, 0, device)

    @classmethod
    def from_process_group(cls, group=None, device: int | None = None):
        """Every rank of `group` (default: the default group) calls this
        together: rank 0's id goes to the others over torch.distributed."""
        import torch
        import torch.distributed as dist

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        if device is None:
            device = torch.cuda.current_device()
        ids = torch.zeros(COMM_ID_BYTES, dtype=torch.uint8)
        if rank == 0:
            ids.copy_(torch.frombuffer(bytearray(cls.unique_id()), dtype=torch.uint8))
        src = dist.get_global_rank(group, 0) if group is not None else 0
        if dist.get_backend(group) == "gloo":
            dist.broadcast(ids, src=src, group=group)
        else:
            dev_ids = ids.to(torch.device("cuda", device))
            dist.broadcast(dev_ids, src=src, group=group)
            ids = dev_ids.cpu()
        return cls(bytes(ids.numpy().tobytes()), world, rank, device)

    @property
    def handle(self):
        return self._h

    def all_gather(self, send, recv, stream):
        """recv = [n_ranks][send.numel() bytes], enqueued on `stream` (a torch stream)."""
        call("och_comm_all_gather", self._h, C.c_void_p(send.data_ptr()), C.c_void_p(recv.data_ptr()),
             send.numel() * send.element_size(), C.c_void_p(stream.cuda_stream))

    def gather(self, send, recv, stream, root: int = 0):
        """Only `root` receives recv = [n_ranks][bytes]; recv may be None elsewhere."""
        call("och_comm_gather", self._h, C.c_void_p(send.data_ptr()),
             C.c_void_p(recv.data_ptr() if recv is not None else 0), send.numel() * send.element_size(), int(root),
             C.c_void_p(stream.cuda_stream))

    @staticmethod
    def available() -> bool:
        """RCCL can be loaded here (och_comm_available; no communicator made)."""
        try:
            call("och_comm_available")
            return True
        except Exception:
            return False

    def abort(self):
        """ncclCommAbort (och_comm_abort), safe from another thread: this rank's
        collectives stop waiting for peers that never come.  close() still frees
        the handle."""
        if getattr(self, "_h", None) and self._h.value:
            call("och_comm_abort", self._h)

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            call("och_comm_destroy", self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardedFrame:
    """Renders frames of one or more equal-size views across the ranks of the
    default process group.

    pool: this rank's GpuPool (same tree on every rank).  Everything runs on
    the current torch stream, which the pool is bound to, so render ->
    all-gather -> unshard are ordered without host synchronisation.  Views
    are rendered by one launch (och_gpu_render_views_dev), gathered by one
    collective and unsharded by one kernel.

    comm: an RcclComm -- the exchange runs on the library's own communicator
    instead of torch.distributed's (the path och_gpu_render_sharded_steps_dev
    issues natively); sharded=True keeps the codes + exchange + shade path at
    world size 1 (the exchange is then the collective's copy), so it runs on a
    one-GPU box.  exchange="gather": only rank 0 (the display) receives the
    slices (ncclSend / ncclRecv through comm); needs comm and shade="display".
    """

    def __init__(self, pool: GpuPool, width: int, height: int, row_chunk: int = 8, n_views: int = 1, group=None,
                 indexed: bool = False, shard: tuple[int, int] | None = None, shade: str = "all",
                 direct: bool = False, deal=None, shade_stream=None, comm: RcclComm | None = None,
                 sharded: bool = False, exchange: str = "all_gather"):
        import torch
        import torch.distributed as dist

        self.pool, self.width, self.height, self.row_chunk = pool, width, height, row_chunk
        self.n_views, self.group = n_views, group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # shard=(rank, world) without a process group: one rank's share of an
        # N-rank frame on this GPU alone (tools/proxy_rank.py); exchange() then
        # shades the gathered buffer without a collective
        self.proxy = shard is not None and not dist.is_initialized()
        if self.proxy:
            self.rank, self.world = shard
            assert 0 <= self.rank < self.world
        # deal: the row chunk -> rank table (och_gpu_set_row_deal; every rank
        # must pass the same one), None for round-robin chunks
        self.deal = None if deal is None else np.ascontiguousarray(deal, np.int32)
        if self.world > 1 or self.deal is not None:
            pool.set_row_deal(height, row_chunk, self.world, self.deal)
        self.rows = pool.slice_rows(height, row_chunk, self.world)
        # indexed=True: ranks render and exchange 1-byte colour codes (OCH_CODE_*)
        # and shade after the gather -- a quarter of the RGBA8 bytes on xGMI,
        # the same frames (needs a palette of <= CODE_MAX_VOXELS ids).
        self.indexed = indexed
        # shade="display": every rank all-gathers the frame (as codes or RGBA8
        # slices), and only rank 0 -- the one that displays it, as the
        # reference's single window does (ORT/test_och_h_octree.cpp:437-457) --
        # turns it into the [views][H][W] RGBA8 frames; the other ranks'
        # `frames` stay unwritten and `gathered` holds their copy of the frame.
        if shade not in ("all", "display"):
            raise ValueError("shade must be 'all' or 'display'")
        self.shade = shade
        # direct=True on a single rank: the fused launch writes the RGBA8 frames
        # themselves (update_image's framebuffer, ORT/test_och_h_octree.cpp:
        # 448-450) -- no slice, no exchange, no shade pass
        self.comm = comm
        if comm is not None and (comm.n_ranks, comm.rank) != (self.world, self.rank):
            raise ValueError(f"communicator rank {comm.rank} of {comm.n_ranks}, frame rank {self.rank} of {self.world}")
        if exchange not in EXCHANGE:
            raise ValueError(f"exchange must be one of {sorted(EXCHANGE)}")
        if exchange == "gather" and (comm is None or shade != "display"):
            raise ValueError("exchange='gather' needs an RcclComm and shade='display'")
        self.exchange_mode = exchange
        self.sharded = bool(sharded) or self.world > 1
        self.direct = bool(direct) and self.world == 1 and not self.proxy and not self.sharded
        dev = torch.device("cuda", torch.cuda.current_device())
        dt = torch.uint8 if indexed else torch.int32
        self.slice = torch.empty((n_views, self.rows, width), dtype=dt, device=dev)
        self.gathered = torch.empty((self.world, n_views, self.rows, width), dtype=dt, device=dev)
        self.frames = torch.empty((n_views, height, width), dtype=torch.int32, device=dev)
        # shade_stream (N > 1): the shade + unshard of the gathered frame runs on
        # this stream, after an event on the gather, so the next frame's render
        # on the frame's own stream does not wait for it; the next gather into
        # this frame's buffer waits for the shade that read it
        self.shade_stream = shade_stream if (self.world > 1 and not self.direct) else None
        if self.shade_stream is not None:
            self._gathered = torch.cuda.Event()
            self._shaded = torch.cuda.Event()
            self._shade_pending = False
        pool.set_stream(torch.cuda.current_stream())

    def render_local(self, cams, bounce: bool = False):
        """This rank's rows of every view; bounce=True renders config 5 (one
        mirrored secondary ray per hit pixel)."""
        if not isinstance(cams, (list, tuple)):
            cams = [cams]
        assert len(cams) == self.n_views
        if self.direct:
            render = self.pool.render_bounce_views_dev if bounce else self.pool.render_views_dev
            render(list(cams), self.frames, self.row_chunk, 0, 1)
            return self.frames
        if self.indexed:
            self.pool.render_codes_views_dev(list(cams), self.slice, self.row_chunk, self.rank, self.world, bounce)
            return self.slice
        render = self.pool.render_bounce_views_dev if bounce else self.pool.render_views_dev
        render(list(cams), self.slice, self.row_chunk, self.rank, self.world)
        return self.slice

    def exchange(self):
        import torch
        import torch.distributed as dist

        if self.direct:
            return self.frames
        src = self.slice
        if self.shade_stream is not None and self._shade_pending:
            torch.cuda.current_stream().wait_event(self._shaded)   # the last shade has read `gathered`
        if self.proxy:
            # the bytes a gather lands in this rank's buffer, written on the
            # device (every slot gets this rank's slice; no xGMI time)
            self.gathered.copy_(self.slice.unsqueeze(0).expand_as(self.gathered))
            src = self.gathered
        elif self.comm is not None:                         # the library's own RCCL communicator
            cur = torch.cuda.current_stream()
            if self.exchange_mode == "gather":
                self.comm.gather(self.slice, self.gathered if self.rank == 0 else None, cur)
            else:
                self.comm.all_gather(self.slice, self.gathered, cur)
            src = self.gathered
        elif self.sharded and (self.world > 1 or dist.is_initialized()):
            if dist.get_backend(self.group) == "gloo":      # host-staged (CPU tests, rehearsal runs)
                host = self.gathered.new_empty(self.gathered.shape, device="cpu")
                dist.all_gather(list(host.unbind(0)), self.slice.cpu(), group=self.group)
                self.gathered.copy_(host)
            else:
                dist.all_gather_into_tensor(self.gathered, self.slice, group=self.group)
            src = self.gathered
        if self.shade == "display" and self.rank != 0:
            return None
        if self.shade_stream is not None:
            cur = torch.cuda.current_stream()
            self._gathered.record(cur)
            self.shade_stream.wait_event(self._gathered)
            self.pool.set_stream(self.shade_stream)
            try:
                self._shade(src)
                self._shaded.record(self.shade_stream)
                self._shade_pending = True
            finally:
                self.pool.set_stream(cur)
            # the frames are still being written on shade_stream: a consumer
            # calls ready() (or waits on shaded_event) before reading them
            return self.frames
        self._shade(src)
        return self.frames

    @property
    def shaded_event(self):
        """With a shade_stream: the event the last shade recorded (None before
        the first one, or without a shade_stream)."""
        if self.shade_stream is None or not self._shade_pending:
            return None
        return self._shaded

    def ready(self, stream=None):
        """Make `stream` (default: the current stream) wait until the frames
        of the last exchange are written.  Needed only with a shade_stream,
        whose shade exchange() leaves in flight; otherwise the frames are
        written on the stream the exchange ran on."""
        import torch

        ev = self.shaded_event
        if ev is not None:
            (stream or torch.cuda.current_stream()).wait_event(ev)
        return self.frames

    def _shade(self, src):
        if self.indexed:
            self.pool.shade_unshard_dev(src, self.frames, self.width, self.height, self.row_chunk, self.world,
                                        self.n_views)
        else:
            self.pool.unshard_dev(src, self.frames, self.width, self.height, self.row_chunk, self.world, self.n_views)
        return self.frames

    def render(self, cams, bounce: bool = False):
        self.render_local(cams, bounce)
        return self.exchange()


class FrameGroup:
    """One process driving several GPUs (och_frame_group_*, the C++ host's
    form of SURVEY §8(e)): a pool replica per device, each renders its row
    chunks, one RCCL all-gather (ncclCommInitAll over the devices) and a
    shade + unshard per device.  `frames(rank)` is device `rank`'s copy of
    the [views][H][W] RGBA8 frames."""

    def __init__(self, nodes: np.ndarray, root: int, depth: int, devices=None, index_base: int = 1,
                 miss_t: float | None = None):
        nodes = np.ascontiguousarray(nodes, np.uint32).reshape(-1, 8)
        if devices is None:
            from .tracer import device_list
            devices = device_list()
        devs = (C.c_int * len(devices))(*devices)
        if miss_t is None:
            miss_t = math.inf if index_base == 1 else 0.0
        self._h = C.c_void_p()
        self.n = len(devices)
        call("och_frame_group_create", C.cast(devs, C.c_void_p), len(devices), nodes.ctypes.data, nodes.shape[0],
             int(root), int(depth), int(index_base), float(miss_t), C.byref(self._h))
        self._shape = None

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            call("och_frame_group_destroy", self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_palette(self, rgba: np.ndarray):
        rgba = np.ascontiguousarray(rgba, np.uint32).reshape(-1)
        if rgba.size % 6:
            raise ValueError("palette must hold 6 colours per voxel id")
        call("och_frame_group_set_palette", self._h, rgba.ctypes.data, rgba.size // 6)

    def set_option(self, name: str, value: int):
        call("och_frame_group_set_option", self._h, GpuPool.OPTIONS[name], int(value))

    def plan(self, cams, row_chunk: int = 8):
        """Cost-planned launch order on every device (och_frame_group_plan)."""
        cams = list(cams) if isinstance(cams, (list, tuple)) else [cams]
        arr = (Camera * len(cams))(*cams)
        call("och_frame_group_plan", self._h, C.cast(arr, C.c_void_p), len(cams), int(row_chunk))

    def render(self, cams, row_chunk: int = 8, bounce: bool = False):
        cams = list(cams) if isinstance(cams, (list, tuple)) else [cams]
        arr = (Camera * len(cams))(*cams)
        call("och_frame_group_render", self._h, C.cast(arr, C.c_void_p), len(cams), int(row_chunk), int(bool(bounce)))
        self._shape = (len(cams), cams[0].height, cams[0].width)

    def render_steps(self, cams, n_steps: int, n_buffers: int = 3, row_chunk: int = 8, bounce: bool = False):
        """n_steps frames issued by the devices' own threads, up to n_buffers
        in flight (och_frame_group_render_steps); download() gives the last."""
        cams = list(cams) if isinstance(cams, (list, tuple)) else [cams]
        arr = (Camera * len(cams))(*cams)
        call("och_frame_group_render_steps", self._h, C.cast(arr, C.c_void_p), len(cams), int(n_steps),
             int(n_buffers), int(row_chunk), int(bool(bounce)))
        self._shape = (len(cams), cams[0].height, cams[0].width)

    def synchronize(self):
        call("och_frame_group_synchronize", self._h)

    def download(self, rank: int = 0) -> np.ndarray:
        out = np.empty(self._shape, np.uint32)
        call("och_frame_group_download", self._h, int(rank), out.ctypes.data)
        return out


class ShardedSteps:
    """A window of sharded frames issued natively (och_gpu_render_sharded_steps_dev):
    frame k renders this rank's rows as colour codes, exchanges them over the
    library's RCCL communicator and (where this rank shades) shades them, all
    on streams[k % B] into frames[k % B]'s buffers -- the work of
    ShardedFrame.render on that stream, with no interpreter between a frame's
    launches.  frames: one ShardedFrame per stream, indexed, sharing one pool
    and made with this comm.  exchange: override the frames' own exchange mode
    ("all_gather" or "gather"; both need every rank's gathered buffer only
    where it receives)."""

    def __init__(self, frames, streams, comm: RcclComm, cams, bounce: bool = False, exchange: str | None = None):
        f0 = frames[0]
        if len(frames) != len(streams) or not all(f.comm is comm and f.indexed and not f.direct for f in frames):
            raise ValueError("one indexed, sharded ShardedFrame per stream, all on this comm")
        self.lib = load()
        self.pool = f0.pool
        self.frames, self.streams, self.comm = list(frames), list(streams), comm
        cams = list(cams) if isinstance(cams, (list, tuple)) else [cams]
        self.cams = (Camera * len(cams))(*cams)
        self.n_views = len(cams)
        B = len(frames)
        mode = f0.exchange_mode if exchange is None else exchange
        if mode not in ("all_gather", "gather"):
            raise ValueError("exchange must be 'all_gather' or 'gather'")
        if mode == "gather" and f0.shade != "display":
            raise ValueError("exchange='gather' needs shade='display'")
        if mode == "all_gather" and f0.shade == "display":
            mode = "display"
        self.mode = mode
        self.exchange = EXCHANGE[mode]
        receives = mode != "gather" or f0.rank == 0
        shades = mode == "all_gather" or f0.rank == 0
        self._streams = (C.c_void_p * B)(*[s.cuda_stream for s in streams])
        self._slices = (C.c_void_p * B)(*[f.slice.data_ptr() for f in frames])
        self._gathered = (C.c_void_p * B)(*[f.gathered.data_ptr() if receives else 0 for f in frames])
        self._frames = (C.c_void_p * B)(*[f.frames.data_ptr() if shades else 0 for f in frames])
        self.row_chunk = f0.row_chunk
        self.bounce = int(bool(bounce))

    def prepare(self, n_steps: int, start_events=None, stop_events=None):
        """The window's call with its arguments built now; returns issue()."""
        fn = self.lib.och_gpu_render_sharded_steps_dev
        e0 = e1 = None
        if start_events is not None:
            e0 = (C.c_void_p * n_steps)(*start_events)
            e1 = (C.c_void_p * n_steps)(*stop_events)
        args = (self.pool._h, self.comm.handle, C.cast(self.cams, C.c_void_p), self.n_views, int(n_steps),
                self._streams, self._slices, self._gathered, self._frames, len(self.frames), e0, e1,
                self.row_chunk, self.bounce, self.exchange)

        def issue():
            if fn(*args):
                raise RuntimeError(f"sharded steps: {self.lib.och_last_error().decode()}")
        return issue

    def run(self, n_steps: int):
        self.prepare(n_steps)()
        return self.frames[(n_steps - 1) % len(self.frames)]
