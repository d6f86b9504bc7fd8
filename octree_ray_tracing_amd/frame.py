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

import numpy as np

from .tracer import GpuPool, shard_rows


def slice_row_map(height: int, row_chunk: int, n_shards: int, shard: int) -> np.ndarray:
    """Global row of each row of `shard`'s compact slice (-1 = padding)."""
    rows = shard_rows(height, row_chunk, n_shards)
    local = np.arange(rows)
    gchunk = (local // row_chunk) * n_shards + shard
    g = gchunk * row_chunk + local % row_chunk
    return np.where(g < height, g, -1)


def unshard_host(gathered: np.ndarray, height: int, row_chunk: int) -> np.ndarray:
    """Host restatement of the unshard kernel: (n, rows, W) slices -> (H, W) frame."""
    n, rows, width = gathered.shape
    frame = np.zeros((height, width), gathered.dtype)
    for s in range(n):
        m = slice_row_map(height, row_chunk, n, s)
        ok = m >= 0
        frame[m[ok]] = gathered[s][ok]
    return frame


class ShardedFrame:
    """Renders frames of one or more equal-size views across the ranks of the
    default process group.

    pool: this rank's GpuPool (same tree on every rank).  Everything runs on
    the current torch stream, which the pool is bound to, so render ->
    all-gather -> unshard are ordered without host synchronisation.  Views
    are rendered by one launch (och_gpu_render_views_dev), gathered by one
    collective and unsharded by one kernel.
    """

    def __init__(self, pool: GpuPool, width: int, height: int, row_chunk: int = 8, n_views: int = 1, group=None,
                 indexed: bool = False):
        import torch
        import torch.distributed as dist

        self.pool, self.width, self.height, self.row_chunk = pool, width, height, row_chunk
        self.n_views, self.group = n_views, group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rows = shard_rows(height, row_chunk, self.world)
        # indexed=True: ranks render and exchange 1-byte colour codes (OCH_CODE_*)
        # and shade after the gather -- a quarter of the RGBA8 bytes on xGMI,
        # the same frames (needs a palette of <= CODE_MAX_VOXELS ids).
        self.indexed = indexed
        dev = torch.device("cuda", torch.cuda.current_device())
        dt = torch.uint8 if indexed else torch.int32
        self.slice = torch.empty((n_views, self.rows, width), dtype=dt, device=dev)
        self.gathered = torch.empty((self.world, n_views, self.rows, width), dtype=dt, device=dev)
        self.frames = torch.empty((n_views, height, width), dtype=torch.int32, device=dev)
        pool.set_stream(torch.cuda.current_stream())

    def render_local(self, cams, bounce: bool = False):
        """This rank's rows of every view; bounce=True renders config 5 (one
        mirrored secondary ray per hit pixel)."""
        if not isinstance(cams, (list, tuple)):
            cams = [cams]
        assert len(cams) == self.n_views
        if self.indexed:
            self.pool.render_codes_views_dev(list(cams), self.slice, self.row_chunk, self.rank, self.world, bounce)
            return self.slice
        render = self.pool.render_bounce_views_dev if bounce else self.pool.render_views_dev
        render(list(cams), self.slice, self.row_chunk, self.rank, self.world)
        return self.slice

    def exchange(self):
        import torch.distributed as dist

        src = self.slice
        if self.world > 1:
            if dist.get_backend(self.group) == "gloo":      # host-staged (CPU tests, rehearsal runs)
                host = self.gathered.new_empty(self.gathered.shape, device="cpu")
                dist.all_gather(list(host.unbind(0)), self.slice.cpu(), group=self.group)
                self.gathered.copy_(host)
            else:
                dist.all_gather_into_tensor(self.gathered, self.slice, group=self.group)
            src = self.gathered
        if self.indexed:
            self.pool.shade_unshard_dev(src, self.frames, self.width, self.height, self.row_chunk, self.world,
                                        self.n_views)
        else:
            self.pool.unshard_dev(src, self.frames, self.width, self.height, self.row_chunk, self.world, self.n_views)
        return self.frames

    def render(self, cams, bounce: bool = False):
        self.render_local(cams, bounce)
        return self.exchange()
