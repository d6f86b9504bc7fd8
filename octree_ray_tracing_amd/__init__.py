"""octree_ray_tracing_amd -- MI355X-native sparse-voxel-octree ray caster.

The hot path (Laine-Karras SVO/SVDAG traversal of the reference's
h_octree::sse_trace / octree::sse_trace, its camera ray generator and its
per-pixel shading loop) runs as hand-written gfx950 HIP kernels in
liboch_gpu.so behind the C ABI of include/och_gpu.h.  This package is the
host-side mirror of the reference interface over that ABI.
"""
from ._lib import OchError, library_path, load
from .builder import NodePool, build_terrain, occupied_box, pack_pool
from .editor import Editor
from .frame import FrameGroup, RcclComm, ShardedFrame, ShardedSteps
from .tracer import (Direction, GpuPool, HOctree, Octree, camera, deal_chunks, display_weight, device_count, device_list, host_rcp_lut,
                     rcp_from_lut, rcp_lut_error, shard_rows, split_defaults)
from .voxels import VoxelData, VoxelDataError

__all__ = ["OchError", "library_path", "load", "NodePool", "build_terrain", "occupied_box", "pack_pool", "Editor", "FrameGroup", "RcclComm", "ShardedFrame", "ShardedSteps", "Direction", "GpuPool",
           "HOctree", "Octree", "camera", "deal_chunks", "display_weight", "device_count", "device_list", "host_rcp_lut", "rcp_from_lut", "rcp_lut_error", "shard_rows", "split_defaults",
           "VoxelData", "VoxelDataError"]
