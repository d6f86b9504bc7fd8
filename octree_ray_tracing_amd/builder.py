"""Terrain builder binding (och_build_terrain in liboch_gpu.so).

Builds the demo world of ORT/test_och_h_octree.cpp:561-787 (heightmap from
simplex noise, grass/dirt cap, simplex tunnels) as a hash-consed DAG in
parallel, breadth-first ordered.  Returns the node pool in the reference's
h_octree layout (1-based, root 1) or och::octree layout (0-based, root 0).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from ._lib import HostPool, TerrainParams, call


@dataclass
class NodePool:
    nodes: np.ndarray            # (n, 8) uint32
    root: int
    depth: int
    index_base: int
    solid_voxels: int = 0
    voxel_hist: list = field(default_factory=list)
    tree_nodes: int = 0
    build_seconds: float = 0.0

    @property
    def n_nodes(self) -> int:
        return self.nodes.shape[0]

    def at(self, x: int, y: int, z: int) -> int:
        """h_octree::at (ORT/och_h_octree.h:239-258)."""
        return call("och_pool_at", self.nodes.ctypes.data, self.root, self.depth, self.index_base, x, y, z)


def build_terrain(depth: int, tunnels: bool = True, dedup: bool = True, rand_kind: str = "glibc",
                  threads: int = 0, use_gpu: bool = True) -> NodePool:
    params = TerrainParams(int(depth), int(tunnels), int(dedup), 1 if rand_kind == "msvc" else 0,
                           int(threads), int(use_gpu))
    hp = HostPool()
    call("och_build_terrain", C.byref(params), C.byref(hp))
    try:
        n = hp.n_nodes
        arr = np.ctypeslib.as_array(hp.nodes, shape=(n * 8,)).reshape(n, 8).copy()
    finally:
        call("och_host_pool_free", C.byref(hp))
    return NodePool(arr, hp.root, hp.depth, hp.index_base, hp.solid_voxels, list(hp.voxel_hist),
                    hp.tree_nodes, hp.build_seconds)


def pack_pool(nodes: np.ndarray, root: int, depth: int, index_base: int = 1):
    """The packed device layout of a pool (och_pool_pack): (packed nodes, packed root)."""
    nodes = np.ascontiguousarray(nodes, np.uint32).reshape(-1, 8)
    n, r = C.c_uint32(), C.c_uint32()
    call("och_pool_pack", nodes.ctypes.data, nodes.shape[0], int(root), int(depth), int(index_base), None, 0,
         C.byref(n), C.byref(r))
    out = np.zeros((n.value, 8), np.uint32)
    call("och_pool_pack", nodes.ctypes.data, nodes.shape[0], int(root), int(depth), int(index_base), out.ctypes.data,
         n.value, C.byref(n), C.byref(r))
    return out, r.value
