"""Terrain builder binding (och_build_terrain in liboch_gpu.so).

Builds the demo world of ORT/test_och_h_octree.cpp:561-787 (heightmap from
simplex noise, grass/dirt cap, simplex tunnels) as a hash-consed DAG in
parallel, breadth-first ordered.  Returns the node pool in the reference's
h_octree layout (1-based, root 1) or och::octree layout (0-based, root 0).
"""
from __future__ import annotations

import ctypes as C
import struct
import zlib
from dataclasses import dataclass, field
from pathlib import Path

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

    # -- linearised node-pool file: a 64-byte header, then the
    # n x 8 little-endian uint32 slots exactly as och_gpu_pool_create takes them.
    # The reference rebuilds its world on every start (ORT/test_och_h_octree.cpp:822);
    # a depth-12 build takes ~30 s even in parallel, a load is one read.
    # Version 2: the CRC-32 covers the header fields (depth, index base, root,
    # node count) and then the slots; version-1 files (slots only) still load.
    _MAGIC = b"OCHPOOL\0"
    _HEADER = struct.Struct("<8sIiiIQI")   # magic, version, depth, index_base, root, n_nodes, crc32
    _VERSION = 2

    @classmethod
    def _crc(cls, version, depth, base, root, n, slots) -> int:
        crc = 0
        if version >= 2:
            crc = zlib.crc32(struct.pack("<IiiIQ", version, depth, base, root, n))
        return zlib.crc32(slots, crc)

    def save(self, path) -> None:
        nodes = np.ascontiguousarray(self.nodes, dtype="<u4").reshape(-1, 8)
        n = nodes.shape[0]
        crc = self._crc(self._VERSION, self.depth, self.index_base, self.root, n, memoryview(nodes).cast("B"))
        head = self._HEADER.pack(self._MAGIC, self._VERSION, self.depth, self.index_base, self.root, n, crc)
        with open(path, "wb") as f:
            f.write(head.ljust(64, b"\0"))
            f.write(memoryview(nodes).cast("B"))

    @classmethod
    def load(cls, path, mmap: bool = False, verify: bool = True) -> "NodePool":
        """Read a pool file.  Raises ValueError on a bad magic/version, a size
        that does not match the header, a depth / index base / root outside
        their ranges, or (verify=True) a checksum mismatch.  mmap=True maps the
        slots read-only instead of reading them."""
        path = Path(path)
        size = path.stat().st_size
        with open(path, "rb") as f:
            raw = f.read(64)
        if len(raw) < 64:
            raise ValueError(f"{path}: truncated header")
        magic, ver, depth, base, root, n, crc = cls._HEADER.unpack(raw[:cls._HEADER.size])
        if magic != cls._MAGIC or ver not in (1, 2):
            raise ValueError(f"{path}: not a version-1/2 node-pool file")
        if size != 64 + n * 32:
            raise ValueError(f"{path}: {size} bytes, header says {n} nodes ({64 + n * 32} bytes)")
        if not 1 <= depth <= 22 or base not in (0, 1):
            raise ValueError(f"{path}: depth {depth} / index base {base} out of range")
        # h_octree: root 0 = empty tree, else 1..n; och::octree: root 0 of n >= 1 nodes
        if (base == 1 and root > n) or (base == 0 and (root != 0 or n == 0)):
            raise ValueError(f"{path}: root {root} outside a {n}-node pool (index base {base})")
        if mmap:
            nodes = np.memmap(path, dtype="<u4", mode="r", offset=64, shape=(n, 8))
        else:
            nodes = np.fromfile(path, dtype="<u4", offset=64, count=n * 8).reshape(n, 8)
        if verify and cls._crc(ver, depth, base, root, n, memoryview(np.ascontiguousarray(nodes)).cast("B")) != crc:
            raise ValueError(f"{path}: checksum mismatch")
        return cls(np.asarray(nodes, dtype=np.uint32), root, depth, base)


def build_terrain(depth: int, tunnels: bool = True, dedup: bool = True, rand_kind: str = "glibc",
                  threads: int = 0, use_gpu: bool = False) -> NodePool:
    """The demo world as a node pool.  use_gpu=True voxelises (and, for a DAG,
    hash-conses) on the current GPU (och_terrain_params.use_gpu; raises
    OchError OCH_E_NODEV without one); the pool is the same either way."""
    params = TerrainParams(int(depth), int(tunnels), int(dedup), 1 if rand_kind == "msvc" else 0,
                           int(threads), int(bool(use_gpu)))
    hp = HostPool()
    call("och_build_terrain", C.byref(params), C.byref(hp))
    try:
        n = hp.n_nodes
        arr = np.ctypeslib.as_array(hp.nodes, shape=(n * 8,)).reshape(n, 8).copy()
    finally:
        call("och_host_pool_free", C.byref(hp))
    return NodePool(arr, hp.root, hp.depth, hp.index_base, hp.solid_voxels, list(hp.voxel_hist),
                    hp.tree_nodes, hp.build_seconds)


def occupied_box(nodes: np.ndarray, root: int, depth: int, index_base: int = 1):
    """Bounding box of the pool's voxels (och_pool_occupied_box): (lo, hi) in
    voxel units, voxel (x, y, z) inside iff lo <= (x, y, z) < hi; lo = hi = 0
    for a pool without voxels.  The kernels' cull box (OCH_OPT_CULL)."""
    nodes = np.ascontiguousarray(nodes, np.uint32).reshape(-1, 8)
    lo, hi = (C.c_int32 * 3)(), (C.c_int32 * 3)()
    call("och_pool_occupied_box", nodes.ctypes.data, nodes.shape[0], int(root), int(depth), int(index_base), lo, hi)
    return tuple(lo), tuple(hi)


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
