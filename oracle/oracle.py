"""oracle/oracle.py -- ctypes wrapper over oracle/build/liboch_oracle.so.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker, never as the thing being
measured or shipped.  See oracle/och_oracle.c for what each entry restates
(reference file:line) and for the parity status ("parity unpinned" per-ray
against a reference binary; pinned by the reference's own noise source and the
SURVEY known-answer values).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "liboch_oracle.so"
REF_HARNESS = HERE / "_ref" / "ref_harness"

INF = float("inf")


class _Pool(C.Structure):
    _fields_ = [("nodes", C.c_void_p), ("root", C.c_uint32), ("depth", C.c_int),
                ("index_base", C.c_int), ("miss_t", C.c_float)]


class _Rcp(C.Structure):
    _fields_ = [("lut", C.c_void_p), ("log2_entries", C.c_int)]


class _Counts(C.Structure):
    _fields_ = [("push", C.c_uint64), ("step", C.c_uint64), ("pop", C.c_uint64)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        L.ora_rcpps_native.restype = C.c_uint32
        L.ora_rcpps_native.argtypes = [C.c_uint32]
        L.ora_rcp_lut.restype = C.c_uint32
        L.ora_rcp_lut.argtypes = [C.c_uint32, C.c_void_p, C.c_int]
        L.ora_trace.restype = None
        L.ora_trace.argtypes = [C.POINTER(_Pool), C.POINTER(_Rcp)] + [C.c_float] * 6 + [
            C.POINTER(C.c_int32), C.POINTER(C.c_uint32), C.POINTER(C.c_float), C.POINTER(_Counts)]
        L.ora_trace_batch.restype = None
        L.ora_trace_batch.argtypes = [C.POINTER(_Pool), C.POINTER(_Rcp), C.c_void_p, C.c_int, C.c_void_p,
                                      C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_int, C.POINTER(_Counts)]
        L.ora_bounce_ray.restype = None
        L.ora_bounce_ray.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_float, C.c_int, C.c_void_p, C.c_void_p]
        L.ora_trace_bounce_batch.restype = None
        L.ora_trace_bounce_batch.argtypes = [C.POINTER(_Pool), C.POINTER(_Rcp), C.c_void_p, C.c_int, C.c_void_p,
                                             C.c_uint64] + [C.c_void_p] * 7 + [C.c_int, C.POINTER(_Counts)]
        L.ora_shade_bounce.restype = C.c_uint32
        L.ora_shade_bounce.argtypes = [C.c_int32, C.c_uint32, C.c_int32, C.c_void_p, C.c_uint32]
        L.ora_raygen.restype = None
        L.ora_raygen.argtypes = [C.c_float, C.c_float, C.c_float, C.c_int, C.c_int, C.c_void_p]
        L.ora_shade.restype = C.c_uint32
        L.ora_shade.argtypes = [C.c_int32, C.c_uint32, C.c_void_p, C.c_uint32]
        L.ora_noise2.restype = C.c_float
        L.ora_noise2.argtypes = [C.c_float] * 3
        L.ora_noise3.restype = C.c_float
        L.ora_noise3.argtypes = [C.c_float] * 4
        L.ora_height.restype = C.c_int
        L.ora_height.argtypes = [C.c_int] * 3
        L.ora_column_tops.restype = None
        L.ora_column_tops.argtypes = [C.c_int, C.c_void_p]
        L.ora_is_tunnel.restype = C.c_int
        L.ora_is_tunnel.argtypes = [C.c_int] * 3
        L.ora_voxel.restype = C.c_uint32
        L.ora_voxel.argtypes = [C.c_int] * 6
        L.ora_height_map.restype = None
        L.ora_height_map.argtypes = [C.c_int, C.c_void_p]
        L.ora_voxel_batch.restype = None
        L.ora_voxel_batch.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_int, C.c_void_p]
        L.ora_build_terrain.restype = C.c_uint32
        L.ora_build_terrain.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_uint32)]
        L.ora_free.restype = None
        L.ora_free.argtypes = [C.c_void_p]
        L.ora_at.restype = C.c_uint32
        L.ora_at.argtypes = [C.POINTER(_Pool), C.c_int, C.c_int, C.c_int]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class OraclePool:
    """A node pool as the oracle sees it: uint32[n, 8], root, depth, index base."""

    def __init__(self, nodes: np.ndarray, root: int, depth: int, index_base: int = 1,
                 miss_t: float | None = None):
        self.nodes = np.ascontiguousarray(nodes, dtype=np.uint32).reshape(-1, 8)
        self.root, self.depth, self.index_base = int(root), int(depth), int(index_base)
        self.miss_t = (INF if index_base == 1 else 0.0) if miss_t is None else float(miss_t)
        self._c = _Pool(self.nodes.ctypes.data, self.root, self.depth, self.index_base, self.miss_t)

    def at(self, x: int, y: int, z: int) -> int:
        return lib().ora_at(C.byref(self._c), x, y, z)


class Rcp:
    """RCPPS model: lut=None -> the host CPU's native instruction."""

    def __init__(self, lut: np.ndarray | None = None):
        self.lut = None if lut is None else np.ascontiguousarray(lut, dtype=np.uint32)
        k = 0 if self.lut is None else int(np.log2(self.lut.size))
        self._c = _Rcp(None if self.lut is None else self.lut.ctypes.data, k)


def trace(pool: OraclePool, rcp: Rcp, o, d):
    dr, vx, t, cnt = C.c_int32(), C.c_uint32(), C.c_float(), _Counts()
    lib().ora_trace(C.byref(pool._c), C.byref(rcp._c), *[float(v) for v in o], *[float(v) for v in d],
                    C.byref(dr), C.byref(vx), C.byref(t), C.byref(cnt))
    return dr.value, vx.value, t.value, (cnt.push, cnt.step, cnt.pop)


def trace_batch(pool: OraclePool, rcp: Rcp, origins: np.ndarray, dirs: np.ndarray,
                nthreads: int = 1, want_push: bool = False):
    """origins: (3,) shared or (n,3) per ray; dirs (n,3).  Returns dict."""
    dirs = np.ascontiguousarray(dirs, dtype=np.float32).reshape(-1, 3)
    n = dirs.shape[0]
    origins = np.ascontiguousarray(origins, dtype=np.float32)
    stride = 0 if origins.size == 3 else 3
    hd = np.empty(n, np.int32)
    hv = np.empty(n, np.uint32)
    ht = np.empty(n, np.float32)
    push = np.empty(n, np.uint32) if want_push else None
    tot = _Counts()
    lib().ora_trace_batch(C.byref(pool._c), C.byref(rcp._c), _ptr(origins), stride, _ptr(dirs), n,
                          _ptr(hd), _ptr(hv), _ptr(ht), None if push is None else _ptr(push),
                          int(nthreads), C.byref(tot))
    return {"dir": hd, "voxel": hv, "t": ht, "push": push,
            "counts": (tot.push, tot.step, tot.pop)}


def bounce_ray(o, d, direction: int, t: float, depth: int):
    """Config 5's secondary ray of a hit (ora_bounce_ray)."""
    o = np.ascontiguousarray(o, np.float32)
    d = np.ascontiguousarray(d, np.float32)
    o2, d2 = np.empty(3, np.float32), np.empty(3, np.float32)
    lib().ora_bounce_ray(_ptr(o), _ptr(d), int(direction), float(t), int(depth), _ptr(o2), _ptr(d2))
    return o2, d2


def trace_bounce_batch(pool: OraclePool, rcp: Rcp, origins: np.ndarray, dirs: np.ndarray,
                       nthreads: int = 1, want_push: bool = False):
    """Primary and secondary records (config 5), as och_gpu_trace_bounce_batch_dev."""
    dirs = np.ascontiguousarray(dirs, dtype=np.float32).reshape(-1, 3)
    n = dirs.shape[0]
    origins = np.ascontiguousarray(origins, dtype=np.float32)
    stride = 0 if origins.size == 3 else 3
    out = {"dir": np.empty(n, np.int32), "voxel": np.empty(n, np.uint32), "t": np.empty(n, np.float32),
           "dir2": np.empty(n, np.int32), "voxel2": np.empty(n, np.uint32), "t2": np.empty(n, np.float32),
           "push": np.empty(n, np.uint32) if want_push else None}
    tot = _Counts()
    lib().ora_trace_bounce_batch(C.byref(pool._c), C.byref(rcp._c), _ptr(origins), stride, _ptr(dirs), n,
                                 _ptr(out["dir"]), _ptr(out["voxel"]), _ptr(out["t"]), _ptr(out["dir2"]),
                                 _ptr(out["voxel2"]), _ptr(out["t2"]),
                                 None if out["push"] is None else _ptr(out["push"]), int(nthreads), C.byref(tot))
    out["counts"] = (tot.push, tot.step, tot.pop)
    return out


def shade_fast(dirs: np.ndarray, voxels: np.ndarray, palette: np.ndarray) -> np.ndarray:
    """Vectorised ora_shade (trace_pixel's colour choice)."""
    palette = np.ascontiguousarray(palette, dtype=np.uint32)
    nvox = palette.size // 6
    dirs = np.asarray(dirs, np.int64)
    voxels = np.asarray(voxels, np.int64)
    ok = (voxels >= 1) & (voxels <= nvox) & (dirs >= 0) & (dirs <= 5)
    idx = np.where(ok, 6 * (voxels - 1) + dirs, 0)
    c = np.where(ok, palette[idx], np.uint32(0xFFFF00FF))
    c = np.where(dirs == 6, np.uint32(0xFFFEBF00), c)
    c = np.where(dirs == 7, np.uint32(0xFF07193F), c)
    return c.astype(np.uint32)


def shade_bounce(dirs: np.ndarray, voxels: np.ndarray, dirs2: np.ndarray, palette: np.ndarray) -> np.ndarray:
    """Config 5 pixels (vectorised restatement of ora_shade_bounce)."""
    c = shade_fast(dirs, voxels, palette)
    dark = (np.asarray(dirs) >= 0) & (np.asarray(dirs) <= 5) & (np.asarray(dirs2) != 6)
    return np.where(dark, ((c >> 1) & np.uint32(0x007F7F7F)) | (c & np.uint32(0xFF000000)), c).astype(np.uint32)


def raygen(yaw: float, pitch: float, fov: float, W: int, H: int) -> np.ndarray:
    rays = np.empty((H * W, 3), np.float32)
    lib().ora_raygen(yaw, pitch, fov, W, H, _ptr(rays))
    return rays


def shade(dirs: np.ndarray, voxels: np.ndarray, palette: np.ndarray) -> np.ndarray:
    palette = np.ascontiguousarray(palette, dtype=np.uint32)
    L = lib()
    nvox = palette.size // 6
    out = np.empty(dirs.shape[0], np.uint32)
    pp = _ptr(palette)
    for i, (dr, vx) in enumerate(zip(dirs.tolist(), voxels.tolist())):
        out[i] = L.ora_shade(dr, vx, pp, nvox)
    return out


def rcpps_native(xbits: int) -> int:
    return lib().ora_rcpps_native(xbits)


def rcp_lut(xbits: int, lut: np.ndarray) -> int:
    lut = np.ascontiguousarray(lut, dtype=np.uint32)
    return lib().ora_rcp_lut(xbits, _ptr(lut), int(np.log2(lut.size)))


def noise2(freq: float, x: float, y: float) -> float:
    return lib().ora_noise2(freq, x, y)


def noise3(freq: float, x: float, y: float, z: float) -> float:
    return lib().ora_noise3(freq, x, y, z)


def height(x: int, y: int, dim: int) -> int:
    return lib().ora_height(x, y, dim)


def column_tops(dim: int) -> np.ndarray:
    tops = np.empty(dim * dim, np.uint8)
    lib().ora_column_tops(dim, _ptr(tops))
    return tops.reshape(dim, dim)


def is_tunnel(x: int, y: int, z: int) -> bool:
    return bool(lib().ora_is_tunnel(x, y, z))


def voxel(x, y, z, h, top, tunnels=True) -> int:
    return lib().ora_voxel(x, y, z, h, top, int(tunnels))


def height_map(dim: int) -> np.ndarray:
    """ora_height for every column: (dim, dim) int32 indexed [y, x]."""
    h = np.empty(dim * dim, np.int32)
    lib().ora_height_map(dim, _ptr(h))
    return h.reshape(dim, dim)


def voxels_at(dim: int, xyz: np.ndarray, tops: np.ndarray, tunnels: bool = True) -> np.ndarray:
    """ora_voxel at many points (n x 3 int32), closed form (ORT/test_och_h_octree.cpp:767-787)."""
    xyz = np.ascontiguousarray(xyz, np.int32).reshape(-1, 3)
    tops = np.ascontiguousarray(tops, np.uint8)
    out = np.empty(xyz.shape[0], np.uint32)
    lib().ora_voxel_batch(dim, _ptr(xyz), xyz.shape[0], _ptr(tops), int(tunnels), _ptr(out))
    return out


def build_terrain(depth: int, tunnels: bool = True, dedup: bool = True) -> OraclePool:
    """Small-depth reference terrain (ORT/test_och_h_octree.cpp:767-787)."""
    p = C.c_void_p()
    root = C.c_uint32()
    n = lib().ora_build_terrain(depth, int(tunnels), int(dedup), C.byref(p), C.byref(root))
    arr = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint32)), shape=(n * 8,)).copy()
    lib().ora_free(p)
    nodes = arr.reshape(n, 8)
    if dedup:
        # slot 0 is the unused "empty" slot; h_octree indices are 1-based into nodes[1:]
        return OraclePool(nodes[1:], root.value, depth, index_base=1)
    return OraclePool(nodes, 0, depth, index_base=0)


def ref_harness_available() -> bool:
    return REF_HARNESS.exists() and os.access(REF_HARNESS, os.X_OK)


def ref_run(mode: str, records: np.ndarray, freq: float = 1.0) -> bytes:
    """Run the reference's own noise / z-order code (compiled where it lies)."""
    out = subprocess.run([str(REF_HARNESS), mode, repr(float(freq))], input=records.tobytes(),
                         capture_output=True, check=True)
    return out.stdout


class HRef:
    """Exact restatement of och::h_octree<L, D>'s hash table and edits
    (ORT/och_h_octree.h:70-258) -- reproduces the reference's table->nodes."""

    def __init__(self, depth: int, log2cap: int):
        L = lib()
        if not hasattr(L, "_href_ready"):
            L.ora_href_new.restype = C.c_void_p
            L.ora_href_new.argtypes = [C.c_int, C.c_int]
            L.ora_href_free.argtypes = [C.c_void_p]
            L.ora_href_set.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_uint32]
            L.ora_href_at.restype = C.c_uint32
            L.ora_href_at.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
            L.ora_href_fill_terrain.argtypes = [C.c_void_p, C.c_int]
            L.ora_href_nodes.restype = C.c_void_p
            L.ora_href_nodes.argtypes = [C.c_void_p]
            for f in ("capacity", "root", "fillcnt", "nodecnt"):
                getattr(L, "ora_href_" + f).restype = C.c_uint32
                getattr(L, "ora_href_" + f).argtypes = [C.c_void_p]
            L.ora_href_overflow.restype = C.c_int
            L.ora_href_overflow.argtypes = [C.c_void_p]
            L._href_ready = True
        self.depth, self.log2cap = depth, log2cap
        self._t = L.ora_href_new(depth, log2cap)

    def __del__(self):
        if getattr(self, "_t", None):
            lib().ora_href_free(self._t)
            self._t = None

    def set(self, x, y, z, v):
        lib().ora_href_set(self._t, x, y, z, v)

    def at(self, x, y, z):
        return lib().ora_href_at(self._t, x, y, z)

    def fill_terrain(self, tunnels: bool = True):
        lib().ora_href_fill_terrain(self._t, int(tunnels))
        if lib().ora_href_overflow(self._t):
            raise RuntimeError("h_octree table overflow (reference would exit(0))")

    @property
    def root(self):
        return lib().ora_href_root(self._t)

    @property
    def fillcnt(self):
        return lib().ora_href_fillcnt(self._t)

    @property
    def nodecnt(self):
        return lib().ora_href_nodecnt(self._t)

    def nodes(self) -> np.ndarray:
        cap = lib().ora_href_capacity(self._t)
        p = lib().ora_href_nodes(self._t)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint32)), shape=(cap * 8,)).reshape(cap, 8).copy()

    def pool(self) -> OraclePool:
        return OraclePool(self.nodes(), self.root, self.depth, index_base=1)


class ORef:
    """Exact restatement of och::octree's table and edits (ORT/och_octree.cpp:14-160):
    capacity-sized, root at 0, free list threaded through children[0], set() /
    unset() / at() as the reference performs them.  nodes() is the reference's
    _table, slot for slot (what a reference user hands to the GPU)."""

    def __init__(self, depth: int, capacity: int):
        L = lib()
        if not hasattr(L, "_oref_ready"):
            L.ora_oref_new.restype = C.c_void_p
            L.ora_oref_new.argtypes = [C.c_int, C.c_uint32]
            L.ora_oref_free.argtypes = [C.c_void_p]
            L.ora_oref_set.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_uint32]
            L.ora_oref_unset.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
            L.ora_oref_at.restype = C.c_uint32
            L.ora_oref_at.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
            L.ora_oref_fill_terrain.argtypes = [C.c_void_p, C.c_int]
            L.ora_oref_nodes.restype = C.c_void_p
            L.ora_oref_nodes.argtypes = [C.c_void_p]
            for f in ("capacity", "head"):
                getattr(L, "ora_oref_" + f).restype = C.c_uint32
                getattr(L, "ora_oref_" + f).argtypes = [C.c_void_p]
            for f in ("node_cnt", "overflow"):
                getattr(L, "ora_oref_" + f).restype = C.c_int
                getattr(L, "ora_oref_" + f).argtypes = [C.c_void_p]
            L._oref_ready = True
        if capacity < 2:
            raise ValueError("capacity must be at least 2")
        self.depth, self.capacity = int(depth), int(capacity)
        self._t = L.ora_oref_new(self.depth, self.capacity)

    def __del__(self):
        if getattr(self, "_t", None):
            lib().ora_oref_free(self._t)
            self._t = None

    def _check(self):
        if lib().ora_oref_overflow(self._t):
            raise RuntimeError("octree table exhausted (reference: 'Too many allocations', exit(0))")

    def set(self, x, y, z, v):
        lib().ora_oref_set(self._t, x, y, z, v)
        self._check()

    def unset(self, x, y, z):
        lib().ora_oref_unset(self._t, x, y, z)

    def at(self, x, y, z):
        return lib().ora_oref_at(self._t, x, y, z)

    def fill_terrain(self, tunnels: str | None = "unset"):
        """Config 1's fill: non-zero set() per column, then the tunnel voxels
        unset() ("unset"), set to 0 ("set0", as remove() does), or kept (None)."""
        mode = {"unset": 0, "set0": 1, None: -1}[tunnels]
        lib().ora_oref_fill_terrain(self._t, mode)
        self._check()

    @property
    def head(self):
        return lib().ora_oref_head(self._t)

    @property
    def node_cnt(self):
        return lib().ora_oref_node_cnt(self._t)

    def nodes(self) -> np.ndarray:
        p = lib().ora_oref_nodes(self._t)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint32)),
                                     shape=(self.capacity * 8,)).reshape(self.capacity, 8).copy()

    def pool(self) -> OraclePool:
        return OraclePool(self.nodes(), 0, self.depth, index_base=0)
