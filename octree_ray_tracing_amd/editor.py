"""Interactive tree editing: h_octree::set / at (ORT/och_h_octree.h:176-258)
in liboch_gpu.so's native editor, mirrored into a device pool by uploading
only the slots an edit wrote (och_editor_* in include/och_gpu.h).

The demo's place/remove keys (ORT/test_och_h_octree.cpp:301-435) call
``tree.set(x, y, z, v)`` and redraw; here that is ``editor.set(...)`` followed
by ``editor.flush(pool)`` before the next frame.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import call
from .tracer import HOctree, _np_ptr


class Editor:
    """A capacity-bounded, 1-based node pool that supports set() edits."""

    def __init__(self, nodes: np.ndarray, root: int, depth: int, capacity: int | None = None):
        nodes = np.ascontiguousarray(nodes, dtype=np.uint32).reshape(-1, 8)
        if capacity is None:
            capacity = max(2 * nodes.shape[0], 64 * int(depth))
        self.depth = int(depth)
        self._h = C.c_void_p()
        call("och_editor_create", _np_ptr(nodes), nodes.shape[0], int(root), self.depth, int(capacity),
             C.byref(self._h))

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            call("och_editor_destroy", self._h)
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

    def set(self, x: int, y: int, z: int, v: int):
        """h_octree::set (ORT/och_h_octree.h:176-237): voxel (x, y, z) := v, 0 removes."""
        call("och_editor_set", self._h, int(x), int(y), int(z), int(v))

    def at(self, x: int, y: int, z: int) -> int:
        """h_octree::at (ORT/och_h_octree.h:239-258)."""
        return int(call("och_editor_at", self._h, int(x), int(y), int(z)))

    def stats(self) -> dict:
        st = _lib.EditorStats()
        call("och_editor_info", self._h, C.byref(st))
        return {f: getattr(st, f) for f, _ in _lib.EditorStats._fields_}

    @property
    def root(self) -> int:
        return self.stats()["root"]

    def nodes(self) -> np.ndarray:
        """A copy of the slot array (capacity x 8; slot s at row s-1)."""
        ptr, n, root = C.POINTER(C.c_uint32)(), C.c_uint32(), C.c_uint32()
        call("och_editor_nodes", self._h, C.byref(ptr), C.byref(n), C.byref(root))
        return np.ctypeslib.as_array(ptr, shape=(n.value, 8)).copy()

    def make_pool(self, device: int = -1) -> HOctree:
        """The device pool that mirrors this editor (same slots, same root)."""
        ptr, n, root = C.POINTER(C.c_uint32)(), C.c_uint32(), C.c_uint32()
        call("och_editor_nodes", self._h, C.byref(ptr), C.byref(n), C.byref(root))
        arr = np.ctypeslib.as_array(ptr, shape=(n.value, 8))
        pool = HOctree(arr, root.value, self.depth, device=device)
        self.flush(pool)   # clears the dirty window the adoption left
        return pool

    def flush(self, pool) -> None:
        """Upload the slots written since the last flush, and the root."""
        call("och_editor_flush", self._h, pool._h)
