"""ctypes binding of liboch_gpu.so (the C ABI declared in include/och_gpu.h).

The library is built in-tree by __graft_entry__.build() (or `make -C
octree_ray_tracing_amd/csrc`).  There is no fallback: if it is missing or
fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "liboch_gpu.so"
HEADER_PATH = PKG_DIR.parent / "include" / "och_gpu.h"

OCH_OK = 0
STATUS_NAMES = {0: "OCH_OK", -1: "OCH_E_INVALID", -2: "OCH_E_HIP", -3: "OCH_E_NODEV",
                -4: "OCH_E_RCP_MODEL", -5: "OCH_E_NOMEM", -6: "OCH_E_CAPACITY"}


class OchError(RuntimeError):
    def __init__(self, status: int, func: str, msg: str):
        self.status = status
        super().__init__(f"{func} -> {STATUS_NAMES.get(status, status)}: {msg}")


class Camera(C.Structure):
    """och_camera: tree_camera::update_position's per-frame uniforms."""
    _fields_ = [("pos", C.c_float * 3), ("rot", C.c_float * 9), ("fov_factor", C.c_float),
                ("aspect", C.c_float), ("view_x", C.c_float), ("view_y", C.c_float),
                ("width", C.c_int32), ("height", C.c_int32)]


class PoolInfo(C.Structure):
    _fields_ = [("device_bytes", C.c_uint64), ("n_nodes", C.c_uint32), ("root", C.c_uint32),
                ("depth", C.c_int32), ("index_base", C.c_int32), ("miss_t", C.c_float),
                ("rcp_log2_entries", C.c_int32), ("device", C.c_int32)]


class EditorStats(C.Structure):
    _fields_ = [("capacity", C.c_uint32), ("live_nodes", C.c_uint32), ("high_water", C.c_uint32),
                ("root", C.c_uint32), ("depth", C.c_int32), ("dirty_first", C.c_uint32), ("dirty_count", C.c_uint32)]


class TerrainParams(C.Structure):
    _fields_ = [("depth", C.c_int32), ("tunnels", C.c_int32), ("dedup", C.c_int32),
                ("rand_kind", C.c_int32), ("threads", C.c_int32), ("use_gpu", C.c_int32)]


class HostPool(C.Structure):
    _fields_ = [("nodes", C.POINTER(C.c_uint32)), ("n_nodes", C.c_uint32), ("root", C.c_uint32),
                ("depth", C.c_int32), ("index_base", C.c_int32), ("solid_voxels", C.c_uint64),
                ("voxel_hist", C.c_uint64 * 8), ("tree_nodes", C.c_uint64), ("build_seconds", C.c_double)]


_P = C.c_void_p
_u32, _i32, _f32 = C.c_uint32, C.c_int32, C.c_float

# name -> (restype, argtypes); int-returning functions are status-checked.
PROTOTYPES = {
    "och_abi_version": (C.c_int, []),
    "och_last_error": (C.c_char_p, []),
    "och_discarded_error": (C.c_int, [C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_char_p, C.c_size_t, C.c_int]),
    "och_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "och_device_list": (C.c_int, [_P, C.c_int, C.POINTER(C.c_int)]),
    "och_host_rcp_lut": (C.c_int, [_P, C.POINTER(C.c_int)]),
    "och_rcp_from_lut": (_u32, [_u32, _P, C.c_int]),
    "och_rcp_lut_error": (C.c_int, [_P, C.c_int, C.POINTER(C.c_double)]),
    "och_gpu_pool_create": (C.c_int, [_P, _u32, _u32, C.c_int, C.c_int, _f32, C.c_int, C.POINTER(_P)]),
    "och_gpu_pool_destroy": (C.c_int, [_P]),
    "och_gpu_pool_info": (C.c_int, [_P, C.POINTER(PoolInfo)]),
    "och_gpu_pool_update": (C.c_int, [_P, _u32, _u32, _P, _u32]),
    "och_gpu_set_rcp_lut": (C.c_int, [_P, _P, C.c_int]),
    "och_gpu_set_palette": (C.c_int, [_P, _P, _u32]),
    "och_gpu_set_stream": (C.c_int, [_P, _P]),
    "och_gpu_synchronize": (C.c_int, [_P]),
    "och_gpu_set_option": (C.c_int, [_P, C.c_int, C.c_int]),
    "och_gpu_get_option": (C.c_int, [_P, C.c_int, C.POINTER(C.c_int)]),
    "och_gpu_set_stamp_buffer": (C.c_int, [_P, _P, _u32]),
    "och_gpu_occupancy": (C.c_int, [_P, C.c_int, C.POINTER(C.c_int)]),
    "och_gpu_last_kernel_ms": (C.c_int, [_P, C.POINTER(C.c_float)]),
    "och_gpu_set_launch_events": (C.c_int, [_P, C.c_void_p, C.c_void_p]),
    "och_gpu_trace": (C.c_int, [_P] + [_f32] * 6 + [C.POINTER(_i32), C.POINTER(_u32), C.POINTER(_f32)]),
    "och_gpu_trace_batch": (C.c_int, [_P, _P, C.c_int, _P, _u32, _P, _P, _P]),
    "och_gpu_trace_batch_dev": (C.c_int, [_P, _P, C.c_int, _P, _u32, _P, _P, _P, _P]),
    "och_gpu_trace_batch_image": (C.c_int, [_P, _P, C.c_int, _P, _u32, _u32, _P, _P, _P]),
    "och_gpu_trace_batch_tiled_dev": (C.c_int, [_P, _P, C.c_int, _P, _u32, _u32, _P, _P, _P, _P]),
    "och_gpu_plan_batch_tiled": (C.c_int, [_P, _P, C.c_int, _P, _u32, _u32]),
    "och_gpu_trace_bounce_batch_dev": (C.c_int, [_P, _P, C.c_int, _P, _u32, _P, _P, _P, _P, _P, _P, _P]),
    "och_camera_setup": (C.c_int, [_f32] * 6 + [C.c_int, C.c_int, C.POINTER(Camera)]),
    "och_gpu_raygen_dev": (C.c_int, [_P, C.POINTER(Camera), _P]),
    "och_gpu_render": (C.c_int, [_P, C.POINTER(Camera), _P]),
    "och_gpu_render_dev": (C.c_int, [_P, C.POINTER(Camera), _P, C.c_int, C.c_int, C.c_int]),
    "och_shard_rows": (C.c_int, [C.c_int, C.c_int, C.c_int]),
    "och_gpu_render_views_dev": (C.c_int, [_P, _P, C.c_int, _P, C.c_int, C.c_int, C.c_int]),
    "och_gpu_plan_views": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int]),
    "och_gpu_render_bounce_views_dev": (C.c_int, [_P, _P, C.c_int, _P, C.c_int, C.c_int, C.c_int]),
    "och_gpu_render_steps_dev": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, _P, C.c_int, _P, _P, C.c_int, C.c_int]),
    "och_gpu_set_row_deal": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, _P]),
    "och_gpu_slice_rows": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]),
    "och_gpu_chunk_costs": (C.c_int, [_P, _P, C.c_int, C.c_int, _P]),
    "och_deal_chunks": (C.c_int, [_P, C.c_int, C.c_int, _P, _P]),
    "och_gpu_unshard_dev": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, C.c_int, C.c_int]),
    "och_gpu_unshard_views_dev": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    "och_gpu_render_codes_views_dev": (C.c_int, [_P, _P, C.c_int, _P, C.c_int, C.c_int, C.c_int, C.c_int]),
    "och_gpu_shade_unshard_views_dev": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    "och_build_terrain": (C.c_int, [C.POINTER(TerrainParams), C.POINTER(HostPool)]),
    "och_host_pool_free": (None, [C.POINTER(HostPool)]),
    "och_pool_pack": (C.c_int, [_P, _u32, _u32, C.c_int, C.c_int, _P, _u32, C.POINTER(_u32), C.POINTER(_u32)]),
    "och_pool_at": (_u32, [_P, _u32, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    "och_pool_occupied_box": (C.c_int, [_P, _u32, _u32, C.c_int, C.c_int, _P, _P]),
    "och_editor_create": (C.c_int, [_P, _u32, _u32, C.c_int, _u32, C.POINTER(_P)]),
    "och_editor_destroy": (C.c_int, [_P]),
    "och_editor_set": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, _u32]),
    "och_editor_at": (_u32, [_P, C.c_int, C.c_int, C.c_int]),
    "och_editor_info": (C.c_int, [_P, C.POINTER(EditorStats)]),
    "och_editor_nodes": (C.c_int, [_P, C.POINTER(C.POINTER(_u32)), C.POINTER(_u32), C.POINTER(_u32)]),
    "och_editor_flush": (C.c_int, [_P, _P]),
    "och_frame_group_create": (C.c_int, [_P, C.c_int, _P, _u32, _u32, C.c_int, C.c_int, _f32, C.POINTER(_P)]),
    "och_frame_group_destroy": (C.c_int, [_P]),
    "och_frame_group_size": (C.c_int, [_P, C.POINTER(C.c_int)]),
    "och_frame_group_pool": (C.c_int, [_P, C.c_int, C.POINTER(_P)]),
    "och_frame_group_set_palette": (C.c_int, [_P, _P, _u32]),
    "och_frame_group_set_option": (C.c_int, [_P, C.c_int, C.c_int]),
    "och_frame_group_render": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int]),
    "och_frame_group_plan": (C.c_int, [_P, _P, C.c_int, C.c_int]),
    "och_frame_group_frames_dev": (C.c_int, [_P, C.c_int, C.POINTER(_P)]),
    "och_frame_group_download": (C.c_int, [_P, C.c_int, _P]),
    "och_frame_group_synchronize": (C.c_int, [_P]),
    "och_frame_group_render_steps": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    "och_comm_unique_id": (C.c_int, [_P]),
    "och_comm_create": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, C.POINTER(_P)]),
    "och_comm_destroy": (C.c_int, [_P]),
    "och_comm_available": (C.c_int, []),
    "och_comm_abort": (C.c_int, [_P]),
    "och_comm_info": (C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "och_comm_all_gather": (C.c_int, [_P, _P, _P, C.c_size_t, _P]),
    "och_comm_gather": (C.c_int, [_P, _P, _P, C.c_size_t, C.c_int, _P]),
    "och_gpu_render_sharded_steps_dev": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, _P, _P, _P, _P, C.c_int, _P, _P,
                                                   C.c_int, C.c_int, C.c_int]),
}

# och_gpu_render_sharded_steps_dev's exchange (include/och_gpu.h OCH_EXCHANGE_*)
EXCHANGE = {"all_gather": 0, "display": 1, "gather": 2}
COMM_ID_BYTES = 128

# Functions whose int return value is data, not a status.
_NOT_STATUS = {"och_abi_version", "och_shard_rows"}

_lib = None


def library_path() -> Path:
    return Path(os.environ.get("OCH_GPU_LIB", LIB_PATH))


def load(path: Path | None = None):
    """Load liboch_gpu.so once.  Raises if it is missing -- there is no fallback."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    explicit = path is not None
    path = Path(path) if explicit else library_path()
    if not path.exists():
        raise OchError(-3, "load", f"{path} is missing: build it with __graft_entry__.build() "
                                   "or `make -C octree_ray_tracing_amd/csrc`")
    # torch (if imported first) already holds libamdhip64.so.7; binding by
    # soname makes this library share that HIP runtime.
    lib = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
    for name, (res, args) in PROTOTYPES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if not explicit:
        _lib = lib
    return lib


def call(name: str, *args):
    lib = load()
    r = getattr(lib, name)(*args)
    if name in _NOT_STATUS or PROTOTYPES[name][0] is not C.c_int:
        return r
    if r != OCH_OK:
        msg = lib.och_last_error()
        raise OchError(r, name, msg.decode() if msg else "")
    return r


def discarded_error(reset: bool = False) -> dict | None:
    """The first pending HIP error a kernel launch found and cleared since the
    last reset (och_discarded_error), or None: {"hip_error", "count", "what"}."""
    code, count = C.c_int(), C.c_int()
    what = C.create_string_buffer(512)
    call("och_discarded_error", C.byref(code), C.byref(count), what, len(what), int(bool(reset)))
    if not count.value:
        return None
    return {"hip_error": code.value, "count": count.value, "what": what.value.decode(errors="replace")}


def exported_symbols() -> list[str]:
    return list(PROTOTYPES)
