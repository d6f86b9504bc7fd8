"""The C ABI library: loads, exports every symbol include/och_gpu.h declares,
and the host-only entry points behave (no GPU compute here)."""
import ctypes as C
import math
import re

import numpy as np
import pytest


def declared_symbols(ort):
    text = ort._lib.HEADER_PATH.read_text()
    return sorted(set(re.findall(r"OCH_API\s+[\w\s\*]+?\b(och_\w+)\s*\(", text)))


def test_header_and_binding_agree(ort):
    assert declared_symbols(ort) == sorted(ort._lib.exported_symbols())


def test_library_exports_every_declared_symbol(ort):
    lib = ort.load()
    for name in declared_symbols(ort):
        assert hasattr(lib, name), name


def test_abi_version(ort):
    assert ort._lib.call("och_abi_version") == 1


def test_rcp_from_lut_matches_oracle(ort, O, intel_lut):
    rng = np.random.default_rng(0)
    for x in rng.integers(0, 1 << 32, 5000, dtype=np.uint64).astype(np.uint32).tolist():
        assert ort.rcp_from_lut(x, intel_lut) == O.rcp_lut(x, intel_lut)


def test_host_rcp_lut(ort, intel_lut):
    lut = ort.host_rcp_lut()
    assert lut.size in (1 << k for k in range(8, 24))
    vendor = open("/proc/cpuinfo").read()
    if "GenuineIntel" in vendor:
        assert np.array_equal(lut, intel_lut)


def test_camera_constants(ort):
    cam = ort.camera((1.5, 1.5, 1.5), 0.3, -0.6, 1.25, 1920, 1080)
    f = np.float32
    assert cam.aspect == f(f(1920) / f(1080))
    assert cam.view_x == f(f(2) / f(1920)) and cam.view_y == f(f(2) / f(1080))
    assert cam.rot[6] == -f(math.sin(f(0.3))) or abs(cam.rot[6] + math.sin(0.3)) < 1e-7
    assert (cam.width, cam.height) == (1920, 1080)


def test_shard_rows(ort):
    assert ort.shard_rows(1080, 1080, 1) == 1080
    assert ort.shard_rows(2160, 8, 8) == 272          # 270 chunks -> 34 per shard
    assert ort.shard_rows(10, 4, 3) == 4


def test_pool_validation_rejects_bad_pools(ort):
    nodes = np.zeros((2, 8), np.uint32)
    nodes[0, 3] = 7                                   # interior slot names node 7 of 2
    with pytest.raises(ort.OchError) as e:
        ort.HOctree(nodes, 1, 3)
    assert e.value.status == -1
    with pytest.raises(ort.OchError):
        ort.HOctree(np.zeros((1, 8), np.uint32), 1, 40)   # depth out of range


def test_pool_create_without_gpu_fails_loudly(ort):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    tree = ort.build_terrain(4)
    with pytest.raises(ort.OchError) as e:
        ort.HOctree(tree.nodes, tree.root, tree.depth)
    assert e.value.status == -3


def test_missing_library_raises(ort, tmp_path):
    with pytest.raises(ort.OchError):
        ort._lib.load(tmp_path / "nope.so")


def test_header_is_plain_c_and_links(ort, tmp_path):
    """include/och_gpu.h is what a C FFI (cgo, ctypes, a C host) binds: it
    compiles as strict C99, and a C program links against liboch_gpu.so and
    runs the host-only entry points (ABI version, camera setup, pool pack /
    at on a tiny tree, the error text of a refused call)."""
    import shutil
    import subprocess
    from pathlib import Path
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no C compiler")
    root = Path(ort._lib.HEADER_PATH).resolve().parents[1]
    libdir = Path(ort.load()._name).resolve().parent
    src = tmp_path / "abi.c"
    src.write_text(r'''
#include <stdio.h>
#include <string.h>
#include "och_gpu.h"
int main(void)
{
    och_camera cam;
    /* one leaf-level node under a root at depth 2: voxel 3 at (0, 0, 0) */
    const uint32_t nodes[2][8] = {{2, 0, 0, 0, 0, 0, 0, 0}, {3, 0, 0, 0, 0, 0, 0, 0}};
    uint32_t packed[3 * 8], n_packed = 0, packed_root = 0;
    och_gpu_pool *pool = NULL;
    if (och_abi_version() != 1) return 1;
    if (och_camera_setup(1.5f, 1.5f, 1.5f, 0.3f, -0.6f, 1.25f, 64, 36, &cam) != OCH_OK) return 2;
    if (och_pool_at(&nodes[0][0], 1, 2, 1, 0, 0, 0) != 3 || och_pool_at(&nodes[0][0], 1, 2, 1, 1, 0, 0) != 0) return 3;
    if (och_pool_pack(&nodes[0][0], 2, 1, 2, 1, packed, 3, &n_packed, &packed_root) != OCH_OK || n_packed != 3)
        return 4;
    /* a refused call reports a status and a message */
    if (och_gpu_pool_create(&nodes[0][0], 2, 1, 0, 1, 0.0f, -1, &pool) == OCH_OK || pool != NULL) return 5;
    if (strlen(och_last_error()) == 0) return 6;
    printf("ok %u %08x\n", n_packed, packed_root);
    return 0;
}
''')
    exe = tmp_path / "abi"
    cc = subprocess.run([gcc, "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror", f"-I{root / 'include'}",
                         str(src), f"-L{libdir}", "-loch_gpu", f"-Wl,-rpath,{libdir}", "-o", str(exe)],
                        capture_output=True, text=True)
    assert cc.returncode == 0, cc.stderr
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert run.returncode == 0 and run.stdout.startswith("ok 3 "), (run.returncode, run.stdout, run.stderr)
