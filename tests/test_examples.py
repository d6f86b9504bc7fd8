"""The C++ boundary, exercised: examples/render_frame (och::gpu::tree --
the reference's tree.sse_trace(o, d, dir&, voxel&, t&) call shape and the
update_image frame), examples/multi_gpu_frame (och::gpu::frame_group, one
process over every GPU, RCCL all-gather) and examples/sharded_frame (one
process per GPU: the RCCL id handed over through a file, the gather to the
display rank, och_gpu_render_sharded_steps_dev) are built by __graft_entry__.build()
against include/och_gpu.hpp, run as programs, and their PPM frames and pick
ray are compared with the oracle."""
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

EX = ROOT / "examples"
ORIGIN = np.array([1.5, 1.5, 1.5], np.float32)


def _ensure_examples():
    if not all((EX / x).exists() for x in ("render_frame", "multi_gpu_frame", "sharded_frame")):
        subprocess.run(["make", "-s", "-C", str(EX)], check=True)


def read_ppm(path):
    data = path.read_bytes()
    m = re.match(rb"P6\n(\d+) (\d+)\n255\n", data)
    w, h = int(m.group(1)), int(m.group(2))
    return np.frombuffer(data[m.end():], np.uint8).reshape(h, w, 3)


def rgb_of(rgba):
    rgba = np.asarray(rgba, np.uint32)
    return np.stack([rgba & 0xFF, (rgba >> 8) & 0xFF, (rgba >> 16) & 0xFF], axis=-1).astype(np.uint8)


def test_examples_build_and_fail_cleanly_without_gpu(ort, tmp_path):
    import torch
    _ensure_examples()
    if torch.cuda.is_available():
        pytest.skip("GPU present: the -m gpu tests run the examples")
    r = subprocess.run([str(EX / "render_frame"), "4", str(tmp_path / "x.ppm"), "64", "36", "0.3", "-0.6"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "och_gpu_pool_create" in r.stderr


@pytest.mark.gpu
def test_render_frame_example(ort, O, gpu_device, tmp_path):
    _ensure_examples()
    depth, W, H, yaw, pitch = 9, 640, 360, 0.3, -0.6
    out = tmp_path / "frame.ppm"
    r = subprocess.run([str(EX / "render_frame"), str(depth), str(out), str(W), str(H), str(yaw), str(pitch)],
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr
    tree = ort.build_terrain(depth)
    pool = O.OraclePool(tree.nodes, tree.root, depth, 1)
    rays = O.raygen(yaw, pitch, 1.25, W, H)
    ref = O.trace_batch(pool, O.Rcp(None), ORIGIN, rays, nthreads=16)
    want = rgb_of(O.shade_fast(ref["dir"], ref["voxel"], ort.VoxelData().get_colours())).reshape(H, W, 3)
    assert np.array_equal(read_ppm(out), want)
    m = re.search(r"pick ray: d (\S+) (\S+) (\S+) direction (\d+) voxel (\d+) t (\S+)", r.stdout)
    d = [float.fromhex(m.group(i)) for i in (1, 2, 3)]
    dr, vx, t, _ = O.trace(pool, O.Rcp(None), ORIGIN, d)
    assert (int(m.group(4)), int(m.group(5))) == (dr, vx)
    assert np.float32(float.fromhex(m.group(6))) == np.float32(t)


@pytest.mark.gpu
def test_multi_gpu_frame_example(ort, O, gpu_device, tmp_path):
    import torch
    _ensure_examples()
    depth, W, H = 10, 800, 450
    n = torch.cuda.device_count()
    for view, pitch in ((0, 0.0), (1, -0.6)):
        out = tmp_path / f"mg{view}.ppm"
        r = subprocess.run([str(EX / "multi_gpu_frame"), str(depth), str(W), str(H), str(out), str(n), "3", str(view)],
                           capture_output=True, text=True, timeout=110)
        assert r.returncode == 0, r.stderr
        tree = ort.build_terrain(depth)
        pool = O.OraclePool(tree.nodes, tree.root, depth, 1)
        ref = O.trace_batch(pool, O.Rcp(None), ORIGIN, O.raygen(0.3, pitch, 1.25, W, H), nthreads=16)
        want = rgb_of(O.shade_fast(ref["dir"], ref["voxel"], ort.VoxelData().get_colours())).reshape(H, W, 3)
        assert np.array_equal(read_ppm(out), want), view


@pytest.mark.gpu
def test_sharded_frame_example(ort, O, gpu_device, tmp_path):
    """One rank (a one-GPU box): the RCCL id through the file, the gather's
    ncclSend / ncclRecv group, the display rank's shade -- the frames of
    och_gpu_render_sharded_steps_dev against the oracle's."""
    _ensure_examples()
    depth, W, H = 10, 800, 450
    tree = ort.build_terrain(depth)
    pool = O.OraclePool(tree.nodes, tree.root, depth, 1)
    for view, pitch in ((0, 0.0), (1, -0.6)):
        out = tmp_path / f"sh{view}.ppm"
        r = subprocess.run([str(EX / "sharded_frame"), str(depth), str(W), str(H), str(out), "0", "1",
                            str(tmp_path / f"id{view}"), "4", str(view)], capture_output=True, text=True, timeout=110)
        assert r.returncode == 0, r.stderr
        assert "rank 0 of 1" in r.stdout
        ref = O.trace_batch(pool, O.Rcp(None), ORIGIN, O.raygen(0.3, pitch, 1.25, W, H), nthreads=16)
        want = rgb_of(O.shade_fast(ref["dir"], ref["voxel"], ort.VoxelData().get_colours())).reshape(H, W, 3)
        assert np.array_equal(read_ppm(out), want), view
