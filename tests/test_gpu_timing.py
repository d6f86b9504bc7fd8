"""Per-launch timing (OCH_OPT_TIMING, och_gpu_set_launch_events): the kernel's
own dispatch records the events (hipExtLaunchKernel), so a frame timer puts no
packets between two launches of a stream.  The frames are the
same in every timing mode; each mode times what it says."""
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def test_timing_modes_and_launch_events(ort, O, gpu_device):
    import torch
    from bench import FenceFreeEvent
    tree = ort.build_terrain(8)
    pal = ort.VoxelData().get_colours()
    pool = ort.HOctree(tree.nodes, tree.root, 8, device=0)
    pool.set_palette(pal)
    stream = torch.cuda.current_stream()
    pool.set_stream(stream)
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, 640, 360) for p in (0.0, -0.6)]
    r = [O.trace_batch(O.OraclePool(tree.nodes, tree.root, 8, 1), O.Rcp(None), np.array([1.5, 1.5, 1.5], np.float32),
                       O.raygen(0.3, p, 1.25, 640, 360)) for p in (0.0, -0.6)]
    want = np.stack([O.shade(x["dir"], x["voxel"], pal).reshape(360, 640) for x in r])
    assert pool.get_option("timing") == 1                       # the dispatch records the pool's events
    for mode in (1, 2, 0):
        pool.set_option("timing", mode)
        frames = torch.zeros((2, 360, 640), dtype=torch.int32, device="cuda")
        pool.render_views_dev(cams, frames)
        torch.cuda.synchronize()
        assert np.array_equal(frames.cpu().numpy().view(np.uint32), want), mode
        if mode:
            assert 0.0 < pool.last_kernel_ms() < 1000.0
        else:
            with pytest.raises(ort.OchError):
                pool.last_kernel_ms()
    # the caller's events, one launch only; the pool's own are not recorded by it
    pool.set_option("timing", 1)
    e0, e1 = FenceFreeEvent(), FenceFreeEvent()
    pool.set_launch_events(e0, e1)
    frames = torch.zeros((2, 360, 640), dtype=torch.int32, device="cuda")
    pool.render_views_dev(cams, frames)
    torch.cuda.synchronize()
    assert 0.0 < e0.elapsed_time(e1) < 1000.0
    assert np.array_equal(frames.cpu().numpy().view(np.uint32), want)
    with pytest.raises(ort.OchError):
        pool.last_kernel_ms()
    pool.render_views_dev(cams, frames)                          # the next launch: the pool's events again
    torch.cuda.synchronize()
    assert pool.last_kernel_ms() > 0.0
    with pytest.raises(ort.OchError):
        pool.set_option("timing", 3)
    pool.close()


def test_render_steps_native_loop(ort, O, gpu_device):
    """och_gpu_render_steps_dev: the frame loop issued by the library -- frame k
    on stream k % B into buffer k % B, its dispatch recording event pair k --
    gives the oracle's frames in every buffer, primary and config 5, and leaves
    the pool's stream as it was."""
    import torch
    from bench import FenceFreeEvent
    tree = ort.build_terrain(8)
    pal = ort.VoxelData().get_colours()
    pool = ort.HOctree(tree.nodes, tree.root, 8, device=0)
    pool.set_palette(pal)
    cur = torch.cuda.current_stream()
    pool.set_stream(cur)
    W, H = 320, 180
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in (0.0, -0.6)]
    r = [O.trace_batch(O.OraclePool(tree.nodes, tree.root, 8, 1), O.Rcp(None), np.array([1.5, 1.5, 1.5], np.float32),
                       O.raygen(0.3, p, 1.25, W, H)) for p in (0.0, -0.6)]
    want = np.stack([O.shade(x["dir"], x["voxel"], pal).reshape(H, W) for x in r])
    streams = [cur] + [torch.cuda.Stream() for _ in range(2)]
    for n_steps in (7, 1, 0):
        frames = [torch.zeros((2, H, W), dtype=torch.int32, device="cuda") for _ in streams]
        events = [(FenceFreeEvent(), FenceFreeEvent()) for _ in range(n_steps)]
        pool.render_steps_dev(cams, frames, streams, n_steps, events)
        torch.cuda.synchronize()
        for b, f in enumerate(frames):
            got = f.cpu().numpy().view(np.uint32)
            if b < n_steps:
                assert np.array_equal(got, want), (n_steps, b)
            else:
                assert not got.any()                           # no frame went to this buffer
        assert all(0.0 < x.elapsed_time(y) < 1000.0 for x, y in events)
    # without events; config 5 through the same loop equals the single-launch render
    frames = [torch.zeros((2, H, W), dtype=torch.int32, device="cuda") for _ in streams]
    pool.render_steps_dev(cams, frames, streams, 4, bounce=True)
    one = torch.zeros((2, H, W), dtype=torch.int32, device="cuda")
    pool.render_bounce_views_dev(cams, one)
    torch.cuda.synchronize()
    for f in frames:
        assert torch.equal(f, one)
    # the pool's own stream is untouched: a plain launch after the loop runs on it
    pool.set_option("timing", 1)
    pool.render_views_dev(cams, one)
    cur.synchronize()
    assert np.array_equal(one.cpu().numpy().view(np.uint32), want)
    with pytest.raises(ValueError):
        pool.render_steps_dev(cams, frames[:2], streams, 3)
    with pytest.raises(ValueError):
        pool.render_steps_dev(cams, frames, streams, 3, [(FenceFreeEvent(), FenceFreeEvent())])
    pool.close()
