"""och_frame_group_*: multi-GPU frames from one host process (SURVEY §8(e):
one process, ncclCommInitAll over the devices, RCCL all-gather of the slices).

On the one-GPU test box the group has one device: the RCCL communicator, the
all-gather and the shade + unshard still run, and the frames must equal the
oracle's (and the single-pool render's) bit for bit."""
import numpy as np
import pytest

ORIGIN = np.array([1.5, 1.5, 1.5], np.float32)
PITCHES = (0.0, -0.6)


def test_group_needs_devices(ort):
    """Argument checks that need no GPU; without one the group reports OCH_E_NODEV."""
    import torch
    nodes = np.zeros((1, 8), np.uint32)
    nodes[0, 0] = 1
    with pytest.raises(ort.OchError):
        ort.FrameGroup(nodes, 1, 1, devices=[])
    if not torch.cuda.is_available():
        with pytest.raises(ort.OchError, match="NODEV"):
            ort.FrameGroup(nodes, 1, 1, devices=[0])


@pytest.mark.gpu
@pytest.mark.parametrize("bounce", [False, True])
def test_group_one_device_matches_oracle(ort, O, gpu_device, bounce):
    depth, W, H = 10, 1280, 720
    tree = ort.build_terrain(depth)
    pal = ort.VoxelData().get_colours()
    g = ort.FrameGroup(tree.nodes, tree.root, depth, devices=[0])
    g.set_palette(pal)
    cams = [ort.camera(tuple(ORIGIN), 0.3, p, 1.25, W, H) for p in PITCHES]
    ref_pool = O.OraclePool(tree.nodes, tree.root, depth, 1)
    want = []
    for p in PITCHES:
        rays = O.raygen(0.3, p, 1.25, W, H)
        if bounce:
            r = O.trace_bounce_batch(ref_pool, O.Rcp(None), ORIGIN, rays, nthreads=16)
            want.append(O.shade_bounce(r["dir"], r["voxel"], r["dir2"], pal).reshape(H, W))
        else:
            r = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, rays, nthreads=16)
            want.append(O.shade_fast(r["dir"], r["voxel"], pal).reshape(H, W))
    for chunk in (8, 5):
        g.render(cams, row_chunk=chunk, bounce=bounce)
        got = g.download(0)
        for v in range(2):
            assert np.array_equal(got[v], want[v]), (chunk, v)
    g.plan(cams, row_chunk=8)                   # planned launch order (tile_order 2)
    g.render(cams, row_chunk=8, bounce=bounce)
    got = g.download(0)
    for v in range(2):
        assert np.array_equal(got[v], want[v]), ("planned", v)
    # a palette of more than OCH_CODE_MAX_VOXELS ids: RGBA8 slices travel instead of codes
    big = np.resize(np.asarray(pal, np.uint32).reshape(-1), 6 * 24)
    g.set_palette(big)
    g.render(cams, row_chunk=8, bounce=bounce)
    got = g.download(0)
    pool = ort.HOctree(tree.nodes, tree.root, depth, device=0)
    pool.set_palette(big)
    for v, cam in enumerate(cams):
        if not bounce:
            assert np.array_equal(got[v], pool.render(cam))
    pool.close()
    g.close()


@pytest.mark.gpu
def test_group_rejects_duplicates(ort, gpu_device):
    tree = ort.build_terrain(4)
    with pytest.raises(ort.OchError):
        ort.FrameGroup(tree.nodes, tree.root, 4, devices=[0, 0])
    import torch
    with pytest.raises(ort.OchError):
        ort.FrameGroup(tree.nodes, tree.root, 4, devices=[torch.cuda.device_count()])


@pytest.mark.gpu
def test_group_checks_before_queueing(ort, O, gpu_device):
    """A frame the group cannot complete is refused before any device queues
    its render or all-gather (a palette-less group cannot shade): the group
    stays usable -- no communicator aborted -- and renders once a palette is
    set; destroy releases the pools before the streams they point at."""
    tree = ort.build_terrain(6)
    g = ort.FrameGroup(tree.nodes, tree.root, 6, devices=[0])
    cams = [ort.camera(tuple(ORIGIN), 0.3, p, 1.25, 64, 40) for p in PITCHES]
    with pytest.raises(ort.OchError, match="palette"):
        g.render(cams)
    pal = ort.VoxelData().get_colours()
    g.set_palette(pal)
    g.render_steps(cams, 3, n_buffers=2)
    got = g.download(0)
    ref_pool = O.OraclePool(tree.nodes, tree.root, 6, 1)
    for v, p in enumerate(PITCHES):
        r = O.trace_batch(ref_pool, O.Rcp(None), ORIGIN, O.raygen(0.3, p, 1.25, 64, 40))
        assert np.array_equal(got[v], O.shade(r["dir"], r["voxel"], pal).reshape(40, 64))
    g.close()
