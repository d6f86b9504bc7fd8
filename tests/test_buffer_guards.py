"""The Python wrappers check device buffers passed as tensors against what a
launch writes (the C ABI takes bare pointers): a frame slice holds whole row
chunks (och_shard_rows), a batch holds 12 B per ray in and 4 B per record out.
CPU tensors stand in for device ones; no launch is made."""
import pytest
import torch

from octree_ray_tracing_amd import tracer


def test_need_accepts_exact_and_larger():
    t = torch.zeros(10, dtype=torch.int32)
    tracer._need(t, 40, "x")
    tracer._need(t, 8, "x")
    tracer._need(12345, 10 ** 9, "a raw pointer is not checked")


def test_need_refuses_short_buffers():
    with pytest.raises(ValueError, match="holds 36 B, the launch needs 40 B"):
        tracer._need(torch.zeros(9, dtype=torch.int32), 40, "frame")


def test_batch_sizes():
    n = 5
    o1 = torch.zeros(3)                           # one shared origin
    d = torch.zeros(3 * n)
    outs = [torch.zeros(n, dtype=torch.int32) for _ in range(3)]
    tracer.GpuPool._need_batch(o1, d, n, 0, outs + [None])
    with pytest.raises(ValueError, match="origins"):
        tracer.GpuPool._need_batch(o1, d, n, 3, outs)        # per-ray origins need 12 B each
    with pytest.raises(ValueError, match="dirs"):
        tracer.GpuPool._need_batch(o1, d[:-1], n, 0, outs)
    with pytest.raises(ValueError, match="hit records"):
        tracer.GpuPool._need_batch(o1, d, n, 0, outs[:2] + [torch.zeros(n - 1, dtype=torch.int32)])


def test_frame_slices_hold_whole_row_chunks():
    """451 rows in chunks of 8: a slice holds 456 rows (och_shard_rows)."""
    assert tracer.shard_rows(451, 8, 1) == 456
    assert tracer.shard_rows(451, 8, 3) == 152
