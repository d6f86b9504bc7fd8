"""bench.py's launch selection and its N > 1 exchange check, on the CPU.

`bench.py --gpus N` must measure N GPUs or fail: without a launcher it starts
N ranks under torch.distributed.run (or, with --launch group, drives N devices
from one process); with fewer than N devices visible it exits non-zero instead
of measuring one.  Before the timed window of an N > 1 run, one exchanged
frame is checked slice by slice (bench.check_exchange); here two gloo ranks run
that check on host tensors, clean and with one corrupted copy."""
import os
import subprocess
import sys
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def test_resolve_launch():
    r = bench.resolve_launch
    assert r(1, {}, "procs", 0) == "rank"                       # N = 1: this process
    assert r(8, {}, "procs", 8) == "procs"                      # no launcher: start 8 ranks
    assert r(2, {}, "group", 2) == "group"
    assert r(1, {}, "group", 1) == "group"
    assert r(8, {"WORLD_SIZE": "8"}, "procs", 8) == "rank"      # the driver's torch.distributed.run
    # the gloo rehearsal shares one GPU between ranks on purpose
    assert r(8, {"WORLD_SIZE": "8", "OCH_DIST_BACKEND": "gloo"}, "procs", 1) == "rank"
    for args in [(8, {}, "procs", 1),                           # fewer devices than --gpus: refuse
                 (2, {}, "group", 1),
                 (8, {"WORLD_SIZE": "8"}, "procs", 4),
                 (8, {"WORLD_SIZE": "4"}, "procs", 8),          # launcher and --gpus disagree
                 (2, {"WORLD_SIZE": "2"}, "group", 2),          # the group is one process
                 (0, {}, "procs", 8)]:
        with pytest.raises(SystemExit):
            r(*args)


@pytest.mark.parametrize("extra", [[], ["--launch", "group"]])
def test_bench_refuses_missing_gpus(extra):
    """No GPU in this container: asking for 2 must exit non-zero at once
    (before any build or timing), never report a one-GPU line."""
    if torch.cuda.device_count() >= 2:
        pytest.skip("enough GPUs visible")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", *extra], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert "GPU(s) visible" in p.stderr
    assert p.stdout.strip() == ""


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "8"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE 4" in p.stderr


def test_slice_checksum_is_order_sensitive():
    a = torch.arange(64, dtype=torch.uint8).reshape(2, 4, 8)
    b = a.flip(-1).contiguous()
    assert int(bench.slice_checksum(a)) != int(bench.slice_checksum(b))
    assert int(bench.slice_checksum(a)) == int(bench.slice_checksum(a.clone()))


def _check_worker(rank, world, port, corrupt, receives_all, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(rank)
    sl = torch.from_numpy(rng.integers(0, 255, (2, 16, 24), dtype=np.uint8))
    outs = [torch.empty_like(sl) for _ in range(world)]
    dist.all_gather(outs, sl)
    gathered = torch.stack(outs)
    if corrupt and rank == 1:
        gathered[0, 1, 3, 5] ^= 1                        # one byte of rank 0's slice, as received by rank 1
    frame = SimpleNamespace(slice=sl, gathered=gathered)
    bad = bench.check_exchange(frame, world, rank, receives_all or rank == 0)
    q.put((rank, bad))
    dist.destroy_process_group()


@pytest.mark.parametrize("corrupt,receives_all,want", [(False, True, 0), (True, True, 1), (True, False, 0)])
def test_check_exchange_gloo_world2(corrupt, receives_all, want):
    """All-gather (every rank receives): a corrupted copy on rank 1 is counted
    on every rank.  Gather to rank 0: rank 1's buffer is not a receive buffer
    and is not checked."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 32500 + os.getpid() % 1000 + 7 * int(corrupt) + 3 * int(receives_all)
    procs = [ctx.Process(target=_check_worker, args=(r, 2, port, corrupt, receives_all, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == {0: want, 1: want}


class _FakeComm:
    closed = False

    def close(self):
        _FakeComm.closed = True


def _comm_worker(rank, world, port, fail_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def make():
        if rank == fail_rank:
            raise RuntimeError("ncclCommInitRank failed (test)")
        return _FakeComm()
    comm = bench.agreed_comm(make, world, torch.device("cpu"), log=lambda *a: None)
    q.put((rank, comm is not None, _FakeComm.closed))
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [-1, 1])
def test_agreed_comm_gloo_world2(fail_rank):
    """The library communicator is used only if every rank made one: when rank 1
    fails, rank 0 closes its own and both fall back together."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33700 + os.getpid() % 1000 + 5 * (fail_rank + 1)
    procs = [ctx.Process(target=_comm_worker, args=(r, 2, port, fail_rank, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, (has, closed)) for r, has, closed in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if fail_rank < 0:
        assert got == {0: (True, False), 1: (True, False)}
    else:
        assert got == {0: (False, True), 1: (False, False)}
