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


def _comm_worker(rank, world, port, fail, q):
    """fail = (step, rank): which agreement step fails on which rank."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    step, bad_rank = fail
    calls = []

    def unique_id():
        calls.append("id")
        if step == "id" and rank == bad_rank:
            raise RuntimeError("ncclGetUniqueId failed (test)")
        return bytes(range(128))

    def available():
        calls.append("available")
        return not (step == "available" and rank == bad_rank)

    def create(uid):
        calls.append("create")
        assert uid == bytes(range(128))               # rank 0's id reached every rank
        if step == "create" and rank == bad_rank:
            raise RuntimeError("ncclCommInitRank failed (test)")
        return _FakeComm()
    comm = bench.agreed_comm(world, rank, torch.device("cpu"), unique_id, available, create, log=lambda *a: None)
    q.put((rank, comm is not None, _FakeComm.closed, tuple(calls)))
    dist.destroy_process_group()


@pytest.mark.parametrize("fail", [("none", -1), ("id", 0), ("available", 1), ("create", 1), ("create", 0)])
def test_agreed_comm_gloo_world2(fail):
    """The library communicator is used only if every rank made one, and no
    rank enters a collective step the others skip: rank 0's failed id travels
    with the id broadcast (no rank calls ncclCommInitRank), a rank that cannot
    load RCCL is known before anyone joins, and a failed join makes the ranks
    that joined close theirs -- all fall back together."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33700 + os.getpid() % 1000 + 11 * ["none", "id", "available", "create"].index(fail[0]) + fail[1] + 1
    procs = [ctx.Process(target=_comm_worker, args=(r, 2, port, fail, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {r: (has, closed, calls) for r, has, closed, calls in (q.get(timeout=120) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    step, bad = fail
    if step == "none":
        assert got == {0: (True, False, ("id", "create")), 1: (True, False, ("available", "create"))}
    elif step in ("id", "available"):
        # nobody joins: no rank is left inside ncclCommInitRank
        assert all(not has and "create" not in calls for has, _, calls in got.values())
    else:
        good = 1 - bad
        assert got[bad][:2] == (False, False) and got[good][:2] == (False, True)


def test_watchdog_in_process():
    """A stage past its deadline: the abort hooks run, one JSON line names the
    stage, the exit status is 3; a stage ended in time never fires."""
    import io
    import json
    import threading
    out, exited, aborted = io.StringIO(), [], []
    done = threading.Event()

    def fake_exit(code):
        exited.append(code)
        done.set()
    wd = bench.Watchdog(0, 8, poll_s=0.02, exit_fn=fake_exit, out=out)
    wd.on_expiry(lambda: aborted.append(1))
    wd.enter("window (headline)", 0.1)
    assert done.wait(10)
    line = json.loads(out.getvalue().strip().splitlines()[-1])
    assert exited == [3] and aborted == [1]
    assert line["stage"] == "window (headline)" and line["value"] is None and line["n_gpus"] == 8
    assert line["communicators_aborted"] == 1 and "deadline" in line["error"]
    wd2 = bench.Watchdog(1, 2, poll_s=0.02, exit_fn=fake_exit, out=io.StringIO())
    wd2.enter("setup", 0.2)
    wd2.done()
    import time
    time.sleep(0.5)
    assert exited == [3]


_WITHHOLD = r"""
import os, sys, time, datetime
from types import SimpleNamespace
sys.path.insert(0, {root!r})
import torch, torch.distributed as dist
import bench
rank = int(sys.argv[1])
dist.init_process_group("gloo", rank=rank, world_size=2, init_method="tcp://127.0.0.1:{port}",
                        timeout=datetime.timedelta(seconds=120))
wd = bench.Watchdog(rank, 2, poll_s=0.05)
wd.enter("exchange check", {deadline} if rank == 0 else 120)
sl = torch.zeros((2, 4, 8), dtype=torch.uint8)
frame = SimpleNamespace(slice=sl, gathered=torch.stack([sl, sl]))
if rank == 1:
    time.sleep(60)                      # withholds its side of the collective
bad = bench.check_exchange(frame, 2, rank, True)
print("returned", bad, flush=True)
"""


def test_watchdog_names_stage_when_a_rank_withholds_gloo_world2():
    """Two gloo ranks: rank 1 never joins the exchange check's collective.
    Rank 0 exits with status 3 within its deadline and prints one JSON line
    naming the stage, instead of waiting out torch's timeout (or the driver's)."""
    import json
    import time
    port = 35100 + os.getpid() % 1000
    code = _WITHHOLD.format(root=str(ROOT), port=port, deadline=4)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r1 = subprocess.Popen([sys.executable, "-c", code, "1"], env=env, stdout=subprocess.PIPE,
                          stderr=subprocess.PIPE, text=True)
    try:
        t0 = time.monotonic()
        r0 = subprocess.run([sys.executable, "-c", code, "0"], env=env, capture_output=True, text=True, timeout=100)
        took = time.monotonic() - t0
    finally:
        r1.kill()
        r1.communicate()
    assert r0.returncode == bench.Watchdog.EXIT, r0.stderr[-2000:]
    assert "returned" not in r0.stdout
    line = json.loads(r0.stdout.strip().splitlines()[-1])
    assert line["stage"] == "exchange check" and line["rank"] == 0 and line["value"] is None
    assert "exchange check" in r0.stderr
    assert took < 60                                    # the deadline (4 s) plus start-up, not torch's 120 s
