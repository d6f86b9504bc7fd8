"""bench.py's multi-GPU launch paths on the one-GPU box, end to end.

* `--launch group --gpus 1`: the one-process device group (och_frame_group_*:
  ncclCommInitAll, one issuing thread per device, RCCL all-gather, shade),
  its last frames checked against the oracle inside the bench line;
* the N > 1 per-process path as two gloo ranks sharing the GPU (the
  driver's 8-GPU form rehearsed at world size 2): the one-frame exchange
  check before the timed window, parity of rank 0's frames against the
  oracle, and scaling_base -- rank 0 alone rendering the same frame the
  N = 1 way, whose frames must equal the sharded run's.
Depth 10 keeps both runs short; the code paths are the depth-12 ones."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SMALL = ["--depth", "10", "--steps", "5", "--warmup", "2", "--sustain", "0", "--no-bounce", "--no-cull-off",
         "--no-cpu-baseline", "--no-other-configs", "--moving-steps", "0"]


def _line(stdout: str) -> dict:
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert lines, stdout[-2000:]
    return json.loads(lines[-1])


def _env():
    return {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "OCH_DIST_BACKEND")}


@pytest.mark.gpu
def test_bench_group_launch_one_device_matches_oracle():
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--launch", "group", *SMALL],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = _line(p.stdout)
    assert line["n_gpus"] == 1 and "och_frame_group" in line["config"]["launch"]
    assert line["parity"]["mismatches"] == 0 and line["parity"]["pixels"] == 2 * 1920 * 1080
    assert line["parity"]["devices_equal_rank0"] is True
    assert line["value"] > 0


@pytest.mark.gpu
def test_bench_two_gloo_ranks_exchange_check_and_scaling_base():
    env = dict(_env(), OCH_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(29600 + os.getpid() % 300), str(ROOT / "bench.py"), "--gpus", "2",
           "--width", "960", "--height", "544", *SMALL]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = _line(p.stdout)
    assert line["n_gpus"] == 2
    assert line["exchange_check"]["mismatches"] == 0 and line["exchange_check"]["slices"] == 2
    assert "gloo" in line["config"]["exchange"] and "rehearsal" in line["config"]["workload"]
    assert line["parity"]["mismatches"] == 0 and line["parity"]["pixels"] == 2 * 960 * 544
    base = line["scaling_base"]
    assert base["frames_equal_sharded"] is True and base["value"] > 0 and base["frames_in_flight"] == 3
