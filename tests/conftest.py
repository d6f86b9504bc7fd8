import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
GOLD = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU check")


def _ensure_built():
    lib = ROOT / "octree_ray_tracing_amd" / "liboch_gpu.so"
    ora = ROOT / "oracle" / "build" / "liboch_oracle.so"
    if not lib.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "octree_ray_tracing_amd" / "csrc")], check=True)
    if not ora.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def ort():
    import octree_ray_tracing_amd as m
    m.load()
    return m


@pytest.fixture(scope="session")
def O():
    from oracle import oracle as m
    return m


@pytest.fixture(scope="session")
def intel_lut():
    import numpy as np
    return np.fromfile(GOLD / "rcp_lut_intel.bin", dtype=np.uint32)


@pytest.fixture(scope="session")
def known():
    import json
    return json.loads((GOLD / "known_answers.json").read_text())


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no GPU visible")
    torch.cuda.set_device(0)
    return 0
