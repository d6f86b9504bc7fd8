import subprocess
import sys
from pathlib import Path

import numpy as np
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


def sparse_dag(depth, voxels):
    """A 1-based, hash-consed h_octree pool holding `voxels` (x, y, z, id > 0);
    child index x | y << 1 | z << 2 (ORT/och_h_octree.h:38-66).  The
    reference's own set() packs coordinates with z_encode_16 and stops at
    depth 16, so deeper test trees are assembled here."""
    table, nodes = {}, []

    def intern(children, lvl):
        key = (lvl, tuple(children))
        if key not in table:
            nodes.append(children)
            table[key] = len(nodes)
        return table[key]

    cells = {}
    for x, y, z, v in voxels:
        cells.setdefault((x >> 1, y >> 1, z >> 1), [0] * 8)[(x & 1) | (y & 1) << 1 | (z & 1) << 2] = v
    ids = {k: intern(c, 0) for k, c in cells.items()}
    for lvl in range(1, depth):
        up = {}
        for (x, y, z), i in ids.items():
            up.setdefault((x >> 1, y >> 1, z >> 1), [0] * 8)[(x & 1) | (y & 1) << 1 | (z & 1) << 2] = i
        ids = {k: intern(c, lvl) for k, c in up.items()}
    return np.array(nodes, np.uint32), ids[(0, 0, 0)]
