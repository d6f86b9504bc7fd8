"""A fixed-seed slice of the randomised parity campaign (tools/fuzz_parity.py):
random scenes (scatter, boxes, slabs, checkerboards, dyadic-corner clusters;
depths 2-16; voxel ids up to 2^32 - 1), random edge-case rays and random
launch options through eleven C-ABI paths (trace, tiled trace, bounce,
och::octree, camera frames in natural or planned order with the heavy-tile
split, sharded colour codes + shade, config-5 frames, the host image entry,
editor flushes, the N = 1 frame loop, the N > 1 window at world size 1), each
against the oracle bit for bit.  Round 6's campaigns:
profiles/r06/INDEX.md (r06n-r06r, prof_r06q)."""
import json
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


def test_fuzz_slice(tmp_path, ort, O, gpu_device):
    sys.path.insert(0, str(ROOT / "tools"))
    import fuzz_parity
    out = tmp_path / "fuzz.jsonl"
    rc = fuzz_parity.main(["--cases", "160", "--seed", "7", "--rays", "20000", "--seconds", "90",
                           "--terrain", "0.1", "--out", str(out)])
    rows = [json.loads(l) for l in out.read_text().splitlines()]
    summary = rows[-1]
    bad = [r for r in rows[:-1] if r["mismatches"]]
    assert rc == 0 and not bad, bad[:3]
    assert summary["cases"] >= 60 and len(summary["by_path"]) == 11, summary
