"""bench.py's host logic on the CPU: the per-world-size pipeline defaults
(frames in flight, hardware queues), the kernel-source digest the PMC summary
is keyed by, and the committed profiles' loaders."""
import sys
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def test_pipeline_defaults_by_world_size():
    assert bench.pipeline_defaults(1) == (3, None)
    assert bench.pipeline_defaults(2) == (3, None)
    assert bench.pipeline_defaults(4) == (3, None)
    assert bench.pipeline_defaults(8) == (6, 8)
    assert bench.pipeline_defaults(8, inflight=3, hw_queues=4) == (3, 4)      # explicit values win
    assert bench.pipeline_defaults(1, inflight=6, hw_queues=8) == (6, 8)
    with pytest.raises(SystemExit):
        bench.pipeline_defaults(1, hw_queues=33)                              # gpurun refuses > 32
    with pytest.raises(SystemExit):
        bench.pipeline_defaults(1, inflight=0)


def test_committed_profiles_match_this_kernel_source():
    pmc, src = bench.load_pmc("k_render_rgba", "d12_1920x1080_n1")
    assert src == "profiles/pmc_summary.json", src
    assert pmc["valu_insts_per_wave"] > 0 and 0 < pmc["valu_lane_utilization"] <= 1
    win = bench.load_window()
    assert win is not None and not win.get("stale")
    assert 0 < win["busy_union_ms_per_step"] <= win["ms_per_step_trace"] + 1e-9
