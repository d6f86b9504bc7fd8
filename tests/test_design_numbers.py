"""DESIGN.md §4's roofline paragraph quotes the committed profile
(profiles/pmc_summary.json): the render launch's VALU count, its VALU per wave
and the PMC passes' mean launch duration.  A refreshed profile without the
paragraph (or the reverse) fails here, as the kernel digest check in
test_bench_host.py fails for a stale profile."""
import json
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _fmt_thousands(x: float, nd: int) -> str:
    whole, _, frac = f"{x:.{nd}f}".partition(".")
    groups = []
    while len(whole) > 3:
        groups.insert(0, whole[-3:])
        whole = whole[:-3]
    groups.insert(0, whole)
    return " ".join(groups) + ("." + frac if frac else "")


def test_design_roofline_quotes_the_committed_profile():
    pmc = json.loads((ROOT / "profiles" / "pmc_summary.json").read_text())["kernels"]["k_render_rgba"]
    design = (ROOT / "DESIGN.md").read_text()
    para = design[design.index("**Roofline numbers.**"):design.index("**Where a slot load's latency comes from**")]
    valu_m = f"{pmc['SQ_INSTS_VALU'] / 1e6:.2f} M"
    assert valu_m in para, f"DESIGN §4 roofline paragraph should quote {valu_m} VALU per launch"
    assert f"`pmc_mean_ms` {pmc['pmc_mean_ms']:.5f} ms" in para or f"`pmc_mean_ms` {pmc['pmc_mean_ms']} ms" in para
    per_wave = _fmt_thousands(pmc["valu_insts_per_wave"], 1)
    assert per_wave in design, f"DESIGN should quote {per_wave} VALU per wave"
    # the fraction over the serialised launch, recomputed from the same two numbers
    frac = pmc["SQ_INSTS_VALU"] / (pmc["pmc_mean_ms"] * 1e-3) / 1e9 / (256 * 4 * 2.4 / 2)
    assert f"{frac:.3f}" in para
