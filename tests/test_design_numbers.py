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


def _bench_line(path: Path) -> dict:
    """The JSON line of a committed bench.py output (the last line that parses)."""
    for line in reversed(path.read_text().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError(f"no JSON line in {path}")


def test_readme_headline_quotes_the_committed_runs():
    """README's headline ranges (20-step window, sustained, the lone launch with
    the headline's split and, from the split arm, without it) are the min-max over the bench runs that
    profiles/r06/headline.json lists -- committed bench.py outputs."""
    spec = json.loads((ROOT / "profiles" / "r06" / "headline.json").read_text())
    lines = [_bench_line(ROOT / f) for f in spec["n1_runs"]]
    readme = (ROOT / "README.md").read_text()
    win = [l["value"] / 1e3 for l in lines]
    sus = [l["sustained"]["value"] / 1e3 for l in lines]
    assert f"{min(sus):.1f}–{max(sus):.1f} G rays/s sustained" in readme
    assert f"{min(win):.1f}–{max(win):.1f} G over the driver's 20-step" in readme
    lone = [l["roofline"]["kernel_ms_serial"] for l in lines]          # the headline's launch
    off = []
    for l in lines:                 # the split arm's launches without the split, one per interleaved round
        off += l["split"]["off"]["kernel_ms_serial"]
    assert all(l["config"]["heavy_tile_split"] != "off" for l in lines)
    assert f"one two-view frame in {min(lone):.3f}–{max(lone):.3f} ms" in readme
    assert off and f"{min(off):.3f}–{max(off):.3f} ms without it" in readme


def test_n8_projection_quotes_the_committed_proxy():
    """The N = 8 numbers README and DESIGN §4d quote (the proxy's slowest shard
    over 20 steps, without and with the split) are the min-max over the
    committed proxy runs profiles/r06/headline.json lists."""
    spec = json.loads((ROOT / "profiles" / "r06" / "headline.json").read_text())
    readme = (ROOT / "README.md").read_text()
    design = (ROOT / "DESIGN.md").read_text()

    def slowest(files):
        out = []
        for f in files:
            rows = json.loads((ROOT / f).read_text())
            out.append(max(r["ms_per_step_20"] for r in rows if "shard" in r))
        return min(out), max(out)
    b, s = slowest(spec["n8_base"]), slowest(spec["n8_split"])
    quote = f"{b[0]:.4f}–{b[1]:.4f} → {s[0]:.4f}–{s[1]:.4f} ms"
    assert quote in readme, quote
    assert quote in design, quote
