"""Summarise a tools/profile.sh output directory (rocprofv3 CSVs) per kernel.

python tools/pmc_summary.py gpurun_out/prof_<tag> [--update profiles/pmc_summary.json --key d12_1920x1080_n1]

Per kernel family (render = the fused raygen+trace+shade launch, trace =
trace_batch, raygen, unshard): dispatch count and mean duration from the
kernel trace, and the mean of every PMC counter per dispatch.  HBM traffic
per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reads half the bytes of 128-B line requests, so
hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.  These counters sit on
the L2's memory side, so Infinity-Cache hits are included: the figure is
"bytes that left L2", an upper bound on DRAM bytes.
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics
import sys
from collections import defaultdict
from pathlib import Path


def family(name: str) -> str:
    if "bitwise_not" in name.lower() or "BitwiseNot" in name:
        return "marker"
    if "CameraSource" in name and "Bounce" in name:
        return "k_render_bounce"
    if "CameraSource" in name and "FrameSink" in name:
        return "k_render_rgba"          # RGBA8 frames: the planning launch, render_views
    if "CameraSource" in name:
        return "k_render"               # indexed-colour codes: the bench's timed launches
    if "ArraySource" in name and "Bounce" in name:
        return "k_trace_bounce"
    if "ArraySource" in name:
        return "k_trace"
    for k in ("k_raygen", "k_unshard"):
        if k in name:
            return k
    return "other"


WINDOW = False     # --window: only the dispatches between bench.py's two marker kernels


def _did(row) -> int:
    return int(row.get("Dispatch_Id") or row.get("Correlation_Id") or 0)


def read_rows(root: Path, need: str):
    for f in sorted(root.rglob("*.csv")):
        with open(f, newline="") as fh:
            r = csv.DictReader(fh)
            if not (r.fieldnames and need in r.fieldnames):
                continue
            rows = list(r)
        if WINDOW:
            # bench.py brackets its headline window with two one-element
            # bitwise_not kernels (outside the timed region): keep what ran between
            marks = sorted({_did(x) for x in rows if family(x["Kernel_Name"]) == "marker"})
            if len(marks) < 2:
                raise SystemExit(f"{f}: no marker pair (run bench.py from this tree)")
            rows = [x for x in rows if marks[0] < _did(x) < marks[1]]
        yield from rows


def summarise(root: Path) -> dict:
    out: dict = defaultdict(dict)
    dur = defaultdict(list)
    for row in read_rows(root / "trace", "Kernel_Name"):
        if "Start_Timestamp" not in row:
            continue
        fam = family(row["Kernel_Name"])
        dur[fam].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
        # register and LDS sizes are not copied from the trace: its VGPR/LDS fields are
        # allocation granules, not counts; the compiler's -Rpass-analysis=kernel-resource-usage
        # figures are in DESIGN.md
        out[fam].setdefault("kernel_name", row["Kernel_Name"][:160])
    for fam, d in dur.items():
        out[fam]["dispatches"] = len(d)
        out[fam]["mean_ms"] = round(statistics.fmean(d), 5)
        out[fam]["median_ms"] = round(statistics.median(d), 5)
    for sub in sorted(p for p in root.iterdir() if p.is_dir() and p.name.startswith("pmc_")):
        per = defaultdict(lambda: defaultdict(float))     # (family, dispatch) -> counter -> value
        span = {}                                            # (family, dispatch) -> duration, if the CSV has it
        for row in read_rows(sub, "Counter_Name"):
            key = (family(row["Kernel_Name"]), row.get("Dispatch_Id") or row.get("Correlation_Id"))
            per[key][row["Counter_Name"]] += float(row["Counter_Value"])
            if row.get("Start_Timestamp") and row.get("End_Timestamp"):
                span[key] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
        if sub.name == "pmc_grbm" and span:
            # the launch duration under counter collection, which serialises dispatches
            by = defaultdict(list)
            for (fam, _), ms in span.items():
                by[fam].append(ms)
            for fam, v in by.items():
                out[fam]["pmc_mean_ms"] = round(statistics.fmean(v), 5)
        acc = defaultdict(lambda: defaultdict(list))
        for (fam, _), cs in per.items():
            for c, v in cs.items():
                acc[fam][c].append(v)
        for fam, cs in acc.items():
            for c, vs in cs.items():
                out[fam][c] = statistics.fmean(vs)
    for fam, d in out.items():
        if "FETCH_SIZE" in d:
            d["hbm_bytes_per_launch"] = int(2 * d["FETCH_SIZE"] * 1024 + d.get("WRITE_SIZE", 0.0) * 1024)
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d and d["TCC_HIT_sum"] + d["TCC_MISS_sum"] > 0:
            d["l2_hit_rate"] = round(d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"]), 4)
        if "SQ_ACTIVE_INST_VALU" in d and d.get("SQ_BUSY_CYCLES"):
            # SQ_ACTIVE_INST_VALU is per-SIMD quad-cycles summed over the chip; normalise by
            # busy cycles x 4 SIMDs x CUs (256) / 4 (quad) -- reported as a ratio, see DESIGN.md
            d["valu_active_per_busy"] = round(d["SQ_ACTIVE_INST_VALU"] / d["SQ_BUSY_CYCLES"], 4)
        if "SQ_THREAD_CYCLES_VALU" in d and d.get("SQ_ACTIVE_INST_VALU"):
            # active lanes per VALU issue cycle / 64 (both counters from the same SQ, same units)
            d["valu_lane_utilization"] = round(d["SQ_THREAD_CYCLES_VALU"] / (64.0 * d["SQ_ACTIVE_INST_VALU"]), 4)
        if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d and d["SQ_WAVES"]:
            d["valu_insts_per_wave"] = round(d["SQ_INSTS_VALU"] / d["SQ_WAVES"], 1)
        # GRBM_GUI_ACTIVE is counted under counter collection (dispatches serialised):
        # over that pass's own launch duration when the CSV carries timestamps
        dur = d.get("pmc_mean_ms") or d.get("mean_ms")
        if "GRBM_GUI_ACTIVE" in d and dur:
            d["effective_clock_ghz"] = round(d["GRBM_GUI_ACTIVE"] / 8 / (dur * 1e-3) / 1e9, 3)
            d["effective_clock_basis"] = "pmc_mean_ms" if d.get("pmc_mean_ms") else "mean_ms (kernel-trace run)"
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--update", default=None, help="profiles/pmc_summary.json to merge into")
    ap.add_argument("--key", default=None, help="config key, e.g. d12_1920x1080_n1")
    ap.add_argument("--window", action="store_true",
                    help="only the bench's headline window (the dispatches between its marker kernels)")
    a = ap.parse_args()
    global WINDOW
    WINDOW = a.window
    s = summarise(Path(a.root))
    print(json.dumps(s, indent=1, sort_keys=True))
    if a.update and a.key:
        # One configuration per file, tied to the kernel sources it was taken
        # of: bench.py uses it only when both match (bench.load_pmc).
        sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
        from bench import kernel_source_digest
        p = Path(a.update)
        p.write_text(json.dumps({"config": a.key, "kernel_source_sha": kernel_source_digest(),
                                 "dispatches": "the bench's headline window only" if a.window else "every dispatch",
                                 "kernels": s}, indent=1, sort_keys=True))
        print(f"wrote {p} [{a.key}]", file=sys.stderr)


if __name__ == "__main__":
    main()
