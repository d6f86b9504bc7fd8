"""Summarise the bench's headline window from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/win -o run -- python bench.py ...
    python tools/window_trace.py gpurun_out/win --steps 20 --out profiles/window_summary.json \
        --csv profiles/r03/window_trace.csv

bench.py brackets its headline window (the `steps` timed steps) with two
one-element bitwise_not kernels, launched outside the timed region.  This
tool takes the kernels that run between them -- the render launches
(k_trace_grid<CameraSource,CodeSink>) and the shade + unshard launches of the
frames in flight on their streams -- and reports, per step:

  ms_per_step_trace      first start to last end of the window's kernels / steps
  busy_union_ms_per_step the union of the kernels' [start, end) intervals / steps:
                         time the GPU had at least one of them running
  kernel_ms_sum_per_step the sum of their durations / steps (> the union when
                         launches overlap)
  mean_concurrency       sum / union: how many of them ran at once on average
  concurrency_hist_ms    per step, the time with exactly k kernels running

With frames in flight a render launch lasts longer than a step; the union
and the concurrency show how the launches of three frames overlap to give
the step time the bench line reports.
"""
from __future__ import annotations

import argparse
import csv
import hashlib
import json
import statistics
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def kernel_source_digest() -> str:
    h = hashlib.sha256()
    for f in ("och_kernels.hip", "och_internal.h", "Makefile"):
        h.update((ROOT / "octree_ray_tracing_amd" / "csrc" / f).read_bytes())
    return h.hexdigest()[:16]


def family(name: str) -> str:
    if "bitwise_not" in name.lower() or "BitwiseNot" in name:
        return "marker"
    if "CameraSource" in name and "Bounce" in name:
        return "k_render_bounce"
    if "CameraSource" in name:
        return "k_render"
    for k in ("k_shade_unshard4", "k_shade_unshard", "k_unshard", "k_raygen"):
        if k in name:
            return k
    if "nccl" in name.lower() or "rccl" in name.lower():
        return "rccl"
    return "other"


def read_trace(root: Path):
    rows = []
    for f in sorted(root.rglob("*kernel_trace.csv")):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                rows.append({"name": r["Kernel_Name"], "fam": family(r["Kernel_Name"]),
                             "start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"]),
                             "queue": r.get("Queue_Id", ""), "stream": r.get("Stream_Id", ""),
                             "dispatch": r.get("Dispatch_Id", "")})
    rows.sort(key=lambda r: r["start"])
    return rows


def window(rows):
    marks = [r for r in rows if r["fam"] == "marker"]
    if len(marks) < 2:
        raise SystemExit("no marker pair in the trace: run bench.py from this tree")
    m0, m1 = marks[0], marks[1]
    return [r for r in rows if r["fam"] != "marker" and r["start"] >= m0["end"] and r["end"] <= m1["start"]]


def summarise(win, steps: int) -> dict:
    # the step kernels; "other" is runtime copies (the window's elapsed-time
    # tensor goes to the device after the host has stopped its clock)
    steps_k = [r for r in win if r["fam"] != "other"] or win
    t0 = min(r["start"] for r in steps_k)
    t1 = max(r["end"] for r in steps_k)
    ev = sorted([(r["start"], 1) for r in steps_k] + [(r["end"], -1) for r in steps_k])
    hist = defaultdict(int)
    busy, k, last = 0, 0, ev[0][0]
    for t, d in ev:
        if k > 0:
            busy += t - last
        hist[k] += t - last
        k += d
        last = t
    total = sum(r["end"] - r["start"] for r in steps_k)
    fams = defaultdict(list)
    for r in win:
        fams[r["fam"]].append((r["end"] - r["start"]) / 1e6)
    return {
        "steps": steps,
        "kernels": {f: {"launches": len(v), "mean_ms": round(statistics.fmean(v), 5),
                        "sum_ms_per_step": round(sum(v) / steps, 5)} for f, v in sorted(fams.items())},
        "ms_per_step_trace": round((t1 - t0) / 1e6 / steps, 5),
        "busy_union_ms_per_step": round(busy / 1e6 / steps, 5),
        "kernel_ms_sum_per_step": round(total / 1e6 / steps, 5),
        "mean_concurrency": round(total / busy, 3),
        "concurrency_hist_ms": {str(c): round(v / 1e6 / steps, 5) for c, v in sorted(hist.items()) if c > 0},
        "render_mean_ms": round(statistics.fmean(fams["k_render"]), 5) if fams.get("k_render") else None,
        "streams": sorted({r["stream"] or r["queue"] for r in win}),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir", help="rocprofv3 output directory, or a window CSV of an earlier run")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--config", default="d12_1920x1080_n1")
    ap.add_argument("--bench-json", help="the bench line printed by the profiled run (its ms_per_step)")
    ap.add_argument("--out")
    ap.add_argument("--csv", help="write the window's kernel rows here")
    a = ap.parse_args()
    if a.trace_dir.endswith(".csv"):          # a window CSV written by --csv (times in us)
        with open(a.trace_dir, newline="") as fh:
            win = [{"name": r["kernel"], "fam": r["kernel"], "stream": r["stream"], "queue": r["queue"],
                    "start": int(float(r["start_us"]) * 1e3), "end": int(float(r["end_us"]) * 1e3)}
                   for r in csv.DictReader(fh)]
    else:
        win = window(read_trace(Path(a.trace_dir)))
    d = {"config": a.config, "kernel_source_sha": kernel_source_digest(), **summarise(win, a.steps)}
    if a.bench_json:
        line = json.loads(Path(a.bench_json).read_text().strip().splitlines()[-1])
        d["bench_ms_per_step"] = line.get("ms_per_step")
        d["bench_value"] = line.get("value")
    if a.csv:
        t0 = min(r["start"] for r in win)
        with open(a.csv, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["kernel", "stream", "queue", "start_us", "end_us", "dur_us"])
            for r in win:
                w.writerow([r["fam"], r["stream"], r["queue"], round((r["start"] - t0) / 1e3, 3),
                            round((r["end"] - t0) / 1e3, 3), round((r["end"] - r["start"]) / 1e3, 3)])
    text = json.dumps(d, indent=1)
    if a.out:
        Path(a.out).write_text(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
