"""Schedule sweep on the GPU: time trace_batch_dev and render_dev per launch
schedule, check each variant's output bit-for-bit against the grid schedule,
and summarise per-wave residency (stamps) for selected variants.

python tools/sweep.py --depth 12 [--quick]
"""
from __future__ import annotations

import argparse
import itertools
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def residency(stamps: np.ndarray, n_waves: int):
    s = stamps[:n_waves]
    s = s[s[:, 1] > 0]
    t0, t1 = s[:, 0].min(), s[:, 1].max()
    span = (t1 - t0) / 100.0                                  # us (100 MHz)
    life = (s[:, 1] - s[:, 0]) / 100.0
    xcc = (s[:, 2] >> 32) & 0xF
    hw = s[:, 2] & 0xFFFFFFFF
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    sh = (hw >> 12) & 0x1
    key = xcc * 1000 + se * 100 + sh * 16 + cu
    n_cu = len(np.unique(key))
    return {"span_us": round(float(span), 1), "waves": int(len(s)), "cus_seen": int(n_cu),
            "wave_life_us_mean": round(float(life.mean()), 2), "wave_life_us_p99": round(float(np.percentile(life, 99)), 2),
            "mean_resident_waves_per_cu": round(float(life.sum() / span / max(n_cu, 1)), 2),
            "tail_us_last_10pct_waves": round(float((t1 - np.percentile(s[:, 1], 90)) / 100.0), 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--out", default="gpurun_out/sweep.json")
    a = ap.parse_args()

    import torch
    import octree_ray_tracing_amd as ort

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    tree = ort.build_terrain(a.depth, use_gpu=True)
    print(f"depth {a.depth}: {tree.n_nodes} nodes, built in {tree.build_seconds:.1f}s", flush=True)
    pool = ort.HOctree(tree.nodes, tree.root, a.depth, device=0)
    pool.set_palette(ort.VoxelData().get_colours())
    stream = torch.cuda.current_stream()
    pool.set_stream(stream)
    W, H = a.width, a.height
    n = W * H
    o = torch.tensor([1.5, 1.5, 1.5], dtype=torch.float32, device=dev)
    dirs = {p: torch.empty(n * 3, dtype=torch.float32, device=dev) for p in (0.0, -0.6)}
    cams = {p: ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, W, H) for p in (0.0, -0.6)}
    for p in dirs:
        pool.raygen_dev(cams[p], dirs[p])
    hd = torch.empty(n, dtype=torch.int32, device=dev)
    hv = torch.empty(n, dtype=torch.int32, device=dev)
    ht = torch.empty(n, dtype=torch.int32, device=dev)
    frame = torch.empty(n, dtype=torch.int32, device=dev)
    stamps = torch.zeros((1 << 17) * 4, dtype=torch.int64, device=dev)

    def timed(fn):
        for _ in range(2):
            fn()
        evs = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            evs.append((e0, e1))
        torch.cuda.synchronize()
        return float(np.median([x.elapsed_time(y) for x, y in evs]))

    # reference outputs (grid schedule)
    ref = {}
    pool.set_option("schedule", 0)
    for p in dirs:
        pool.trace_batch_dev(o, dirs[p], hd, hv, ht)
        pool.render_dev(cams[p], frame)
        torch.cuda.synchronize()
        ref[p] = (hd.clone(), hv.clone(), ht.clone(), frame.clone())

    variants = [("grid", 0, b, 0, 0) for b in (64, 128, 256, 512)] + [("grid-raw", 0, b, 0, 0) for b in (64, 256)]
    wpc = (16, 32) if a.quick else (8, 16, 24, 32)
    rf = (8, 32) if a.quick else (1, 8, 16, 32, 48, 64)
    for b, w, r in itertools.product((64, 256), wpc, rf):
        variants.append(("persistent", 1, b, w, r))
    results = []
    for name, sched, block, w, r in variants:
        pool.set_option("schedule", sched)
        pool.set_option("block", block)
        pool.set_option("layout", 0 if name == "grid-raw" else 1)
        if sched:
            pool.set_option("waves_per_cu", w)
            pool.set_option("refill", r)
        row = {"schedule": name, "block": block, "waves_per_cu": w, "refill": r}
        ok = True
        for p in dirs:
            tt = timed(lambda: pool.trace_batch_dev(o, dirs[p], hd, hv, ht))
            tr = timed(lambda: pool.render_dev(cams[p], frame))
            ok &= bool(torch.equal(hd, ref[p][0]) and torch.equal(hv, ref[p][1]) and torch.equal(ht, ref[p][2])
                       and torch.equal(frame, ref[p][3]))
            row[f"trace_ms_p{p}"] = round(tt, 4)
            row[f"render_ms_p{p}"] = round(tr, 4)
        both = torch.empty(2 * n, dtype=torch.int32, device=dev)
        tv = timed(lambda: pool.render_views_dev([cams[0.0], cams[-0.6]], both))
        ok &= bool(torch.equal(both[:n], ref[0.0][3]) and torch.equal(both[n:], ref[-0.6][3]))
        row["render2_ms"] = round(tv, 4)
        row["render2_mrays_s"] = round(2 * n / tv / 1e3, 1)
        row["trace_mrays_s"] = round(2 * n / (row["trace_ms_p0.0"] + row["trace_ms_p-0.6"]) / 1e3, 1)
        row["render_mrays_s"] = round(2 * n / (row["render_ms_p0.0"] + row["render_ms_p-0.6"]) / 1e3, 1)
        row["bit_exact_vs_grid"] = ok
        results.append(row)
        print(json.dumps(row), flush=True)
    # residency of the default grid and of the best persistent variant
    best = max((r for r in results if r["schedule"] == "persistent"), key=lambda r: r["render_mrays_s"])
    res = {}
    pool.set_option("layout", 1)
    for tag, cfg in (("grid256", (0, 256, 0, 0)), ("best_persistent", (1, best["block"], best["waves_per_cu"], best["refill"]))):
        pool.set_option("schedule", cfg[0])
        pool.set_option("block", cfg[1])
        if cfg[0]:
            pool.set_option("waves_per_cu", cfg[2])
            pool.set_option("refill", cfg[3])
        stamps.zero_()
        pool.set_stamp_buffer(stamps, 1 << 17)
        pool.render_dev(cams[-0.6], frame)
        torch.cuda.synchronize()
        pool.set_stamp_buffer(None, 0)
        res[tag] = residency(stamps.cpu().numpy().reshape(-1, 4).astype(np.uint64), 1 << 17)
        print(tag, json.dumps(res[tag]), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps({"depth": a.depth, "W": W, "H": H, "results": results, "residency": res,
                                       "best_persistent": best}, indent=1))
    pool.close()


if __name__ == "__main__":
    main()
