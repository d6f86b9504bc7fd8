"""Regenerate tests/golden/ (run in the build container, where /root/reference exists).

    python tests/make_golden.py

Fixtures (all small, data only):
  rcp_lut_intel.bin   RCPPS of this container's Intel CPU for inputs -(1 + k/2048), k < 2048,
                      captured with the product's och_host_rcp_lut; sha256 must equal the
                      value SURVEY.md §8c records (5d532f85...3f31aba1).
  noise_ref.npz       inputs and outputs of the REFERENCE's och::simplex_n (ORT/och_noise.h),
                      compiled where it lies by oracle/Makefile (oracle/_ref/ref_harness).
  zorder_ref.npz      the reference's och::z_encode_16 (ORT/och_z_order.cpp) on sample inputs.
  trace_d6.npz        a depth-6 terrain pool, ray sets (camera, random, edge cases) and the
                      oracle's hit records under the Intel table (regression vectors; the
                      oracle itself is pinned by known_answers.json).
  known_answers.json  values SURVEY.md reports from the reference run in this container.
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
GOLD = ROOT / "tests" / "golden"

SURVEY_LUT_SHA256 = "5d532f854e820a0f024be14265a0cd345232384ae7cf712c9c75cb4b3f31aba1"


def edge_rays():
    """Origins/directions that exercise the reference's corner cases."""
    o, d = [], []
    mids = [1.5, 1.25, 1.75, 1.125, 1.0625]
    dirs = [(0, 0, -1), (0, 0, 1), (1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0),
            (0.6, 0.8, 0), (0.6, 0, -0.8), (0, 0.6, -0.8), (1e-9, 1e-9, -1), (-1e-9, 1e-9, -1),
            (0.577, 0.577, -0.577), (-0.577, -0.577, -0.577), (1e-30, -1, 1e-30), (-0.0, -0.0, -1),
            (0.0, -0.0, 1.0), (1.0, 1.0, 1.0), (-1e-40, 0.5, -0.5)]
    for x in mids:
        for y in mids:
            for z in (1.5, 1.9, 1.1, 1.2):
                for dd in dirs:
                    o.append((x, y, z))
                    d.append(dd)
    return np.array(o, np.float32), np.array(d, np.float32)


def main():
    import octree_ray_tracing_amd as ort
    from oracle import oracle as O

    GOLD.mkdir(parents=True, exist_ok=True)
    # RCPPS table of this host.
    lut = ort.host_rcp_lut()
    sha = hashlib.sha256(lut.tobytes()).hexdigest()
    if sha != SURVEY_LUT_SHA256:
        raise SystemExit(f"this host's RCPPS table {sha} is not the survey's Intel table")
    (GOLD / "rcp_lut_intel.bin").write_bytes(lut.tobytes())

    if not O.ref_harness_available():
        raise SystemExit("oracle/_ref/ref_harness missing: run make -C oracle with /root/reference present")
    rng = np.random.default_rng(2024)
    # 2-D inputs: the terrain's own (x*4/dim for dim 16..4096) and random.
    xs = []
    for dim in (16, 64, 256, 1024, 4096):
        c = rng.integers(0, dim, (400, 2))
        xs.append((c * 4).astype(np.float32) / np.float32(dim))
    xs.append(rng.uniform(0, 300, (2000, 2)).astype(np.float32))
    n2_in = np.ascontiguousarray(np.concatenate(xs), np.float32)
    n2_out = np.frombuffer(O.ref_run("noise2", n2_in, 0.5), np.float32)
    # 3-D inputs: the tunnels' own (voxel/16) and random.
    v = rng.integers(0, 4096, (3000, 3)).astype(np.float32) * np.float32(1.0 / 16.0)
    n3_in = np.ascontiguousarray(np.concatenate([v, rng.uniform(0, 300, (2000, 3)).astype(np.float32)]), np.float32)
    n3_out = np.frombuffer(O.ref_run("noise3", n3_in, 0.5), np.float32)
    np.savez_compressed(GOLD / "noise_ref.npz", n2_in=n2_in, n2_out=n2_out, n3_in=n3_in, n3_out=n3_out)

    zin = rng.integers(0, 65536, (2000, 3)).astype(np.uint16)
    zout = np.frombuffer(O.ref_run("zenc", zin), np.uint64)
    np.savez_compressed(GOLD / "zorder_ref.npz", zin=zin, zout=zout)

    # Tracing regression vectors on a depth-6 terrain.
    tree = ort.build_terrain(6)
    pool = O.OraclePool(tree.nodes, tree.root, 6, 1)
    rcp = O.Rcp(lut)
    cam = O.raygen(0.3, -0.6, 1.25, 64, 36)
    rd = rng.uniform(-1, 1, (4096, 3)).astype(np.float32)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    ro = rng.uniform(1.01, 1.99, (4096, 3)).astype(np.float32)
    eo, ed = edge_rays()
    out = {"nodes": tree.nodes, "root": np.uint32(tree.root), "depth": np.int32(6)}
    for name, (o, d) in {"cam": (np.array([1.5, 1.5, 1.5], np.float32), cam), "rnd": (ro, rd),
                         "edge": (eo, ed)}.items():
        r = O.trace_batch(pool, rcp, o, d, want_push=True)
        out[f"{name}_o"], out[f"{name}_d"] = o, d
        out[f"{name}_dir"], out[f"{name}_vox"] = r["dir"], r["voxel"]
        out[f"{name}_t"], out[f"{name}_push"] = r["t"].view(np.uint32), r["push"]
    np.savez_compressed(GOLD / "trace_d6.npz", **out)
    print("golden fixtures written to", GOLD)


if __name__ == "__main__":
    main()
