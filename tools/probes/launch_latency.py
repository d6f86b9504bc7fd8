"""Host-to-GPU latency of the first launch after a synchronize (run under
rocprofv3 --kernel-trace; tools/probes/launch_latency_report.py lines the host
clock readings up with the trace).  Variants: the pool's render launch timed by
its dispatch (OCH_OPT_TIMING 1), untimed (0), a torch kernel; after an idle
spin of 0 / 0.1 / 1 / 10 ms; on the current stream and on a second stream."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def spin(us):
    t = time.monotonic_ns() + int(us * 1e3)
    while time.monotonic_ns() < t:
        pass


def main():
    import numpy as np
    import torch
    import octree_ray_tracing_amd as ort
    torch.cuda.set_device(0)
    z = np.load("/tmp/och_tree_d12.npz") if Path("/tmp/och_tree_d12.npz").exists() else None
    if z is not None and int(z["depth"]) == 12:
        nodes, root = z["nodes"], int(z["root"])
    else:
        t = ort.build_terrain(12, use_gpu=True)
        nodes, root = t.nodes, t.root
        np.savez("/tmp/och_tree_d12.npz", nodes=nodes, root=root, depth=12)
    pool = ort.HOctree(nodes, root, 12, device=0)
    pool.set_palette(ort.VoxelData().get_colours())
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    cams = [ort.camera((1.5, 1.5, 1.5), 0.3, p, 1.25, 1920, 1080) for p in (0.0, -0.6)]
    frames = torch.zeros((2, 1080, 1920), dtype=torch.int32, device="cuda")
    x = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = []
    for rep in range(3):
        for what in ("render_t1", "render_t0", "torch"):
            for idle_us in (0, 100, 1000, 10000):
                for sname, s in (("s0", s0), ("s1", s1)):
                    pool.set_stream(s)
                    pool.set_option("timing", 1 if what == "render_t1" else 0)
                    torch.cuda.synchronize()
                    spin(idle_us)
                    with torch.cuda.stream(s):
                        h0 = time.monotonic_ns()
                        if what == "torch":
                            torch.bitwise_not(x, out=x)
                        else:
                            pool.render_views_dev(cams, frames)
                        h1 = time.monotonic_ns()
                    torch.cuda.synchronize()
                    out.append({"what": what, "idle_us": idle_us, "stream": sname, "h0": h0, "h1": h1})
    pool.set_stream(s0)
    print(json.dumps(out))
    pool.close()


if __name__ == "__main__":
    main()
