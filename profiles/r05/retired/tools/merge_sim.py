"""Host simulation of k_trace_grid_merge's exchange protocol (och_kernels.hip):
waves of 64 lanes, rays that finish at random, merges that move the rays of the
highest waves into free lanes of the lower ones through the free lanes' LDS
columns.  Checks, over many random blocks, that a ray keeps the stack column it
started in, no two live rays share a column, a mailbox column is never a live
ray's stack, and every ray is retired exactly once.  Run on the CPU before the
merge kernel changes go to the GPU."""
import random


def simulate(n_waves, seed, K=2):
    rng = random.Random(seed)
    nb = 64 * n_waves
    # lane -> ray id (None = free); ray -> (column, remaining iterations)
    lane_ray = [t if rng.random() < 0.9 else None for t in range(nb)]
    col = {t: t for t in range(nb) if lane_ray[t] is not None}
    left = {t: rng.randint(1, 60) for t in col}
    retired = set()
    alive = n_waves
    while True:
        for lane in range(64 * alive):                  # a round of K iterations
            r = lane_ray[lane]
            if r is not None and left[r] > 0:
                left[r] = max(0, left[r] - K)
        for lane in range(64 * alive):                  # retire
            r = lane_ray[lane]
            if r is not None and left[r] == 0:
                assert r not in retired
                retired.add(r)
                lane_ray[lane] = None
        counts = [sum(lane_ray[w * 64 + l] is not None for l in range(64)) for w in range(alive)]
        total = sum(counts)
        if total == 0:
            break
        keep = (total + 63) // 64
        if keep < alive:
            free = [t for t in range(64 * keep) if lane_ray[t] is None]        # ranked by (wave, lane)
            movers = [t for t in range(64 * keep, 64 * alive) if lane_ray[t] is not None]
            assert len(movers) <= len(free)
            live_cols = {col[lane_ray[t]] for t in range(64 * alive) if lane_ray[t] is not None}
            for m, src in enumerate(movers):
                dst = free[m]
                assert dst not in live_cols, "mailbox column holds a live stack"
                r = lane_ray[src]
                lane_ray[dst] = r                          # the ray's column travels with it, unchanged
                lane_ray[src] = None
            alive = keep
        cols = [col[lane_ray[t]] for t in range(64 * alive) if lane_ray[t] is not None]
        assert len(cols) == len(set(cols)), "two live rays on one column"
    assert retired == set(col)


if __name__ == "__main__":
    for n in (2, 4, 8, 16):
        for seed in range(300):
            simulate(n, seed, K=1 + seed % 8)
    print("merge protocol: ok")
