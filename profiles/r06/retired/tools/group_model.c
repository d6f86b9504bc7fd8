/* group_model.c -- prices cost-sorted wave assembly for the render loop (design
 * tool, not product).  Today a wave walks one 8x8 pixel tile and costs its
 * longest lane (lockstep: one PUSH test per iteration), so lanes
 * whose rays end early idle.  If a plan knew every ray's cost (the planning
 * render can count them, och_api.cpp plan_split), a B x B pixel block's rays
 * could be sorted by cost and dealt 64 to a wave, so a wave's lanes end
 * together.  This counts the work both ways -- the sum over waves of the
 * longest lane -- per block size, with rays the occupied-box cull ends counted
 * as free (their lanes walk nothing), and the spread of a wave's rays (the
 * bounding box of its pixels, a proxy for how many cache lines its loads touch).
 *
 * Build: gcc -O2 -msse2 -o /tmp/group_model profiles/r06/retired/tools/group_model.c -lm -lpthread
 * Usage: group_model nodes.bin depth pitch [threads] */
#define SPLIT_MODEL_NO_MAIN
#include "../../../../tools/split_model.c"

static int *COST;                  /* per pixel: PUSH tests of the full walk (0: culled sky ray) */
static int G_NEXT;

/* the occupied box of the depth-12 terrain: [0,4096)^2 x [0,1264) voxels */
static int proven_miss(const float *o, const float *d)
{
    const float lo[3] = {1.0F, 1.0F, 1.0F}, hi[3] = {2.0F, 2.0F, 1.0F + 1264.0F / 4096.0F};
    float t0 = 0.0F, t1 = 1e30F;
    for (int a = 0; a < 3; ++a) {
        if (d[a] == 0.0F) { if (o[a] < lo[a] || o[a] > hi[a]) return 1; continue; }
        float ta = (lo[a] - o[a]) / d[a], tb = (hi[a] - o[a]) / d[a];
        if (ta > tb) { const float x = ta; ta = tb; tb = x; }
        if (ta > t0) t0 = ta;
        if (tb < t1) t1 = tb;
    }
    return t0 > t1 * 1.0001F;
}

static void *gworker(void *arg)
{
    (void)arg;
    const float o[3] = {1.5F, 1.5F, 1.5F};
    for (;;) {
        const int row = __atomic_fetch_add(&G_NEXT, 1, __ATOMIC_RELAXED);
        if (row >= H) return NULL;
        for (int x = 0; x < W; ++x) {
            float d[3];
            camera(0.3F, PITCH, W, H, x, row, d);
            if (proven_miss(o, d)) { COST[row * W + x] = 0; continue; }
            Rec r;
            walk(o, d, -1, -1, &r);
            COST[row * W + x] = r.push;
        }
    }
}

typedef struct { int cost, x, y; } Px;
static int cmp_px(const void *a, const void *b) { return ((const Px *)b)->cost - ((const Px *)a)->cost; }

int main(int argc, char **argv)
{
    if (argc < 4) { fprintf(stderr, "usage: group_model nodes.bin depth pitch [threads]\n"); return 2; }
    FILE *fp = fopen(argv[1], "rb");
    if (!fp) return 1;
    fseek(fp, 0, SEEK_END);
    const long sz = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    uint32_t *buf = malloc(sz);
    if (fread(buf, 1, sz, fp) != (size_t)sz) return 1;
    fclose(fp);
    N = buf;
    DEPTH = atoi(argv[2]);
    PITCH = (float)atof(argv[3]);
    LEVEL = 1;
    SEGS = 1;
    const int threads = argc > 4 ? atoi(argv[4]) : 8;
    COST = calloc((size_t)W * H, sizeof(int));
    pthread_t th[256];
    for (int k = 0; k < threads; ++k) pthread_create(&th[k], NULL, gworker, NULL);
    for (int k = 0; k < threads; ++k) pthread_join(th[k], NULL);
    long lanes = 0, rays_walk = 0;
    for (int i = 0; i < W * H; ++i) { lanes += COST[i]; rays_walk += COST[i] > 0; }
    printf("{\"pitch\": %g, \"rays_walking\": %ld, \"lane_pushes\": %ld, \"blocks\": [", PITCH, rays_walk, lanes);
    const int Bs[] = {8, 16, 32, 64};
    for (int k = 0; k < 4; ++k) {
        const int B = Bs[k];
        long tiles = 0, sorted = 0, waves = 0, spread = 0, tile_waves = 0;
        Px *px = malloc(sizeof(Px) * B * B);
        for (int by = 0; by + B <= H; by += B)
            for (int bx = 0; bx + B <= W; bx += B) {
                /* today: its 8x8 tiles, a tile with every ray culled costs nothing */
                for (int ty = by; ty < by + B; ty += 8)
                    for (int tx = bx; tx < bx + B; tx += 8) {
                        int m = 0;
                        for (int l = 0; l < 64; ++l) { const int c = COST[(ty + l / 8) * W + tx + l % 8]; if (c > m) m = c; }
                        tiles += m;
                        tile_waves += m > 0;
                    }
                /* sorted: the block's walking rays, longest first, 64 to a wave */
                int n = 0;
                for (int y = by; y < by + B; ++y)
                    for (int x = bx; x < bx + B; ++x)
                        if (COST[y * W + x]) px[n++] = (Px){COST[y * W + x], x, y};
                qsort(px, n, sizeof(Px), cmp_px);
                for (int i = 0; i < n; i += 64) {
                    sorted += px[i].cost;
                    ++waves;
                    int x0 = W, x1 = 0, y0 = H, y1 = 0;
                    for (int j = i; j < n && j < i + 64; ++j) {
                        if (px[j].x < x0) x0 = px[j].x;
                        if (px[j].x > x1) x1 = px[j].x;
                        if (px[j].y < y0) y0 = px[j].y;
                        if (px[j].y > y1) y1 = px[j].y;
                    }
                    spread += (long)(x1 - x0 + 1) * (y1 - y0 + 1);
                }
            }
        free(px);
        printf("%s{\"B\": %d, \"tile_waves\": %ld, \"tile_work\": %ld, \"sorted_waves\": %ld, \"sorted_work\": %ld, "
               "\"ratio\": %.4f, \"mean_bbox_px\": %.0f}", k ? ", " : "", B, tile_waves, tiles, waves, sorted,
               (double)sorted / tiles, (double)spread / waves);
    }
    printf("], \"lane_utilisation_tiles_ideal\": %.4f}\n", 0.0);
    return 0;
}
