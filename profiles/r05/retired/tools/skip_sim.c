/* skip_sim.c -- prices an exact per-node skip before it is built (design tool,
 * not product, not a checker).
 *
 * The occupied-box cull ends a ray that never enters the
 * bounding box of ALL voxels.  The same argument holds for any node: every
 * cell the walk enters satisfies max_a t_a(hi_a) <= t_min <= min_a t_a(lo_a)
 * in the walk's own arithmetic, so a ray that fails that test for the
 * bounding box of the voxels under child C never enters a cell of C that
 * holds a voxel -- it cannot hit inside C.  Treating C as empty at its PUSH
 * then leaves the walk in the state the excursion through C would end in
 * (the POP-chain argument, DESIGN.md §4: the exit of C is the same plane at
 * the same t), so records are unchanged.  This walks the bench's camera
 * frames over the packed depth-12 DAG twice -- the reference walk and the
 * walk with the skip -- checks every record is identical, and reports the
 * PUSHes (and the costliest 8x8 tiles, which set a frame's latency), and the
 * descents (PUSHes that find their child: one dependent load each) with each
 * tile's lockstep maximum -- what a wave costs.
 *
 * Input: packed nodes (och_pool_pack, n x 8 u32, row 0 padding), node levels
 * (u8 per row) and per-node boxes (6 x u8 per row: lo x,y,z then hi x,y,z in
 * 1/Q of the node's own cell, world orientation), written by
 * tools/skip_model.py, which builds them and runs this.
 * Build: gcc -O2 -msse2 -o /tmp/skip_sim tools/skip_sim.c -lm -lpthread
 * Usage: skip_sim packed.bin levels.bin boxes.bin depth root_id Q pitch [min_level] */
#include <immintrin.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static const uint32_t *N;
static const uint8_t *LV, *BX;
static int DEPTH, Q, MINLV;
static uint32_t ROOT;

typedef struct { int dir; uint32_t voxel; uint32_t t; int push; int desc; int skips; } Rec;

/* ORT/och_h_octree.h:292-447 over the packed pool (child id in the low 24 bits),
 * host RCPPS; skip = 1: a present child whose voxel box the ray provably
 * misses is treated as empty. */
static Rec trace(const float *o, const float *d, int skip)
{
    float c[3], b[3];
    uint32_t p[3];
    int inv = 0, idx = 0, ok = 1;
    for (int a = 0; a < 3; ++a) {
        const int pos = 0.0F < d[a];
        inv |= pos << a;
        const float dn = u2f(f2u(d[a]) | 0x80000000u);
        const float refl = fabsf((pos ? 3.0F : 0.0F) - o[a]);
        c[a] = _mm_cvtss_f32(_mm_rcp_ss(_mm_set_ss(dn)));
        b[a] = u2f(f2u(c[a] * refl) ^ 0x80000000u);
        p[a] = f2u(refl) & 0x3FC00000u;
        if (u2f(p[a]) == 1.5F) idx |= 1 << a;
        const uint32_t e = (f2u(c[a]) >> 23) & 0xFFu;
        ok &= e - 1u < 251u;
        ok &= o[a] > 1.0F && o[a] < 2.0F;
    }
    uint32_t dim = 1u << 22, stack[32], node = ROOT;
    int sp = 0, level = 1, axis = 8;
    float tmin = 0.0F;
    Rec r = {0, 0, 0, 0, 0, 0};
    enum { PUSH, STEP, POP } st = PUSH;
    for (;;) {
        if (st == PUSH) {
            ++r.push;
            const uint32_t w = N[(size_t)node * 8 + ((idx ^ inv) & 7)];
            uint32_t child = level == DEPTH ? w : (w & 0xFFFFFFu);
            if (child && skip && ok && level < DEPTH && level + 1 >= MINLV) {
                /* child cell in the reflected frame: [p_a, p_a + size), size = dim ulps */
                const uint8_t *bx = BX + (size_t)child * 6;
                float enter = -INFINITY, leave = INFINITY;
                for (int a = 0; a < 3; ++a) {
                    int lo = bx[a], hi = bx[3 + a];
                    if ((inv >> a) & 1) { const int t = lo; lo = Q - hi; hi = Q - t; }   /* reflected */
                    const uint32_t step = dim / (uint32_t)Q;
                    const float plo = u2f(p[a] + (uint32_t)lo * step), phi = u2f(p[a] + (uint32_t)hi * step);
                    const float tlo = fmaf(plo, c[a], b[a]), thi = fmaf(phi, c[a], b[a]);
                    enter = fmaxf(enter, thi);
                    leave = fminf(leave, tlo);
                }
                if (enter > leave || leave < tmin) { child = 0; ++r.skips; }
            }
            if (!child) { st = STEP; continue; }
            ++r.desc;                      /* a descent or the HIT: one dependent load */
            if (level++ == DEPTH) {
                r.voxel = child;
                r.dir = (axis >> 1) + 3 * ((inv & axis) == 0);
                r.t = f2u(tmin);
                return r;
            }
            stack[sp++] = node;
            node = child;
            dim >>= 1;
            idx = 0;
            for (int a = 0; a < 3; ++a) {
                const float tm = fmaf(u2f(p[a] | dim), c[a], b[a]);
                if (tm >= tmin) { idx |= 1 << a; p[a] |= dim; }
            }
        } else if (st == STEP) {
            uint32_t t[3];
            for (int a = 0; a < 3; ++a) t[a] = f2u(fmaf(u2f(p[a]), c[a], b[a]));
            int a;
            if (t[0] <= t[1] && t[0] <= t[2]) a = 0;
            else if (t[1] < t[0] && t[1] <= t[2]) a = 1;
            else a = 2;
            axis = 1 << a;
            tmin = u2f(t[a]);
            if (!(idx & axis)) { st = POP; continue; }
            p[a] &= ~dim;
            idx ^= axis;
            st = PUSH;
        } else {
            if (--level == 0) { r.dir = 6; r.voxel = 0; r.t = 0x7F800000u; return r; }
            node = stack[--sp];
            for (int a = 0; a < 3; ++a) p[a] &= ~dim;
            dim <<= 1;
            idx = 0;
            for (int a = 0; a < 3; ++a) if ((p[a] & dim) == dim) idx |= 1 << a;
            st = STEP;
        }
    }
}

static void camera(float yaw, float pitch, int W, int H, int col, int row, float *d)
{
    const float aspect = (float)W / (float)H, fov = 1.25F;
    const float f = 1.0F / tanf(fov / 2);
    const float sb = sinf(yaw), cb = cosf(yaw), sc = sinf(pitch), cc = cosf(pitch);
    const float m[9] = {cb, sb * sc, sb * cc, 0, cc, -sc, -sb, cb * sc, cb * cc};
    const float u = aspect * ((2.0F / W) * col - 1.0F), v = (2.0F / H) * row - 1.0F;
    const float ru = u * m[0] + v * m[1] + f * m[2];
    const float rv = u * m[3] + v * m[4] + f * m[5];
    const float rw = u * m[6] + v * m[7] + f * m[8];
    const float rm = 1.0F / sqrtf(ru * ru + rv * rv + rw * rw);
    d[0] = rw * rm; d[1] = ru * rm; d[2] = -rv * rm;
}

static float PITCH;
enum { W = 1920, H = 1080, TX = W / 8, TY = H / 8, NT = 16 };
static long tile_push[2][TX * TY];
static long tile_desc_max[3][TX * TY], tile_push_max[2][TX * TY], desc_sum[3][NT];
static long mism[NT], hits[NT];

static uint64_t lcg(uint64_t *s) { *s = *s * 6364136223846793005ull + 1442695040888963407ull; return *s >> 33; }

static void *worker(void *arg)
{
    const int id = (int)(intptr_t)arg;
    float o[3] = {1.5F, 1.5F, 1.5F};
    uint64_t seed = 12345u + (uint64_t)id * 7919u;
    for (int t = id; t < TX * TY; t += NT) {
        const int tx = t % TX, ty = t / TX;
        for (int l = 0; l < 64; ++l) {
            float d[3];
            if (PITCH > 9.0F) {            /* random rays: origins in (1.01, 1.99)^3, directions in a cube */
                for (int a = 0; a < 3; ++a) {
                    o[a] = 1.01F + 0.98F * (float)(lcg(&seed) % 1000000u) / 1e6F;
                    d[a] = -1.0F + 2.0F * (float)(lcg(&seed) % 1000000u) / 1e6F;
                }
            } else
                camera(0.3F, PITCH, W, H, tx * 8 + l % 8, ty * 8 + l / 8, d);
            const Rec a = trace(o, d, 0), b = trace(o, d, 1);
            tile_push[0][t] += a.push;
            tile_push[1][t] += b.push;
            /* the lockstep cost of the tile's wave: its longest lane */
            if (a.desc > tile_desc_max[0][t]) tile_desc_max[0][t] = a.desc;
            if (b.desc > tile_desc_max[1][t]) tile_desc_max[1][t] = b.desc;
            if (a.push > tile_push_max[0][t]) tile_push_max[0][t] = a.push;
            if (b.push > tile_push_max[1][t]) tile_push_max[1][t] = b.push;
            desc_sum[0][id] += a.desc;
            desc_sum[1][id] += b.desc;
            /* the GPU's skip tests a child's box after descending into it: each
               skipped child still costs its descent */
            if (b.desc + b.skips > tile_desc_max[2][t]) tile_desc_max[2][t] = b.desc + b.skips;
            desc_sum[2][id] += b.desc + b.skips;
            mism[id] += a.dir != b.dir || a.voxel != b.voxel || a.t != b.t;
            hits[id] += a.dir < 6;
        }
    }
    return NULL;
}

static int cmp_desc(const void *x, const void *y)
{
    const long a = *(const long *)x, b = *(const long *)y;
    return a < b ? 1 : a > b ? -1 : 0;
}

static void *load(const char *path, long *size)
{
    FILE *fp = fopen(path, "rb");
    if (!fp) { perror(path); exit(1); }
    fseek(fp, 0, SEEK_END);
    *size = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    void *buf = malloc(*size);
    if (fread(buf, 1, *size, fp) != (size_t)*size) exit(1);
    fclose(fp);
    return buf;
}

int main(int argc, char **argv)
{
    if (argc < 8) { fprintf(stderr, "usage: skip_sim packed levels boxes depth root Q pitch [min_level]\n"); return 2; }
    long sz;
    N = load(argv[1], &sz);
    LV = load(argv[2], &sz);
    BX = load(argv[3], &sz);
    DEPTH = atoi(argv[4]);
    ROOT = (uint32_t)atoi(argv[5]);
    Q = atoi(argv[6]);
    PITCH = (float)atof(argv[7]);
    MINLV = argc > 8 ? atoi(argv[8]) : 2;
    pthread_t th[NT];
    for (int i = 0; i < NT; ++i) pthread_create(&th[i], NULL, worker, (void *)(intptr_t)i);
    for (int i = 0; i < NT; ++i) pthread_join(th[i], NULL);
    long tot[2] = {0, 0}, mm = 0, hh = 0;
    for (int t = 0; t < TX * TY; ++t) { tot[0] += tile_push[0][t]; tot[1] += tile_push[1][t]; }
    for (int i = 0; i < NT; ++i) { mm += mism[i]; hh += hits[i]; }
    long dm[3] = {0, 0, 0}, pm[2] = {0, 0}, ds[3] = {0, 0, 0};
    for (int t = 0; t < TX * TY; ++t) {
        for (int k = 0; k < 3; ++k) dm[k] += tile_desc_max[k][t];
        for (int k = 0; k < 2; ++k) pm[k] += tile_push_max[k][t];
    }
    for (int i = 0; i < NT; ++i)
        for (int k = 0; k < 3; ++k) ds[k] += desc_sum[k][i];
    printf("{\"pitch\": %.2f, \"descents_per_ray\": [%.3f, %.3f, %.3f], \"sum_tile_max_descents\": [%ld, %ld, %ld], "
           "\"sum_tile_max_push\": [%ld, %ld]}   (reference, skip tested before the descent, skip after it)\n",
           PITCH, ds[0] / (double)(W * H), ds[1] / (double)(W * H), ds[2] / (double)(W * H), dm[0], dm[1], dm[2],
           pm[0], pm[1]);
    qsort(tile_push[0], TX * TY, sizeof(long), cmp_desc);
    qsort(tile_push[1], TX * TY, sizeof(long), cmp_desc);
    printf("{\"pitch\": %.2f, \"Q\": %d, \"min_level\": %d, \"rays\": %d, \"hits\": %ld, \"mismatches\": %ld, "
           "\"push_per_ray\": [%.3f, %.3f], \"max_tile_push\": [%ld, %ld], \"top10_tile_push\": [%ld, %ld], "
           "\"top100_tile_push_mean\": [%.0f, %.0f]}\n",
           PITCH, Q, MINLV, W * H, hh, mm, tot[0] / (double)(W * H), tot[1] / (double)(W * H), tile_push[0][0],
           tile_push[1][0], tile_push[0][9], tile_push[1][9],
           ({ double s = 0; for (int i = 0; i < 100; ++i) s += tile_push[0][i]; s / 100; }),
           ({ double s = 0; for (int i = 0; i < 100; ++i) s += tile_push[1][i]; s / 100; }));
    return 0;
}
