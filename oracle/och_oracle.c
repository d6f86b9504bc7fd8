/*
 * oracle/och_oracle.c -- CPU ORACLE.  TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's hot path, used only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER.
 * Nothing in octree_ray_tracing_amd/ links, loads or calls this file; the
 * product path is the HIP library (octree_ray_tracing_amd/csrc) and fails
 * loudly when that library is missing.
 *
 * Parity status: the reference tracer (ORT/och_h_octree.h, ORT/och_octree.cpp)
 * cannot be compiled in this image without stand-ins (MSVC-only <intrin.h> and
 * the MSVC-only __m128::m128_f32 / m128_u32 members), so this restatement is
 * pinned by (a) the reference's own och_noise.h compiled as it lies
 * (oracle/_ref/ref_harness, see oracle/Makefile), (b) the known-answer values
 * SURVEY.md records from the reference run in this container (§4, §6, §7,
 * §8c: depth-3 zero-direction KAT, depth-8/10 node and voxel counts, mean
 * PUSH/STEP/POP per ray, hit fractions) and (c) the host's own RCPPS
 * instruction.  Per-ray hit records beyond those are "parity unpinned"
 * against a reference binary; see DESIGN.md §3.
 *
 * ORT/ = /root/reference/Octree_Ray_Tracing/.  Compile with
 * -ffp-contract=off (the reference pins fused ops with explicit intrinsics and
 * everything else must stay unfused).  Never enable FTZ/DAZ.
 */
#include <immintrin.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORA_API __attribute__((visibility("default")))

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* ------------------------------------------------------------------ RCPPS */

/* The reference takes 1/d with _mm_rcp_ps (ORT/och_h_octree.h:316,
 * ORT/och_octree.cpp:191): an approximate, CPU-defined reciprocal. */
ORA_API uint32_t ora_rcpps_native(uint32_t xbits)
{
    __m128 r = _mm_rcp_ps(_mm_castsi128_ps(_mm_set1_epi32((int)xbits)));
    return (uint32_t)_mm_cvtsi128_si32(_mm_castps_si128(r));
}

/* Table model of RCPPS: entry k = RCPPS(-(1 + k/2^L)) (exponent 127 input);
 * other exponents shift the result exponent; zero/denormal inputs give inf,
 * results below the normal range flush to zero.  Only valid where the host's
 * RCPPS actually follows this model (checked by tests/test_rcp.py). */
ORA_API uint32_t ora_rcp_lut(uint32_t x, const uint32_t *lut, int log2_entries)
{
    uint32_t sign = x & 0x80000000u, e = (x >> 23) & 0xFFu;
    if (e == 0) return sign | 0x7F800000u;
    if (e == 0xFF) return (x & 0x7FFFFFu) ? (x | 0x400000u) : sign;
    uint32_t ent = lut[(x & 0x7FFFFFu) >> (23 - log2_entries)];
    int ne = (int)((ent >> 23) & 0xFFu) + 127 - (int)e;
    if (ne <= 0) return sign;
    return sign | ((uint32_t)ne << 23) | (ent & 0x7FFFFFu);
}

/* ---------------------------------------------------------------- tracer */

typedef struct ora_pool {
    const uint32_t *nodes;   /* n x 8 child slots                         */
    uint32_t root;           /* root index in the pool's own numbering    */
    int depth;               /* levels; leaf level children are voxel ids */
    int index_base;          /* 1 = h_octree (1-based), 0 = octree        */
    float miss_t;            /* +INF (h_octree :429) or 0.0F (octree :302)*/
} ora_pool;

typedef struct ora_rcp {
    const uint32_t *lut;     /* NULL -> native RCPPS of this host */
    int log2_entries;
} ora_rcp;

typedef struct ora_counts { uint64_t push, step, pop; } ora_counts;

static inline float ora_rcp_eval(const ora_rcp *r, float x)
{
    uint32_t b = f2u(x);
    return u2f(r->lut ? ora_rcp_lut(b, r->lut, r->log2_entries) : ora_rcpps_native(b));
}

/* Laine-Karras traversal in the reflected frame, ORT/och_h_octree.h:292-447
 * (DAG, 1-based, miss t = INF) and ORT/och_octree.cpp:167-320 (pointer tree,
 * 0-based, miss t = 0).  Written as an explicit state machine over the three
 * labels of the reference (PUSH :342, STEP :378, POP :421). */
ORA_API void ora_trace(const ora_pool *P, const ora_rcp *R,
                       float ox, float oy, float oz, float dx, float dy, float dz,
                       int32_t *hit_dir, uint32_t *hit_voxel, float *hit_time,
                       ora_counts *cnt)
{
    const float o[3] = {ox, oy, oz}, d[3] = {dx, dy, dz};
    float coef[3], bias[3];
    uint32_t pos[3];
    int inv_signs = 0, idx = 0;

    /* setup, :306-338 */
    for (int a = 0; a < 3; ++a) {
        const int positive = 0.0F < d[a];                           /* :310 */
        inv_signs |= positive << a;                                 /* :322 */
        const float dneg = u2f(f2u(d[a]) | 0x80000000u);            /* :312 */
        const float orefl = fabsf((positive ? 3.0F : 0.0F) - o[a]); /* :314 */
        coef[a] = ora_rcp_eval(R, dneg);                            /* :316 */
        bias[a] = u2f(f2u(coef[a] * orefl) ^ 0x80000000u);          /* :318 */
        pos[a] = f2u(orefl) & 0x3FC00000u;                          /* :320 */
        if (u2f(pos[a]) == 1.5F) idx |= 1 << a;                     /* :324 */
    }

    uint32_t dim_bit = 1u << 22;                                    /* :326 */
    uint32_t parents[32];
    int sp = 0;
    uint32_t node = P->root;
    int level = 1, min_t_idx = 8;
    float t_min = 0.0F;
    const int base = P->index_base;

    enum { S_PUSH, S_STEP, S_POP } state = S_PUSH;
    for (;;) {
        if (state == S_PUSH) {
            if (cnt) ++cnt->push;
            const uint32_t child = P->nodes[(size_t)(node - base) * 8 + ((idx ^ inv_signs) & 7)];
            if (!child) { state = S_STEP; continue; }
            if (level++ == P->depth) {                              /* HIT :346-355 */
                *hit_voxel = child;
                *hit_dir = (min_t_idx >> 1) + 3 * ((inv_signs & min_t_idx) == 0);
                *hit_time = t_min;
                return;
            }
            parents[sp++] = node;                                   /* :357-359 */
            node = child;
            dim_bit >>= 1;                                          /* :361 */
            idx = 0;
            for (int a = 0; a < 3; ++a) {                           /* :363-373 */
                const float t_mid = fmaf(u2f(pos[a] | dim_bit), coef[a], bias[a]);
                if (t_mid >= t_min) { idx |= 1 << a; pos[a] |= dim_bit; }
            }
        } else if (state == S_STEP) {
            if (cnt) ++cnt->step;
            uint32_t t[3];
            for (int a = 0; a < 3; ++a)                             /* :380 */
                t[a] = f2u(fmaf(u2f(pos[a]), coef[a], bias[a]));
            int a;                                                  /* :388-406, unsigned */
            if (t[0] <= t[1] && t[0] <= t[2]) a = 0;
            else if (t[1] < t[0] && t[1] <= t[2]) a = 1;
            else a = 2;
            min_t_idx = 1 << a;
            t_min = u2f(t[a]);
            if (!(idx & min_t_idx)) { state = S_POP; continue; }    /* :410 */
            pos[a] &= ~dim_bit;                                     /* :413-417 */
            idx ^= min_t_idx;
            state = S_PUSH;
        } else {
            if (cnt) ++cnt->pop;
            if (--level == 0) {                                     /* MISS :423-431 */
                *hit_dir = 6;
                *hit_voxel = 0;
                *hit_time = P->miss_t;
                return;
            }
            node = parents[--sp];                                   /* :434 */
            for (int a = 0; a < 3; ++a) pos[a] &= ~dim_bit;         /* :436 */
            dim_bit <<= 1;                                          /* :438 */
            idx = 0;
            for (int a = 0; a < 3; ++a)                             /* :440-444 */
                if (u2f(dim_bit) == u2f(pos[a] & dim_bit)) idx |= 1 << a;
            state = S_STEP;
        }
    }
}

typedef struct ora_batch_job {
    const ora_pool *P; const ora_rcp *R;
    const float *origin; int origin_stride; const float *dirs;
    int32_t *hit_dir; uint32_t *hit_voxel; float *hit_time; uint32_t *push;
    uint64_t *next, n;          /* shared work counter: rays are handed out ORA_GRAIN at a time */
    ora_counts cnt;
} ora_batch_job;

/* Dynamic hand-out keeps the threads balanced: sky rows trace in a few
 * steps, terrain rows in hundreds, so contiguous ranges would idle most
 * threads behind the one holding the horizon. */
#define ORA_GRAIN 256u

static int ora_next_range(uint64_t *next, uint64_t n, uint64_t *b, uint64_t *e)
{
    *b = __atomic_fetch_add(next, ORA_GRAIN, __ATOMIC_RELAXED);
    if (*b >= n) return 0;
    *e = *b + ORA_GRAIN < n ? *b + ORA_GRAIN : n;
    return 1;
}

static void *ora_batch_worker(void *arg)
{
    ora_batch_job *j = (ora_batch_job *)arg;
    memset(&j->cnt, 0, sizeof j->cnt);
    uint64_t b, e;
    while (ora_next_range(j->next, j->n, &b, &e))
    for (uint64_t i = b; i < e; ++i) {
        const float *o = j->origin + (size_t)i * j->origin_stride;
        const float *d = j->dirs + 3 * i;
        uint64_t p0 = j->cnt.push;
        ora_trace(j->P, j->R, o[0], o[1], o[2], d[0], d[1], d[2],
                  &j->hit_dir[i], &j->hit_voxel[i], &j->hit_time[i], &j->cnt);
        if (j->push) j->push[i] = (uint32_t)(j->cnt.push - p0);
    }
    return NULL;
}

/* The reference's per-pixel loop (ORT/test_och_h_octree.cpp:448-450) traced
 * over a batch; nthreads > 1 shares it out ORA_GRAIN rays at a time. */
ORA_API void ora_trace_batch(const ora_pool *P, const ora_rcp *R,
                             const float *origin, int origin_stride, const float *dirs, uint64_t n,
                             int32_t *hit_dir, uint32_t *hit_voxel, float *hit_time, uint32_t *push,
                             int nthreads, ora_counts *total)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    ora_batch_job jobs[256];
    pthread_t th[256];
    uint64_t next = 0;
    for (int k = 0; k < nthreads; ++k) {
        jobs[k] = (ora_batch_job){P, R, origin, origin_stride, dirs, hit_dir, hit_voxel, hit_time, push,
                                  &next, n, {0, 0, 0}};
        if (nthreads == 1) ora_batch_worker(&jobs[k]);
        else pthread_create(&th[k], NULL, ora_batch_worker, &jobs[k]);
    }
    if (total) memset(total, 0, sizeof *total);
    for (int k = 0; k < nthreads; ++k) {
        if (nthreads > 1) pthread_join(th[k], NULL);
        if (total) { total->push += jobs[k].cnt.push; total->step += jobs[k].cnt.step; total->pop += jobs[k].cnt.pop; }
    }
}

/* ------------------------------------------------------- secondary rays */

/* Config 5's bounce (build-defined; the reference traces primary rays only):
 * origin o + d*t - offset, with get_directional_hit_offset's +-voxel_dim/2 on
 * the hit axis (ORT/test_och_h_octree.cpp:487-502; voxel_dim = 1.0F / dim,
 * ORT/och_h_octree.h:28) subtracted as for the editor's placement point
 * (:385, :418); direction mirrored on the hit axis.  float3 arithmetic:
 * products rounded, then sums (-ffp-contract=off). */
ORA_API void ora_bounce_ray(const float *o, const float *d, int32_t dir, float t, int depth, float *o2, float *d2)
{
    const float half = (1.0F / (float)(1 << depth)) / 2;
    const int axis = dir % 3;
    const float off = dir < 3 ? half : -half;
    for (int a = 0; a < 3; ++a) {
        const float q = o[a] + d[a] * t;
        o2[a] = q - (a == axis ? off : 0.0F);
        d2[a] = a == axis ? -d[a] : d[a];
    }
}

typedef struct ora_bounce_job {
    const ora_pool *P; const ora_rcp *R;
    const float *origin; int origin_stride; const float *dirs;
    int32_t *hd; uint32_t *hv; float *ht; int32_t *hd2; uint32_t *hv2; float *ht2; uint32_t *push;
    uint64_t *next, n;
    ora_counts cnt;
} ora_bounce_job;

static void *ora_bounce_worker(void *arg)
{
    ora_bounce_job *j = (ora_bounce_job *)arg;
    memset(&j->cnt, 0, sizeof j->cnt);
    uint64_t b, e;
    while (ora_next_range(j->next, j->n, &b, &e))
    for (uint64_t i = b; i < e; ++i) {
        const float *o = j->origin + (size_t)i * j->origin_stride;
        const float *d = j->dirs + 3 * i;
        const uint64_t p0 = j->cnt.push;
        ora_trace(j->P, j->R, o[0], o[1], o[2], d[0], d[1], d[2], &j->hd[i], &j->hv[i], &j->ht[i], &j->cnt);
        if (j->hd[i] < 6) {
            float o2[3], d2[3];
            ora_bounce_ray(o, d, j->hd[i], j->ht[i], j->P->depth, o2, d2);
            ora_trace(j->P, j->R, o2[0], o2[1], o2[2], d2[0], d2[1], d2[2], &j->hd2[i], &j->hv2[i], &j->ht2[i], &j->cnt);
        } else {
            j->hd2[i] = -1; j->hv2[i] = 0; j->ht2[i] = 0.0F;
        }
        if (j->push) j->push[i] = (uint32_t)(j->cnt.push - p0);
    }
    return NULL;
}

/* Primary + secondary records of a batch (the GPU's och_gpu_trace_bounce_batch_dev). */
ORA_API void ora_trace_bounce_batch(const ora_pool *P, const ora_rcp *R, const float *origin, int origin_stride,
                                    const float *dirs, uint64_t n, int32_t *hd, uint32_t *hv, float *ht,
                                    int32_t *hd2, uint32_t *hv2, float *ht2, uint32_t *push, int nthreads,
                                    ora_counts *total)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    ora_bounce_job jobs[256];
    pthread_t th[256];
    uint64_t next = 0;
    for (int k = 0; k < nthreads; ++k) {
        jobs[k] = (ora_bounce_job){P, R, origin, origin_stride, dirs, hd, hv, ht, hd2, hv2, ht2, push,
                                   &next, n, {0, 0, 0}};
        if (nthreads == 1) ora_bounce_worker(&jobs[k]);
        else pthread_create(&th[k], NULL, ora_bounce_worker, &jobs[k]);
    }
    if (total) memset(total, 0, sizeof *total);
    for (int k = 0; k < nthreads; ++k) {
        if (nthreads > 1) pthread_join(th[k], NULL);
        if (total) { total->push += jobs[k].cnt.push; total->step += jobs[k].cnt.step; total->pop += jobs[k].cnt.pop; }
    }
}

/* ---------------------------------------------------------------- camera */

/* tree_camera::update_position, ORT/test_och_h_octree.cpp:87-138.
 * yaw = dir.x, pitch = dir.y (:53, :102-105); roll fixed (sin_a 0, cos_a 1). */
ORA_API void ora_raygen(float yaw, float pitch, float fov, int W, int H, float *rays)
{
    const float aspect = (float)W / (float)H;                       /* :89 */
    const float view_x = 2.0F / (float)W;                           /* :91 */
    const float view_y = 2.0F / (float)H;                           /* :93 */
    const float fov_factor = 1 / tanf(fov / 2);                     /* :97 */
    const float sa = 0, ca = 1;                                     /* :100-101 */
    const float sb = sinf(yaw), cb = cosf(yaw), sc = sinf(pitch), cc = cosf(pitch);
    const float m[9] = {                                            /* :107-115 */
        ca * cb, ca * sb * sc - sa * cc, ca * sb * cc + sa * sc,
        sa * cb, sa * sb * sc + ca * cc, sa * sb * cc - ca * sc,
        -sb,     cb * sc,                cb * cc};
    size_t k = 0;
    for (int row = 0; row < H; ++row)
        for (int col = 0; col < W; ++col) {
            const float u = aspect * (view_x * (float)col - 1.0F);  /* :123 */
            const float v = view_y * (float)row - 1.0F;             /* :125 */
            const float ru = u * m[0] + v * m[1] + fov_factor * m[2];
            const float rv = u * m[3] + v * m[4] + fov_factor * m[5];
            const float rw = u * m[6] + v * m[7] + fov_factor * m[8];
            const float rmag = 1 / sqrtf(ru * ru + rv * rv + rw * rw); /* :133 */
            rays[k++] = rw * rmag;                                  /* :135 */
            rays[k++] = ru * rmag;
            rays[k++] = -rv * rmag;
        }
}

/* tree_camera::trace_pixel colour choice, ORT/test_och_h_octree.cpp:76-84,
 * as olc::Pixel packed RGBA8 (r in the low byte). */
ORA_API uint32_t ora_shade(int32_t dir, uint32_t voxel, const uint32_t *palette, uint32_t n_voxels)
{
    if (dir == 6) return 0xFFFEBF00u;                               /* exit colour 00 BF FE */
    if (dir == 7) return 0xFF07193Fu;                               /* inside colour 3F 19 07 */
    if (voxel == 0 || voxel > n_voxels || dir < 0 || dir > 5) return 0xFFFF00FFu;
    return palette[6 * (voxel - 1) + (uint32_t)dir];
}

/* Config 5 pixel: the primary colour, halved (RGB >> 1, alpha kept) when
 * the pixel's secondary ray is blocked (anything but exit). */
ORA_API uint32_t ora_shade_bounce(int32_t dir, uint32_t voxel, int32_t dir2, const uint32_t *palette, uint32_t n_voxels)
{
    const uint32_t c = ora_shade(dir, voxel, palette, n_voxels);
    if (dir < 0 || dir > 5 || dir2 == 6) return c;
    return ((c >> 1) & 0x007F7F7Fu) | (c & 0xFF000000u);
}

/* ----------------------------------------------------------------- noise */

/* och::simplex_n (ORT/och_noise.h:18-367), float arithmetic in the same
 * evaluation order.  Used to restate the terrain fill (§3.2 of SURVEY). */
static const uint8_t ora_perm[256] = {
    151, 160, 137, 91, 90, 15, 131, 13, 201, 95, 96, 53, 194, 233, 7, 225,
    140, 36, 103, 30, 69, 142, 8, 99, 37, 240, 21, 10, 23, 190, 6, 148,
    247, 120, 234, 75, 0, 26, 197, 62, 94, 252, 219, 203, 117, 35, 11, 32,
    57, 177, 33, 88, 237, 149, 56, 87, 174, 20, 125, 136, 171, 168, 68, 175,
    74, 165, 71, 134, 139, 48, 27, 166, 77, 146, 158, 231, 83, 111, 229, 122,
    60, 211, 133, 230, 220, 105, 92, 41, 55, 46, 245, 40, 244, 102, 143, 54,
    65, 25, 63, 161, 1, 216, 80, 73, 209, 76, 132, 187, 208, 89, 18, 169,
    200, 196, 135, 130, 116, 188, 159, 86, 164, 100, 109, 198, 173, 186, 3, 64,
    52, 217, 226, 250, 124, 123, 5, 202, 38, 147, 118, 126, 255, 82, 85, 212,
    207, 206, 59, 227, 47, 16, 58, 17, 182, 189, 28, 42, 223, 183, 170, 213,
    119, 248, 152, 2, 44, 154, 163, 70, 221, 153, 101, 155, 167, 43, 172, 9,
    129, 22, 39, 253, 19, 98, 108, 110, 79, 113, 224, 232, 178, 185, 112, 104,
    218, 246, 97, 228, 251, 34, 242, 193, 238, 210, 144, 12, 191, 179, 162, 241,
    81, 51, 145, 235, 249, 14, 239, 107, 49, 192, 214, 31, 181, 199, 106, 157,
    184, 84, 204, 176, 115, 121, 50, 45, 127, 4, 150, 254, 138, 236, 205, 93,
    222, 114, 67, 29, 24, 72, 243, 141, 128, 195, 78, 66, 215, 61, 156, 180};

static const float ora_grad[12][3] = {
    {1, 1, 0}, {-1, 1, 0}, {1, -1, 0}, {-1, -1, 0}, {1, 0, 1}, {-1, 0, 1},
    {1, 0, -1}, {-1, 0, -1}, {0, 1, 1}, {0, -1, 1}, {0, 1, -1}, {0, -1, -1}};

static inline int P8(int v) { return ora_perm[v & 255]; }

/* 2-D simplex, ORT/och_noise.h:73-179 */
ORA_API float ora_noise2(float freq, float x, float y)
{
    x *= freq; y *= freq;
    const float F2 = 0.5F * (0.73205078F);
    const float G2 = (3.0F - 1.73205078F) / 6.0F;
    const float s = (x + y) * F2;
    const int i = (int)(x + s), j = (int)(y + s);
    const float t = (float)(i + j) * G2;
    const float x0 = x - ((float)i - t), y0 = y - ((float)j - t);
    const int i1 = x0 > y0, j1 = !(x0 > y0);
    const float cx[3] = {x0, x0 - (float)i1 + G2, x0 - 1.0F + 2.0F * G2};
    const float cy[3] = {y0, y0 - (float)j1 + G2, y0 - 1.0F + 2.0F * G2};
    const int ii = i & 255, jj = j & 255;
    const int gi[3] = {P8(ii + P8(jj)) % 12, P8(ii + i1 + P8(jj + j1)) % 12, P8(ii + 1 + P8(jj + 1)) % 12};
    float n[3];
    for (int c = 0; c < 3; ++c) {
        float tc = 0.5F - cx[c] * cx[c] - cy[c] * cy[c];
        if (tc < 0) { n[c] = 0.0F; continue; }
        tc *= tc;
        n[c] = tc * tc * (ora_grad[gi[c]][0] * cx[c] + ora_grad[gi[c]][1] * cy[c]);
    }
    return 70.0F * (n[0] + n[1] + n[2]);
}

/* 3-D simplex, ORT/och_noise.h:181-366 */
ORA_API float ora_noise3(float freq, float x, float y, float z)
{
    x *= freq; y *= freq; z *= freq;
    const float F3 = 1.0F / 3.0F, G3 = 1.0F / 6.0F;
    const float s = (x + y + z) * F3;
    const int i = (int)(x + s), j = (int)(y + s), k = (int)(z + s);
    const float t = (float)(i + j + k) * G3;
    const float x0 = x - ((float)i - t), y0 = y - ((float)j - t), z0 = z - ((float)k - t);
    int o1[3], o2[3];                                   /* :224-281 */
    if (x0 >= y0) {
        if (y0 >= z0)      { o1[0]=1; o1[1]=0; o1[2]=0; o2[0]=1; o2[1]=1; o2[2]=0; }
        else if (x0 >= z0) { o1[0]=1; o1[1]=0; o1[2]=0; o2[0]=1; o2[1]=0; o2[2]=1; }
        else               { o1[0]=0; o1[1]=0; o1[2]=1; o2[0]=1; o2[1]=0; o2[2]=1; }
    } else {
        if (y0 < z0)       { o1[0]=0; o1[1]=0; o1[2]=1; o2[0]=0; o2[1]=1; o2[2]=1; }
        else if (x0 < z0)  { o1[0]=0; o1[1]=1; o1[2]=0; o2[0]=0; o2[1]=1; o2[2]=1; }
        else               { o1[0]=0; o1[1]=1; o1[2]=0; o2[0]=1; o2[1]=1; o2[2]=0; }
    }
    const float px[4] = {x0, x0 - (float)o1[0] + G3, x0 - (float)o2[0] + G3 * 2.0F, x0 - 1.0F + G3 * 3.0F};
    const float py[4] = {y0, y0 - (float)o1[1] + G3, y0 - (float)o2[1] + G3 * 2.0F, y0 - 1.0F + G3 * 3.0F};
    const float pz[4] = {z0, z0 - (float)o1[2] + G3, z0 - (float)o2[2] + G3 * 2.0F, z0 - 1.0F + G3 * 3.0F};
    const int ii = i & 255, jj = j & 255, kk = k & 255;
    const int gi[4] = {
        P8(ii + P8(jj + P8(kk))) % 12,
        P8(ii + o1[0] + P8(jj + o1[1] + P8(kk + o1[2]))) % 12,
        P8(ii + o2[0] + P8(jj + o2[1] + P8(kk + o2[2]))) % 12,
        P8(ii + 1 + P8(jj + 1 + P8(kk + 1))) % 12};
    float n[4];
    for (int c = 0; c < 4; ++c) {
        float tc = 0.6F - px[c] * px[c] - py[c] * py[c] - pz[c] * pz[c];
        if (tc < 0) { n[c] = 0.0F; continue; }
        tc *= tc;
        const float *g = ora_grad[gi[c]];
        n[c] = tc * tc * (g[0] * px[c] + g[1] * py[c] + g[2] * pz[c]);
    }
    return 32.0F * (n[0] + n[1] + n[2] + n[3]);
}

/* ---------------------------------------------------------------- terrain */

/* get_terrain_heigth, ORT/test_och_h_octree.cpp:561-569 (global noise at
 * frequency 0.5, :35), generalised from tree_t::dim to 1 << depth. */
ORA_API int ora_height(int x, int y, int dim)
{
    const float px = (float)(x * 4) / (float)dim;
    const float py = (float)(y * 4) / (float)dim;
    return (int)(ora_noise2(0.5F, px, py) * (float)dim / 16.0F + (float)(dim / 4));
}

/* The top voxel of each column: 2 + (rand() > RAND_MAX / 2), one rand() per
 * column, y outer, x inner, default seed (ORT/test_och_h_octree.cpp:776-780).
 * Uses this platform's rand() (glibc here and on the GPU box). */
ORA_API void ora_column_tops(int dim, uint8_t *tops)
{
    srand(1);
    for (int y = 0; y < dim; ++y)
        for (int x = 0; x < dim; ++x)
            tops[(size_t)y * dim + x] = (uint8_t)(2 + (rand() > RAND_MAX / 2));
}

/* tunnels: splatter_noise(-0.5, 1, 0, 1/16) evaluated through the global
 * simplex_n(0.5) (ORT/test_och_h_octree.cpp:745-765, :770, :786). */
ORA_API int ora_is_tunnel(int x, int y, int z)
{
    const float sc = 1.0F / 16.0F;
    return !(ora_noise3(0.5F, (float)x * sc, (float)y * sc, (float)z * sc) >= -0.5F);
}

/* Final voxel value after initialize_h_octree (ORT/test_och_h_octree.cpp:767-787):
 * create_volume fills z <= h with 1 (:651-695), the column pass writes the
 * top and the two voxels under it (:776-783), then tunnels clear (:786). */
ORA_API uint32_t ora_voxel(int x, int y, int z, int h, int top, int tunnels)
{
    if (z > h) return 0;
    if (tunnels && ora_is_tunnel(x, y, z)) return 0;
    if (z == h) return (uint32_t)top;
    if (z >= h - 2) return 4;
    return 1;
}

/* The whole height map, row-major h[y * dim + x]. */
ORA_API void ora_height_map(int dim, int32_t *h)
{
    for (int y = 0; y < dim; ++y)
        for (int x = 0; x < dim; ++x) h[(size_t)y * dim + x] = ora_height(x, y, dim);
}

/* ora_voxel at n points (x, y, z triples) of a dim^3 world; tops = the
 * dim x dim column tops (ora_column_tops).  Test helper for large trees. */
ORA_API void ora_voxel_batch(int dim, const int32_t *xyz, uint64_t n, const uint8_t *tops, int tunnels, uint32_t *out)
{
    for (uint64_t i = 0; i < n; ++i) {
        const int x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
        out[i] = ora_voxel(x, y, z, ora_height(x, y, dim), tops[(size_t)y * dim + x], tunnels);
    }
}

/* ---------------------------------------------------- small DAG builder */

/* Hash-consed bottom-up build of the terrain for small depths (<= 9): the
 * same canonical DAG that h_octree::register_node/set produce
 * (ORT/och_h_octree.h:110-237): identical subtrees share one node and
 * all-empty subtrees are 0.  Output is 1-based (index 0 unused); when
 * dedup == 0 the tree is expanded instead (och::octree, 0-based root 0,
 * ORT/och_octree.cpp:74-91). */
typedef struct ora_builder {
    int dim, depth, tunnels, dedup;
    const int *heights; const uint8_t *tops;
    uint32_t *nodes; uint32_t n, cap;
    uint32_t *table; uint32_t table_mask;
} ora_builder;

static uint32_t ora_hash8(const uint32_t *c)
{
    uint32_t h = 0x811C9DC5u;
    const uint8_t *b = (const uint8_t *)c;
    for (int i = 0; i < 32; ++i) h = (h ^ b[i]) * 0x01000193u;
    return h;
}

static uint32_t ora_intern(ora_builder *B, const uint32_t *c)
{
    if (B->n >= B->cap) {
        B->cap *= 2;
        B->nodes = (uint32_t *)realloc(B->nodes, (size_t)B->cap * 32);
    }
    if (!B->dedup) {
        memcpy(B->nodes + (size_t)B->n * 8, c, 32);
        return B->n++;
    }
    uint32_t s = ora_hash8(c) & B->table_mask;
    while (B->table[s]) {
        if (!memcmp(B->nodes + (size_t)B->table[s] * 8, c, 32)) return B->table[s];
        s = (s + 1) & B->table_mask;
    }
    memcpy(B->nodes + (size_t)B->n * 8, c, 32);
    B->table[s] = B->n;
    return B->n++;
}

static uint32_t ora_build_rec(ora_builder *B, int x, int y, int z, int lvl_size)
{
    uint32_t c[8];
    int any = 0;
    const int half = lvl_size >> 1;
    if (!B->dedup && lvl_size == B->dim) {
        /* pointer octree: reserve slot 0 for the root before its children */
        if (B->n == 0) { memset(B->nodes, 0, 32); B->n = 1; }
    }
    for (int k = 0; k < 8; ++k) {
        const int cx = x + (k & 1) * half, cy = y + ((k >> 1) & 1) * half, cz = z + ((k >> 2) & 1) * half;
        if (half == 1) {
            const size_t col = (size_t)cy * B->dim + cx;
            c[k] = ora_voxel(cx, cy, cz, B->heights[col], B->tops[col], B->tunnels);
        } else {
            c[k] = ora_build_rec(B, cx, cy, cz, half);
        }
        any |= c[k] != 0;
    }
    if (!any) return 0;
    if (!B->dedup && lvl_size == B->dim) { memcpy(B->nodes, c, 32); return 0; }
    return ora_intern(B, c);
}

/* Returns the node count (including the unused/reserved slot 0) and the root. */
ORA_API uint32_t ora_build_terrain(int depth, int tunnels, int dedup, uint32_t **nodes_out, uint32_t *root_out)
{
    ora_builder B;
    memset(&B, 0, sizeof B);
    B.depth = depth; B.dim = 1 << depth; B.tunnels = tunnels; B.dedup = dedup;
    int *h = (int *)malloc(sizeof(int) * (size_t)B.dim * B.dim);
    uint8_t *tops = (uint8_t *)malloc((size_t)B.dim * B.dim);
    for (int y = 0; y < B.dim; ++y)
        for (int x = 0; x < B.dim; ++x) h[(size_t)y * B.dim + x] = ora_height(x, y, B.dim);
    ora_column_tops(B.dim, tops);
    B.heights = h; B.tops = tops;
    B.cap = 1024;
    B.nodes = (uint32_t *)malloc((size_t)B.cap * 32);
    memset(B.nodes, 0, 32);
    B.n = 1;                          /* index 0 = empty / reserved */
    if (dedup) {
        B.table_mask = (1u << 24) - 1;
        B.table = (uint32_t *)calloc((size_t)B.table_mask + 1, 4);
    } else {
        B.n = 0;
    }
    uint32_t root = ora_build_rec(&B, 0, 0, 0, B.dim);
    free(h); free(tops); free(B.table);
    *nodes_out = B.nodes;
    *root_out = root;
    return B.n;
}

ORA_API void ora_free(void *p) { free(p); }

/* h_octree::at / octree::at (ORT/och_h_octree.h:239-258, ORT/och_octree.cpp:141-160) */
ORA_API uint32_t ora_at(const ora_pool *P, int x, int y, int z)
{
    uint32_t cur = P->root;
    if (P->index_base == 1 && cur == 0) return 0;
    for (int l = P->depth - 1; l >= 0; --l) {
        const int c = ((x >> l) & 1) | (((y >> l) & 1) << 1) | (((z >> l) & 1) << 2);
        const uint32_t nx = P->nodes[(size_t)(cur - P->index_base) * 8 + c];
        if (l == 0) return nx;
        if (!nx) return 0;
        cur = nx;
    }
    return 0;
}

/* ------------------------------------- h_octree hash table, restated exactly */

/* och::h_octree<L, D>'s node_hashtable and edit operations
 * (ORT/och_h_octree.h:70-83 table, :52-65 hash, :110-160 register_node,
 * :162-174 remove_node, :176-237 set, :239-258 at) and the demo's fill
 * sequence initialize_h_octree (ORT/test_och_h_octree.cpp:651-695, :767-787).
 * Reproduces the reference's table->nodes array slot for slot, so the GPU can
 * be fed exactly what a reference user would hand over. */
typedef struct ora_href {
    int log2cap, depth, dim;
    uint32_t cap, idx_mask;
    uint8_t *cashes; uint32_t *refcounts; uint32_t *nodes;
    uint32_t root, fillcnt, nodecnt;
    int overflow;
} ora_href;

static uint32_t href_hash(const uint32_t *c)                       /* :52-65 */
{
    const signed char *b = (const signed char *)c;   /* MSVC/x86 char is signed */
    uint32_t h = 0x811C9DC5u;
    for (int i = 0; i < 32; ++i) h = ((uint32_t)(int32_t)b[i] ^ h) * 0x01000193u;
    return h;
}

static uint32_t href_register(ora_href *T, const uint32_t *n)       /* :110-160 */
{
    if (T->fillcnt > (uint32_t)((float)T->cap * 0.9375F)) { T->overflow = 1; return 0; }
    const uint32_t hash = href_hash(n);
    uint32_t index = hash & T->idx_mask;
    uint8_t cash = (uint8_t)(hash >> T->log2cap);
    if (cash == 0) cash = 1;
    else if (cash == 0xFF) cash = 0x7F;
    uint32_t last_grave = 0xFFFFFFFFu;
    while (T->cashes[index]) {
        if (T->cashes[index] == 0xFF) last_grave = index;
        if (T->cashes[index] == cash && !memcmp(T->nodes + (size_t)index * 8, n, 32)) {
            ++T->nodecnt;
            ++T->refcounts[index];
            return index + 1;
        }
        index = (index + 1) & (T->cap - 1);
    }
    ++T->nodecnt; ++T->fillcnt;
    if (last_grave != 0xFFFFFFFFu) index = last_grave;
    T->cashes[index] = cash;
    memcpy(T->nodes + (size_t)index * 8, n, 32);
    T->refcounts[index] = 1;
    return index + 1;
}

static void href_remove(ora_href *T, uint32_t idx)                  /* :162-174 */
{
    --T->refcounts[idx - 1];
    --T->nodecnt;
    if (!T->refcounts[idx - 1]) { --T->fillcnt; T->cashes[idx - 1] = 0xFF; }
}

static inline int href_child_of(int x, int y, int z, int level)     /* z_encode_16 digit */
{
    return ((x >> level) & 1) | (((y >> level) & 1) << 1) | (((z >> level) & 1) << 2);
}

ORA_API void ora_href_set(ora_href *T, int xi, int yi, int zi, uint32_t v)   /* :176-237 */
{
    const uint16_t x = (uint16_t)xi, y = (uint16_t)yi, z = (uint16_t)zi;
    if ((x | y | z) >= T->dim) return;
    uint32_t stk[32];
    int d = T->depth - 1;
    for (uint32_t curr = T->root; curr && d >= 0; --d) {
        stk[d] = curr;
        curr = T->nodes[(size_t)(curr - 1) * 8 + href_child_of(x, y, z, d)];
    }
    uint32_t child = v;
    int _d = 0;
    if (++d) {
        if (!v) return;
        while (_d != d) {
            uint32_t n[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            n[href_child_of(x, y, z, _d)] = child;
            ++_d;
            child = href_register(T, n);
        }
    }
    for (int i = d; i != T->depth; ++i) {
        href_remove(T, stk[i]);
        uint32_t n[8];
        memcpy(n, T->nodes + (size_t)(stk[i] - 1) * 8, 32);
        n[href_child_of(x, y, z, i)] = child;
        int zero = 1;
        for (int k = 0; k < 8; ++k) zero &= n[k] == 0;
        child = zero ? 0 : href_register(T, n);
    }
    T->root = child;
}

ORA_API uint32_t ora_href_at(const ora_href *T, int x, int y, int z)   /* :239-258 */
{
    uint32_t curr = T->root;
    for (int i = T->depth - 1; i != 0; --i) {
        const uint32_t nx = T->nodes[(size_t)(curr - 1) * 8 + href_child_of(x, y, z, i)];
        if (!nx) return 0;
        curr = nx;
    }
    return T->nodes[(size_t)(curr - 1) * 8 + href_child_of(x, y, z, 0)];
}

/* create_volume, ORT/test_och_h_octree.cpp:651-695 (voxel value 1, :600-603) */
static uint32_t href_create_volume(ora_href *T, const int *h, int x, int y, int z, int depth)
{
    const int dim = 1 << depth;
    int active = 0;
    for (int yy = 0; yy < dim && !active; ++yy)
        for (int xx = 0; xx < dim; ++xx)
            if (z <= h[(size_t)(y + yy) * T->dim + (x + xx)]) { active = 1; break; }
    if (!active) return 0;
    uint32_t n[8];
    if (depth != 1) {
        const int hd = 1 << (depth - 1);
        for (int k = 0; k < 8; ++k)
            n[k] = href_create_volume(T, h, x + (k & 1) * hd, y + ((k >> 1) & 1) * hd, z + ((k >> 2) & 1) * hd, depth - 1);
    } else {
        for (int k = 0; k < 8; ++k)
            n[k] = (z + ((k >> 2) & 1)) <= h[(size_t)(y + ((k >> 1) & 1)) * T->dim + (x + (k & 1))] ? 1u : 0u;
    }
    return href_register(T, n);
}

ORA_API ora_href *ora_href_new(int depth, int log2cap)
{
    ora_href *T = (ora_href *)calloc(1, sizeof *T);
    T->depth = depth; T->dim = 1 << depth; T->log2cap = log2cap;
    T->cap = 1u << log2cap;
    T->idx_mask = ((T->cap - 1) >> 4) << 4;
    T->cashes = (uint8_t *)calloc(T->cap, 1);
    T->refcounts = (uint32_t *)calloc(T->cap, 4);
    T->nodes = (uint32_t *)calloc((size_t)T->cap * 8, 4);
    return T;
}

ORA_API void ora_href_free(ora_href *T)
{
    if (!T) return;
    free(T->cashes); free(T->refcounts); free(T->nodes); free(T);
}

/* initialize_h_octree, ORT/test_och_h_octree.cpp:767-787. */
ORA_API void ora_href_fill_terrain(ora_href *T, int tunnels)
{
    const int dim = T->dim;
    int *h = (int *)malloc(sizeof(int) * (size_t)dim * dim);
    for (int y = 0; y < dim; ++y)
        for (int x = 0; x < dim; ++x) h[(size_t)y * dim + x] = ora_height(x, y, dim);
    T->root = href_create_volume(T, h, 0, 0, 0, T->depth);
    srand(1);
    for (int y = 0; y < dim; ++y)
        for (int x = 0; x < dim; ++x) {
            const uint16_t z = (uint16_t)h[(size_t)y * dim + x];
            ora_href_set(T, x, y, z, 2 + (rand() > RAND_MAX / 2));
            ora_href_set(T, x, y, (uint16_t)(z - 1), 4);
            ora_href_set(T, x, y, (uint16_t)(z - 2), 4);
        }
    if (tunnels)
        for (int z = 0; z < dim; ++z)
            for (int y = 0; y < dim; ++y)
                for (int x = 0; x < dim; ++x)
                    if (ora_is_tunnel(x, y, z)) ora_href_set(T, x, y, z, 0);
    free(h);
}

/* ------------------------------------- och::octree's table, restated exactly */

/* och::octree (ORT/och_octree.h:10-69, ORT/och_octree.cpp:14-160): a
 * capacity-sized table of 8 x u32 nodes, the root fixed at index 0, children
 * 0-based (0 = empty), a free list threaded through children[0] of the free
 * nodes (create_table :21-34, alloc :46-63, dealloc :65-72).  set() allocates
 * the missing path and writes the voxel, 0 included (:74-91), so set(..., 0)
 * leaves allocated empty nodes reachable; unset() clears the voxel and
 * deallocates the nodes it empties, bottom-up (:93-139) -- the root too,
 * which then gets the free list's head written into its children[0] and
 * leaves head = 0.  The reference exit(0)s when alloc() finds head == 0
 * (:50-54); here that sets `overflow` and the edit stops. */
typedef struct ora_oref {
    int depth, dim;
    uint32_t cap;
    uint32_t *nodes;                 /* cap x 8 */
    uint32_t head;                   /* och_octree.h:27 */
    int node_cnt;                    /* och_octree.h:28, OCH_IF_DEBUG counter */
    int overflow;
} ora_oref;

ORA_API ora_oref *ora_oref_new(int depth, uint32_t capacity)          /* :14, create_table :21-34 */
{
    if (capacity < 2) return NULL;
    ora_oref *T = (ora_oref *)calloc(1, sizeof *T);
    T->depth = depth; T->dim = 1 << depth; T->cap = capacity;
    T->nodes = (uint32_t *)calloc((size_t)capacity * 8, 4);
    for (uint32_t i = 1; i != capacity; ++i) T->nodes[(size_t)i * 8] = i + 1;
    T->nodes[(size_t)(capacity - 1) * 8] = 0;
    T->head = 1;
    T->node_cnt = 1;
    return T;
}

ORA_API void ora_oref_free(ora_oref *T)
{
    if (!T) return;
    free(T->nodes); free(T);
}

static uint32_t oref_alloc(ora_oref *T)                               /* :46-63 */
{
    ++T->node_cnt;
    if (!T->head) { T->overflow = 1; return 0; }                     /* "Too many allocations", exit(0) */
    const uint32_t old = T->head;
    T->head = T->nodes[(size_t)old * 8];
    memset(T->nodes + (size_t)old * 8, 0, 32);
    return old;
}

static void oref_dealloc(ora_oref *T, uint32_t idx)                   /* :65-72 */
{
    --T->node_cnt;
    T->nodes[(size_t)idx * 8] = T->head;
    T->head = idx;
}

static int oref_is_empty(const ora_oref *T, uint32_t idx)             /* :41-44 */
{
    const uint32_t *c = T->nodes + (size_t)idx * 8;
    for (int k = 0; k < 8; ++k) if (c[k]) return 0;
    return 1;
}

/* The child digit of level i of z_encode_16(x, y, z) (ORT/och_z_order.cpp:191-196). */
static inline int oref_digit(int x, int y, int z, int i)
{
    return ((x >> i) & 1) | (((y >> i) & 1) << 1) | (((z >> i) & 1) << 2);
}

ORA_API void ora_oref_set(ora_oref *T, int x, int y, int z, uint32_t vx)   /* :74-91 */
{
    if (T->overflow) return;
    uint32_t curr = 0;                                                /* root */
    for (int i = T->depth - 1; i != 0; --i) {
        const int k = oref_digit(x, y, z, i);
        if (!T->nodes[(size_t)curr * 8 + k]) {
            const uint32_t n = oref_alloc(T);
            if (T->overflow) return;
            T->nodes[(size_t)curr * 8 + k] = n;
        }
        curr = T->nodes[(size_t)curr * 8 + k];
    }
    T->nodes[(size_t)curr * 8 + oref_digit(x, y, z, 0)] = vx;
}

ORA_API void ora_oref_unset(ora_oref *T, int x, int y, int z)         /* :93-139 */
{
    if (T->overflow) return;
    uint32_t curr = 0, stack[32];
    int sptr = 0;
    for (int i = T->depth - 1; i != 0; --i) {
        const uint32_t child = T->nodes[(size_t)curr * 8 + oref_digit(x, y, z, i)];
        if (!child) return;
        stack[sptr++] = curr;
        curr = child;
    }
    T->nodes[(size_t)curr * 8 + oref_digit(x, y, z, 0)] = 0;
    if (oref_is_empty(T, curr)) oref_dealloc(T, curr);
    else return;
    for (int i = 1; i != T->depth; ++i) {
        --sptr;
        T->nodes[(size_t)stack[sptr] * 8 + oref_digit(x, y, z, i)] = 0;
        if (oref_is_empty(T, stack[sptr])) oref_dealloc(T, stack[sptr]);   /* the root too: dealloc(0) */
        else return;
    }
}

ORA_API uint32_t ora_oref_at(const ora_oref *T, int x, int y, int z)  /* :141-160 */
{
    uint32_t curr = 0;
    for (int i = T->depth - 1; i > 0; --i) {
        const uint32_t c = T->nodes[(size_t)curr * 8 + oref_digit(x, y, z, i)];
        if (!c) return 0;
        curr = c;
    }
    return T->nodes[(size_t)curr * 8 + oref_digit(x, y, z, 0)];
}

/* Config 1's och::octree, filled the reference's way: the demo
 * terrain's columns with non-zero set() calls (y outer, x inner, z upward;
 * one rand() per column for the top voxel, ORT/test_och_h_octree.cpp:776-783),
 * then remove()'s pass over every voxel, z outer, x inner (:735-743), for the
 * tunnel voxels (:745-765, :786): tunnel_mode 0 unset()s them, tunnel_mode 1
 * set()s them to 0 as remove() does on the h_octree (leaving allocated empty
 * nodes reachable, air voxels included), tunnel_mode -1 skips the pass. */
ORA_API void ora_oref_fill_terrain(ora_oref *T, int tunnel_mode)
{
    const int dim = T->dim;
    int *h = (int *)malloc(sizeof(int) * (size_t)dim * dim);
    for (int y = 0; y < dim; ++y)
        for (int x = 0; x < dim; ++x) h[(size_t)y * dim + x] = ora_height(x, y, dim);
    srand(1);
    for (int y = 0; y < dim && !T->overflow; ++y)
        for (int x = 0; x < dim; ++x) {
            const int hh = h[(size_t)y * dim + x];
            const int top = 2 + (rand() > RAND_MAX / 2);
            for (int z = 0; z <= hh && z < dim; ++z) ora_oref_set(T, x, y, z, ora_voxel(x, y, z, hh, top, 0));
        }
    if (tunnel_mode >= 0)
        for (int z = 0; z < dim; ++z)
            for (int y = 0; y < dim; ++y)
                for (int x = 0; x < dim; ++x)
                    if (ora_is_tunnel(x, y, z)) {
                        if (tunnel_mode == 0) ora_oref_unset(T, x, y, z);
                        else ora_oref_set(T, x, y, z, 0);
                    }
    free(h);
}

ORA_API const uint32_t *ora_oref_nodes(const ora_oref *T) { return T->nodes; }
ORA_API uint32_t ora_oref_capacity(const ora_oref *T) { return T->cap; }
ORA_API uint32_t ora_oref_head(const ora_oref *T) { return T->head; }
ORA_API int ora_oref_node_cnt(const ora_oref *T) { return T->node_cnt; }
ORA_API int ora_oref_overflow(const ora_oref *T) { return T->overflow; }

ORA_API const uint32_t *ora_href_nodes(const ora_href *T) { return T->nodes; }
ORA_API uint32_t ora_href_capacity(const ora_href *T) { return T->cap; }
ORA_API uint32_t ora_href_root(const ora_href *T) { return T->root; }
ORA_API uint32_t ora_href_fillcnt(const ora_href *T) { return T->fillcnt; }
ORA_API uint32_t ora_href_nodecnt(const ora_href *T) { return T->nodecnt; }
ORA_API int ora_href_overflow(const ora_href *T) { return T->overflow; }
