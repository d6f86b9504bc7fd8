/* split_model.c -- checks and prices splitting one ray's walk over S lanes.
 *
 * Design tool only (not product, not a checker): its own restatement of the
 * walk (ORT/och_h_octree.h:292-447) with the host's RCPPS, on a raw 1-based
 * pool.
 *
 * The decomposition.  Call the cells of level L (size 2^-L) the walk tests at
 * a PUSH and finds present its "segments", numbered 0, 1, 2, ... in walk
 * order.  What the walk does at levels <= L does not depend on what it does
 * inside a segment: it enters a present level-L cell, walks below it, and
 * POPs back to level L with the position bits, child index and child size it
 * had before the PUSH (a POP clears exactly the bits the descent set), and
 * its next STEP at level L computes the same t values -- the same state a
 * walk that found the cell empty reaches by STEPping at once.  So a lane that
 * treats every segment but its own (ordinal % S == s) as empty walks the same
 * levels <= L, enters its own segments in the same state as the full walk,
 * and finds the same hit there if the hit lies there.  The ray's record is
 * then the hit of the lowest segment ordinal any lane found, or the MISS.
 * This tool checks that claim ray by ray against the full walk (also for the
 * dynamic variant: a ray's lanes claim segments first come, first served), and
 * prices the split with the lockstep model (a wave costs its longest lane's PUSH
 * tests, one per iteration of the render loop).
 *
 * Build: gcc -O2 -msse2 -o /tmp/split_model tools/split_model.c -lm -lpthread
 * Input: raw uint32 nodes[n][8] of a 1-based h_octree pool, root 1, e.g.
 *   ort.build_terrain(12).nodes.astype(np.uint32).tofile("d12_nodes.bin")
 * Usage: split_model nodes.bin depth pitch L S [threads [early [theta]]]
 *   early 1: a lane stops at the first segment past the ray's hit (ideal: as if
 *   the lane that finds the hit told the others at once).
 *   theta: the per-ray variant splits only the rays of a split tile longer than
 *   theta % of its longest, the others walking whole on one lane (default 50). */
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
static int DEPTH, LEVEL, SEGS, EARLY, THETA;

typedef struct { int32_t dir; uint32_t voxel, t; int ord; int push; } Rec;

/* seg < 0: the full walk; else only segments with ordinal % SEGS == seg are
 * entered.  ord: the hit's segment ordinal (-1: MISS). */
static void walk(const float *o, const float *d, int seg, int stop_ord, Rec *out)
{
    float c[3], b[3];
    uint32_t p[3], stack[32];
    int inv = 0, idx = 0, sp = 0, level = 1, axis = 8, ord = 0, push = 0;
    for (int a = 0; a < 3; ++a) {
        const int pos = 0.0F < d[a];
        inv |= pos << a;
        const float refl = fabsf((pos ? 3.0F : 0.0F) - o[a]);
        c[a] = _mm_cvtss_f32(_mm_rcp_ss(_mm_set_ss(u2f(f2u(d[a]) | 0x80000000u))));
        b[a] = u2f(f2u(c[a] * refl) ^ 0x80000000u);
        p[a] = f2u(refl) & 0x3FC00000u;
        if (p[a] == 0x3FC00000u) idx |= 1 << a;
    }
    uint32_t dim = 1u << 22, node = 1, t_min = 0;
    int cur_ord = -1;                       /* the segment the walk is inside (level > LEVEL) */
    enum { PUSH, STEP, POP } st = PUSH;
    for (;;) {
        if (st == PUSH) {
            ++push;
            const uint32_t ch = N[(size_t)(node - 1) * 8 + ((idx ^ inv) & 7)];
            if (!ch) { st = STEP; continue; }
            if (level == LEVEL) {           /* a present level-L cell: segment ord */
                const int k = ord++;
                if (stop_ord >= 0 && k > stop_ord) {    /* past the ray's first hit: no later segment can win */
                    out->dir = 6; out->voxel = 0; out->t = 0x7F800000u; out->ord = -1; out->push = push;
                    return;
                }
                if (seg >= 0 && k % SEGS != seg) { st = STEP; continue; }
                cur_ord = k;
            }
            if (level++ == DEPTH) {
                out->dir = (axis >> 1) + 3 * ((inv & axis) == 0);
                out->voxel = ch;
                out->t = t_min;
                out->ord = cur_ord;
                out->push = push;
                return;
            }
            stack[sp++] = node;
            node = ch;
            dim >>= 1;
            idx = 0;
            for (int a = 0; a < 3; ++a)
                if (fmaf(u2f(p[a] | dim), c[a], b[a]) >= u2f(t_min)) { idx |= 1 << a; p[a] |= dim; }
        } else if (st == STEP) {
            uint32_t t[3];
            for (int a = 0; a < 3; ++a) t[a] = f2u(fmaf(u2f(p[a]), c[a], b[a]));
            const int a = (t[0] <= t[1] && t[0] <= t[2]) ? 0 : (t[1] < t[0] && t[1] <= t[2]) ? 1 : 2;
            axis = 1 << a;
            t_min = t[a];
            if (!(idx & axis)) { st = POP; continue; }
            p[a] &= ~dim;
            idx ^= axis;
            st = PUSH;
        } else {
            if (--level == 0) {
                out->dir = 6; out->voxel = 0; out->t = 0x7F800000u; out->ord = -1; out->push = push;
                return;
            }
            node = stack[--sp];
            for (int a = 0; a < 3; ++a) p[a] &= ~dim;
            dim <<= 1;
            idx = 0;
            for (int a = 0; a < 3; ++a)
                if (u2f(dim) == u2f(p[a] & dim)) idx |= 1 << a;
            st = STEP;
        }
    }
}

/* Dynamic claiming (the alternative to ordinal % S): every lane of a ray walks
 * the levels <= L and claims each present level-L cell it reaches that no lane
 * of the ray has claimed yet (claimed = the next unclaimed ordinal), so a lane
 * busy inside a segment leaves the next ones to the others; a lane also stops
 * at a cell past the lowest HIT found so far (hitmin).  Lanes step in lockstep,
 * one PUSH test per iteration, as the render loop does. */
typedef struct { int claimed, hitmin, closed; } Shared;   /* closed: no segment left to claim */
typedef struct {
    float c[3], b[3];
    uint32_t p[3], stack[32], dim, node, t_min;
    int inv, idx, sp, level, axis, ord, push, cur_ord, st, done;
    Rec rec;
} Lane;

static void lane_init(Lane *L, const float *o, const float *d)
{
    memset(L, 0, sizeof *L);
    for (int a = 0; a < 3; ++a) {
        const int pos = 0.0F < d[a];
        L->inv |= pos << a;
        const float refl = fabsf((pos ? 3.0F : 0.0F) - o[a]);
        L->c[a] = _mm_cvtss_f32(_mm_rcp_ss(_mm_set_ss(u2f(f2u(d[a]) | 0x80000000u))));
        L->b[a] = u2f(f2u(L->c[a] * refl) ^ 0x80000000u);
        L->p[a] = f2u(refl) & 0x3FC00000u;
        if (L->p[a] == 0x3FC00000u) L->idx |= 1 << a;
    }
    L->dim = 1u << 22; L->node = 1; L->level = 1; L->axis = 8; L->cur_ord = -1; L->st = 0;
}

static void lane_finish(Lane *L, int hit, uint32_t voxel)
{
    L->done = 1;
    if (hit) { L->rec = (Rec){(L->axis >> 1) + 3 * ((L->inv & L->axis) == 0), voxel, L->t_min, L->cur_ord, L->push}; }
    else L->rec = (Rec){6, 0, 0x7F800000u, -1, L->push};
}

/* run until one PUSH test is done (or the lane finishes) */
static void lane_iter(Lane *L, Shared *sh)
{
    /* inside a segment past the ray's lowest HIT so far: nothing it finds can win */
    if (sh->hitmin >= 0 && L->cur_ord > sh->hitmin && L->level > LEVEL) { lane_finish(L, 0, 0); return; }
    for (;;) {
        if (L->st == 0) {                                   /* PUSH */
            ++L->push;
            const uint32_t ch = N[(size_t)(L->node - 1) * 8 + ((L->idx ^ L->inv) & 7)];
            if (!ch) { L->st = 1; return; }
            if (L->level == LEVEL) {
                const int k = L->ord++;
                if ((sh->hitmin >= 0 && k > sh->hitmin) || sh->closed) { lane_finish(L, 0, 0); return; }
                if (sh->claimed > k) { L->st = 1; return; }   /* another lane's */
                sh->claimed = k + 1;
                L->cur_ord = k;
            }
            if (L->level++ == DEPTH) {
                lane_finish(L, 1, ch);
                if (sh->hitmin < 0 || L->cur_ord < sh->hitmin) sh->hitmin = L->cur_ord;
                return;
            }
            L->stack[L->sp++] = L->node;
            L->node = ch;
            L->dim >>= 1;
            L->idx = 0;
            for (int a = 0; a < 3; ++a)
                if (fmaf(u2f(L->p[a] | L->dim), L->c[a], L->b[a]) >= u2f(L->t_min)) { L->idx |= 1 << a; L->p[a] |= L->dim; }
            return;
        } else if (L->st == 1) {                            /* STEP */
            uint32_t t[3];
            for (int a = 0; a < 3; ++a) t[a] = f2u(fmaf(u2f(L->p[a]), L->c[a], L->b[a]));
            const int a = (t[0] <= t[1] && t[0] <= t[2]) ? 0 : (t[1] < t[0] && t[1] <= t[2]) ? 1 : 2;
            L->axis = 1 << a;
            L->t_min = t[a];
            if (!(L->idx & L->axis)) { L->st = 2; continue; }
            L->p[a] &= ~L->dim;
            L->idx ^= L->axis;
            L->st = 0;
        } else {                                            /* POP */
            if (--L->level == 0) { lane_finish(L, 0, 0); return; }
            L->node = L->stack[--L->sp];
            for (int a = 0; a < 3; ++a) L->p[a] &= ~L->dim;
            L->dim <<= 1;
            L->idx = 0;
            for (int a = 0; a < 3; ++a)
                if (u2f(L->dim) == u2f(L->p[a] & L->dim)) L->idx |= 1 << a;
            L->st = 1;
        }
    }
}

/* S lanes of one ray in lockstep: returns the iterations of the slowest (the
 * ray's critical path), the merged record in *m and the lanes' summed iterations. */
static int ray_dynamic(const float *o, const float *d, int S, Rec *m, int *lane_sum)
{
    Lane L[16];
    Shared sh = {0, -1, 0};
    for (int s = 0; s < S; ++s) lane_init(&L[s], o, d);
    int rounds = 0, left = S;
    while (left) {
        ++rounds;
        for (int s = 0; s < S; ++s)
            if (!L[s].done) { lane_iter(&L[s], &sh); if (L[s].done) --left; }
    }
    int best = -1, sum = 0;
    for (int s = 0; s < S; ++s) {
        sum += L[s].push;
        if (L[s].rec.ord >= 0 && (best < 0 || L[s].rec.ord < L[best].rec.ord)) best = s;
    }
    *m = best < 0 ? (Rec){6, 0, 0x7F800000u, -1, 0} : L[best].rec;
    *lane_sum = sum;
    return rounds;
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

enum { W = 1920, H = 1080, TX = W / 8, TY = H / 8 };
static float PITCH;
static int *FULL, *SPLIT;        /* per tile: longest lane, full walk / split (max over its S x 64 lane tasks) */
static long *SPLIT_WORK;         /* per tile: sum over the S waves of their longest lane */
static int *RSPLIT;              /* per tile, per-ray split: longest task */
static long *RSPLIT_WORK;        /* per tile, per-ray split: waves' longest tasks summed (tasks packed longest first) */
static int *DSPLIT;              /* per tile, per-ray split with dynamic claiming: longest task */
static long *DSPLIT_WORK;
static long BAD, RAYS;
static int NEXT;
static pthread_mutex_t MU = PTHREAD_MUTEX_INITIALIZER;

static void *worker(void *arg)
{
    (void)arg;
    const float o[3] = {1.5F, 1.5F, 1.5F};
    Rec seg[64];
    int full_push[64], seg_push[64][16], dyn_rounds[64];
    for (;;) {
        const int tile = __atomic_fetch_add(&NEXT, 1, __ATOMIC_RELAXED);
        if (tile >= TX * TY) return NULL;
        const int tx = tile % TX, ty = tile / TX;
        int full_max = 0, split_max = 0;
        int wave_max[64] = {0};                 /* S waves of 64 / S rays x S segments */
        long bad = 0;
        for (int l = 0; l < 64; ++l) {
            float d[3];
            camera(0.3F, PITCH, W, H, tx * 8 + l % 8, ty * 8 + l / 8, d);
            Rec full;
            walk(o, d, -1, -1, &full);
            full_push[l] = full.push;
            if (full.push > full_max) full_max = full.push;
            int best = -1;
            for (int s = 0; s < SEGS; ++s) {
                walk(o, d, s, EARLY ? full.ord : -1, &seg[s]);
                seg_push[l][s] = seg[s].push;
                if (seg[s].push > split_max) split_max = seg[s].push;
                const int w = l / (64 / SEGS);
                if (seg[s].push > wave_max[w]) wave_max[w] = seg[s].push;
                if (seg[s].ord >= 0 && (best < 0 || seg[s].ord < seg[best].ord)) best = s;
            }
            const Rec m = best < 0 ? (Rec){6, 0, 0x7F800000u, -1, 0} : seg[best];
            if (m.dir != full.dir || m.voxel != full.voxel || m.t != full.t) ++bad;
            Rec md;
            int lsum;
            dyn_rounds[l] = ray_dynamic(o, d, SEGS, &md, &lsum);
            if (md.dir != full.dir || md.voxel != full.voxel || md.t != full.t) ++bad;
        }
        long work = 0;
        for (int w = 0; w < SEGS; ++w) work += wave_max[w];
        /* per-ray split: rays longer than THETA % of the tile's longest take SEGS lanes */
        {
            int task[64 * 16], nt = 0, lmax = 0;
            for (int l = 0; l < 64; ++l) {
                if (full_push[l] * 100 > THETA * full_max) {
                    for (int s = 0; s < SEGS; ++s) task[nt++] = seg_push[l][s];
                } else
                    task[nt++] = full_push[l];
            }
            /* longest first, 64 to a wave */
            for (int i = 1; i < nt; ++i) { int v = task[i], j = i; while (j > 0 && task[j - 1] < v) { task[j] = task[j - 1]; --j; } task[j] = v; }
            long rw = 0;
            for (int i = 0; i < nt; i += 64) rw += task[i];
            lmax = task[0];
            RSPLIT[tile] = lmax;
            RSPLIT_WORK[tile] = rw;
            /* the same with dynamic claiming: a long ray's S lanes each cost its lockstep rounds */
            nt = 0;
            for (int l = 0; l < 64; ++l) {
                if (full_push[l] * 100 > THETA * full_max) {
                    for (int s = 0; s < SEGS; ++s) task[nt++] = dyn_rounds[l];
                } else
                    task[nt++] = full_push[l];
            }
            for (int i = 1; i < nt; ++i) { int v = task[i], j = i; while (j > 0 && task[j - 1] < v) { task[j] = task[j - 1]; --j; } task[j] = v; }
            rw = 0;
            for (int i = 0; i < nt; i += 64) rw += task[i];
            DSPLIT[tile] = task[0];
            DSPLIT_WORK[tile] = rw;
        }
        FULL[tile] = full_max;
        SPLIT[tile] = split_max;
        SPLIT_WORK[tile] = work;
        pthread_mutex_lock(&MU);
        BAD += bad;
        RAYS += 64;
        pthread_mutex_unlock(&MU);
    }
}

static int cmp_desc(const void *a, const void *b) { return *(const int *)b - *(const int *)a; }

#ifndef SPLIT_MODEL_NO_MAIN
int main(int argc, char **argv)
{
    if (argc < 6) { fprintf(stderr, "usage: split_model nodes.bin depth pitch L S [threads]\n"); return 2; }
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
    LEVEL = atoi(argv[4]);
    SEGS = atoi(argv[5]);
    const int threads = argc > 6 ? atoi(argv[6]) : 8;
    EARLY = argc > 7 ? atoi(argv[7]) : 0;
    THETA = argc > 8 ? atoi(argv[8]) : 50;
    if (LEVEL < 1 || LEVEL >= DEPTH || SEGS < 1 || 64 % SEGS) { fprintf(stderr, "need 1 <= L < depth, S | 64\n"); return 2; }
    FULL = calloc(TX * TY, sizeof *FULL);
    SPLIT = calloc(TX * TY, sizeof *SPLIT);
    SPLIT_WORK = calloc(TX * TY, sizeof *SPLIT_WORK);
    RSPLIT = calloc(TX * TY, sizeof *RSPLIT);
    RSPLIT_WORK = calloc(TX * TY, sizeof *RSPLIT_WORK);
    DSPLIT = calloc(TX * TY, sizeof *DSPLIT);
    DSPLIT_WORK = calloc(TX * TY, sizeof *DSPLIT_WORK);
    pthread_t th[256];
    for (int k = 0; k < threads; ++k) pthread_create(&th[k], NULL, worker, NULL);
    for (int k = 0; k < threads; ++k) pthread_join(th[k], NULL);
    int *sorted = malloc(sizeof(int) * TX * TY);
    memcpy(sorted, FULL, sizeof(int) * TX * TY);
    qsort(sorted, TX * TY, sizeof(int), cmp_desc);
    printf("{\"early\": %d, \"pitch\": %g, \"L\": %d, \"S\": %d, \"rays\": %ld, \"records_differ\": %ld, "
           "\"longest_tile_full\": %d, \"tile_full_p99.9\": %d, \"tile_full_p99\": %d, \"tile_full_p90\": %d,",
           EARLY, PITCH, LEVEL, SEGS, RAYS, BAD, sorted[0], sorted[TX * TY / 1000], sorted[TX * TY / 100], sorted[TX * TY / 10]);
    /* split the tiles whose longest lane exceeds T: the critical path becomes the
     * longest lane of what is left (unsplit tiles' longest lane, split tiles'
     * longest segment lane); the work, the sum of the waves' longest lanes */
    printf(" \"by_threshold\": [");
    const int Ts[] = {400, 300, 250, 200, 150, 100};
    for (size_t k = 0; k < sizeof Ts / sizeof Ts[0]; ++k) {
        long base = 0, work = 0;
        int crit = 0, n = 0;
        for (int t = 0; t < TX * TY; ++t) {
            base += FULL[t];
            if (FULL[t] > Ts[k]) {
                ++n;
                work += SPLIT_WORK[t];
                if (SPLIT[t] > crit) crit = SPLIT[t];
            } else {
                work += FULL[t];
                if (FULL[t] > crit) crit = FULL[t];
            }
        }
        long rwork = 0, dwork = 0;
        int rcrit = 0, dcrit = 0;
        for (int t = 0; t < TX * TY; ++t) {
            if (FULL[t] > Ts[k]) { rwork += RSPLIT_WORK[t]; if (RSPLIT[t] > rcrit) rcrit = RSPLIT[t];
                                   dwork += DSPLIT_WORK[t]; if (DSPLIT[t] > dcrit) dcrit = DSPLIT[t]; }
            else { rwork += FULL[t]; if (FULL[t] > rcrit) rcrit = FULL[t]; dwork += FULL[t]; if (FULL[t] > dcrit) dcrit = FULL[t]; }
        }
        printf("%s{\"T\": %d, \"tiles_split\": %d, \"critical_path\": %d, \"work_vs_unsplit\": %.4f, "
               "\"per_ray_critical_path\": %d, \"per_ray_work_vs_unsplit\": %.4f, "
               "\"dynamic_critical_path\": %d, \"dynamic_work_vs_unsplit\": %.4f}", k ? ", " : "",
               Ts[k], n, crit, (double)work / base, rcrit, (double)rwork / base, dcrit, (double)dwork / base);
    }
    printf("]}\n");
    return BAD != 0;
}
#endif
