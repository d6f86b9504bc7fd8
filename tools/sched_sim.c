/* sched_sim.c -- lockstep model of one 64-lane wavefront running the render
 * kernel's traversal loop (och_kernels.hip ray_iterate, packed layout), to
 * price schedule changes before writing them in HIP.
 *
 * Design tool only (not product, not a checker): it walks the DAG with the
 * host's own RCPPS, runs 64 rays of an 8x8 tile in lockstep through the
 * kernel's phases, and charges each phase's VALU instruction count (taken
 * from the gfx950 ISA of the current kernel, see the table below) whenever
 * at least one lane of the wave executes it.  Output: VALU instructions per
 * wave, iterations per wave and per-phase lane utilisation, per schedule.
 *
 * Build: gcc -O2 -msse2 -o /tmp/sched_sim tools/sched_sim.c -lm
 * Input: raw uint32 nodes[n][8] (1-based h_octree pool), e.g. written by
 *   ort.build_terrain(12).nodes.astype(np.uint32).tofile("d12_nodes.bin")
 * Usage: sched_sim nodes.bin depth pitch [tile_stride [schedule [threshold]]]
 * (Schedule 4, in-block wave merging, went with the retired merge arm:
 * profiles/r05/retired/tools/sched_sim_merge.diff.) */
#include <immintrin.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

typedef struct {
    float c[3], b[3];
    uint32_t p[3], inv, idx, dim, cur, t_min, axis, child;
    uint32_t stack[32];
    int sp, level, stepping, pending, done;
    int iters, push, step, pop;
} Ray;

static const uint32_t *N;
static int DEPTH;

static void ray_setup(Ray *r, const float *o, const float *d)
{
    memset(r, 0, sizeof *r);
    for (int a = 0; a < 3; ++a) {
        const int pos = 0.0F < d[a];
        r->inv |= pos << a;
        const float refl = fabsf((pos ? 3.0F : 0.0F) - o[a]);
        const float dn = u2f(f2u(d[a]) | 0x80000000u);
        float c = _mm_cvtss_f32(_mm_rcp_ss(_mm_set_ss(dn)));
        r->c[a] = c;
        r->b[a] = u2f(f2u(c * refl) ^ 0x80000000u);
        if ((f2u(c) & 0x7FFFFFFFu) == 0x7F800000u) { r->c[a] = 0.0F; r->b[a] = u2f(0xFFC00000u); }
        r->p[a] = f2u(refl) & 0x3FC00000u;
        r->idx |= (r->p[a] == 0x3FC00000u) << a;
    }
    r->dim = 1u << 22;
    r->cur = 1;   /* root id (1-based) */
    r->level = 1;
    r->axis = 8;
}

/* the PUSH test: child of cur at (idx ^ inv) */
static void push(Ray *r)
{
    ++r->push;
    const uint32_t ch = N[(size_t)(r->cur - 1) * 8 + ((r->idx ^ r->inv) & 7)];
    if (ch) { r->child = ch; r->pending = 1; }
    else r->stepping = 1;
}

static int active(const Ray *r) { return r->level >= 1 && r->level <= DEPTH; }

/* ISA VALU counts per block of the current packed render loop (gfx950). */
enum { C_STEP = 10, C_ADV = 7, C_POPPRE = 3, C_POP = 14, C_DESCPRE = 3, C_DESC = 22, C_PUSHPRE = 2,
       C_PUSHTEST = 4, C_PUSHLOAD = 4, C_LOOP = 1 };

typedef struct { double valu, iters, waves, lane_step, lane_desc, lane_push, exec_step, exec_desc, exec_push, rays_it, exec_adv, exec_popper, exec_pop, exec_descbody, exec_load; } Stats;

/* STEP of one lane (+ advance or POP).  Returns 1 advance, 2 POP, 3 MISS. */
static int step_one(Ray *r)
{
    ++r->step;
    uint32_t t[3];
    for (int a = 0; a < 3; ++a) t[a] = f2u(fmaf(u2f(r->p[a]), r->c[a], r->b[a]));
    uint32_t tm = t[0] < t[1] ? t[0] : t[1]; tm = tm < t[2] ? tm : t[2];
    const int ax = t[0] == tm ? 0 : (t[1] == tm ? 1 : 2);
    r->axis = 1u << ax; r->t_min = tm;
    if (r->idx & r->axis) { r->p[ax] ^= r->dim; r->idx ^= r->axis; r->stepping = 0; return 1; }
    ++r->pop;
    if (--r->level == 0) return 3;
    r->cur = r->stack[--r->sp];
    for (int a = 0; a < 3; ++a) r->p[a] &= ~r->dim;
    r->dim <<= 1;
    r->idx = 0;
    for (int a = 0; a < 3; ++a) r->idx |= ((r->p[a] & r->dim) != 0) << a;
    return 2;
}

static int SCHED = 0;
/* schedule 0: iterations in which some lane's PUSH loads a slot word at a node of
 * level <= DEPTH - 2 (the loads left if the bottom two levels' occupancy rode in
 * registers), and loads per node level */
static double IT_LOAD_ABOVE2 = 0, LOADS_AT[40];
static int THRESH = 0;   /* schedule 0: skip a phase needed by fewer than THRESH lanes (at most one iteration) */

/* schedule 0: the current kernel (step, descend, push; each phase skipped when no lane needs it) */
static void wave_sched0(Ray *R, int n, Stats *S)
{
    for (int i = 0; i < n; ++i) push(&R[i]);
    int skipped_step = 0, skipped_desc = 0;
    for (;;) {
        int any = 0;
        for (int i = 0; i < n; ++i) any |= active(&R[i]);
        if (!any) break;
        S->iters += 1;
        int nload_above2 = 0; int ns = 0, nadv = 0, npopper = 0, npop = 0, nd = 0, ndesc = 0, np = 0, nload = 0;
        int want_step = 0, want_desc = 0;
        for (int i = 0; i < n; ++i) { want_step += active(&R[i]) && R[i].stepping; want_desc += R[i].pending; }
        const int run_step = want_step >= THRESH || skipped_step;
        const int run_desc = want_desc >= THRESH || skipped_desc;
        skipped_step = want_step && !run_step;
        skipped_desc = want_desc && !run_desc;
        for (int i = 0; i < n; ++i) {
            Ray *r = &R[i];
            if (!active(r)) continue;
            ++r->iters;
            if (r->stepping && run_step) {
                ++ns; ++r->step;
                uint32_t t[3];
                for (int a = 0; a < 3; ++a) t[a] = f2u(fmaf(u2f(r->p[a]), r->c[a], r->b[a]));
                uint32_t tm = t[0] < t[1] ? t[0] : t[1]; tm = tm < t[2] ? tm : t[2];
                const int ax = t[0] == tm ? 0 : (t[1] == tm ? 1 : 2);
                r->axis = 1u << ax; r->t_min = tm;
                if (r->idx & r->axis) { ++nadv; r->p[ax] ^= r->dim; r->idx ^= r->axis; r->stepping = 0; }
                else {
                    ++npopper; ++r->pop;
                    if (--r->level == 0) continue;
                    ++npop;
                    r->cur = r->stack[--r->sp];
                    for (int a = 0; a < 3; ++a) r->p[a] &= ~r->dim;
                    r->dim <<= 1;
                    r->idx = 0;
                    for (int a = 0; a < 3; ++a) r->idx |= ((r->p[a] & r->dim) != 0) << a;
                }
            }
        }
        for (int i = 0; i < n; ++i) {
            Ray *r = &R[i];
            if (!r->pending || !run_desc) continue;
            r->pending = 0; ++nd;
            if (r->level == DEPTH) { r->level = DEPTH + 1; continue; }
            ++ndesc;
            r->stack[r->sp++] = r->cur; ++r->level; r->cur = r->child; r->dim >>= 1;
            uint32_t ni = 0;
            for (int a = 0; a < 3; ++a) {
                const uint32_t mid = r->p[a] | r->dim;
                const int up = fmaf(u2f(mid), r->c[a], r->b[a]) >= u2f(r->t_min);
                ni |= up << a; if (up) r->p[a] = mid;
            }
            r->idx = ni;
        }
        int fresh[64] = {0};
        for (int i = 0; i < n; ++i) {
            Ray *r = &R[i];
            if (r->stepping || r->pending || !active(r)) continue;
            ++np; push(r); nload += r->pending;
            if (r->pending) { LOADS_AT[r->level] += 1; nload_above2 += r->level <= DEPTH - 2; }
            fresh[i] = r->stepping;
        }
        if (SCHED == 1) {     /* second STEP + PUSH test in the same iteration for lanes whose PUSH failed */
            int n2 = 0, nadv2 = 0, npop2 = 0, np2 = 0, nload2 = 0;
            for (int i = 0; i < n; ++i) {
                Ray *r = &R[i];
                if (!fresh[i] || !active(r)) continue;
                ++n2;
                const int k = step_one(r);
                nadv2 += k == 1; npop2 += k == 2;
                if (k == 1) { ++np2; push(r); nload2 += r->pending; }
            }
            if (n2) S->valu += C_STEP + C_POPPRE;
            if (nadv2) S->valu += C_ADV;
            if (npop2) S->valu += C_POP;
            if (np2) S->valu += C_PUSHTEST;
            if (nload2) S->valu += C_PUSHLOAD;
        }
        S->valu += C_LOOP + C_PUSHPRE;
        if (ns) { S->valu += C_STEP; S->exec_step += 1; S->lane_step += ns; }
        if (nadv) { S->valu += C_ADV; S->exec_adv += 1; }
        if (npopper) { S->valu += C_POPPRE; S->exec_popper += 1; }
        if (npop) { S->valu += C_POP; S->exec_pop += 1; }
        if (nd) { S->valu += C_DESCPRE; S->exec_desc += 1; S->lane_desc += nd; }
        if (ndesc) { S->valu += C_DESC; S->exec_descbody += 1; }
        if (np) { S->valu += C_PUSHTEST; S->exec_push += 1; S->lane_push += np; }
        if (nload) { S->valu += C_PUSHLOAD; S->exec_load += 1; }
        if (nload_above2) IT_LOAD_ABOVE2 += 1;
    }
    for (int i = 0; i < n; ++i) S->rays_it += R[i].iters;
    S->waves += 1;
}

/* schedules 2 and 3: the merged kernel (och_kernels.hip ray_push_descend,
 * OCH_MERGED_DESCEND): phase A = STEP (+ advance or POP) for stepping lanes,
 * phase B = PUSH (+ descent when the child is present) for the others.
 * Schedule 3 repeats phase A for lanes that just popped until none pops.
 * VALU per block from the gfx950 ISA of the merged loop. */
enum { M_LOOP = 4, M_AENTRY = 1, M_STEP = 10, M_ADV = 7, M_POP = 15, M_BENTRY = 8, M_DESC = 25 };

static void wave_merged(Ray *R, int n, Stats *S, int popwhile)
{
    int mode[64];   /* 0 push, 1 stepping */
    for (int i = 0; i < n; ++i) mode[i] = R[i].stepping ? 1 : 0;
    for (;;) {
        int any = 0;
        for (int i = 0; i < n; ++i) any |= active(&R[i]);
        if (!any) break;
        S->iters += 1;
        S->valu += M_LOOP + M_AENTRY;
        int popped[64];
        for (int i = 0; i < n; ++i) popped[i] = 1;   /* first pass: every stepping lane */
        for (int pass = 0;; ++pass) {
            int ns = 0, nadv = 0, npop = 0;
            int again[64] = {0};
            for (int i = 0; i < n; ++i) {
                Ray *r = &R[i];
                if (!active(r) || mode[i] != 1 || !popped[i]) continue;
                ++ns;
                if (pass == 0) ++r->iters;
                const int k = step_one(r);
                if (k == 1) { ++nadv; mode[i] = 0; }
                else { ++npop; again[i] = k == 2; }
            }
            if (ns) S->valu += M_STEP;
            if (nadv) S->valu += M_ADV;
            if (npop) S->valu += M_POP;
            if (pass) S->valu += 3;                       /* the repeat test */
            if (!popwhile) break;
            int more = 0;
            for (int i = 0; i < n; ++i) { popped[i] = again[i]; more |= again[i]; }
            if (!more) break;
        }
        int nb = 0, npres = 0;
        for (int i = 0; i < n; ++i) {
            Ray *r = &R[i];
            if (!active(r) || mode[i] != 0) continue;
            ++nb; ++r->push;
            const uint32_t ch = N[(size_t)(r->cur - 1) * 8 + ((r->idx ^ r->inv) & 7)];
            if (!ch) { mode[i] = 1; continue; }
            ++npres;
            if (r->level == DEPTH) { r->level = DEPTH + 1; continue; }
            r->stack[r->sp++] = r->cur; ++r->level; r->cur = ch; r->dim >>= 1;
            uint32_t ni = 0;
            for (int a = 0; a < 3; ++a) {
                const uint32_t mid = r->p[a] | r->dim;
                const int up = fmaf(u2f(mid), r->c[a], r->b[a]) >= u2f(r->t_min);
                ni |= up << a; if (up) r->p[a] = mid;
            }
            r->idx = ni;
        }
        if (nb) S->valu += M_BENTRY;
        if (npres) S->valu += M_DESC;
    }
    for (int i = 0; i < n; ++i) S->rays_it += R[i].iters;
    S->waves += 1;
}

static void wave_merged_init(Ray *R, int n, Stats *S, int popwhile) { wave_merged(R, n, S, popwhile); }

/* schedule 5: the round-5 kernel -- merged PUSH + descend, STEP with the POP
 * chain (a POP goes straight to the level of p_a's lowest set bit above the
 * current one and advances there; t < 0 or NaN: one POP).  Counts, per
 * iteration, whether any lane runs each block of the loop (the wave issues a
 * block's VALU when one lane needs it), and the lanes in it. */
static double CH_IT, CH_STEP, CH_POP, CH_ADV, CH_PUSH, CH_DESC, CH_LSTEP, CH_LPOP, CH_LADV, CH_LPUSH, CH_LDESC, CH_ACT;
static int ctz32(uint32_t x) { return __builtin_ctz(x); }
static void wave_chain(Ray *R, int n, Stats *S)
{
    int mode[64];   /* 0 STEP due, 1 PUSH due */
    for (int i = 0; i < n; ++i) mode[i] = R[i].stepping ? 0 : 1;
    for (;;) {
        int act = 0;
        for (int i = 0; i < n; ++i) act += active(&R[i]);
        if (!act) break;
        CH_IT += 1; CH_ACT += act;
        int ns = 0, npop = 0, nadv = 0, np = 0, nd = 0;
        for (int i = 0; i < n; ++i) {
            Ray *r = &R[i];
            if (!active(r) || mode[i] != 0) continue;
            ++ns; ++r->iters;
            uint32_t t[3];
            for (int a = 0; a < 3; ++a) t[a] = f2u(fmaf(u2f(r->p[a]), r->c[a], r->b[a]));
            uint32_t tm = t[0] < t[1] ? t[0] : t[1]; tm = tm < t[2] ? tm : t[2];
            const int ax = t[0] == tm ? 0 : (t[1] == tm ? 1 : 2);
            r->axis = 1u << ax; r->t_min = tm;
            if (r->idx & r->axis) { ++nadv; r->p[ax] ^= r->dim; r->idx ^= r->axis; mode[i] = 1; continue; }
            ++npop;
            uint32_t mx = t[0] > t[1] ? t[0] : t[1]; mx = mx > t[2] ? mx : t[2];
            const int chain = mx < 0x80000000u;
            const uint32_t nd2 = 0u - 2u * r->dim;
            const uint32_t up = ((chain ? r->p[ax] : nd2) & nd2) | (1u << 23);
            const int k = ctz32(up);
            const int lv_new = 23 - k;          /* node level of the popped-to cell: dim = 1 << k */
            if (k >= 23) { r->level = 0; continue; }   /* MISS */
            r->sp -= r->level - lv_new; r->level = lv_new;
            r->cur = r->stack[r->sp];
            for (int a = 0; a < 3; ++a) r->p[a] &= 0u - (1u << k);
            r->dim = 1u << k;
            r->idx = 0;
            for (int a = 0; a < 3; ++a) r->idx |= ((r->p[a] >> k) & 1u) << a;
            if (chain) { ++nadv; r->p[ax] ^= r->dim; r->idx ^= r->axis; mode[i] = 1; }
        }
        for (int i = 0; i < n; ++i) {
            Ray *r = &R[i];
            if (!active(r) || mode[i] != 1) continue;
            ++np; ++r->push;
            const uint32_t ch = N[(size_t)(r->cur - 1) * 8 + ((r->idx ^ r->inv) & 7)];
            if (!ch) { mode[i] = 0; continue; }
            ++nd;
            if (r->level == DEPTH) { r->level = DEPTH + 1; continue; }
            r->stack[r->sp++] = r->cur; ++r->level; r->cur = ch; r->dim >>= 1;
            uint32_t ni = 0;
            for (int a = 0; a < 3; ++a) {
                const uint32_t mid = r->p[a] | r->dim;
                const int up = fmaf(u2f(mid), r->c[a], r->b[a]) >= u2f(r->t_min);
                ni |= up << a; if (up) r->p[a] = mid;
            }
            r->idx = ni;
        }
        CH_STEP += ns > 0; CH_POP += npop > 0; CH_ADV += nadv > 0; CH_PUSH += np > 0; CH_DESC += nd > 0;
        CH_LSTEP += ns; CH_LPOP += npop; CH_LADV += nadv; CH_LPUSH += np; CH_LDESC += nd;
        S->iters += 1;
    }
    for (int i = 0; i < n; ++i) S->rays_it += R[i].iters;
    S->waves += 1;
}

static void camera(float yaw, float pitch, int W, int H, int col, int row, float *d)
{
    /* tree_camera::update_position (ORT/test_och_h_octree.cpp:87-138), float math */
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

int main(int argc, char **argv)
{
    if (argc < 4) { fprintf(stderr, "usage: sched_sim nodes.bin depth pitch [tile_stride]\n"); return 2; }
    FILE *fp = fopen(argv[1], "rb");
    fseek(fp, 0, SEEK_END); long sz = ftell(fp); fseek(fp, 0, SEEK_SET);
    uint32_t *buf = malloc(sz);
    if (fread(buf, 1, sz, fp) != (size_t)sz) return 1;
    fclose(fp);
    N = buf; DEPTH = atoi(argv[2]);
    const float pitch = (float)atof(argv[3]);
    const int stride = argc > 4 ? atoi(argv[4]) : 1;
    SCHED = argc > 5 ? atoi(argv[5]) : 0;
    THRESH = argc > 6 ? atoi(argv[6]) : 0;
    const int W = 1920, H = 1080;
    const float o[3] = {1.5F, 1.5F, 1.5F};
    Stats S = {0};
    Ray R[64];
    int tile = 0;
    for (int ty = 0; ty < H / 8; ++ty)
        for (int tx = 0; tx < W / 8; ++tx, ++tile) {
            if (tile % stride) continue;
            for (int l = 0; l < 64; ++l) {
                float d[3];
                camera(0.3F, pitch, W, H, tx * 8 + l % 8, ty * 8 + l / 8, d);
                ray_setup(&R[l], o, d);
            }
            if (SCHED >= 2) {
                /* merged kernel: ray_init does the root PUSH + descent itself */
                for (int l = 0; l < 64; ++l) {
                    Ray *r = &R[l];
                    const uint32_t ch = N[(size_t)(r->cur - 1) * 8 + ((r->idx ^ r->inv) & 7)];
                    ++r->push;
                    if (!ch) { r->stepping = 1; continue; }
                    r->stack[r->sp++] = r->cur; ++r->level; r->cur = ch; r->dim >>= 1;
                    uint32_t ni = 0;
                    for (int a = 0; a < 3; ++a) {
                        const uint32_t mid = r->p[a] | r->dim;
                        const int up = fmaf(u2f(mid), r->c[a], r->b[a]) >= u2f(r->t_min);
                        ni |= up << a; if (up) r->p[a] = mid;
                    }
                    r->idx = ni;
                }
                /* mode from the root PUSH: stepping lanes start in phase A */
                Ray tmp[64];
                memcpy(tmp, R, sizeof tmp);
                if (SCHED == 5) wave_chain(R, 64, &S); else wave_merged_init(R, 64, &S, SCHED == 3);
            } else
                wave_sched0(R, 64, &S);
        }
    printf("{\"waves\": %.0f, \"valu_per_wave\": %.1f, \"iters_per_wave\": %.2f, \"ray_iters\": %.2f, "
           "\"lane_util_iter\": %.3f, \"step_util\": %.3f, \"desc_util\": %.3f, \"push_util\": %.3f, "
           "\"step_exec_frac\": %.3f, \"desc_exec_frac\": %.3f, \"adv_frac\": %.3f, \"pop_frac\": %.3f, "
           "\"load_frac\": %.3f}\n",
           S.waves, S.valu / S.waves, S.iters / S.waves, S.rays_it / S.waves / 64, S.rays_it / S.iters / 64,
           S.lane_step / S.exec_step / 64, S.lane_desc / S.exec_desc / 64, S.lane_push / S.exec_push / 64,
           S.exec_step / S.iters, S.exec_desc / S.iters, S.exec_adv / S.iters, S.exec_popper / S.iters,
           S.exec_load / S.iters);
    if (SCHED == 0) {
        fprintf(stderr, "load_frac_above_bottom2 %.3f\nloads per node level:", IT_LOAD_ABOVE2 / S.iters);
        for (int l = 1; l <= DEPTH; ++l) fprintf(stderr, " %.0f", LOADS_AT[l]);
        fprintf(stderr, "\n");
    }
    if (SCHED == 5)
        printf("{\"iters\": %.0f, \"active_lanes\": %.2f, \"wave_frac\": {\"step\": %.3f, \"pop\": %.3f, \"advance\": %.3f, "
               "\"push\": %.3f, \"descent\": %.3f}, \"lanes_when_run\": {\"step\": %.1f, \"pop\": %.1f, \"advance\": %.1f, "
               "\"push\": %.1f, \"descent\": %.1f}}\n",
               CH_IT, CH_ACT / CH_IT, CH_STEP / CH_IT, CH_POP / CH_IT, CH_ADV / CH_IT, CH_PUSH / CH_IT, CH_DESC / CH_IT,
               CH_LSTEP / CH_STEP, CH_LPOP / CH_POP, CH_LADV / CH_ADV, CH_LPUSH / CH_PUSH, CH_LDESC / CH_DESC);
    return 0;
}
