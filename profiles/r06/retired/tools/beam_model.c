/* beam_model.c -- prices a per-tile "beam" start for camera rays (design tool,
 * not product).  Laine & Karras' beam optimisation starts a tile's rays at a
 * distance the tile's beam provably reaches before any voxel.  In the walk's
 * own arithmetic (tools/split_model.c's restatement of ORT/och_h_octree.h:292-447)
 * the exact form is a PUSH test: a present child whose exit t (the minimum of
 * its three lower planes' t, what the next STEP would compute) is below the
 * tile's bound t_b is treated as empty.  Every voxel inside that child is
 * entered at a t no larger than the child's exit t, so it cannot be a hit at or
 * beyond t_b.
 *
 * This tool takes the ideal bound -- t_b = the smallest hit t of the tile's 64
 * rays, which no beam pass can beat -- and counts, per wave (an 8x8 tile), the
 * longest lane's PUSH tests and descents with and without it, and checks every
 * record against the full walk.  If the ideal does not pay, no beam does.
 *
 * Build: gcc -O2 -msse2 -o /tmp/beam_model profiles/r06/retired/tools/beam_model.c -lm -lpthread
 * Usage: beam_model nodes.bin depth pitch [threads [margin_ulps]]
 *   margin_ulps: t_b lowered by this many float ulps (0 = the ideal bound). */
#define SPLIT_MODEL_NO_MAIN
#include "../../../../tools/split_model.c"

static int MARGIN;

/* The full walk, with present children exiting below tb (unsigned, non-negative
 * floats) treated as empty.  push/desc: PUSH tests, descents (slot loads). */
static void walk_beam(const float *o, const float *d, uint32_t tb, Rec *out, int *desc_out)
{
    float c[3], b[3];
    uint32_t p[3], stack[32];
    int inv = 0, idx = 0, sp = 0, level = 1, axis = 8, push = 0, desc = 0;
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
    enum { PUSH, STEP, POP } st = PUSH;
    for (;;) {
        if (st == PUSH) {
            ++push;
            const uint32_t ch = N[(size_t)(node - 1) * 8 + ((idx ^ inv) & 7)];
            if (!ch) { st = STEP; continue; }
            if (tb) {
                uint32_t e = 0xFFFFFFFFu;
                for (int a = 0; a < 3; ++a) {
                    const uint32_t t = f2u(fmaf(u2f(p[a]), c[a], b[a]));
                    if (t < e) e = t;
                }
                if (e < tb) { st = STEP; continue; }
            }
            ++desc;
            if (level++ == DEPTH) {
                out->dir = (axis >> 1) + 3 * ((inv & axis) == 0);
                out->voxel = ch;
                out->t = t_min;
                out->ord = 0;
                out->push = push;
                *desc_out = desc;
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
                *desc_out = desc;
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

static long S_PUSH[2], S_DESC[2], S_BAD, S_RAYS, S_TILES_WALK;
static int B_NEXT;
static int *TILE_PUSH[2];

static void *bworker(void *arg)
{
    (void)arg;
    const float o[3] = {1.5F, 1.5F, 1.5F};
    for (;;) {
        const int tile = __atomic_fetch_add(&B_NEXT, 1, __ATOMIC_RELAXED);
        if (tile >= TX * TY) return NULL;
        const int tx = tile % TX, ty = tile / TX;
        float dirs[64][3];
        Rec full[64];
        int dfull[64];
        uint32_t tb = 0xFFFFFFFFu;
        for (int l = 0; l < 64; ++l) {
            camera(0.3F, PITCH, W, H, tx * 8 + l % 8, ty * 8 + l / 8, dirs[l]);
            walk_beam((const float *)(const void *)&(float[3]){1.5F, 1.5F, 1.5F}, dirs[l], 0, &full[l], &dfull[l]);
            if (full[l].voxel && full[l].t < tb) tb = full[l].t;
        }
        if (tb == 0xFFFFFFFFu) tb = 0;                  /* no hit in the tile: nothing to bound by */
        else tb = tb > (uint32_t)MARGIN ? tb - (uint32_t)MARGIN : 0;
        int mp[2] = {0, 0}, md[2] = {0, 0};
        long bad = 0;
        for (int l = 0; l < 64; ++l) {
            if (full[l].push > mp[0]) mp[0] = full[l].push;
            if (dfull[l] > md[0]) md[0] = dfull[l];
            Rec r;
            int dd;
            walk_beam(o, dirs[l], tb, &r, &dd);
            if (r.dir != full[l].dir || r.voxel != full[l].voxel || r.t != full[l].t) ++bad;
            if (r.push > mp[1]) mp[1] = r.push;
            if (dd > md[1]) md[1] = dd;
        }
        TILE_PUSH[0][tile] = mp[0];
        TILE_PUSH[1][tile] = mp[1];
        pthread_mutex_lock(&MU);
        for (int k = 0; k < 2; ++k) { S_PUSH[k] += mp[k]; S_DESC[k] += md[k]; }
        S_BAD += bad;
        S_RAYS += 64;
        S_TILES_WALK += tb != 0;
        pthread_mutex_unlock(&MU);
    }
}

int main(int argc, char **argv)
{
    if (argc < 4) { fprintf(stderr, "usage: beam_model nodes.bin depth pitch [threads [margin_ulps]]\n"); return 2; }
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
    const int threads = argc > 4 ? atoi(argv[4]) : 8;
    MARGIN = argc > 5 ? atoi(argv[5]) : 0;
    for (int k = 0; k < 2; ++k) TILE_PUSH[k] = calloc(TX * TY, sizeof(int));
    pthread_t th[256];
    for (int k = 0; k < threads; ++k) pthread_create(&th[k], NULL, bworker, NULL);
    for (int k = 0; k < threads; ++k) pthread_join(th[k], NULL);
    int crit[2] = {0, 0};
    for (int t = 0; t < TX * TY; ++t)
        for (int k = 0; k < 2; ++k) if (TILE_PUSH[k][t] > crit[k]) crit[k] = TILE_PUSH[k][t];
    printf("{\"pitch\": %g, \"margin_ulps\": %d, \"rays\": %ld, \"records_differ\": %ld, \"tiles_with_hits\": %ld, "
           "\"wave_push\": [%ld, %ld], \"wave_desc\": [%ld, %ld], \"push_ratio\": %.4f, \"desc_ratio\": %.4f, "
           "\"longest_tile_push\": [%d, %d]}\n",
           PITCH, MARGIN, S_RAYS, S_BAD, S_TILES_WALK, S_PUSH[0], S_PUSH[1], S_DESC[0], S_DESC[1],
           (double)S_PUSH[1] / S_PUSH[0], (double)S_DESC[1] / S_DESC[0], crit[0], crit[1]);
    return S_BAD != 0;
}
