/* help_model.c -- prices "helper lanes" for the render loop's throughput
 * (design tool, not product).  A wave of 64 rays (an 8x8 tile) runs until its
 * longest ray ends; lanes whose rays end early idle (lane utilisation 0.53).
 * Here a lane whose ray has ended joins a ray of its wave that is still
 * walking: it walks that ray from the root and claims the present level-L
 * cells no lane of that ray has claimed yet (first come, first served, the
 * split's dynamic claiming, tools/split_model.c), so the ray's remaining
 * segments are shared.  Exact by the split's argument.  Lockstep model: one
 * PUSH test per lane per iteration; a lane switching to a ray pays `setup`
 * iterations first.  Output: iterations per wave against the plain walk, and
 * the lane utilisation.
 *
 * Build: gcc -O2 -msse2 -o /tmp/help_model profiles/r06/retired/tools/help_model.c -lm -lpthread
 * Usage: help_model nodes.bin depth pitch L setup [threads [tile_stride]] */
#define SPLIT_MODEL_NO_MAIN
#include "../../../../tools/split_model.c"

static int SETUP, STRIDE = 1;
static long BASE_IT, HELP_IT, RAY_IT;
static int NEXT2;

typedef struct { Lane L; int ray, wait, owner; } HLane;

static void *hworker(void *arg)
{
    (void)arg;
    const float o[3] = {1.5F, 1.5F, 1.5F};
    float dirs[64][3];
    for (;;) {
        const int tile = __atomic_fetch_add(&NEXT2, STRIDE, __ATOMIC_RELAXED);
        if (tile >= TX * TY) return NULL;
        const int tx = tile % TX, ty = tile / TX;
        Shared sh[64];
        int alive[64], lanes_on[64], owner_on[64];
        HLane HL[64];
        long base = 0, ray_it = 0;
        for (int l = 0; l < 64; ++l) {
            camera(0.3F, PITCH, W, H, tx * 8 + l % 8, ty * 8 + l / 8, dirs[l]);
            Rec full;
            walk(o, dirs[l], -1, -1, &full);
            if (full.push > base) base = full.push;
            sh[l] = (Shared){0, -1, 0};
            lane_init(&HL[l].L, o, dirs[l]);
            HL[l].ray = l;
            HL[l].wait = 0;
            HL[l].owner = 1;
            alive[l] = 1;
            lanes_on[l] = 1;
            owner_on[l] = 1;
        }
        int rounds = 0;
        for (;;) {
            if (rounds > 100000) { fprintf(stderr, "runaway tile %d\n", tile); break; }
            int any = 0;
            for (int l = 0; l < 64; ++l) any |= alive[l];
            if (!any) break;
            ++rounds;
            for (int l = 0; l < 64; ++l) {
                HLane *h = &HL[l];
                if (h->ray < 0) continue;
                if (h->wait) { --h->wait; ++ray_it; continue; }
                if (!h->L.done) { lane_iter(&h->L, &sh[h->ray]); ++ray_it; }
                if (h->L.done) {
                    --lanes_on[h->ray];
                    if (h->owner) { owner_on[h->ray] = 0; sh[h->ray].closed = 1; }   /* every segment taken, or its HIT found */
                    if (lanes_on[h->ray] == 0) alive[h->ray] = 0;
                    h->owner = 0;
                    /* join the ray with the fewest lanes among those whose owner still walks */
                    int best = -1;
                    for (int r = 0; r < 64; ++r)
                        if (owner_on[r] && (best < 0 || lanes_on[r] < lanes_on[best])) best = r;
                    h->ray = best;
                    if (best >= 0) {
                        ++lanes_on[best];
                        lane_init(&h->L, o, dirs[best]);
                        h->wait = SETUP;
                    }
                }
            }
        }
        pthread_mutex_lock(&MU);
        BASE_IT += base;
        HELP_IT += rounds;
        RAY_IT += ray_it;
        pthread_mutex_unlock(&MU);
    }
}

int main(int argc, char **argv)
{
    if (argc < 6) { fprintf(stderr, "usage: help_model nodes.bin depth pitch L setup [threads]\n"); return 2; }
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
    SETUP = atoi(argv[5]);
    const int threads = argc > 6 ? atoi(argv[6]) : 8;
    STRIDE = argc > 7 ? atoi(argv[7]) : 1;
    pthread_t th[256];
    for (int k = 0; k < threads; ++k) pthread_create(&th[k], NULL, hworker, NULL);
    for (int k = 0; k < threads; ++k) pthread_join(th[k], NULL);
    printf("{\"pitch\": %g, \"L\": %d, \"setup\": %d, \"wave_iterations_plain\": %ld, \"wave_iterations_helped\": %ld, "
           "\"ratio\": %.4f}\n", PITCH, LEVEL, SETUP, BASE_IT, HELP_IT, (double)HELP_IT / BASE_IT);
    return 0;
}
