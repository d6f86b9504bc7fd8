// och_kernels.hip -- gfx950 (CDNA4) kernels of the SVO-DAG ray caster.
//
// One ray per lane of a 64-wide wavefront.  Per-ray state (reflected-frame
// position bits, ray coefficients, child index, child size) lives in VGPRs;
// the parent stack lives in LDS, lane-strided so a wave's 64 pushes hit 64
// distinct banks.  Every floating-point step reproduces the reference's SSE
// sequence bit for bit: fused only where the reference calls _mm_fmadd_ps,
// RCPPS emulated from a host-captured table, x86's default NaN restored
// before the unsigned t compare, denormal masks compared as integers.
// Build with -ffp-contract=off and without denormal flushing.
//
// One schedule: a grid of one ray per thread, the hardware dispatcher
// balancing waves, in an optional cost-planned workgroup order.  Three ray
// sources (a ray array, the same rays as an image walked 8x8 tile per wave,
// or the camera of tree_camera::update_position mapped 8x8-pixel tile per
// wave) and the sinks (hit records, the shaded RGBA8 framebuffer of
// update_image, or 1-byte colour codes for the multi-GPU exchange) make up
// trace_batch and render.  Config 5 (secondary rays) compacts each block's
// bounced rays through an LDS queue (ballot + popcount).
//
// Arms measured and retired (persistent and refill schedules, in-block wave
// merging, the per-node voxel-box skip, the column cull, LDS-resident top
// levels, two rays per lane, the step-run walk, the secondary walk restarted
// on the primary's stack, packed FMAs, non-temporal frame stores) are kept as
// a diff under profiles/r05/retired/ (DESIGN.md §8).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "och_internal.h"

// Every launch here clears the thread's last HIP error first and reports
// hipGetLastError() after it: that call also returns an error left behind by
// any earlier HIP call of the thread (another library's -- RCCL's communicator
// init, say), which is not this launch's.  The cleared error is kept for
// och_discarded_error (clear_pending_error, och_api.cpp).
// A traversal launch, timed by the dispatch itself when the schedule carries
// events (Schedule::ev_start / ev_stop, OCH_OPT_TIMING): hipExtLaunchKernel
// takes the kernel's own start and end times, with no packets of its own
// between two launches of a stream.
#define OCH_LAUNCH_TIMED(sc, kernel, grid, block, lds, stream, ...)                                                   \
    do {                                                                                                             \
        clear_pending_error(__func__);                                                                               \
        if ((sc).ev_start || (sc).ev_stop)                                                                           \
            hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)(lds), stream, (sc).ev_start, (sc).ev_stop, 0u,     \
                                  __VA_ARGS__);                                                                      \
        else                                                                                                         \
            hipLaunchKernelGGL(kernel, grid, block, lds, stream, __VA_ARGS__);                                       \
    } while (0)

namespace och {
namespace {

constexpr uint32_t kX86DefaultNaN = 0xFFC00000u;

constexpr int kMaxViews = OCH_MAX_VIEWS;

__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float ffrom(uint32_t u) { return __uint_as_float(u); }

// RCPPS model (ORT/och_h_octree.h:316): the table holds RCPPS(-(1 + m/2^k))
// for exponent-127 inputs; other exponents move the result exponent.
// ent = lut[(x & 0x7FFFFF) >> shift], read by the caller for every input (the
// index is in range for any x), so a ray's three lookups are in flight together.
__device__ __forceinline__ uint32_t rcpps_model(uint32_t x, uint32_t ent)
{
    const uint32_t sign = x & 0x80000000u, e = (x >> 23) & 0xFFu;
    const int ne = (int)((ent >> 23) & 0xFFu) + 127 - (int)e;
    uint32_t r = ne <= 0 ? sign : (sign | ((uint32_t)ne << 23) | (ent & 0x7FFFFFu));
    r = e == 0 ? (sign | 0x7F800000u) : r;                              // +-0, denormal -> inf
    r = e == 0xFFu ? ((x & 0x7FFFFFu) ? (x | 0x400000u) : sign) : r;    // NaN (quietened), inf -> 0
    return r;
}

// The same for x = -|d| (sign set) from the device table, whose entries carry
// + 127 << 23 (och_api.cpp upload_lut): while the result exponent ent_e + 127 - e
// stays in 1..254 -- every x whose exponent bits lie in [xlo, xlo + xspan), a
// range the host derives from the table (DevPool::rcp_xlo / rcp_xspan) -- the
// model is one subtraction of x's exponent bits from the entry.  Other x
// (zero, denormal, huge, inf, NaN; none of the bench's rays) take the model.
__device__ __forceinline__ uint32_t rcpps(uint32_t x, uint32_t adj, uint32_t xlo, uint32_t xspan)
{
    const uint32_t xe = x & 0x7F800000u;
    uint32_t r = adj - xe;
    if (xe - xlo >= xspan) r = rcpps_model(x, adj - (127u << 23));
    return r;
}

struct Hit {
    int32_t dir;
    uint32_t voxel;
    uint32_t t;
    uint32_t push;
};

// Traversal state of one ray between iterations.
struct Ray {
    float c[3], b[3];     // coefficient (RCPPS of -|d|) and bias (-c * o') per axis
    uint32_t p[3];        // position bits in the reflected frame
    uint32_t inv;         // direction-sign mask (1 = positive) | 24: idx ^ inv = 24 + child index,
                          // the bit of that child in a packed slot word
    uint32_t idx;         // child index bits at the current level
    uint32_t dim;         // mantissa bit of the current child size: level L <-> 1 << (23 - L)
    uint32_t cur;         // the current node: packed slot word (id | child mask << 24), or raw index
    uint32_t sp;          // LDS byte address of this lane's stack slot for the current level (parents below it)
    uint32_t sp23;        // sp at dim = 1 (slot 23): sp = sp23 - ctz(dim) * 4 * stride (the POP chain)
    uint32_t t_min;       // bits of the entry t of the current cell
    uint32_t min_axis;    // 1, 2, 4 (last STEP axis) or 8 (none yet)
    uint32_t child;       // raw layout: slot word loaded by the last PUSH (pending); the voxel id after a hit
    uint32_t mode;        // see below
    uint32_t push;
    bool inside;          // wave-uniform: every ray of the wave starts inside the root (ray_trace)
    // Split walks only (kSplit, k_trace_grid's heavy tiles): the PUSH test of a
    // present cell of child size split_dim is segment `ord` of the walk, which
    // this lane enters only when ord & split_mask == split_seg; hit_ord: the
    // last segment it entered (the segment of its HIT).
    uint32_t split_dim, split_mask, split_seg, ord, hit_ord;
};

// Ray phase.  Packed layout (one merged PUSH + descend phase): kStepping (0)
// when due to STEP, any nonzero value when due to PUSH -- the advanced axis
// (1, 2, 4) or the present bit, so no phase copies are made at the loop's
// joins (2 VALU per iteration, +0.6 % pipelined, profiles/r02/ab/ab_mode.txt).
// Raw layout (three phases): kAtPush, kStepping, or kPending (a PUSH's slot
// load is in flight).
constexpr uint32_t kAtPush = 1, kStepping = 0, kPending = 8;

// The phase is one VGPR value, opaque to the compiler at each test, so a
// phase test is one compare; as two bools the compiler carried lane masks
// through every join of the loop body (1.5x the SALU instructions, measured).
__device__ __forceinline__ bool in_mode(Ray &r, uint32_t m)
{
    asm volatile("" : "+v"(r.mode));
    return r.mode == m;
}

// The parent stacks (stack_column): per lane, depth + 1 word slots `stride`
// words apart in the block's LDS, and beside each word slot, at its byte
// address / 4, one byte holding the child index the walk took at that level.
// A descent writes both; a POP reads both, so it needs no rebuild of idx from
// the position bits (three bit extracts and two shift-ors per POP).
typedef __attribute__((address_space(3))) uint32_t lds_word;
typedef __attribute__((address_space(3))) uint8_t lds_byte;
__device__ __forceinline__ lds_word *stack_word(uint32_t a) { return (lds_word *)(uintptr_t)a; }
__device__ __forceinline__ lds_byte *stack_idx(uint32_t a) { return (lds_byte *)(uintptr_t)(a >> 2); }

// This lane's stack column (the LDS byte address of its slot 0).  The word
// plane starts at wb with wb / 4 >= the dynamic area's start (the idx plane
// stays clear of static LDS) and wb / 4 + e <= wb (it stays below the word
// plane): e = (depth + 1) * blockDim slots.  stack_bytes sizes the area.
__device__ __forceinline__ uint32_t stack_column(const uint32_t *lds, uint32_t depth)
{
    const uint32_t base = (uint32_t)(uintptr_t)(const lds_word *)lds;
    const uint32_t e = (depth + 1u) * blockDim.x;
    const uint32_t wb = 4u * max(base, (e + 2u) / 3u);
    return wb + 4u * threadIdx.x;
}

// Word index of child slot c24 - 24 of the node whose slot word is w, from
// the node pool's base minus 24 words: id * 8 + c24, id = w's low 24 bits --
// one v_mad_u32_u24 (the compiler turns the mul24 by 8 into a shift and a
// mask, one VALU more per descent).  The descent's buffer load scales it by
// the descriptor's 4-byte stride, so no shift to bytes either.
__device__ __forceinline__ uint32_t slot_index(uint32_t w, uint32_t c24)
{
    uint32_t t;
    asm("v_mad_u32_u24 %0, %1, 8, %2" : "=v"(t) : "v"(w), "v"(c24));
    return t;
}

// The node array as a structured buffer of 4-byte records starting 24 words
// before it (so slot_index needs no bias), bounds-checked against the array:
// an index past it reads 0 instead of faulting.  Built from kernel arguments
// only, so it stays in SGPRs.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slot_buffer(const DevPool &P)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(P.nodes - 24), 4, (int)(P.n_slots + 24u),
                                             0x00020000);
}

// The raw layout's PUSH (ORT/och_h_octree.h:342-344): the slot must be loaded
// to be tested, which happens when the load has landed (ray_phase_descend).
template <bool kCount>
__device__ __forceinline__ void ray_push_raw(Ray &r, const DevPool &P)
{
    if (kCount) ++r.push;
    const uint32_t c24 = r.idx ^ r.inv;                                     // 24 + child index
    r.mode = kPending;
    r.child = (P.nodes - 24)[8u * r.cur + c24];
}

template <bool kCount, bool kAsm, bool kIdxPlane, bool kSplit = false>
__device__ __forceinline__ void ray_push_descend(Ray &r, const DevPool &P, uint32_t stride);

// Occupied-box cull (OCH_OPT_CULL; DESIGN.md §4b has the proof).  With
// t_a(q) = fma(q, c_a, b_a), the walk's t of plane q on axis a in the
// reflected frame (non-increasing in q when c_a < 0), every cell the walk
// enters -- the HIT cell included -- satisfies
//     max_a t_a(hi_a) <= t_min <= min_a t_a(lo_a),  t_min >= +0,
// (its far planes are not yet crossed, its near planes are), so a box holding
// every voxel that fails  max_a t_a(B.hi_a) <= min_a t_a(B.lo_a) >= 0  is
// never entered and the ray ends in the MISS the walk would reach.  Holds
// for c_a negative normal with |c_a| < 2^125 (finite t) and an origin inside
// the root, (1, 2)^3; other rays walk.
__device__ __forceinline__ bool ray_cull(const Ray &r, const DevPool &P, const float *o)
{
    bool ok = true;
    float enter = -INFINITY, leave = INFINITY;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const uint32_t e = (fbits(r.c[a]) >> 23) & 0xFFu;
        ok &= e - 1u < 251u;                                                // 1..251
        ok &= o[a] > 1.0F && o[a] < 2.0F;
        // the box's two planes in the reflected frame, |K - Q| as setup reflects
        // the origin (:314): exact, K - Q lies in [1, 2] or is -Q
        const float k = (r.inv >> a) & 1u ? 3.0F : 0.0F;
        const float t1 = __builtin_fmaf(fabsf(__fsub_rn(k, P.cull_lo[a])), r.c[a], r.b[a]);
        const float t2 = __builtin_fmaf(fabsf(__fsub_rn(k, P.cull_hi[a])), r.c[a], r.b[a]);
        enter = fmaxf(enter, fminf(t1, t2));        // t of the far plane (the larger q)
        leave = fminf(leave, fmaxf(t1, t2));
    }
    return ok && (enter > leave || leave < 0.0F);
}

// Setup, ORT/och_h_octree.h:294-338, up to, not including, the root PUSH.
// stack: this lane's LDS column (stack_column), depth + 1 slots `stride` words apart.
// kCull: a ray that ray_cull proves a miss ends here (false: ray_active
// false, ray_result the miss record, 0 PUSHes).  Launches that count PUSHes
// cull only at OCH_OPT_CULL = 2 (a diagnostic: how many PUSHes the culled
// launch walks), so their counts stay the reference's.  exact = false
// (wave-uniform) leaves the ray to walk: a camera ray that camera_proven_miss
// already tested (DevPool::cam_cull) -- the two tests differ only for rays
// grazing the box within that test's margin, which then walk to the same MISS.
template <bool kCount, bool kCull>
__device__ __forceinline__ bool ray_setup(Ray &r, const DevPool &P, const float *o, const float *d, uint32_t stack,
                                          uint32_t stride, bool exact = true)
{
    r.inv = 24;
    r.idx = 0;
    uint32_t outside = 0;
    uint32_t ent[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) ent[a] = P.lut[(fbits(d[a]) & 0x7FFFFFu) >> P.lut_shift];
    asm volatile("" : "+v"(ent[0]), "+v"(ent[1]), "+v"(ent[2]));   // three loads issued, then one wait
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const uint32_t db = fbits(d[a]);
        const bool positive = (int32_t)db > 0 && db <= 0x7F800000u;          // 0 < d, :310
        r.inv |= (uint32_t)positive << a;
        const float refl = fabsf(__fsub_rn(positive ? 3.0F : 0.0F, o[a]));   // :314
        const uint32_t cb = rcpps(db | 0x80000000u, ent[a], P.rcp_xlo, P.rcp_xspan);   // :312, :316
        r.c[a] = ffrom(cb);
        r.b[a] = ffrom(fbits(__fmul_rn(r.c[a], refl)) ^ 0x80000000u);       // :318
        // A zero or denormal d gives c = -inf, b = +inf and t = fma(p, -inf,
        // +inf) = NaN at every STEP, which the unsigned compare (:384-406)
        // must see as x86's default NaN 0xFFC00000.  Pin it independently of
        // the GPU's default NaN: fma(p, 0, NaN) returns its NaN operand
        // (measured on gfx950, tools/probes/nan_probe.hip), so c = 0 and
        // b = 0xFFC00000 give that pattern at every STEP and every t_mid.
        if ((cb & 0x7FFFFFFFu) == 0x7F800000u) {
            r.c[a] = 0.0F;
            r.b[a] = ffrom(kX86DefaultNaN);
        }
        r.p[a] = fbits(refl) & 0x3FC00000u;                                 // :320
        r.idx |= (uint32_t)(r.p[a] == 0x3FC00000u) << a;                    // :324
        outside |= (r.p[a] >> 23) ^ 0x7Fu;                                  // p not 1.0 or 1.5
    }
    // An origin inside the root, (1, 2)^3, reflects to p = 1.0 or 1.5 on every
    // axis.  Then a POP's child index (:440-444, the position bits at the new
    // level) is the one the descent took there, which the stack's idx plane
    // holds (setup's idx at the root included), and every position has bit 23
    // set (the exponent's), so the POP chain finds a bit at or below 23 without
    // forcing one in.  A wave holding a ray from outside the root walks with the
    // rebuild and the forced bit (ray_trace).
    r.inside = __ballot(outside != 0) == 0;
    r.dim = 1u << 22;                                                       // :326
    r.cur = P.root;
    r.sp = stack + 4u * stride;                                             // slot 0: the miss POP's dummy read
    r.sp23 = stack + 92u * stride;                                          // slot 23 - ctz(dim)
    r.t_min = 0;                                                            // +0.0F
    r.min_axis = 8;
    r.mode = kAtPush;
    r.child = 0;
    r.push = 0;
    if (kCull && exact && (kCount ? P.cull == 2 : P.cull != 0) && ray_cull(r, P, o)) {
        r.dim = 1u << 23;                                                   // finished: the MISS
        r.mode = kStepping;
        return false;
    }
    return true;
}


// The PUSH / STEP / POP machine (ORT/och_h_octree.h:342-446,
// ORT/och_octree.cpp:217-319) in phases per iteration, software-pipelined so
// that a slot load is in flight while other lanes STEP:
//   step    -- lanes due to STEP do so, then advance to a sibling or POP;
//   push + descend (packed) -- lanes due to PUSH test the child in the held
//              node word and, if present, descend and issue the load of the
//              child's slot word (ray_push_descend).
// The raw layout must load every PUSH's slot to test it, so it resolves the
// slot first (descend, step, push): an empty child then STEPs in the same
// iteration.  stride: words between two levels of one lane's LDS stack.
// kIdxPlane: every ray of the wave starts inside the root (Ray::inside), so a
// POP reads idx from the stack's idx plane, else it rebuilds it from the
// position bits.
template <int kPacked, bool kIdxPlane>
__device__ __forceinline__ void ray_phase_step(Ray &r, uint32_t stride)
{
    // STEP :378-419.  The reference's cascade (x if tx <= ty && tx <= tz,
    // else y if ty < tx && ty <= tz, else z) picks the first axis holding
    // the unsigned minimum.
    const uint32_t tx = fbits(__builtin_fmaf(ffrom(r.p[0]), r.c[0], r.b[0]));
    const uint32_t ty = fbits(__builtin_fmaf(ffrom(r.p[1]), r.c[1], r.b[1]));
    const uint32_t tz = fbits(__builtin_fmaf(ffrom(r.p[2]), r.c[2], r.b[2]));
    const uint32_t tm = min(min(tx, ty), tz);
    const bool sx = tx == tm;
    const bool sy = !sx && ty == tm;
    const bool sz = !sx && !sy;
    const uint32_t axis = sx ? 1u : (sy ? 2u : 4u);
    r.min_axis = axis;
    r.t_min = tm;
    if (kPacked) {
        // the phase register holds the advance test itself: nonzero (a PUSH is
        // due) after an advance, kStepping (0) while POPs are left to do
        r.mode = r.idx & axis;
        // POP chain.  After a POP (:421-446) the next STEP sees the parent's
        // lower planes: on the exit axis a the same plane (the child was the
        // lower half there), on every other axis the same or a lower one, whose
        // t is the same or larger.  When all three t are non-negative floats
        // (so the unsigned compare of :384-406 is the float order) that STEP
        // picks axis a again with the same t_min, and it POPs again while the
        // position bit of axis a is clear at that level.  So the walk POPs to
        // the level of the lowest set bit of p_a above the current one and
        // advances there on axis a -- or, with no such bit, POPs past the root
        // (the MISS).  Nothing in between is counted or recorded; the chain
        // lands in the state the POP-by-POP walk reaches, one STEP of it later.
        // Rays with a negative or NaN t (zero / denormal direction components,
        // origins outside the root) take one POP as before.
        if (!r.mode) {
            const bool chain = max(max(tx, ty), tz) < 0x80000000u;
            const uint32_t pa = sx ? r.p[0] : (sy ? r.p[1] : r.p[2]);
            // bit 23 stands for "past the root": the MISS, also when p_a has no
            // bit at 23 (an origin outside the root reflects to p = 0 or below 1).
            // Branch-free: a single POP is the chain from pa = d2 (d2 & -d2 = d2).
            // -2 dim in one 24-bit multiply (dim <= 2^22, one VALU instead of a
            // shift and a negation: +1.7 %, profiles/r05/r05e/); a single POP is
            // the chain from -2 dim itself, whose lowest set bit is 2 dim
            uint32_t nd2;
            asm("v_mul_i32_i24 %0, -2, %1" : "=v"(nd2) : "v"(r.dim));
            const uint32_t up = ((chain ? pa : nd2) & nd2) | (kIdxPlane ? 0u : 1u << 23);
            uint32_t k = __builtin_ctz(up);                                 // the new level's bit
            asm volatile("" : "+v"(k));        // 1 << k, not re-folded into up & -up (one VALU more)
            const uint32_t nd = 1u << k;                                    // new child-size bit
            // sp23 - k * 4 stride in one 24-bit multiply-add (k < 32, stride <= 1024 words);
            // written out, as the compiler re-derives sp23 from the setup and
            // takes a 64-bit multiply-add
            asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r.sp) : "v"(k), "s"(-4 * (int)stride), "v"(r.sp23));
            r.cur = *stack_word(r.sp);                                      // :434 (slot 0 after the MISS)
            if (kIdxPlane) r.idx = *stack_idx(r.sp);                        // :440-444, as the descent left it
            const uint32_t keep = 0u - nd;                                  // clears the levels popped, :436
            r.p[0] &= keep;
            r.p[1] &= keep;
            r.p[2] &= keep;
            r.dim = nd;
            const bool past = nd > (1u << 22);                              // past the root: the MISS
            if (!kIdxPlane) {
                uint32_t zy = (__builtin_amdgcn_ubfe(r.p[2], k, 1) << 1) | __builtin_amdgcn_ubfe(r.p[1], k, 1);
                asm volatile("" : "+v"(zy));
                r.idx = (zy << 1) | __builtin_amdgcn_ubfe(r.p[0], k, 1);    // :440-444
            }
            r.mode = chain && !past ? axis : 0u;                            // the advance at that level
        }
        if (r.mode) {                                                       // advance :413-419
            r.p[0] ^= sx ? r.dim : 0u;
            r.p[1] ^= sy ? r.dim : 0u;
            r.p[2] ^= sz ? r.dim : 0u;
            r.idx ^= axis;
        }
        return;
    }
    if (r.idx & axis) {                                                     // advance :413-419
        // idx bit `axis` set <=> that axis's position has the dim bit set,
        // so clearing it (:415) is a toggle.
        r.p[0] ^= sx ? r.dim : 0u;
        r.p[1] ^= sy ? r.dim : 0u;
        r.p[2] ^= sz ? r.dim : 0u;
        r.idx ^= axis;
        r.mode = kAtPush;
        return;
    }
    // POP :421-446.  At the root this is the MISS (:423-431): dim leaves the
    // walk's range, and the rest of the POP runs on dead state (its stack read
    // lands in the column's spare slot 0) rather than behind a branch.
    r.sp -= 4u * stride;
    r.cur = *stack_word(r.sp);                                              // :434
#pragma unroll
    for (int a = 0; a < 3; ++a) r.p[a] &= ~r.dim;                           // :436
    r.dim <<= 1;                                                            // :438
    const uint32_t k = __builtin_ctz(r.dim);                                // :440-444, bit k of each position
    uint32_t zy = (__builtin_amdgcn_ubfe(r.p[2], k, 1) << 1) | __builtin_amdgcn_ubfe(r.p[1], k, 1);
    asm volatile("" : "+v"(zy));          // two shift-ors, not two shifts and an or3
    r.idx = (zy << 1) | __builtin_amdgcn_ubfe(r.p[0], k, 1);
}

// The raw layout's descend phase: the PUSH's slot word has landed.
__device__ __forceinline__ void ray_phase_descend_raw(Ray &r, uint32_t stride)
{
    r.mode = kAtPush;
    const uint32_t child = r.child;
    if (child == 0) {                                                       // empty child
        r.mode = kStepping;
        return;
    }
    // HIT :346-355 when the PUSH was at the leaf level: dim drops below the
    // walk's range (finished) exactly as a descent halves it, the voxel id
    // stays in r.child (no later load overwrites a finished lane's), and the
    // rest of the descent runs on dead state (its stack write lands in the
    // column's spare top slot) rather than behind a branch.
    *stack_word(r.sp) = r.cur;                                              // :357
    r.sp += 4u * stride;
    r.cur = child;
    r.dim >>= 1;                                                            // :361
    const float tm = ffrom(r.t_min);
    uint32_t nidx = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {                                           // :363-373
        const uint32_t mid = r.p[a] | r.dim;
        const bool upper = __builtin_fmaf(ffrom(mid), r.c[a], r.b[a]) >= tm;
        nidx |= (uint32_t)upper << a;
        r.p[a] = upper ? mid : r.p[a];
    }
    r.idx = nidx;
}

// Still walking: the child-size bit is in the range of levels 1..depth (a
// MISS shifts it past 1 << 22, a HIT below 1 << (23 - depth)), so no level
// counter is kept.
__device__ __forceinline__ bool ray_active(const Ray &r, const DevPool &P)
{
    return r.dim - P.dim_lo <= P.dim_span;
}

// The descent's slot-word load into cur is issued by inline asm, so the
// compiler's waitcnt pass does not see it in flight.  Its only readers are the
// next PUSH and ray_result, each behind an explicit `s_waitcnt vmcnt(0)` that
// takes cur as an operand (so no read of cur is scheduled above it).  What the
// compiler's view saves is the vmcnt(0) it puts at the POP chain: the chain
// writes cur (the popped word, an LDS read) in lanes that are STEPping, and a
// load into cur may still be in flight for the lanes that descended.  Those
// lanes are disjoint (a lane that descended is due to PUSH and skips the STEP
// phase), and a load writes only the lanes active at its issue, so no lane
// sees the other's write; the wave no longer waits for its descents' loads
// before popping.
// The build checks the compiler's output for what this relies on
// (tools/isa_check.py, run by `make` and __graft_entry__.build()): in every
// kernel that issues the load, the load and every wait name one register, and
// on every path from a load to the next vmcnt(0) wait no instruction reads
// that register before writing it (a read there would see the word before
// the load lands -- a copy of cur at a join, a spill, a full-wave select).
// Writes there are the lane-disjoint temporaries of the STEP phase above.
// OCH_ASM_LOAD=0 builds the compiler's own load (tests/test_isa_check.py).
#ifndef OCH_ASM_LOAD
#define OCH_ASM_LOAD 1
#endif
constexpr bool kAsmLoad = OCH_ASM_LOAD != 0;
template <bool kAsm>
__device__ __forceinline__ void wait_cur(Ray &r)
{
    // the comment names cur's register in the compiler's assembly, for the
    // build's ISA check (tools/isa_check.py)
    if (kAsm) asm volatile("s_waitcnt vmcnt(0) ; och_cur_wait %0" : "+v"(r.cur) : : "memory");
}

// Packed layout, PUSH and descent in one phase: the child's presence is a bit
// of the held node word and the descent's geometry (:357-373) does not depend
// on the child's own slot word, so a PUSH that finds its child descends at
// once: the parent to the stack, the child's slot word loaded straight into
// cur -- the node of the next PUSH, or the voxel id of a HIT -- and the child
// cell chosen.  The next PUSH takes the word after the other lanes' STEP phase
// has hidden the load.
template <bool kCount, bool kAsm, bool kIdxPlane, bool kSplit>
__device__ __forceinline__ void ray_push_descend(Ray &r, const DevPool &P, uint32_t stride)
{
    wait_cur<kAsm>(r);
    // Every lane runs the PUSH test (no branch around it: the PUSH phase runs in
    // 96-99 % of a wave's iterations anyway, tools/sched_sim.c schedule 5); a lane
    // due to STEP (mode 0) keeps mode 0 and does not descend.  Two SALU and a
    // branch fewer per iteration: +2.4 % over 20 steps, a lone launch -7 %
    // (profiles/r05/r05r/).
    if (kCount) r.push += r.mode != kStepping;
    const uint32_t c24 = r.idx ^ r.inv;                                     // 24 + child index
    uint32_t present = __builtin_amdgcn_ubfe(r.cur, c24, 1u);
    if (kSplit) {
        // A present cell of the split level due to PUSH is segment ord of the
        // walk; another lane's segment counts as empty here (the walk above
        // the split level does not depend on what happens inside a segment,
        // DESIGN.md §4d).
        if (r.mode != kStepping && present && r.dim == r.split_dim) {
            const bool mine = (r.ord & r.split_mask) == r.split_seg;
            r.hit_ord = mine ? r.ord : r.hit_ord;
            present = mine ? 1u : 0u;
            ++r.ord;
        }
    }
    r.mode = min(r.mode, present);          // kStepping (0), or 1: "PUSH due" after the descent
    const bool go = r.mode != kStepping;    // compared before the barrier: no copy of mode
    asm volatile("" : "+v"(r.mode));
    if (!go) return;
    // the child's slot: one 24-bit multiply-add gives its index in the
    // structured buffer (slot_buffer), the descriptor's stride scales it
    const uint32_t slot = slot_index(r.cur, c24);
    // descent (:357-373); at the leaf level this is the HIT (:346-355): dim
    // drops below the walk's range, the stack write lands in the spare top slot
    *stack_word(r.sp) = r.cur;              // the parent, before its register takes the child's word
    if (kIdxPlane) *stack_idx(r.sp) = (uint8_t)r.idx;   // and the child index taken, for the POP back here
    if (kAsm)
        asm volatile("buffer_load_dword %0, %1, %2, 0 idxen ; och_cur_load"
                     : "+v"(r.cur)
                     : "v"(slot), "s"(slot_buffer(P))
                     : "memory");
    else
        r.cur = (P.nodes - 24)[slot];       // the compiler's own load (OCH_ASM_LOAD=0 builds)
    r.dim >>= 1;
    const float tm = ffrom(r.t_min);
    uint32_t nidx;
    // z, y, x: idx = 2 idx + upper as one v_addc_co_u32 with the compare's
    // mask as carry-in (the compiler builds 3 v_cndmask + v_or3 instead).  A VALU
    // write of vcc is read as a lane mask two wait states later at the soonest
    // (the compiler's own code keeps that distance; tools/isa_check.py check 3
    // holds this asm to it): the next axis's mid-plane and t fill the two states
    // after the z and y compares, and the stack pointer's step (sp += 4 stride as
    // sp - (-4 stride): the POP chain's SGPR, not one more) one after the x compare.
    const uint32_t m2 = r.p[2] | r.dim;
    const float t2 = __builtin_fmaf(ffrom(m2), r.c[2], r.b[2]);
    uint32_t m1, m0, t1, t0;
    asm volatile("v_cmp_ge_f32_e32 vcc, %[t2], %[tm]\n\t"
                 "v_or_b32_e32 %[m1], %[dim], %[p1]\n\t"
                 "v_fma_f32 %[t1], %[m1], %[c1], %[b1]\n\t"
                 "v_cndmask_b32_e32 %[p2], %[p2], %[m2], vcc\n\t"
                 "v_cndmask_b32_e64 %[idx], 0, 1, vcc\n\t"
                 "v_cmp_ge_f32_e32 vcc, %[t1], %[tm]\n\t"
                 "v_or_b32_e32 %[m0], %[dim], %[p0]\n\t"
                 "v_fma_f32 %[t0], %[m0], %[c0], %[b0]\n\t"
                 "v_cndmask_b32_e32 %[p1], %[p1], %[m1], vcc\n\t"
                 "v_addc_co_u32_e32 %[idx], vcc, %[idx], %[idx], vcc\n\t"
                 "v_cmp_ge_f32_e32 vcc, %[t0], %[tm]\n\t"
                 "v_subrev_u32 %[sp], %[n4s], %[sp]\n\t"
                 "s_nop 0\n\t"
                 "v_cndmask_b32_e32 %[p0], %[p0], %[m0], vcc\n\t"
                 "v_addc_co_u32_e32 %[idx], vcc, %[idx], %[idx], vcc"
                 : [p2] "+v"(r.p[2]), [p1] "+v"(r.p[1]), [p0] "+v"(r.p[0]), [sp] "+v"(r.sp), [idx] "=&v"(nidx), [m1] "=&v"(m1),
                   [m0] "=&v"(m0), [t1] "=&v"(t1), [t0] "=&v"(t0)
                 : [t2] "v"(t2), [tm] "v"(tm), [m2] "v"(m2), [dim] "v"(r.dim), [c1] "v"(r.c[1]), [b1] "v"(r.b[1]),
                   [c0] "v"(r.c[0]), [b0] "v"(r.b[0]), [n4s] "s"(-4 * (int)stride)
                 : "vcc");
    r.idx = nidx;
}

template <int kPacked, bool kCount, bool kAsm = false, bool kIdxPlane = false, bool kSplit = false>
__device__ __forceinline__ void ray_iterate(Ray &r, const DevPool &P, uint32_t stride)
{
    if (kPacked) {
        // mode is already behind a barrier (ray_push_descend, and before it below),
        // so no second one here: that one cost an s_nop before this compare
        if (r.mode == kStepping) ray_phase_step<kPacked, kIdxPlane>(r, stride);
        // no activity test: a miss leaves the lane kStepping, a HIT ends in this
        // phase; every lane takes the PUSH test (ray_push_descend)
        asm volatile("" : "+v"(r.mode));
        ray_push_descend<kCount, kAsm, kIdxPlane, kSplit>(r, P, stride);
        return;
    }
    if (in_mode(r, kPending)) ray_phase_descend_raw(r, stride);
    if (in_mode(r, kStepping)) ray_phase_step<kPacked, false>(r, stride);
    if (in_mode(r, kAtPush) && ray_active(r, P)) ray_push_raw<kCount>(r, P);   // PUSH :342-344
}

// The root PUSH (ray_setup leaves the ray due to PUSH at the root), then the
// walk to its HIT or MISS.
// (A lane mask of active lanes cleared by the MISS and HIT compares instead
// of the activity test -- two VALU per iteration -- measured 5 % slower: it
// added a compare to the descent and SALU to every block, profiles/r05/r05e/.)
template <int kPacked, bool kCount, bool kAsm, bool kIdxPlane, bool kSplit = false>
__device__ __forceinline__ void ray_walk(Ray &r, const DevPool &P, uint32_t stride)
{
    if (kPacked)
        ray_push_descend<kCount, kAsm, kIdxPlane, kSplit>(r, P, stride);
    else
        ray_push_raw<kCount>(r, P);
    // the activity test's two constants in VGPRs: as SGPRs the compiler re-loads
    // them from the kernel arguments in every iteration when the kernel's SGPR
    // budget (80, for 8 waves per SIMD) is tight.  Derived from depth (which
    // setup has loaded) rather than read as dim_lo / dim_span: those two share
    // one scalar load with the cull box, and in the split kernel that load was
    // hoisted to the entry, live across setup, and spilled to VGPR lanes
    uint32_t lo = 1u << (23 - P.depth), span = (1u << 22) - lo;
    asm volatile("" : "+v"(lo), "+v"(span));
    if (r.dim - lo <= span) do {
        ray_iterate<kPacked, kCount, kAsm, kIdxPlane, kSplit>(r, P, stride);
    } while (r.dim - lo <= span);
}

// Setup, then the walk.  The branch on inside (wave-uniform) comes
// before the root PUSH issues its asm load, so no copy of cur is made at a
// join while a load is in flight (tools/isa_check.py).
template <int kPacked, bool kCount, bool kCull = false, bool kAsm = false, bool kSplit = false>
__device__ __forceinline__ void ray_trace(Ray &r, const DevPool &P, const float *o, const float *d, uint32_t stack,
                                          uint32_t stride, bool exact = true)
{
    if (!ray_setup<kCount, kCull>(r, P, o, d, stack, stride, exact)) return;
    // A split walk is exact only where a POP restores the child index the
    // descent took: in waves whose rays all start inside the
    // root.  Elsewhere a POP rebuilds idx from the position bits (:440-444),
    // which can differ from what a lane that skipped the segment holds, so
    // every lane of such a wave enters every segment (the whole walk).
    if (kSplit && !r.inside) {
        r.split_mask = 0;
        r.split_seg = 0;
    }
    if (kPacked && r.inside)
        ray_walk<kPacked, kCount, kAsm, true, kSplit>(r, P, stride);
    else
        ray_walk<kPacked, kCount, kAsm, false, kSplit>(r, P, stride);
}

// The hit record of a finished ray (:346-355 hit, :423-431 miss).  The packed
// walk leaves a HIT's voxel id in cur, the raw walk in child.
template <int kPacked, bool kAsm = false>
__device__ __forceinline__ Hit ray_result(Ray &r, const DevPool &P)
{
    Hit h;
    wait_cur<kAsm>(r);                      // a HIT's voxel id load (the asm load)
    const uint32_t cur = r.cur;
    if (r.dim > (1u << 22)) {
        h.dir = OCH_EXIT;
        h.voxel = 0;
        h.t = P.miss_bits;
    } else {
        h.dir = (int32_t)((r.min_axis >> 1) + 3u * ((r.inv & r.min_axis & 7u) == 0));
        h.voxel = kPacked ? cur : r.child;
        h.t = r.t_min;
    }
    h.push = r.push;
    return h;
}

// Secondary ray of a hit, config 5 (BASELINE configs[4]; build-defined, as
// SURVEY §8(a) A10 proposes): from the point half a voxel in front of the hit
// face -- o + d * t - offset, the editor's placement point
// (ORT/test_och_h_octree.cpp:385, :418) with get_directional_hit_offset's
// +-voxel_dim / 2 on the hit axis (:487-502) -- along d mirrored on that axis.
// Products rounded, then sums, as float3's operators evaluate them.
__device__ __forceinline__ void bounce_ray(const float *o, const float *d, const Hit &h, float half, float *o2, float *d2)
{
    const float t = ffrom(h.t);
    const int axis = h.dir % 3;
    const float off = h.dir < 3 ? half : -half;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float q = __fadd_rn(o[a], __fmul_rn(d[a], t));
        o2[a] = __fsub_rn(q, a == axis ? off : 0.0F);
        d2[a] = a == axis ? -d[a] : d[a];
    }
}

// ---------------------------------------------------------------- sources

// Rays from arrays: shared (stride 0) or per-ray (stride 3) origin, AoS float3 dirs.
struct ArraySource {
    static constexpr bool kProvenMiss = false;    // no camera_proven_miss before setup
    static constexpr bool kSplittable = false;    // split plans come from och_gpu_plan_views (camera rays)
    const float *origin;
    const float *dirs;
    int origin_stride;
    uint32_t n;
    __device__ __forceinline__ uint32_t count() const { return n; }
    __device__ __forceinline__ bool get(uint32_t i, float *o, float *d, uint32_t &out) const
    {
        const float *po = origin + (size_t)origin_stride * i;
        const float *pd = dirs + 3 * (size_t)i;
        o[0] = po[0]; o[1] = po[1]; o[2] = po[2];
        d[0] = pd[0]; d[1] = pd[1]; d[2] = pd[2];
        out = i;
        return true;
    }
    // Arbitrary rays: no camera shortcut (see CameraSource::get_wave_culled);
    // ray_setup's exact cull still applies.
    __device__ __forceinline__ bool get_wave_culled(uint32_t wave_base, uint32_t lane, const DevPool &, bool,
                                                    float *o, float *d, uint32_t &out, bool &miss) const
    {
        miss = false;
        return get(wave_base + lane, o, d, out);
    }
};

// tree_camera::update_position per pixel (ORT/test_och_h_octree.cpp:119-136):
// products rounded, sums left to right, correctly rounded sqrt and divide.
__device__ __forceinline__ void camera_rot(const och_camera &C, int col, int row, float &ru, float &rv, float &rw)
{
    const float u = __fmul_rn(C.aspect, __fsub_rn(__fmul_rn(C.view_x, (float)col), 1.0F));
    const float v = __fsub_rn(__fmul_rn(C.view_y, (float)row), 1.0F);
    const float f = C.fov_factor;
    const float *m = C.rot;
    ru = __fadd_rn(__fadd_rn(__fmul_rn(u, m[0]), __fmul_rn(v, m[1])), __fmul_rn(f, m[2]));
    rv = __fadd_rn(__fadd_rn(__fmul_rn(u, m[3]), __fmul_rn(v, m[4])), __fmul_rn(f, m[5]));
    rw = __fadd_rn(__fadd_rn(__fmul_rn(u, m[6]), __fmul_rn(v, m[7])), __fmul_rn(f, m[8]));
}

// Proven sky before the ray is set up (OCH_OPT_CULL).  The
// camera ray's direction is D * R per component, D = (rw, ru, -rv) and R the
// rounded 1 / |D|, each product rounded.  The walk's t of a plane q on axis a
// (ray_cull) is then (q - o_a) / D_a times a common factor 1 / R, times a
// per-axis factor within 2^-9 of 1 (the RCPPS table's relative error, at
// most kCameraCullRcpError = 2^-10 -- x86 RCPPS: 1.5 * 2^-12 -- plus the
// roundings of d, b and the fma, a few 2^-24), plus a shift worth less than
// 2^-21 world units of plane position (the roundings of b and of the
// reflected origin).  So with the box grown by 2^-16 on every side: if the
// ray leaves the grown box behind it (far t < 0), or enters it after leaving
// it by a relative margin of 2^-7 (> (1 + 2^-9) / (1 - 2^-9) - 1 with room for
// this test's own roundings), ray_cull's exact test is true for the real box
// and the ray ends as the MISS -- decided here with an approximate
// reciprocal and no correctly rounded divide or square root.  A pool whose
// table exceeds the bound (P.cam_cull = 0, och_api.cpp upload_lut) skips
// this test and leaves every ray to ray_cull.  Same preconditions as
// ray_cull: origin inside (1, 2)^3, no component below 2^-60 of the largest
// (so every c_a is a normal float below 2^61).  Rays that fail the test take
// the full setup and ray_cull decides them exactly.
// The camera's terms of the test are the view's, computed once per launch on
// the host in the same float operations (CameraView, camera_source): the
// grown box's planes relative to the camera, and whether the camera lies
// inside the root.
struct CameraView {
    float lo[3], hi[3];   // (cull_lo - 2^-16) - pos, (cull_hi + 2^-16) - pos
    int32_t pos_ok;       // 1 < pos < 2 on every axis
};

__device__ __forceinline__ bool camera_proven_miss(const CameraView &V, float ru, float rv, float rw)
{
    const float D[3] = {rw, ru, -rv};
    const float dmax = fmaxf(fmaxf(fabsf(D[0]), fabsf(D[1])), fabsf(D[2]));
    bool ok = V.pos_ok != 0 && dmax > 0x1p-100F;
    float tn = -INFINITY, tf = INFINITY;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        ok &= fabsf(D[a]) >= dmax * 0x1p-60F;
        const float inv = __builtin_amdgcn_rcpf(D[a]);
        const float t1 = V.lo[a] * inv, t2 = V.hi[a] * inv;
        tn = fmaxf(tn, fminf(t1, t2));
        tf = fminf(tf, fmaxf(t1, t2));
    }
    return ok && (tf < 0.0F || tn > tf * (1.0F + 0x1p-7F));
}

// Correctly rounded sqrt(x) for x in [2^-96, 2^96): v_sqrt_f32 (1 ulp) and
// the residual test of its two neighbours -- __builtin_sqrtf's expansion
// without the scaling of small inputs and the zero / inf class test.
__device__ __forceinline__ float sqrt_rn_mid(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = ffrom(fbits(s) - 1u), sp = ffrom(fbits(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x), rp = __builtin_fmaf(-sp, s, x);
    float y = rm <= 0.0F ? sm : s;
    y = rp > 0.0F ? sp : y;
    return y;
}

// Correctly rounded 1 / s for s in [2^-60, 2^60): v_rcp_f32 and one Newton
// step, r + r (1 - s r) with one fma each -- in place of the divide's scale,
// four fmas and fixup.  Both verified bit for bit against __builtin_sqrtf /
// __fdiv_rn over every float of those ranges on gfx950
// (tools/probes/rcp_probe.hip, profiles/r05/r05f/rcp_probe.txt).
__device__ __forceinline__ float rcp_rn_mid(float s)
{
    const float r = __builtin_amdgcn_rcpf(s);
    return __builtin_fmaf(__builtin_fmaf(-s, r, 1.0F), r, r);
}

__device__ __forceinline__ void camera_ray_from(float ru, float rv, float rw, float *d)
{
    const float mag2 = __fadd_rn(__fadd_rn(__fmul_rn(ru, ru), __fmul_rn(rv, rv)), __fmul_rn(rw, rw));
    // RN(1 / RN(sqrt(mag2))): the short forms wherever they are verified exact
    // (every camera ray of a non-degenerate camera: |(u, v, fov factor)|^2), the
    // general expansions elsewhere.  __builtin_sqrtf lowers to the correctly
    // rounded expansion; __fsqrt_rn is a bare v_sqrt_f32 (1 ulp).
    float rmag;
    if (mag2 >= 0x1p-96F && mag2 < 0x1p96F)
        rmag = rcp_rn_mid(sqrt_rn_mid(mag2));
    else
        rmag = __fdiv_rn(1.0F, __builtin_sqrtf(mag2));
    d[0] = __fmul_rn(rw, rmag);
    d[1] = __fmul_rn(ru, rmag);
    d[2] = __fmul_rn(-rv, rmag);
}

__device__ __forceinline__ void camera_ray(const och_camera &C, int col, int row, float *d)
{
    float ru, rv, rw;
    camera_rot(C, col, row, ru, rv, rw);
    camera_ray_from(ru, rv, rw, d);
}

// Pixel tile of one wave: kTileW x kTileH = 64 pixels.
constexpr uint32_t kTileW = 8, kTileH = 64 / kTileW;

// Division by a launch constant: n / d = (mulhi(n, m) + n) >> s for every
// 32-bit n, with m, s from the host (round-up multiplier; checked against
// plain division over all 32-bit edge cases).  A wave-uniform n stays on the
// scalar unit; the integer-division expansion it replaces is ~10 VALU each.
struct FastDiv {
    uint32_t d, m, s;
    __host__ void init(uint32_t divisor)
    {
        d = divisor ? divisor : 1u;      // callers validate sizes; never divide by zero here
        divisor = d;
        s = 0;
        while ((1ull << s) < divisor) ++s;
        m = (uint32_t)((((1ull << s) - divisor) << 32) / divisor + 1);
    }
    __device__ __forceinline__ uint32_t div(uint32_t n) const
    {
        return (uint32_t)(((uint64_t)__umulhi(n, m) + n) >> s);
    }
};

// Resident rays of a row-major image `width` rays wide (a camera's rays as
// update_position lays them out, ORT/test_och_h_octree.cpp:135, x + y * W),
// walked one 8x8 tile per wave as CameraSource walks pixels: neighbouring
// rays share the DAG's top nodes and finish after similar walks, where a
// wave of 64 consecutive rays of one row spreads over a 64 x 1 strip.  Ray
// i = row * width + col, records in the caller's order.  The tile arithmetic
// of a wave runs on the scalar unit.
struct TiledArraySource {
    static constexpr bool kProvenMiss = false;
    static constexpr bool kSplittable = false;
    const float *origin;
    const float *dirs;
    int origin_stride;
    uint32_t n, width, tiles_x, tiles;
    FastDiv by_tiles_x;
    __host__ __device__ __forceinline__ uint32_t count() const { return tiles * 64u; }
    __device__ __forceinline__ bool at(uint32_t tile, uint32_t lane, float *o, float *d, uint32_t &out) const
    {
        const uint32_t ty = by_tiles_x.div(tile), tx = tile - ty * tiles_x;
        const uint32_t col = tx * 8u + (lane & 7u), row = ty * 8u + (lane >> 3);
        if (col >= width) return false;
        const uint32_t i = row * width + col;
        if (i >= n) return false;
        const float *po = origin + (size_t)origin_stride * i;
        const float *pd = dirs + 3 * (size_t)i;
        o[0] = po[0]; o[1] = po[1]; o[2] = po[2];
        d[0] = pd[0]; d[1] = pd[1]; d[2] = pd[2];
        out = i;
        return true;
    }
    // Arbitrary rays: no camera shortcut; ray_setup's exact cull still applies.
    __device__ __forceinline__ bool get_wave_culled(uint32_t wave_base, uint32_t lane, const DevPool &, bool,
                                                    float *o, float *d, uint32_t &out, bool &miss) const
    {
        miss = false;
        return at(__builtin_amdgcn_readfirstlane(wave_base >> 6), lane, o, d, out);
    }
};

// Camera rays of one shard's slice for up to kMaxViews cameras of equal size,
// enumerated view after view, 8x8 pixel tile after tile, so a wave's 64 rays
// are one tile of one view (ray i -> tile i / 64, pixel i % 64).  Tiles run
// row-major (order 0) or in 64x64-pixel supertiles of 8x8 tiles (order 1),
// which the grid kernel hands to one XCD as a unit (see xcd_block).  The
// output token is view * slice_pixels + slice pixel.
struct CameraSource {
    static constexpr bool kProvenMiss = true;     // get_wave_culled runs camera_proven_miss when P.cam_cull
    static constexpr bool kSplittable = true;     // heavy tiles' long rays split over lanes (kSplit launches)
    och_camera cam[kMaxViews];
    CameraView view[kMaxViews];
    int32_t n_views, row_chunk, shard, n_shards, slice_rows, width, height, order;
    uint32_t tiles_x, supertiles_x, per_view, slice_pixels;
    FastDiv by_per_view, by_tiles_x, by_supertiles_x, by_row_chunk;
    // Row deal (och_gpu_set_row_deal): the global chunk of each of this
    // shard's local chunks, -1 past its last; null = round-robin.
    const int32_t *chunk_map;
    // Global row of local chunk `chunk`, row `within` of it; height (no ray)
    // for a padding chunk of a dealt slice.
    __device__ __forceinline__ int global_row(int chunk, int within) const
    {
        const int g = chunk_map ? chunk_map[chunk] : chunk * n_shards + shard;
        return g < 0 ? height : g * row_chunk + within;
    }
    __host__ __device__ __forceinline__ uint32_t count() const { return per_view * (uint32_t)n_views; }
    // Tile of ray i.
    __device__ __forceinline__ void tile_of(uint32_t i, uint32_t &view, uint32_t &tx, uint32_t &ty) const
    {
        view = by_per_view.div(i);
        const uint32_t tile = (i - view * per_view) >> 6;
        if (order == 1) {
            const uint32_t st = tile >> 6, sub = tile & 63u, sy = by_supertiles_x.div(st);
            tx = (st - sy * supertiles_x) * 8u + (sub & 7u);
            ty = sy * 8u + (sub >> 3);
        } else {
            ty = by_tiles_x.div(tile);
            tx = tile - ty * tiles_x;
        }
    }
    // One wave's tile, or miss = true without a ray when camera_proven_miss
    // shows the ray ends as the MISS (cull: the launch may cull,
    // OCH_OPT_CULL).  wave_base (a multiple of 64, wave-uniform) moves the tile
    // arithmetic, divisions included, to the scalar unit.
    __device__ __forceinline__ bool get_wave_culled(uint32_t wave_base, uint32_t lane, const DevPool &P, bool cull,
                                                    float *o, float *d, uint32_t &out, bool &miss) const
    {
        uint32_t view;
        int col, srow, row;
        miss = false;
        if (!locate_wave(wave_base, lane, view, col, srow, row)) return false;
        const och_camera &C = cam[view];
        out = view * slice_pixels + (uint32_t)srow * (uint32_t)width + (uint32_t)col;
        float ru, rv, rw;
        camera_rot(C, col, row, ru, rv, rw);
        if (cull && P.cam_cull && camera_proven_miss(this->view[view], ru, rv, rw)) {
            miss = true;
            return true;
        }
        o[0] = C.pos[0]; o[1] = C.pos[1]; o[2] = C.pos[2];
        camera_ray_from(ru, rv, rw, d);
        return true;
    }
    __device__ __forceinline__ bool locate_wave(uint32_t wave_base, uint32_t lane, uint32_t &view, int &col, int &srow,
                                                int &row) const
    {
        uint32_t tx, ty;
        tile_of(__builtin_amdgcn_readfirstlane(wave_base), view, tx, ty);
        view = __builtin_amdgcn_readfirstlane(view);
        tx = __builtin_amdgcn_readfirstlane(tx);
        ty = __builtin_amdgcn_readfirstlane(ty);
        col = (int)(tx * kTileW + lane % kTileW);
        const int srow0 = (int)(ty * kTileH);
        srow = srow0 + (int)(lane / kTileW);
        if (col >= width || srow >= slice_rows) return false;
        if (row_chunk % (int)kTileH == 0) {                // the tile lies inside one row chunk
            const int chunk = __builtin_amdgcn_readfirstlane((int)by_row_chunk.div((uint32_t)srow0));
            row = global_row(chunk, srow - chunk * row_chunk);
        } else {
            const int chunk = (int)by_row_chunk.div((uint32_t)srow);
            row = global_row(chunk, srow - chunk * row_chunk);
        }
        return row < height;
    }
};

// ---------------------------------------------------------------- sinks

template <bool kCount>
struct HitSink {
    int32_t *dir;
    uint32_t *voxel;
    uint32_t *t;
    uint32_t *push;
    __device__ __forceinline__ void put(uint32_t i, const Hit &h) const
    {
        dir[i] = h.dir;
        voxel[i] = h.voxel;
        t[i] = h.t;
        if (kCount) push[i] = h.push;
    }
};

// Walked PUSH counts per pixel of a camera launch, saturated to 16 bits: the
// split planner's per-ray costs (och_api.cpp plan_split).
struct PushSink {
    uint16_t *push;
    __device__ __forceinline__ void put(uint32_t i, const Hit &h) const { push[i] = (uint16_t)min(h.push, 65535u); }
};

// trace_pixel's colour choice (ORT/test_och_h_octree.cpp:76-84) as olc::Pixel RGBA8.
__device__ __forceinline__ uint32_t pixel_colour(const Hit &h, const uint32_t *palette, uint32_t n_voxels)
{
    if (h.dir == OCH_EXIT) return 0xFFFEBF00u;            // {0x00, 0xBF, 0xFE}
    if (h.dir == OCH_INSIDE) return 0xFF07193Fu;          // {0x3F, 0x19, 0x07}
    if (h.voxel == 0 || h.voxel > n_voxels) return 0xFFFF00FFu;
    return palette[6u * (h.voxel - 1u) + (uint32_t)h.dir];
}

struct FrameSink {
    uint32_t *out;
    const uint32_t *palette;
    uint32_t n_voxels;
    __device__ __forceinline__ void put(uint32_t i, const Hit &h) const { out[i] = pixel_colour(h, palette, n_voxels); }
};

// Config 5 sinks.  put_primary stores what is final for a ray without a
// bounce and returns the payload its secondary ray carries; put_secondary
// completes a bounced ray.
// Shading of a bounced pixel (build-defined): the hit face's colour when the
// mirrored ray escapes to the sky, half of it (RGB >> 1) when it is blocked.
struct BounceFrameSink {
    FrameSink f;
    __device__ __forceinline__ uint32_t put_primary(uint32_t i, const Hit &h, bool bounced) const
    {
        const uint32_t c = pixel_colour(h, f.palette, f.n_voxels);
        if (!bounced) f.out[i] = c;
        return c;
    }
    __device__ __forceinline__ void put_secondary(uint32_t i, uint32_t c, const Hit &h2) const
    {
        f.out[i] = h2.dir == OCH_EXIT ? c : (((c >> 1) & 0x007F7F7Fu) | (c & 0xFF000000u));
    }
};

// Indexed-colour frames (the multi-GPU exchange format, 1 B per pixel): the
// palette index 6 * (voxel - 1) + dir of a hit face, OCH_CODE_MAGENTA /
// _INSIDE / _SKY for the other cases of pixel_colour, + OCH_CODE_BLOCKED
// when a config-5 secondary ray is blocked.  k_shade_unshard turns codes
// into the same RGBA8 words pixel_colour and BounceFrameSink produce.
__device__ __forceinline__ uint32_t pixel_code(const Hit &h, uint32_t n_voxels)
{
    if (h.dir == OCH_EXIT) return OCH_CODE_SKY;
    if (h.dir == OCH_INSIDE) return OCH_CODE_INSIDE;
    if (h.voxel == 0 || h.voxel > n_voxels) return OCH_CODE_MAGENTA;
    return 6u * (h.voxel - 1u) + (uint32_t)h.dir;
}

struct CodeSink {
    uint8_t *out;
    uint32_t n_voxels;
    __device__ __forceinline__ void put(uint32_t i, const Hit &h) const { out[i] = (uint8_t)pixel_code(h, n_voxels); }
};

struct BounceCodeSink {
    CodeSink f;
    __device__ __forceinline__ uint32_t put_primary(uint32_t i, const Hit &h, bool bounced) const
    {
        const uint32_t c = pixel_code(h, f.n_voxels);
        if (!bounced) f.out[i] = (uint8_t)c;
        return c;
    }
    __device__ __forceinline__ void put_secondary(uint32_t i, uint32_t c, const Hit &h2) const
    {
        f.out[i] = (uint8_t)(h2.dir == OCH_EXIT ? c : c | OCH_CODE_BLOCKED);
    }
};

template <bool kCount>
struct BounceHitSink {
    HitSink<kCount> h;
    int32_t *dir2;
    uint32_t *voxel2;
    uint32_t *t2;
    __device__ __forceinline__ uint32_t put_primary(uint32_t i, const Hit &h1, bool bounced) const
    {
        h.dir[i] = h1.dir;
        h.voxel[i] = h1.voxel;
        h.t[i] = h1.t;
        if (!bounced) {
            dir2[i] = -1;
            voxel2[i] = 0;
            t2[i] = 0;
            if (kCount) h.push[i] = h1.push;
        }
        return h1.push;
    }
    __device__ __forceinline__ void put_secondary(uint32_t i, uint32_t push1, const Hit &h2) const
    {
        dir2[i] = h2.dir;
        voxel2[i] = h2.voxel;
        t2[i] = h2.t;
        if (kCount) h.push[i] = push1 + h2.push;
    }
};

// ---------------------------------------------------------------- stamps

// Diagnostic residency record per wave: {start, end} in s_memrealtime ticks
// (100 MHz), HW_ID | XCC_ID << 32, rays finished.  Off when stamps == null.
__device__ __forceinline__ uint64_t realtime() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ uint64_t hw_ids()
{
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    return (uint64_t)hw | ((uint64_t)xcc << 32);
}

__device__ __forceinline__ void stamp(uint64_t *stamps, uint32_t cap, uint64_t t0, uint64_t rays)
{
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0 && wave < cap) {
        uint64_t *s = stamps + 4 * (size_t)wave;
        s[0] = t0;
        s[1] = realtime();
        s[2] = hw_ids();
        s[3] = rays;
    }
}

// ---------------------------------------------------------------- kernels

// A heavy tile's rays, the long ones walked by S lanes each (kSplit launches,
// OCH_OPT_SPLIT).  The workgroup is one wave of lane tasks from
// the plan's task table (och_api.cpp plan_split): word 0 the tile, then per
// lane pixel | seg << 6 | log2(S) << 10, or ~0 for an idle lane.  A lane walks
// its ray's whole walk above the split level but enters only the present
// split-level cells (segments) whose ordinal is seg modulo S (S = 1: all, the
// plain walk).  The ray's record is the HIT of the lowest segment ordinal any
// of its lanes found, or the MISS -- the full walk's record, bit for bit,
// because the walk above the split level does not depend on what it does
// inside a segment.  The lanes agree through one LDS word per pixel (atomic
// min of ordinal << 6 | lane); the winning lane stores its record, or, with no
// HIT, the ray's segment-0 lane stores the MISS.
template <class Src, class Sink, int kPacked>
__device__ __forceinline__ void split_tile(const DevPool &P, const Src &S, const Sink &K, uint32_t ent,
                                           const uint32_t *__restrict__ tasks, uint32_t level, uint32_t *lds_stack)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t *w = tasks + (size_t)(ent & 0x7FFFFFFFu) * 65u;
    const uint32_t tile = __builtin_amdgcn_readfirstlane(w[0]);
    const uint32_t task = w[1u + lane];
    const uint32_t pix = task & 63u, seg = (task >> 6) & 15u, log2s = (task >> 10) & 7u;
    const uint32_t stack = stack_column(lds_stack, P.depth);
    float o[3], d[3];
    uint32_t out = 0, key = ~0u;
    bool miss = false;
    Hit h{OCH_EXIT, 0u, P.miss_bits, 0u};
    const bool valid = task != ~0u && tile * 64u + pix < S.count() &&
                       S.get_wave_culled(tile * 64u, pix, P, P.cull != 0, o, d, out, miss);
    if (valid && !miss) {
        Ray r;
        r.split_dim = 1u << (23u - level);
        r.split_mask = (1u << log2s) - 1u;
        r.split_seg = seg;
        r.ord = 0;
        r.hit_ord = ~0u;
        ray_trace<kPacked, false, true, kAsmLoad, true>(r, P, o, d, stack, blockDim.x,
                                                       !(Src::kProvenMiss && P.cam_cull));
        h = ray_result<kPacked, kAsmLoad>(r, P);
        key = r.dim > (1u << 22) ? ~0u : r.hit_ord;                         // a MISS loses to any HIT
    }
    // one word per pixel: slot 0 of lane `pixel`'s stack column (the walks are over)
    const uint32_t best0 = (stack - (uint32_t)(uintptr_t)(const lds_word *)lds_stack) / 4u - threadIdx.x;
    __syncthreads();
    lds_stack[best0 + lane] = ~0u;
    __syncthreads();
    if (key != ~0u) atomicMin(&lds_stack[best0 + pix], (key << 6) | lane);   // ordinals < 2^26
    __syncthreads();
    if (valid) {
        const uint32_t b = lds_stack[best0 + pix];
        if (b == ~0u ? seg == 0u : (b & 63u) == lane) K.put(out, h);
    }
}

// Workgroups are dealt round-robin over the 8 XCDs (blocks b, b + 8, ... share
// one XCD and its L2).  Remap so each XCD receives runs of `group`
// consecutive logical blocks -- one supertile of neighbouring rays, which walk
// the same DAG nodes -- instead of every eighth block.  A bijection on the
// grid; placement only changes speed, never results.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb, uint32_t group)
{
    if (group == 0) return b;
    const uint32_t span = 8u * group, full = nb - nb % span;
    if (b >= full) return b;
    const uint32_t x = b & 7u, s = b >> 3;
    return ((s / group) * 8u + x) * group + s % group;
}

// order: optional block permutation (a cost-planned launch order: the
// most expensive workgroups of the planning frame first, so the frame does not
// end on a few late grazing tiles); cost: optional per-block duration in
// shader clocks (the planning launch).  Placement only: results are the same.
// The traversal kernels are capped at 80 SGPRs: above 80 a SIMD admits 7 waves, not 8
// (MI355X_MICROARCH.md, residency; the compiler's occupancy note says 8 there), and 8
// give +5 % sustained.  tools/isa_check.py check 4 holds every
// traversal kernel to 8 waves per SIMD.
// kSplit: order entries with bit 31 set are split waves (split_tile): their
// task table row, split_level the split's level.
template <class Src, class Sink, int kPacked, bool kCount, bool kSplit>
__global__ __attribute__((amdgpu_num_sgpr(80))) void k_trace_grid(DevPool P, Src S, Sink K, uint32_t xcd_group, const uint32_t *__restrict__ order,
                             uint32_t *__restrict__ cost, uint64_t *stamps, uint32_t stamp_cap,
                             const uint32_t *__restrict__ split_tasks, uint32_t split_level)
{
    extern __shared__ uint32_t lds_stack[];
    const uint64_t t0 = stamps ? realtime() : 0;
    const uint64_t c0 = cost ? __builtin_amdgcn_s_memtime() : 0;
    const uint32_t blk = order ? order[blockIdx.x] : xcd_block(blockIdx.x, gridDim.x, xcd_group);
    if (kSplit && (blk >> 31)) {                    // a split wave (wave-uniform)
        split_tile<Src, Sink, kPacked>(P, S, K, blk, split_tasks, split_level, lds_stack);
        if (stamps) stamp(stamps, stamp_cap, t0, 64);
        return;
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave_base = blk * blockDim.x + (threadIdx.x & ~63u);
    float o[3], d[3];
    uint32_t out;
    bool miss;
    if (wave_base + lane < S.count() &&
        S.get_wave_culled(wave_base, lane, P, kCount ? P.cull == 2 : P.cull != 0, o, d, out, miss)) {
        if (miss) {                                 // proven before setup: the MISS record, 0 PUSHes
            K.put(out, Hit{OCH_EXIT, 0u, P.miss_bits, 0u});
        } else {
            Ray r;
            ray_trace<kPacked, kCount, true, kAsmLoad>(r, P, o, d, stack_column(lds_stack, P.depth), blockDim.x,
                                                      !(Src::kProvenMiss && P.cam_cull));
            K.put(out, ray_result<kPacked, kAsmLoad>(r, P));
        }
    }
    if (cost && threadIdx.x == 0) cost[blk] = (uint32_t)(__builtin_amdgcn_s_memtime() - c0);
    if (stamps) stamp(stamps, stamp_cap, t0, 64);
}

// Config 5: primary rays, then wavefront compaction -- the block's hit
// lanes (ballot + popcount per wave, wave offsets through LDS) write their
// secondary rays into an LDS queue, and the first lanes of the block trace
// them, so waves whose tiles mostly missed retire instead of idling beside
// a few bounced lanes.  The queue (8 words per thread, SoA) reuses the
// parent stacks' LDS between the passes.
// compact (OCH_OPT_BOUNCE_COMPACT): 0 = every secondary ray in place (by the
// lane that walked its primary); 1 = always through the queue; 2 = per block:
// through the queue when it packs the block's secondary rays into fewer waves
// than hold them in place, else in place.  On the bench's terrain 98.7 % of
// the secondary rays sit in waves whose 64 lanes all bounce, so the queue
// frees few waves and the three modes are within about 1 %.
template <int kPacked, bool kCount, class Sink>
__device__ __forceinline__ void bounce_in_place(const DevPool &P, const Sink &K, uint32_t stack, uint32_t nb,
                                                const float *o2, const float *d2, uint32_t out, uint32_t payload)
{
    Ray r;
    ray_trace<kPacked, kCount, true, kAsmLoad>(r, P, o2, d2, stack, nb);
    K.put_secondary(out, payload, ray_result<kPacked, kAsmLoad>(r, P));
}

template <class Src, class Sink, int kPacked, bool kCount>
__global__ __attribute__((amdgpu_num_sgpr(80))) void k_trace_bounce(DevPool P, Src S, Sink K, int compact, const uint32_t *__restrict__ order,
                               uint32_t *__restrict__ cost, uint64_t *stamps, uint32_t stamp_cap)
{
    extern __shared__ uint32_t lds_stack[];
    __shared__ uint32_t wave_count[16];
    const uint64_t c0 = cost ? __builtin_amdgcn_s_memtime() : 0;
    const uint32_t blk = order ? order[blockIdx.x] : blockIdx.x;
    const uint64_t t0 = stamps ? realtime() : 0;
    const uint32_t stack = stack_column(lds_stack, P.depth);
    uint32_t *queue = lds_stack;
    const uint32_t nb = blockDim.x;
    const uint32_t wave_base = blk * nb + (threadIdx.x & ~63u);
    float o[3], d[3], o2[3], d2[3];
    uint32_t out = 0, payload = 0;
    bool want = false;
    bool miss;
    if (wave_base + (threadIdx.x & 63u) < S.count() &&
        S.get_wave_culled(wave_base, threadIdx.x & 63u, P, kCount ? P.cull == 2 : P.cull != 0, o, d, out, miss)) {
        if (miss) {                                 // proven before setup: the MISS, no secondary ray
            K.put_primary(out, Hit{OCH_EXIT, 0u, P.miss_bits, 0u}, false);
        } else {
            Ray r;
            ray_trace<kPacked, kCount, true, kAsmLoad>(r, P, o, d, stack, nb, !(Src::kProvenMiss && P.cam_cull));
            const Hit h1 = ray_result<kPacked, kAsmLoad>(r, P);
            want = h1.dir < OCH_EXIT;
            if (want) bounce_ray(o, d, h1, P.half_voxel, o2, d2);
            payload = K.put_primary(out, h1, want);
            if (want && compact == 0)                                       // in place, no compaction
                bounce_in_place<kPacked, kCount>(P, K, stack, nb, o2, d2, out, payload);
        }
    }
    if (compact == 0) {
        if (cost && threadIdx.x == 0) cost[blk] = (uint32_t)(__builtin_amdgcn_s_memtime() - c0);
        if (stamps) stamp(stamps, stamp_cap, t0, 0);
        return;
    }
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t bal = __ballot(want);
    if (lane == 0) wave_count[wave] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t base = 0, total = 0, holding = 0;
    for (uint32_t w = 0; w < (nb >> 6); ++w) {
        const uint32_t cnt = wave_count[w];
        base += w < wave ? cnt : 0u;
        total += cnt;
        holding += cnt != 0u;
    }
    if (compact == 2 && (total + 63u) / 64u >= holding) {
        // the queue would not free a wave (block-uniform): in place
        if (want) bounce_in_place<kPacked, kCount>(P, K, stack, nb, o2, d2, out, payload);
        if (cost && threadIdx.x == 0) cost[blk] = (uint32_t)(__builtin_amdgcn_s_memtime() - c0);
        if (stamps) stamp(stamps, stamp_cap, t0, 0);
        return;
    }
    if (want) {
        const uint32_t q = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        queue[0 * nb + q] = fbits(o2[0]);
        queue[1 * nb + q] = fbits(o2[1]);
        queue[2 * nb + q] = fbits(o2[2]);
        queue[3 * nb + q] = fbits(d2[0]);
        queue[4 * nb + q] = fbits(d2[1]);
        queue[5 * nb + q] = fbits(d2[2]);
        queue[6 * nb + q] = out;
        queue[7 * nb + q] = payload;
    }
    __syncthreads();
    float so[3], sd[3];
    uint32_t sout = 0, spay = 0;
    const bool has = threadIdx.x < total;
    if (has) {
        const uint32_t q = threadIdx.x;
        so[0] = ffrom(queue[0 * nb + q]); so[1] = ffrom(queue[1 * nb + q]); so[2] = ffrom(queue[2 * nb + q]);
        sd[0] = ffrom(queue[3 * nb + q]); sd[1] = ffrom(queue[4 * nb + q]); sd[2] = ffrom(queue[5 * nb + q]);
        sout = queue[6 * nb + q];
        spay = queue[7 * nb + q];
    }
    __syncthreads();                                  // the queue is read: its LDS becomes stacks again
    if (has) {
        Ray r;
        ray_trace<kPacked, kCount, true, kAsmLoad>(r, P, so, sd, stack, nb);
        K.put_secondary(sout, spay, ray_result<kPacked, kAsmLoad>(r, P));
    }
    if (cost && threadIdx.x == 0) cost[blk] = (uint32_t)(__builtin_amdgcn_s_memtime() - c0);
    if (stamps) stamp(stamps, stamp_cap, t0, total);
}

__global__ __launch_bounds__(256) void k_raygen(och_camera C, float *__restrict__ dirs)
{
    const int col = blockIdx.x * 16 + (threadIdx.x & 15);
    const int row = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (col >= C.width || row >= C.height) return;
    float d[3];
    camera_ray(C, col, row, d);
    const size_t k = 3 * ((size_t)row * C.width + col);
    dirs[k] = d[0];
    dirs[k + 1] = d[1];
    dirs[k + 2] = d[2];
}

// gathered: [n_shards][n_views][slice_rows][width] -> frames: [n_views][height][width]
// Source row of global row `row` in the gathered slices [n_shards][n_views]
// [slice_rows][W]: round-robin chunks, or the row deal's owner table
// (owner[gchunk] = shard << 16 | local chunk).
__device__ __forceinline__ size_t gathered_row(int row, int row_chunk, int n_shards, int slice_rows, int n_views,
                                               int view, const int32_t *__restrict__ owner)
{
    const int gchunk = row / row_chunk, within = row - gchunk * row_chunk;
    int shard, lchunk;
    if (owner) {
        const int32_t w = owner[gchunk];
        shard = w >> 16;
        lchunk = w & 0xFFFF;
    } else {
        shard = gchunk % n_shards;
        lchunk = gchunk / n_shards;
    }
    return ((size_t)shard * n_views + view) * slice_rows + (size_t)lchunk * row_chunk + within;
}

__global__ __launch_bounds__(256) void k_unshard(const uint32_t *__restrict__ gathered, uint32_t *__restrict__ frames,
                                                 int width, int height, int row_chunk, int n_shards, int slice_rows,
                                                 int n_views, const int32_t *__restrict__ owner)
{
    const int col = blockIdx.x * 256 + threadIdx.x;
    const int row = blockIdx.y, view = blockIdx.z;
    if (col >= width || row >= height) return;
    const size_t src = gathered_row(row, row_chunk, n_shards, slice_rows, n_views, view, owner) * width + col;
    frames[((size_t)view * height + row) * width + col] = gathered[src];
}

// gathered codes [n_shards][n_views][slice_rows][width] -> RGBA8 frames
// [n_views][height][width] through the 256-entry code table (och_api.cpp
// code_table: palette words, the fixed colours, the halved blocked variants).
__global__ __launch_bounds__(256) void k_shade_unshard(const uint8_t *__restrict__ gathered, uint32_t *__restrict__ frames,
                                                       const uint32_t *__restrict__ table, int width, int height,
                                                       int row_chunk, int n_shards, int slice_rows, int n_views,
                                                       const int32_t *__restrict__ owner)
{
    __shared__ uint32_t lut[256];
    lut[threadIdx.x] = table[threadIdx.x];
    __syncthreads();
    const int col = blockIdx.x * 256 + threadIdx.x;
    const int row = blockIdx.y, view = blockIdx.z;
    if (col >= width || row >= height) return;
    const size_t src = gathered_row(row, row_chunk, n_shards, slice_rows, n_views, view, owner) * width + col;
    frames[((size_t)view * height + row) * width + col] = lut[gathered[src]];
}

// The same for width % 4 == 0: four pixels per thread, one 4-B code load and
// one 16-B store, a quarter of the waves (they share the CUs with the render
// launches of the frames in flight).
__global__ __launch_bounds__(256) void k_shade_unshard4(const uint8_t *__restrict__ gathered, uint32_t *__restrict__ frames,
                                                        const uint32_t *__restrict__ table, int width, int height,
                                                        int row_chunk, int n_shards, int slice_rows, int n_views,
                                                        const int32_t *__restrict__ owner)
{
    __shared__ uint32_t lut[256];
    lut[threadIdx.x] = table[threadIdx.x];
    __syncthreads();
    const int col = (blockIdx.x * 256 + threadIdx.x) * 4;
    const int row = blockIdx.y, view = blockIdx.z;
    if (col >= width || row >= height) return;
    const size_t src = gathered_row(row, row_chunk, n_shards, slice_rows, n_views, view, owner) * width + col;
    // streaming accesses: the codes are read once and the frame is not read
    // back here, so neither should evict the DAG's lines from L2 / MALL
    const uint32_t c = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(gathered + src));
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 px = {lut[c & 0xFFu], lut[(c >> 8) & 0xFFu], lut[(c >> 16) & 0xFFu], lut[c >> 24]};
    __builtin_nontemporal_store(px, reinterpret_cast<u32x4 *>(frames + ((size_t)view * height + row) * width + col));
}

// Editor flush: `count` staged slots (8 words each, raw and optionally packed)
// scattered to their slot ids in both device layouts; one thread per word.
__global__ __launch_bounds__(256) void k_scatter_slots(const uint32_t *__restrict__ ids,
                                                       const uint32_t *__restrict__ raw,
                                                       const uint32_t *__restrict__ packed, uint32_t count,
                                                       uint32_t *__restrict__ d_raw, uint32_t *__restrict__ d_packed)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= count * 8u) return;
    const uint32_t slot = ids[i >> 3], w = i & 7u;
    d_raw[(size_t)slot * 8 + w] = raw[i];
    if (packed) d_packed[(size_t)slot * 8 + w] = packed[i];
}

// Per lane: parents of levels 1..depth-1 in slots 1..depth-1, plus a spare
// slot below (the miss POP's read) and above (the hit descent's write); the
// word plane, and below it the idx plane (stack_column), for a dynamic LDS
// area that starts at most kStaticLds bytes in (k_trace_bounce's wave counts).
constexpr size_t kStaticLds = 64;
size_t stack_bytes(int depth, int block)
{
    const size_t e = (size_t)(depth + 1) * block, c = (e + 2) / 3;
    return 4 * (c > kStaticLds ? c : kStaticLds) + 4 * e;
}

template <class Src, class Sink, int kPacked, bool kCount>
hipError_t launch_as(const DevPool &p, const Src &s, const Sink &k, uint32_t n, const Schedule &sc, hipStream_t stream,
                     uint32_t supertile_rays)
{
    if (n == 0) return hipSuccess;
    const int block = sc.block;
    const size_t lds = stack_bytes(p.depth, block);
    const uint32_t xcd_group = supertile_rays >= (uint32_t)block ? supertile_rays / (uint32_t)block : 0u;
    const uint32_t grid = (n + (uint32_t)block - 1) / (uint32_t)block;
    if constexpr (Src::kSplittable && kPacked && !kCount) {
        // a split plan (och_api.cpp plan_split): this grid's workgroups, the
        // heavy ones replaced by their parts; one wave per workgroup
        if (sc.split_tasks && sc.order && block == 64 && sc.order_n == grid + sc.split_extra) {
            OCH_LAUNCH_TIMED(sc, (k_trace_grid<Src, Sink, kPacked, kCount, true>), dim3(sc.order_n), dim3(block), lds,
                             stream, p, s, k, 0u, sc.order, sc.cost, sc.stamps, sc.stamp_cap, sc.split_tasks,
                             sc.split_level);
            return hipGetLastError();
        }
    }
    // a plan is a permutation of exactly this grid's workgroups; any other
    // (stale or for another block size) would index past it
    OCH_LAUNCH_TIMED(sc, (k_trace_grid<Src, Sink, kPacked, kCount, false>), dim3(grid), dim3(block), lds, stream, p, s,
                     k, xcd_group, sc.order_n == grid ? sc.order : nullptr, sc.cost, sc.stamps, sc.stamp_cap, nullptr,
                     0u);
    return hipGetLastError();
}

template <class Src, class Sink, bool kCount>
hipError_t launch(const DevPool &p, const Src &s, const Sink &k, uint32_t n, const Schedule &sc, hipStream_t stream,
                  uint32_t supertile_rays = 0)
{
    return p.packed ? launch_as<Src, Sink, 1, kCount>(p, s, k, n, sc, stream, supertile_rays)
                    : launch_as<Src, Sink, 0, kCount>(p, s, k, n, sc, stream, supertile_rays);
}

template <class Src, class Sink, bool kCount>
hipError_t launch_bounce(const DevPool &p, const Src &s, const Sink &k, uint32_t n, const Schedule &sc, hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    const int block = sc.block > kBounceBlock ? sc.block : kBounceBlock;
    const size_t queue = 8u * (size_t)block * sizeof(uint32_t);
    const size_t lds = stack_bytes(p.depth, block) > queue ? stack_bytes(p.depth, block) : queue;
    const dim3 grid((n + block - 1) / block);
    const uint32_t *order = sc.order_n == grid.x ? sc.order : nullptr;   // a plan of exactly this grid
    if (p.packed)
        OCH_LAUNCH_TIMED(sc, (k_trace_bounce<Src, Sink, 1, kCount>), grid, dim3(block), lds, stream, p, s, k,
                         sc.bounce_compact, order, sc.cost, sc.stamps, sc.stamp_cap);
    else
        OCH_LAUNCH_TIMED(sc, (k_trace_bounce<Src, Sink, 0, kCount>), grid, dim3(block), lds, stream, p, s, k,
                         sc.bounce_compact, order, sc.cost, sc.stamps, sc.stamp_cap);
    return hipGetLastError();
}

CameraSource camera_source(const DevPool &p, const DevFrame &f, const Schedule &sc)
{
    CameraSource src;
    for (int v = 0; v < f.n_views; ++v) {
        src.cam[v] = f.cams[v];
        CameraView &V = src.view[v];
        V.pos_ok = 1;
        for (int a = 0; a < 3; ++a) {
            const float o = f.cams[v].pos[a];
            // the device's operations in IEEE single, one rounding each (no contraction)
            const float lo = p.cull_lo[a] - 0x1p-16F, hi = p.cull_hi[a] + 0x1p-16F;
            V.lo[a] = lo - o;
            V.hi[a] = hi - o;
            V.pos_ok &= (o > 1.0F && o < 2.0F) ? 1 : 0;
        }
    }
    src.n_views = f.n_views;
    src.row_chunk = f.row_chunk;
    src.shard = f.shard;
    src.n_shards = f.n_shards;
    src.slice_rows = f.slice_rows;
    src.width = f.cams[0].width;
    src.height = f.cams[0].height;
    src.tiles_x = (uint32_t)(src.width + kTileW - 1) / kTileW;
    src.order = sc.tile_order == 1 ? 1 : 0;       // 2 = row-major tiles in a planned launch order
    const uint32_t tiles_y = (uint32_t)(f.slice_rows + kTileH - 1) / kTileH;
    src.supertiles_x = (src.tiles_x + 7) / 8;
    src.per_view = sc.tile_order == 1 ? src.supertiles_x * ((tiles_y + 7) / 8) * 64u * 64u : src.tiles_x * tiles_y * 64u;
    src.slice_pixels = (uint32_t)f.slice_rows * (uint32_t)src.width;
    src.by_per_view.init(src.per_view);
    src.by_tiles_x.init(src.tiles_x);
    src.by_supertiles_x.init(src.supertiles_x);
    src.by_row_chunk.init((uint32_t)src.row_chunk);
    src.chunk_map = f.chunk_map;
    return src;
}

}  // namespace

hipError_t occupancy_blocks_per_cu(int kind, int block, int depth, int *blocks)
{
    const size_t lds = stack_bytes(depth, block);
    switch (kind) {
    case 0:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, k_trace_grid<CameraSource, FrameSink, 1, false, false>,
                                                            block, lds);
    case 2:
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks,
                                                            k_trace_grid<ArraySource, HitSink<false>, 1, false, false>,
                                                            block, lds);
    default:
        return hipErrorInvalidValue;
    }
}

hipError_t launch_trace_batch(const DevPool &p, const float *origin, int origin_stride, const float *dirs,
                              uint32_t n, int32_t *hit_dir, uint32_t *hit_voxel, uint32_t *hit_time,
                              uint32_t *push_count, const Schedule &sc, hipStream_t stream)
{
    const ArraySource src{origin, dirs, origin_stride, n};
    if (push_count)
        return launch<ArraySource, HitSink<true>, true>(p, src, HitSink<true>{hit_dir, hit_voxel, hit_time, push_count},
                                                        n, sc, stream);
    return launch<ArraySource, HitSink<false>, false>(p, src, HitSink<false>{hit_dir, hit_voxel, hit_time, nullptr}, n,
                                                      sc, stream);
}

hipError_t launch_trace_batch_tiled(const DevPool &p, const float *origin, int origin_stride, const float *dirs,
                                    uint32_t n, uint32_t width, int32_t *hit_dir, uint32_t *hit_voxel,
                                    uint32_t *hit_time, uint32_t *push_count, const Schedule &sc, hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    TiledArraySource src;
    src.origin = origin;
    src.dirs = dirs;
    src.origin_stride = origin_stride;
    src.n = n;
    src.width = width;
    src.tiles_x = (width + 7) / 8;
    src.tiles = src.tiles_x * ((((n + width - 1) / width) + 7) / 8);
    src.by_tiles_x.init(src.tiles_x);
    if (push_count)
        return launch<TiledArraySource, HitSink<true>, true>(
            p, src, HitSink<true>{hit_dir, hit_voxel, hit_time, push_count}, src.count(), sc, stream);
    return launch<TiledArraySource, HitSink<false>, false>(p, src, HitSink<false>{hit_dir, hit_voxel, hit_time, nullptr},
                                                           src.count(), sc, stream);
}

hipError_t launch_raygen(const och_camera &cam, float *dirs, hipStream_t stream)
{
    const dim3 grid((cam.width + 15) / 16, (cam.height + 15) / 16);
    clear_pending_error(__func__);
    hipLaunchKernelGGL(k_raygen, grid, dim3(256), 0, stream, cam, dirs);
    return hipGetLastError();
}

hipError_t launch_render(const DevPool &p, const DevFrame &f, const Schedule &sc, hipStream_t stream)
{
    if (f.n_views < 1 || f.n_views > kMaxViews) return hipErrorInvalidValue;
    const CameraSource src = camera_source(p, f, sc);
    return launch<CameraSource, FrameSink, false>(p, src, FrameSink{f.out, f.palette, f.n_voxels}, src.count(), sc,
                                                  stream, sc.tile_order == 1 ? 64u * 64u : 0u);
}

hipError_t launch_render_push(const DevPool &p, const DevFrame &f, const Schedule &sc, uint16_t *push, hipStream_t stream)
{
    if (f.n_views < 1 || f.n_views > kMaxViews) return hipErrorInvalidValue;
    DevPool q = p;
    q.cull = 2;                                 // a counting launch culls only at 2: the PUSHes the render walks
    const CameraSource src = camera_source(q, f, sc);
    return launch<CameraSource, PushSink, true>(q, src, PushSink{push}, src.count(), sc, stream);
}

hipError_t launch_render_bounce(const DevPool &p, const DevFrame &f, const Schedule &sc, hipStream_t stream)
{
    if (f.n_views < 1 || f.n_views > kMaxViews) return hipErrorInvalidValue;
    const CameraSource src = camera_source(p, f, sc);
    return launch_bounce<CameraSource, BounceFrameSink, false>(
        p, src, BounceFrameSink{FrameSink{f.out, f.palette, f.n_voxels}}, src.count(), sc, stream);
}

hipError_t launch_render_codes(const DevPool &p, const DevFrame &f, const Schedule &sc, bool bounce, hipStream_t stream)
{
    if (f.n_views < 1 || f.n_views > kMaxViews) return hipErrorInvalidValue;
    const CameraSource src = camera_source(p, f, sc);
    const CodeSink k{f.codes, f.n_voxels};
    if (bounce) return launch_bounce<CameraSource, BounceCodeSink, false>(p, src, BounceCodeSink{k}, src.count(), sc, stream);
    return launch<CameraSource, CodeSink, false>(p, src, k, src.count(), sc, stream,
                                                 sc.tile_order == 1 ? 64u * 64u : 0u);
}

hipError_t launch_shade_unshard(const uint8_t *gathered, uint32_t *frames, const uint32_t *table, int width, int height,
                                int row_chunk, int n_shards, int slice_rows, int n_views, const int32_t *owner,
                                hipStream_t stream)
{
    const bool vec4 = width % 4 == 0 && ((uintptr_t)gathered & 3u) == 0 && ((uintptr_t)frames & 15u) == 0;
    if (vec4) {
        const dim3 grid((width / 4 + 255) / 256, height, n_views);
        clear_pending_error(__func__);
        hipLaunchKernelGGL(k_shade_unshard4, grid, dim3(256), 0, stream, gathered, frames, table, width, height,
                           row_chunk, n_shards, slice_rows, n_views, owner);
        return hipGetLastError();
    }
    const dim3 grid((width + 255) / 256, height, n_views);
    clear_pending_error(__func__);
    hipLaunchKernelGGL(k_shade_unshard, grid, dim3(256), 0, stream, gathered, frames, table, width, height, row_chunk,
                       n_shards, slice_rows, n_views, owner);
    return hipGetLastError();
}

hipError_t launch_trace_bounce_batch(const DevPool &p, const float *origin, int origin_stride, const float *dirs,
                                     uint32_t n, int32_t *hit_dir, uint32_t *hit_voxel, uint32_t *hit_time,
                                     int32_t *bounce_dir, uint32_t *bounce_voxel, uint32_t *bounce_time,
                                     uint32_t *push_count, const Schedule &sc, hipStream_t stream)
{
    const ArraySource src{origin, dirs, origin_stride, n};
    if (push_count)
        return launch_bounce<ArraySource, BounceHitSink<true>, true>(
            p, src, BounceHitSink<true>{HitSink<true>{hit_dir, hit_voxel, hit_time, push_count}, bounce_dir, bounce_voxel,
                                        bounce_time},
            n, sc, stream);
    return launch_bounce<ArraySource, BounceHitSink<false>, false>(
        p, src, BounceHitSink<false>{HitSink<false>{hit_dir, hit_voxel, hit_time, nullptr}, bounce_dir, bounce_voxel,
                                     bounce_time},
        n, sc, stream);
}

hipError_t launch_scatter_slots(const uint32_t *ids, const uint32_t *raw, const uint32_t *packed, uint32_t count,
                                uint32_t *d_raw, uint32_t *d_packed, hipStream_t stream)
{
    if (count == 0) return hipSuccess;
    clear_pending_error(__func__);
    hipLaunchKernelGGL(k_scatter_slots, dim3((count * 8u + 255u) / 256u), dim3(256), 0, stream, ids, raw, packed, count,
                       d_raw, d_packed);
    return hipGetLastError();
}

hipError_t launch_unshard(const uint32_t *gathered, uint32_t *frames, int width, int height, int row_chunk,
                          int n_shards, int slice_rows, int n_views, const int32_t *owner, hipStream_t stream)
{
    const dim3 grid((width + 255) / 256, height, n_views);
    clear_pending_error(__func__);
    hipLaunchKernelGGL(k_unshard, grid, dim3(256), 0, stream, gathered, frames, width, height, row_chunk, n_shards,
                       slice_rows, n_views, owner);
    return hipGetLastError();
}

}  // namespace och
