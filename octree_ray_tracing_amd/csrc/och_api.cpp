// och_api.cpp -- the C ABI (include/och_gpu.h): pools, RCPPS capture, camera
// constants, synchronous and asynchronous trace / render entry points.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "och_internal.h"

namespace {

constexpr uint32_t kIdLimit = 1u << 24;   // packed ids are 24 bits

thread_local std::string g_error;

thread_local const char *t_entry = nullptr;     // outermost C-ABI entry of this thread

// The first pending HIP error a launcher cleared since the last reset, process
// wide (the frame group issues from one thread per device), and how many.
struct Discarded {
    std::mutex m;
    int code = 0;
    int count = 0;
    std::string what;
};

Discarded &discarded()
{
    static Discarded d;
    return d;
}

int fail(int status, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_error = buf;
    return status;
}

#define OCH_HIP(expr)                                                                        \
    do {                                                                                     \
        const hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) return fail(OCH_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

// Keep the caller's current device (torch sets one per rank) across calls.
struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// ------------------------------------------------------------ RCPPS capture

inline uint32_t rcpps_native(uint32_t x)
{
    const __m128 r = _mm_rcp_ps(_mm_castsi128_ps(_mm_set1_epi32((int)x)));
    return (uint32_t)_mm_cvtsi128_si32(_mm_castps_si128(r));
}

struct HostRcp {
    int status = OCH_OK;
    int log2_entries = 0;
    std::vector<uint32_t> lut;
    std::string error;
};

const HostRcp &host_rcp()
{
    static HostRcp cap;
    static std::once_flag once;
    std::call_once(once, [] {
        const uint32_t n = 1u << 23;
        std::vector<uint32_t> full(n);
        for (uint32_t m = 0; m < n; m += 4) {
            const __m128i x = _mm_set_epi32((int)(0xBF800000u | (m + 3)), (int)(0xBF800000u | (m + 2)),
                                            (int)(0xBF800000u | (m + 1)), (int)(0xBF800000u | m));
            _mm_storeu_si128((__m128i *)&full[m], _mm_castps_si128(_mm_rcp_ps(_mm_castsi128_ps(x))));
        }
        // Smallest k such that the result only depends on the top k mantissa bits.
        int k = 23;
        for (int cand = 8; cand <= 23; ++cand) {
            const uint32_t block = 1u << (23 - cand);
            bool ok = true;
            for (uint32_t m = 0; m < n && ok; ++m) ok = full[m] == full[m & ~(block - 1)];
            if (ok) { k = cand; break; }
        }
        cap.log2_entries = k;
        cap.lut.resize(1u << k);
        for (uint32_t i = 0; i < (1u << k); ++i) cap.lut[i] = full[(size_t)i << (23 - k)];
        // Check the exponent model on every exponent (negative inputs, as the tracer uses).
        for (uint32_t e = 0; e < 256 && cap.status == OCH_OK; ++e)
            for (uint32_t m = 0; m < n; m += (e == 127 ? 1u : 997u)) {
                const uint32_t x = 0x80000000u | (e << 23) | m;
                if (e == 255 && m) continue;   // NaN payload handling is not used by the tracer
                const uint32_t want = rcpps_native(x);
                const uint32_t got = och_rcp_from_lut(x, cap.lut.data(), k);
                if (want != got) {
                    cap.status = OCH_E_RCP_MODEL;
                    char buf[160];
                    snprintf(buf, sizeof buf, "host RCPPS(0x%08x) = 0x%08x, table model gives 0x%08x", x, want, got);
                    cap.error = buf;
                    break;
                }
            }
    });
    return cap;
}

}  // namespace

// ------------------------------------------------------------ pool object

struct och_gpu_pool {
    int device = 0;
    uint32_t *d_nodes = nullptr;    // with one padding node in front for 1-based pools
    uint32_t n_nodes = 0;           // nodes in d_nodes
    uint32_t root = 0;
    int depth = 0;
    int index_base = 1;
    float miss_t = INFINITY;
    uint32_t *d_lut = nullptr;
    int lut_log2 = 0;
    uint32_t rcp_xlo = 0, rcp_xspan = 0;   // DevPool::rcp_xlo / rcp_xspan of the uploaded table
    double lut_error = INFINITY;    // maximum relative error of the table (lut_max_rel_error)
    uint32_t *d_palette = nullptr;
    uint32_t n_voxels = 0;
    uint32_t *d_code_table = nullptr;   // OCH_CODE_* -> RGBA8 (256 words), when n_voxels <= OCH_CODE_MAX_VOXELS
    hipStream_t own_stream = nullptr;
    hipStream_t ext_stream = nullptr;
    bool use_ext = false;           // och_gpu_set_stream called: ext_stream (NULL = null stream)
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    bool timed = false;
    // schedule (och_gpu_set_option)
    int opt_block = 64;
    uint64_t *stamps = nullptr;
    uint32_t stamp_cap = 0;
    // host mirror of the uploaded nodes (user numbering), for validating edits
    std::vector<uint32_t> mirror;
    // packed layout (see och_internal.h DevPool)
    uint32_t *d_packed = nullptr;
    uint32_t packed_root = 0;
    uint32_t packed_nodes = 0;
    bool packed_by_slot = false;    // d_packed numbered like d_nodes (editor flushes)
    uint64_t serial = 0;            // process-unique, never reused (och::pool_serial)
    uint64_t last_writer = 0;       // editor id of the last och::pool_commit, 0 otherwise
    bool torn = false;              // a failed editor flush left the slots half written (och::pool_mark_torn)
    int opt_layout = 1;
    int opt_tile_order = 0;
    int opt_bounce_compact = 1;
    int opt_cull = 1;
    int opt_timing = 1;                        // OCH_OPT_TIMING
    int opt_plan = 10;                         // OCH_OPT_PLAN (shape of och_gpu_plan_views' order)
    int opt_split = 0;                         // OCH_OPT_SPLIT: heavy-tile threshold, % of the costliest tile (0 off)
    int opt_split_segs = 4;                    // OCH_OPT_SPLIT_SEGS: lanes per heavy tile's ray (2, 4, 8, 16)
    int opt_split_level = 6;                   // OCH_OPT_SPLIT_LEVEL: the level whose cells are the segments
    hipEvent_t next_ev_start = nullptr;        // och_gpu_set_launch_events: the next launch's events
    hipEvent_t next_ev_stop = nullptr;
    // bounding box of the pool's voxels (voxel units, [lo, hi)), for the cull
    bool box_any = false;
    int32_t box_lo[3] = {0, 0, 0}, box_hi[3] = {0, 0, 0};
    // host-call staging
    void *d_scratch = nullptr;
    size_t scratch_bytes = 0;
    // editor flush staging (och::pool_scatter_slots): pinned host + device, grown on demand
    uint32_t *h_stage = nullptr, *d_stage = nullptr;
    size_t stage_words = 0;
    // cost-planned launch order (och_gpu_plan_views, OCH_OPT_TILE_ORDER = 2)
    // [0] primary frames (grid kernel), [1] config-5 frames (bounce kernel),
    // [2] tiled trace batches (och_gpu_plan_batch_tiled)
    uint32_t *d_order[3] = {nullptr, nullptr, nullptr};
    uint32_t *d_order_xcd[3] = {nullptr, nullptr, nullptr};   // OCH_OPT_TILE_ORDER = 3: grouped per XCD
    uint32_t order_blocks[3] = {0, 0, 0};     // allocated entries
    uint32_t plan_blocks[3] = {0, 0, 0};      // entries of the current plan (its launch's grid)
    int64_t plan_key[3][9] = {};
    // the primary plan's split form (OCH_OPT_SPLIT, plan_split): the heavy tiles'
    // split waves first, then the plan's other workgroups, and the waves' task
    // rows; valid with plan_key[0] while split_params matches the options it was
    // made with
    uint32_t *d_order_split = nullptr, *d_split_tasks = nullptr;
    uint32_t split_alloc = 0, task_alloc = 0, split_n = 0, split_extra = 0, split_tiles = 0;
    int split_params[3] = {0, 0, 0};          // threshold, segments, level
    // row deal (och_gpu_set_row_deal): for frames of deal_h rows in chunks of
    // deal_chunk over deal_n shards, chunk g belongs to a chosen shard instead
    // of g % n; slices hold deal_max chunks (the largest shard's, the rest padded)
    int deal_h = 0, deal_chunk = 0, deal_n = 0, deal_max = 0;
    uint64_t deal_serial = 0;                 // changes with every deal (plan keys)
    int32_t *d_chunk_map = nullptr;           // [deal_n][deal_max] global chunk, -1 = padding
    int32_t *d_owner = nullptr;               // [n_chunks] shard << 16 | local chunk
    std::vector<int32_t> deal_table;          // the chunk -> shard table as set
    bool deal_for(int H, int rc, int n) const { return deal_n && H == deal_h && rc == deal_chunk && n == deal_n; }
    int slice_rows(int H, int rc, int n) const { return deal_for(H, rc, n) ? deal_max * rc : och_shard_rows(H, rc, n); }

    hipStream_t stream() const { return use_ext ? ext_stream : own_stream; }

    och::Schedule schedule() const
    {
        och::Schedule sc;
        sc.block = opt_block;
        sc.tile_order = opt_tile_order;
        sc.bounce_compact = opt_bounce_compact;
        sc.stamps = stamps;
        sc.stamp_cap = stamp_cap;
        sc.order = nullptr;
        sc.order_n = 0;
        sc.cost = nullptr;
        sc.split_tasks = nullptr;
        sc.split_level = 0;
        sc.split_extra = 0;
        sc.ev_start = nullptr;
        sc.ev_stop = nullptr;
        return sc;
    }

    och::DevPool dev() const
    {
        och::DevPool p;
        const bool pk = opt_layout == 1 && d_packed;
        p.nodes = pk ? d_packed : d_nodes;
        p.n_slots = 8u * (pk ? packed_nodes : n_nodes);
        p.packed = pk ? 1 : 0;
        p.lut = d_lut;
        p.rcp_xlo = rcp_xlo;
        p.rcp_xspan = rcp_xspan;
        p.root = pk ? packed_root : root;
        p.depth = depth;
        p.lut_shift = 23 - lut_log2;
        uint32_t mb;
        std::memcpy(&mb, &miss_t, 4);
        p.miss_bits = mb;
        p.half_voxel = std::ldexp(1.0F, -(depth + 1));
        p.dim_lo = 1u << (23 - depth);
        p.dim_span = (1u << 22) - p.dim_lo;
        // 1 + k / 2^depth is an exact float for depth <= 22
        p.cull = box_any ? opt_cull : 0;
        p.cam_cull = lut_error <= och::kCameraCullRcpError ? 1 : 0;
        for (int a = 0; a < 3; ++a) {
            p.cull_lo[a] = 1.0F + std::ldexp((float)box_lo[a], -depth);
            p.cull_hi[a] = 1.0F + std::ldexp((float)box_hi[a], -depth);
        }
        return p;
    }
};

namespace {

int ensure_scratch(och_gpu_pool *p, size_t bytes)
{
    if (bytes <= p->scratch_bytes) return OCH_OK;
    if (p->d_scratch) OCH_HIP(hipFree(p->d_scratch));
    p->d_scratch = nullptr;
    p->scratch_bytes = 0;
    OCH_HIP(hipMalloc(&p->d_scratch, bytes));
    p->scratch_bytes = bytes;
    return OCH_OK;
}

// Launches refuse a pool that a failed editor flush left half written: its
// slots may name nodes that were never uploaded.
int check_ready(const och_gpu_pool *p)
{
    if (p->torn)
        return fail(OCH_E_INVALID, "pool left half written by a failed och_editor_flush: flush the editor again");
    if (!p->d_lut) return fail(OCH_E_RCP_MODEL, "no RCPPS table on this pool (call och_gpu_set_rcp_lut)");
    return OCH_OK;
}

// Walk every reachable (node, level) pair once and check that interior slots
// name nodes inside the pool, so no kernel can read out of bounds.
int validate_pool(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth, int base)
{
    if (depth < 1 || depth > 22) return fail(OCH_E_INVALID, "depth %d outside 1..22", depth);
    if (n_nodes == 0) return fail(OCH_E_INVALID, "empty node array");
    if ((uint64_t)n_nodes + 1 >= (1ull << 29)) return fail(OCH_E_INVALID, "pool of %u nodes exceeds 2^29", n_nodes);
    auto in_range = [&](uint32_t v) { return base == 1 ? (v >= 1 && v <= n_nodes) : (v < n_nodes); };
    if (base == 1 && root == 0) return OCH_OK;   // empty h_octree: every ray misses
    if (!in_range(root)) return fail(OCH_E_INVALID, "root %u outside the pool", root);
    std::vector<uint32_t> seen(n_nodes, 0);
    std::vector<uint32_t> cur{root}, next;
    seen[root - base] |= 1u << 1;
    for (int level = 1; level < depth; ++level) {
        next.clear();
        for (uint32_t v : cur) {
            const uint32_t *c = nodes + (size_t)(v - base) * 8;
            for (int k = 0; k < 8; ++k) {
                if (!c[k]) continue;
                if (!in_range(c[k]) || (base == 0 && c[k] == 0))
                    return fail(OCH_E_INVALID, "node %u (level %d) slot %d names %u, outside the pool", v, level, k, c[k]);
                uint32_t &s = seen[c[k] - base];
                if (!(s & (1u << (level + 1)))) {
                    s |= 1u << (level + 1);
                    next.push_back(c[k]);
                }
            }
        }
        cur.swap(next);
    }
    return OCH_OK;
}

}  // namespace

// Bounding box of the voxels: one post-order walk over the (node, level)
// pairs, each box memoised in node-local voxel units (a DAG shares subtrees;
// a node the caller's table shares between levels gets one entry per level).
bool och::occupied_box(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth, int base, int32_t lo[3],
                       int32_t hi[3])
{
    struct Box {
        int32_t lo[3], hi[3];
        bool empty() const { return lo[0] >= hi[0]; }
    };
    if ((base == 1 && root == 0) || n_nodes == 0) return false;
    std::vector<uint8_t> memo_level(n_nodes, 0);     // level + 1 of memo[i], 0 = none
    std::vector<Box> memo(n_nodes);
    std::unordered_map<uint64_t, Box> extra;
    auto walk = [&](auto &self, uint32_t v, int level) -> Box {
        const uint32_t i = v - base;
        const uint64_t key = ((uint64_t)i << 5) | (uint64_t)level;
        if (memo_level[i] == level + 1) return memo[i];
        if (memo_level[i]) {
            auto it = extra.find(key);
            if (it != extra.end()) return it->second;
        }
        Box b{{INT32_MAX, INT32_MAX, INT32_MAX}, {INT32_MIN, INT32_MIN, INT32_MIN}};
        const int32_t half = 1 << (depth - level - 1);   // a child's size in voxels
        const uint32_t *c = nodes + (size_t)i * 8;
        for (int k = 0; k < 8; ++k) {
            if (!c[k]) continue;
            Box cb{{0, 0, 0}, {1, 1, 1}};                // leaf level: the voxel itself
            if (level + 1 < depth) {
                cb = self(self, c[k], level + 1);
                if (cb.empty()) continue;
            }
            for (int a = 0; a < 3; ++a) {
                const int32_t off = ((k >> a) & 1) * half;
                b.lo[a] = std::min(b.lo[a], off + cb.lo[a]);
                b.hi[a] = std::max(b.hi[a], off + cb.hi[a]);
            }
        }
        if (b.lo[0] == INT32_MAX) b = Box{{0, 0, 0}, {0, 0, 0}};
        if (!memo_level[i]) {
            memo_level[i] = (uint8_t)(level + 1);
            memo[i] = b;
        } else {
            extra.emplace(key, b);
        }
        return b;
    };
    const Box b = walk(walk, root, 0);
    if (b.empty()) return false;
    for (int a = 0; a < 3; ++a) {
        lo[a] = b.lo[a];
        hi[a] = b.hi[a];
    }
    return true;
}

namespace {

void set_box(och_gpu_pool *p, const uint32_t *nodes, uint32_t n_nodes)
{
    p->box_any = och::occupied_box(nodes, n_nodes, p->root, p->depth, p->index_base, p->box_lo, p->box_hi);
}

// Packed layout: every reachable (node, level) pair gets a breadth-first id
// (1-based; 0 is a zero padding node).  Interior slots become
// child_id | child_mask << 24, leaf-level slots keep the voxel ids.  A node
// the caller's table shares between levels (h_octree hash-conses by content
// alone) is simply emitted once per level.  Returns false when more than
// 2^24 - 1 ids would be needed.
bool pack_pool(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth, int base,
               std::vector<uint32_t> &out, uint32_t &packed_root)
{
    auto mask_of = [&](uint32_t v) {
        const uint32_t *c = nodes + (size_t)(v - base) * 8;
        uint32_t m = 0;
        for (int k = 0; k < 8; ++k) m |= (uint32_t)(c[k] != 0) << k;
        return m;
    };
    out.assign(8, 0u);                               // padding node 0
    if (base == 1 && root == 0) {
        packed_root = 0;
        return true;
    }
    // id of (v, level): first_level[v] / first_id[v] hold the common case, a
    // map holds the rare extra levels.
    std::vector<uint8_t> first_level(n_nodes, 0);
    std::vector<uint32_t> first_id(n_nodes, 0);
    std::unordered_map<uint64_t, uint32_t> extra;
    std::vector<uint32_t> order_v;
    std::vector<uint8_t> order_l;
    uint32_t next = 1;
    auto id_of = [&](uint32_t v, int level, bool create) -> uint32_t {
        const uint32_t i = v - base;
        if (first_level[i] == level) return first_id[i];
        if (first_level[i] == 0) {
            if (!create) return 0;
            first_level[i] = (uint8_t)level;
            first_id[i] = next;
            order_v.push_back(v);
            order_l.push_back((uint8_t)level);
            return next++;
        }
        const uint64_t key = ((uint64_t)i << 5) | (uint64_t)level;
        auto it = extra.find(key);
        if (it != extra.end()) return it->second;
        if (!create) return 0;
        extra.emplace(key, next);
        order_v.push_back(v);
        order_l.push_back((uint8_t)level);
        return next++;
    };
    id_of(root, 1, true);
    for (size_t q = 0; q < order_v.size(); ++q) {        // breadth-first: order grows as we go
        const int level = order_l[q];
        if (level >= depth) continue;
        const uint32_t *c = nodes + (size_t)(order_v[q] - base) * 8;
        for (int k = 0; k < 8; ++k)
            if (c[k]) id_of(c[k], level + 1, true);
        if (next > kIdLimit) return false;
    }
    out.resize((size_t)next * 8, 0u);
    for (size_t q = 0; q < order_v.size(); ++q) {
        const uint32_t v = order_v[q];
        const int level = order_l[q];
        const uint32_t *c = nodes + (size_t)(v - base) * 8;
        uint32_t *o = out.data() + (q + 1) * 8;
        for (int k = 0; k < 8; ++k) {
            if (!c[k]) continue;
            o[k] = level == depth ? c[k] : (id_of(c[k], level + 1, false) | (mask_of(c[k]) << 24));
        }
    }
    packed_root = 1u | (mask_of(root) << 24);
    return true;
}

int upload_packed(och_gpu_pool *p, const uint32_t *nodes, uint32_t n_nodes)
{
    std::vector<uint32_t> packed;
    uint32_t proot = 0;
    if (p->d_packed) OCH_HIP(hipFree(p->d_packed));
    p->d_packed = nullptr;
    p->packed_nodes = 0;
    p->packed_by_slot = false;
    if (!pack_pool(nodes, n_nodes, p->root, p->depth, p->index_base, packed, proot))
        return OCH_OK;   // raw only
    OCH_HIP(hipMalloc(&p->d_packed, packed.size() * 4));
    OCH_HIP(hipMemcpy(p->d_packed, packed.data(), packed.size() * 4, hipMemcpyHostToDevice));
    p->packed_root = proot;
    p->packed_nodes = (uint32_t)(packed.size() / 8);
    return OCH_OK;
}

// Largest relative error |r * x - 1| of the table model over x in [-2, -1):
// entry k serves the mantissa bin [k, k + 1) / 2^L, so the extremes are at
// the bin's ends.  Non-finite or zero entries count as an infinite error.
double lut_max_rel_error(const uint32_t *lut, int log2_entries)
{
    const uint32_t n = 1u << log2_entries;
    double worst = 0.0;
    for (uint32_t k = 0; k < n; ++k) {
        float r;
        std::memcpy(&r, &lut[k], 4);
        if (!std::isfinite(r) || r == 0.0F) return INFINITY;
        const double lo = -(1.0 + (double)k / n), hi = -(1.0 + (double)(k + 1) / n);
        worst = std::max({worst, std::fabs((double)r * lo - 1.0), std::fabs((double)r * hi - 1.0)});
    }
    return worst;
}

int upload_lut(och_gpu_pool *p, const uint32_t *lut, int log2_entries)
{
    if (!lut || log2_entries < 1 || log2_entries > 23) return fail(OCH_E_INVALID, "bad RCPPS table");
    if (p->d_lut) OCH_HIP(hipFree(p->d_lut));
    p->d_lut = nullptr;
    const size_t bytes = sizeof(uint32_t) << log2_entries;
    // The device table holds every entry + (127 << 23): the kernels' RCPPS of
    // x = -|d| is then entry - (x's exponent bits) wherever the model's result
    // exponent ent_e + 127 - e stays in 1..254 and the entry is negative -- for
    // e in [max(1, max_e - 127), min_e + 126] over this table's entries (och_kernels.hip
    // rcpps); other x, and every x of a table with a non-negative entry, take
    // the model itself.
    const uint32_t n = 1u << log2_entries;
    std::vector<uint32_t> adj(n);
    int min_e = 255, max_e = 0;
    bool negative = true;
    for (uint32_t k = 0; k < n; ++k) {
        const int e = (int)((lut[k] >> 23) & 0xFFu);
        min_e = std::min(min_e, e);
        max_e = std::max(max_e, e);
        negative = negative && (lut[k] >> 31) != 0;
        adj[k] = lut[k] + (127u << 23);
    }
    const int e_lo = std::max(1, max_e - 127), e_hi = std::min(254, min_e + 126);
    p->rcp_xlo = (uint32_t)e_lo << 23;
    p->rcp_xspan = negative && e_hi >= e_lo ? (uint32_t)(e_hi - e_lo + 1) << 23 : 0u;
    OCH_HIP(hipMalloc(&p->d_lut, bytes));
    OCH_HIP(hipMemcpy(p->d_lut, adj.data(), bytes, hipMemcpyHostToDevice));
    p->lut_log2 = log2_entries;
    // camera_proven_miss budgets the table's error; a coarser table leaves
    // every camera ray to the exact ray_cull
    p->lut_error = lut_max_rel_error(lut, log2_entries);
    return OCH_OK;
}

}  // namespace

extern "C" {

OCH_API int och_abi_version(void) { return OCH_GPU_ABI_VERSION; }

OCH_API const char *och_last_error(void) { return g_error.c_str(); }

OCH_API int och_discarded_error(int *hip_error, int *count, char *what, size_t what_cap, int reset)
{
    auto &d = discarded();
    std::lock_guard<std::mutex> lk(d.m);
    if (hip_error) *hip_error = d.code;
    if (count) *count = d.count;
    if (what && what_cap) snprintf(what, what_cap, "%s", d.what.c_str());
    if (reset) {
        d.code = d.count = 0;
        d.what.clear();
    }
    return OCH_OK;
}

OCH_API int och_device_list(int *devices, int capacity, int *count)
{
    if (!count || (capacity > 0 && !devices)) return fail(OCH_E_INVALID, "NULL argument");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    int gfx950 = 0;
    for (int i = 0; i < n; ++i) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, i) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0) {
            if (gfx950 < capacity) devices[gfx950] = i;
            ++gfx950;
        }
    }
    *count = gfx950;
    return OCH_OK;
}

OCH_API int och_device_count(int *count)
{
    if (!count) return fail(OCH_E_INVALID, "count is NULL");
    return och_device_list(nullptr, 0, count);
}

OCH_API uint32_t och_rcp_from_lut(uint32_t x, const uint32_t *lut, int log2_entries)
{
    const uint32_t sign = x & 0x80000000u, e = (x >> 23) & 0xFFu;
    if (e == 0) return sign | 0x7F800000u;
    if (e == 0xFFu) return (x & 0x7FFFFFu) ? (x | 0x400000u) : sign;
    const uint32_t ent = lut[(x & 0x7FFFFFu) >> (23 - log2_entries)];
    const int ne = (int)((ent >> 23) & 0xFFu) + 127 - (int)e;
    return ne <= 0 ? sign : (sign | ((uint32_t)ne << 23) | (ent & 0x7FFFFFu));
}

OCH_API int och_rcp_lut_error(const uint32_t *lut, int log2_entries, double *max_rel_error)
{
    if (!lut || !max_rel_error || log2_entries < 1 || log2_entries > 23) return fail(OCH_E_INVALID, "bad RCPPS table");
    *max_rel_error = lut_max_rel_error(lut, log2_entries);
    return OCH_OK;
}

OCH_API int och_host_rcp_lut(uint32_t *lut, int *log2_entries)
{
    const HostRcp &c = host_rcp();
    if (c.status != OCH_OK) return fail(c.status, "%s", c.error.c_str());
    if (lut) std::memcpy(lut, c.lut.data(), c.lut.size() * sizeof(uint32_t));
    if (log2_entries) *log2_entries = c.log2_entries;
    return OCH_OK;
}

OCH_API int och_gpu_pool_create(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth, int index_base,
                                float miss_t, int device, och_gpu_pool **out)
{
    if (!nodes || !out) return fail(OCH_E_INVALID, "nodes/out is NULL");
    if (index_base != 0 && index_base != 1) return fail(OCH_E_INVALID, "index_base must be 0 or 1");
    *out = nullptr;
    int st = validate_pool(nodes, n_nodes, root, depth, index_base);
    if (st != OCH_OK) return st;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(OCH_E_NODEV, "no HIP device visible");
    if (device < 0) OCH_HIP(hipGetDevice(&device));
    if (device >= ndev) return fail(OCH_E_NODEV, "device %d of %d", device, ndev);
    DeviceGuard g(device);
    if (!g.ok) return fail(OCH_E_HIP, "hipSetDevice(%d) failed", device);

    och_gpu_pool *p = new och_gpu_pool;
    static std::atomic<uint64_t> next_serial{1};
    p->serial = next_serial.fetch_add(1);
    p->device = device;
    p->depth = depth;
    p->index_base = index_base;
    p->miss_t = miss_t;
    p->root = root;
    p->n_nodes = n_nodes + (uint32_t)index_base;   // padding node 0 for 1-based pools
    const size_t bytes = (size_t)p->n_nodes * 32;
    auto bail = [&](int s) { och_gpu_pool_destroy(p); return s; };
    if (hipMalloc(&p->d_nodes, bytes) != hipSuccess) return bail(fail(OCH_E_NOMEM, "hipMalloc(%zu) failed", bytes));
    if (index_base == 1 && hipMemset(p->d_nodes, 0, 32) != hipSuccess) return bail(fail(OCH_E_HIP, "hipMemset failed"));
    if (hipMemcpy(p->d_nodes + 8 * index_base, nodes, (size_t)n_nodes * 32, hipMemcpyHostToDevice) != hipSuccess)
        return bail(fail(OCH_E_HIP, "node upload failed"));
    p->mirror.assign(nodes, nodes + (size_t)n_nodes * 8);
    set_box(p, nodes, n_nodes);
    st = upload_packed(p, nodes, n_nodes);
    if (st != OCH_OK) return bail(st);
    if (hipStreamCreateWithFlags(&p->own_stream, hipStreamNonBlocking) != hipSuccess ||
        // timing only: no system-scope release at the timed kernel's end
        hipEventCreateWithFlags(&p->ev_start, hipEventDisableSystemFence) != hipSuccess ||
        hipEventCreateWithFlags(&p->ev_stop, hipEventDisableSystemFence) != hipSuccess)
        return bail(fail(OCH_E_HIP, "stream/event creation failed"));
    const HostRcp &rc = host_rcp();
    if (rc.status == OCH_OK) {
        st = upload_lut(p, rc.lut.data(), rc.log2_entries);
        if (st != OCH_OK) return bail(st);
    }
    // A host whose RCPPS does not fit the model leaves the pool without a table:
    // tracing then fails with OCH_E_RCP_MODEL until och_gpu_set_rcp_lut is called.
    *out = p;
    return OCH_OK;
}

OCH_API int och_gpu_pool_destroy(och_gpu_pool *p)
{
    if (!p) return OCH_OK;
    DeviceGuard g(p->device);
    if (p->own_stream) (void)hipStreamSynchronize(p->own_stream);
    if (p->use_ext) (void)hipStreamSynchronize(p->ext_stream);
    if (p->d_nodes) (void)hipFree(p->d_nodes);
    if (p->d_packed) (void)hipFree(p->d_packed);
    if (p->d_lut) (void)hipFree(p->d_lut);
    if (p->d_palette) (void)hipFree(p->d_palette);
    if (p->d_code_table) (void)hipFree(p->d_code_table);
    if (p->d_scratch) (void)hipFree(p->d_scratch);
    if (p->h_stage) (void)hipHostFree(p->h_stage);
    if (p->d_stage) (void)hipFree(p->d_stage);
    for (uint32_t *o : p->d_order)
        if (o) (void)hipFree(o);
    if (p->d_order_split) (void)hipFree(p->d_order_split);
    if (p->d_split_tasks) (void)hipFree(p->d_split_tasks);
    for (uint32_t *o : p->d_order_xcd)
        if (o) (void)hipFree(o);
    if (p->d_chunk_map) (void)hipFree(p->d_chunk_map);
    if (p->d_owner) (void)hipFree(p->d_owner);
    if (p->ev_start) (void)hipEventDestroy(p->ev_start);
    if (p->ev_stop) (void)hipEventDestroy(p->ev_stop);
    if (p->own_stream) (void)hipStreamDestroy(p->own_stream);
    delete p;
    return OCH_OK;
}

OCH_API int och_gpu_pool_info(const och_gpu_pool *p, och_pool_info *info)
{
    if (!p || !info) return fail(OCH_E_INVALID, "pool/info is NULL");
    info->device_bytes = (uint64_t)p->n_nodes * 32;
    info->n_nodes = p->n_nodes;
    info->root = p->root;
    info->depth = p->depth;
    info->index_base = p->index_base;
    info->miss_t = p->miss_t;
    info->rcp_log2_entries = p->d_lut ? p->lut_log2 : 0;
    info->device = p->device;
    return OCH_OK;
}

OCH_API int och_gpu_pool_update(och_gpu_pool *p, uint32_t first, uint32_t count, const uint32_t *nodes, uint32_t root)
{
    OCH_ENTRY();
    if (!p || (count && !nodes)) return fail(OCH_E_INVALID, "pool/nodes is NULL");
    if (p->torn) return fail(OCH_E_INVALID, "pool left half written by a failed och_editor_flush: flush the editor again");
    const uint32_t n_user = p->n_nodes - (uint32_t)p->index_base;
    const uint32_t lo = p->index_base == 1 ? 1u : 0u;
    if (count && (first < lo || (uint64_t)first - lo + count > n_user))
        return fail(OCH_E_INVALID, "update [%u, +%u) outside the pool", first, count);
    // Apply to the host mirror and re-validate everything reachable from the
    // new root before any byte reaches the device (h_octree::set keeps the
    // pool consistent, ORT/och_h_octree.h:176-237; a bad edit must not fault).
    const size_t off = (size_t)(first - lo) * 8;
    std::vector<uint32_t> saved(p->mirror.begin() + off, p->mirror.begin() + off + (size_t)count * 8);
    std::memcpy(p->mirror.data() + off, nodes, (size_t)count * 32);
    const int st = validate_pool(p->mirror.data(), n_user, root, p->depth, p->index_base);
    if (st != OCH_OK) {
        std::memcpy(p->mirror.data() + off, saved.data(), saved.size() * 4);
        return st;
    }
    // slots are rewritten in place: kernels of frames in flight on any stream
    // may still walk them (as the editor's flush)
    int ds = och::pool_drain(p);
    if (ds != OCH_OK) return ds;
    DeviceGuard g(p->device);
    if (count)
        OCH_HIP(hipMemcpyAsync(p->d_nodes + 8 * (size_t)(first - lo + p->index_base), p->mirror.data() + off,
                               (size_t)count * 32, hipMemcpyHostToDevice, p->stream()));
    OCH_HIP(hipStreamSynchronize(p->stream()));
    p->root = root;
    p->last_writer = 0;
    set_box(p, p->mirror.data(), n_user);
    return upload_packed(p, p->mirror.data(), n_user);
}

}  // extern "C"

int och::report(int status, const char *msg) { return fail(status, "%s", msg); }

// ------------------------------------------------------------ discarded errors


och::EntryScope::EntryScope(const char *name) : prev(t_entry)
{
    if (!t_entry) t_entry = name;
}

och::EntryScope::~EntryScope() { t_entry = prev; }

void och::clear_pending_error(const char *launcher)
{
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return;
    Discarded &d = discarded();
    std::lock_guard<std::mutex> lk(d.m);
    if (d.count++ == 0) {
        char buf[320];
        snprintf(buf, sizeof buf, "%s (%d) pending at %s, cleared by %s", hipGetErrorName(e), (int)e,
                 t_entry ? t_entry : "an internal call", launcher);
        d.code = (int)e;
        d.what = buf;
    }
}

uint64_t och::pool_serial(const och_gpu_pool *p) { return p ? p->serial : 0; }
void *och::pool_stream(const och_gpu_pool *p) { return p ? static_cast<void *>(p->stream()) : nullptr; }
int och::pool_palette_size(const och_gpu_pool *p, int *n)
{
    if (!p || !n) return fail(OCH_E_INVALID, "NULL argument");
    *n = (int)p->n_voxels;
    return OCH_OK;
}
uint64_t och::pool_last_writer(const och_gpu_pool *p) { return p ? p->last_writer : 0; }

int och::pool_drain(och_gpu_pool *p)
{
    if (!p) return fail(OCH_E_INVALID, "pool is NULL");
    DeviceGuard g(p->device);
    // Every stream, not just the pool's: bench and frame code rotate the pool
    // over several streams with frames in flight, and a kernel still walking a
    // slot that is rewritten in place could read a torn DAG.
    OCH_HIP(hipDeviceSynchronize());
    return OCH_OK;
}

int och::pool_write_slots(och_gpu_pool *p, uint32_t first, uint32_t count, const uint32_t *raw,
                          const uint32_t *packed, bool full)
{
    if (!p || p->index_base != 1 || (count && !raw)) return fail(OCH_E_INVALID, "bad editor flush");
    if ((uint64_t)first + count > p->n_nodes || (full && (first != 0 || count != p->n_nodes)))
        return fail(OCH_E_INVALID, "editor window [%u, +%u) outside the pool", first, count);
    if (packed && p->n_nodes > kIdLimit) return fail(OCH_E_INVALID, "packed ids exceed 24 bits");
    if (packed && !full && (!p->d_packed || !p->packed_by_slot))
        return fail(OCH_E_INVALID, "packed buffer is not in editor numbering");
    DeviceGuard g(p->device);
    p->last_writer = 0;                 // until pool_commit: a failed flush forces a full rewrite
    // mirror and raw device slots: slot 0 is the padding node, never written
    const uint32_t lo = first ? first : 1;
    const uint32_t skip = lo - first;
    if (count > skip) {
        const size_t n = (size_t)(count - skip) * 8;
        std::memcpy(p->mirror.data() + (size_t)(lo - 1) * 8, raw + (size_t)skip * 8, n * 4);
        OCH_HIP(hipMemcpy(p->d_nodes + (size_t)lo * 8, raw + (size_t)skip * 8, n * 4, hipMemcpyHostToDevice));
    }
    if (!packed) return OCH_OK;
    if (full && (!p->d_packed || !p->packed_by_slot || p->packed_nodes != p->n_nodes)) {
        if (p->d_packed) OCH_HIP(hipFree(p->d_packed));
        p->d_packed = nullptr;
        p->packed_nodes = 0;
        p->packed_by_slot = false;
        OCH_HIP(hipMalloc(&p->d_packed, (size_t)p->n_nodes * 32));
        p->packed_nodes = p->n_nodes;
        p->packed_by_slot = true;
    }
    if (count)
        OCH_HIP(hipMemcpy(p->d_packed + (size_t)first * 8, packed, (size_t)count * 32, hipMemcpyHostToDevice));
    return OCH_OK;
}

int och::pool_scatter_slots(och_gpu_pool *p, const uint32_t *ids, uint32_t count, const uint32_t *raw,
                            const uint32_t *packed)
{
    if (!p || p->index_base != 1 || (count && (!ids || !raw))) return fail(OCH_E_INVALID, "bad editor flush");
    if (packed && (!p->d_packed || !p->packed_by_slot))
        return fail(OCH_E_INVALID, "packed buffer is not in editor numbering");
    if (count == 0) return OCH_OK;
    for (uint32_t i = 0; i < count; ++i)
        if (ids[i] == 0 || ids[i] >= p->n_nodes) return fail(OCH_E_INVALID, "editor slot %u outside the pool", ids[i]);
    DeviceGuard g(p->device);
    p->last_writer = 0;                 // until pool_commit
    // staging: [ids | raw | packed]
    const size_t words = (size_t)count * (packed ? 17 : 9);
    if (words > p->stage_words) {
        if (p->h_stage) OCH_HIP(hipHostFree(p->h_stage));
        if (p->d_stage) OCH_HIP(hipFree(p->d_stage));
        p->h_stage = p->d_stage = nullptr;
        p->stage_words = 0;
        const size_t cap = std::max<size_t>(words, 1 << 16);
        OCH_HIP(hipHostMalloc(&p->h_stage, cap * 4, hipHostMallocDefault));
        OCH_HIP(hipMalloc(&p->d_stage, cap * 4));
        p->stage_words = cap;
    }
    std::memcpy(p->h_stage, ids, (size_t)count * 4);
    std::memcpy(p->h_stage + count, raw, (size_t)count * 32);
    if (packed) std::memcpy(p->h_stage + 9 * (size_t)count, packed, (size_t)count * 32);
    for (uint32_t i = 0; i < count; ++i)       // host mirror (user numbering, slot s at row s - 1)
        std::memcpy(p->mirror.data() + (size_t)(ids[i] - 1) * 8, raw + (size_t)i * 8, 32);
    const hipStream_t s = p->stream();
    OCH_HIP(hipMemcpyAsync(p->d_stage, p->h_stage, words * 4, hipMemcpyHostToDevice, s));
    OCH_HIP(och::launch_scatter_slots(p->d_stage, p->d_stage + count, packed ? p->d_stage + 9 * (size_t)count : nullptr,
                                      count, p->d_nodes, packed ? p->d_packed : nullptr, s));
    OCH_HIP(hipStreamSynchronize(s));
    return OCH_OK;
}

int och::pool_commit(och_gpu_pool *p, uint32_t root, uint32_t packed_root, bool packed, uint64_t writer,
                     const int32_t *box_lo, const int32_t *box_hi)
{
    if (!p || p->index_base != 1) return fail(OCH_E_INVALID, "bad editor flush");
    if (packed && (!p->d_packed || !p->packed_by_slot))
        return fail(OCH_E_INVALID, "packed buffer is not in editor numbering");
    DeviceGuard g(p->device);
    if (!packed && p->d_packed) {
        OCH_HIP(hipFree(p->d_packed));
        p->d_packed = nullptr;
        p->packed_nodes = 0;
        p->packed_by_slot = false;
    }
    p->root = root;
    p->packed_root = packed ? packed_root : 0;
    p->box_any = box_lo && box_hi;
    for (int a = 0; a < 3; ++a) {
        p->box_lo[a] = p->box_any ? box_lo[a] : 0;
        p->box_hi[a] = p->box_any ? box_hi[a] : 0;
    }
    p->last_writer = writer;
    p->torn = false;
    return OCH_OK;
}

int och::pool_mark_torn(och_gpu_pool *p)
{
    if (!p) return OCH_E_INVALID;
    DeviceGuard g(p->device);
    (void)hipDeviceSynchronize();
    if (p->d_packed) (void)hipFree(p->d_packed);
    p->d_packed = nullptr;
    p->packed_nodes = 0;
    p->packed_by_slot = false;
    p->packed_root = 0;
    p->root = 0;
    p->box_any = false;
    p->last_writer = 0;
    p->torn = true;
    return OCH_OK;
}

extern "C" {

OCH_API int och_gpu_set_rcp_lut(och_gpu_pool *p, const uint32_t *lut, int log2_entries)
{
    if (!p) return fail(OCH_E_INVALID, "pool is NULL");
    DeviceGuard g(p->device);
    OCH_HIP(hipStreamSynchronize(p->stream()));
    return upload_lut(p, lut, log2_entries);
}

OCH_API int och_gpu_set_palette(och_gpu_pool *p, const uint32_t *rgba, uint32_t n_voxels)
{
    if (!p || (n_voxels && !rgba)) return fail(OCH_E_INVALID, "pool/palette is NULL");
    DeviceGuard g(p->device);
    OCH_HIP(hipStreamSynchronize(p->stream()));
    if (p->d_palette) OCH_HIP(hipFree(p->d_palette));
    if (p->d_code_table) OCH_HIP(hipFree(p->d_code_table));
    p->d_palette = nullptr;
    p->d_code_table = nullptr;
    p->n_voxels = 0;
    if (n_voxels <= OCH_CODE_MAX_VOXELS) {
        // Indexed-colour frames: trace_pixel's colour per code
        // (ORT/test_och_h_octree.cpp:76-84), then config 5's blocked (halved) variants.
        std::vector<uint32_t> t(256, 0xFFFF00FFu);
        for (uint32_t c = 0; c < 6 * n_voxels; ++c) t[c] = rgba[c];
        t[OCH_CODE_INSIDE] = 0xFF07193Fu;
        t[OCH_CODE_SKY] = 0xFFFEBF00u;
        for (uint32_t c = 0; c < OCH_CODE_BLOCKED; ++c)
            t[c | OCH_CODE_BLOCKED] = ((t[c] >> 1) & 0x007F7F7Fu) | (t[c] & 0xFF000000u);
        OCH_HIP(hipMalloc(&p->d_code_table, 256 * 4));
        OCH_HIP(hipMemcpy(p->d_code_table, t.data(), 256 * 4, hipMemcpyHostToDevice));
    }
    if (!n_voxels) return OCH_OK;
    OCH_HIP(hipMalloc(&p->d_palette, (size_t)n_voxels * 6 * 4));
    OCH_HIP(hipMemcpy(p->d_palette, rgba, (size_t)n_voxels * 6 * 4, hipMemcpyHostToDevice));
    p->n_voxels = n_voxels;
    return OCH_OK;
}

OCH_API int och_gpu_set_stream(och_gpu_pool *p, void *stream)
{
    if (!p) return fail(OCH_E_INVALID, "pool is NULL");
    p->ext_stream = (hipStream_t)stream;
    p->use_ext = true;
    return OCH_OK;
}

// Option ids retired in round 5 (measured slower on every scene, DESIGN.md
// §8): 0 schedule (persistent / refill), 2 waves per CU, 3 refill, 7 chunk
// tiles, 9 merge, 12 per-node skip, 13 column cull.  Their ids stay unused.
static int retired_option(int option)
{
    return fail(OCH_E_INVALID, "option %d was retired (the grid schedule alone remains; DESIGN.md section 8)", option);
}

OCH_API int och_gpu_set_option(och_gpu_pool *p, int option, int value)
{
    if (!p) return fail(OCH_E_INVALID, "pool is NULL");
    switch (option) {
    case OCH_OPT_BLOCK:
        if (value < 64 || value > 1024 || value % 64) return fail(OCH_E_INVALID, "block %d", value);
        p->opt_block = value;
        return OCH_OK;
    case OCH_OPT_LAYOUT:
        if (value != 0 && value != 1) return fail(OCH_E_INVALID, "layout must be 0 or 1");
        if (value == 1 && !p->d_packed) return fail(OCH_E_INVALID, "pool too large for the packed layout");
        p->opt_layout = value;
        return OCH_OK;
    case OCH_OPT_TILE_ORDER:
        if (value < 0 || value > 3) return fail(OCH_E_INVALID, "tile order must be 0..3");
        p->opt_tile_order = value;
        return OCH_OK;
    case OCH_OPT_BOUNCE_COMPACT:
        if (value < 0 || value > 2) return fail(OCH_E_INVALID, "bounce compaction must be 0, 1 or 2");
        p->opt_bounce_compact = value;
        return OCH_OK;
    case OCH_OPT_CULL:
        if (value < 0 || value > 2) return fail(OCH_E_INVALID, "cull must be 0, 1 or 2");
        p->opt_cull = value;
        return OCH_OK;
    case OCH_OPT_TIMING:
        if (value < 0 || value > 2) return fail(OCH_E_INVALID, "timing must be 0, 1 or 2");
        p->opt_timing = value;
        return OCH_OK;
    case OCH_OPT_PLAN:
        if (value < 0 || value > 100) return fail(OCH_E_INVALID, "plan shape must be 0..100");
        p->opt_plan = value;
        return OCH_OK;
    case OCH_OPT_SPLIT:
        if (value < 0 || value > 100) return fail(OCH_E_INVALID, "split threshold must be 0..100 (%% of the costliest tile)");
        p->opt_split = value;
        return OCH_OK;
    case OCH_OPT_SPLIT_SEGS:
        if (value != 2 && value != 4 && value != 8 && value != 16) return fail(OCH_E_INVALID, "split segments must be 2, 4, 8 or 16");
        p->opt_split_segs = value;
        return OCH_OK;
    case OCH_OPT_SPLIT_LEVEL:
        if (value < 1 || value > 21) return fail(OCH_E_INVALID, "split level must be 1..21");
        p->opt_split_level = value;
        return OCH_OK;
    case OCH_OPT_SPLIT_TILES:
        return fail(OCH_E_INVALID, "OCH_OPT_SPLIT_TILES is read-only");
    case 0: case 2: case 3: case 7: case 9: case 12: case 13:
        return retired_option(option);
    default:
        return fail(OCH_E_INVALID, "unknown option %d", option);
    }
}

OCH_API int och_gpu_get_option(const och_gpu_pool *p, int option, int *value)
{
    if (!p || !value) return fail(OCH_E_INVALID, "NULL argument");
    switch (option) {
    case OCH_OPT_BLOCK: *value = p->opt_block; return OCH_OK;
    case OCH_OPT_LAYOUT: *value = (p->opt_layout == 1 && p->d_packed) ? 1 : 0; return OCH_OK;
    case OCH_OPT_TILE_ORDER: *value = p->opt_tile_order; return OCH_OK;
    case OCH_OPT_BOUNCE_COMPACT: *value = p->opt_bounce_compact; return OCH_OK;
    case OCH_OPT_CULL: *value = p->opt_cull; return OCH_OK;
    case OCH_OPT_TIMING: *value = p->opt_timing; return OCH_OK;
    case OCH_OPT_PLAN: *value = p->opt_plan; return OCH_OK;
    case OCH_OPT_SPLIT: *value = p->opt_split; return OCH_OK;
    case OCH_OPT_SPLIT_SEGS: *value = p->opt_split_segs; return OCH_OK;
    case OCH_OPT_SPLIT_LEVEL: *value = p->opt_split_level; return OCH_OK;
    case OCH_OPT_SPLIT_TILES: *value = (int)p->split_tiles; return OCH_OK;
    case 0: case 2: case 3: case 7: case 9: case 12: case 13:
        return retired_option(option);
    default: return fail(OCH_E_INVALID, "unknown option %d", option);
    }
}

OCH_API int och_gpu_occupancy(const och_gpu_pool *p, int kind, int *blocks_per_cu)
{
    if (!p || !blocks_per_cu) return fail(OCH_E_INVALID, "NULL argument");
    DeviceGuard g(p->device);
    OCH_HIP(och::occupancy_blocks_per_cu(kind, p->opt_block, p->depth, blocks_per_cu));
    return OCH_OK;
}

OCH_API int och_gpu_set_stamp_buffer(och_gpu_pool *p, uint64_t *stamps, uint32_t capacity_waves)
{
    if (!p) return fail(OCH_E_INVALID, "pool is NULL");
    p->stamps = capacity_waves ? stamps : nullptr;
    p->stamp_cap = stamps ? capacity_waves : 0;
    return OCH_OK;
}

namespace {

// Per-launch timing of the traversal kernel (OCH_OPT_TIMING).  1 (default):
// the dispatch itself records the pool's events (hipExtLaunchKernel, no
// packets of its own); 2: hipEventRecord before and after the launch (two
// marker packets, each with a system-scope release: ~10 us of idle GPU
// between two launches of a stream); 0: none.  Events handed
// over by och_gpu_set_launch_events take the place of the pool's for one launch.
och::Schedule timed_schedule(och_gpu_pool *p, int &st)
{
    och::Schedule sc = p->schedule();
    st = OCH_OK;
    if (p->next_ev_start || p->next_ev_stop) {
        sc.ev_start = p->next_ev_start;
        sc.ev_stop = p->next_ev_stop;
        p->next_ev_start = p->next_ev_stop = nullptr;
    } else if (p->opt_timing == 1) {
        sc.ev_start = p->ev_start;
        sc.ev_stop = p->ev_stop;
    } else if (p->opt_timing == 2 && hipEventRecord(p->ev_start, p->stream()) != hipSuccess) {
        st = fail(OCH_E_HIP, "hipEventRecord: %s", hipGetErrorString(hipGetLastError()));
    }
    return sc;
}

// After the launch: och_gpu_last_kernel_ms reads the pool's events only if
// this launch recorded them (n = 0 launches nothing).
int timed_done(och_gpu_pool *p, const och::Schedule &sc, bool launched)
{
    if (sc.ev_start == p->ev_start && sc.ev_start) {
        p->timed = launched;
    } else if (!sc.ev_start && !sc.ev_stop && p->opt_timing == 2) {
        OCH_HIP(hipEventRecord(p->ev_stop, p->stream()));
        p->timed = true;
    } else {
        p->timed = false;
    }
    return OCH_OK;
}

}  // namespace

OCH_API int och_gpu_set_launch_events(och_gpu_pool *p, void *start_event, void *stop_event)
{
    if (!p) return fail(OCH_E_INVALID, "pool is NULL");
    p->next_ev_start = static_cast<hipEvent_t>(start_event);
    p->next_ev_stop = static_cast<hipEvent_t>(stop_event);
    return OCH_OK;
}

OCH_API int och_gpu_synchronize(och_gpu_pool *p)
{
    if (!p) return fail(OCH_E_INVALID, "pool is NULL");
    DeviceGuard g(p->device);
    OCH_HIP(hipStreamSynchronize(p->stream()));
    return OCH_OK;
}

OCH_API int och_gpu_last_kernel_ms(och_gpu_pool *p, float *ms)
{
    if (!p || !ms) return fail(OCH_E_INVALID, "pool/ms is NULL");
    if (!p->timed)
        return fail(OCH_E_INVALID, "the last launch on this pool was not timed (none yet, n = 0, OCH_OPT_TIMING 0, "
                                   "or the caller's events)");
    DeviceGuard g(p->device);
    OCH_HIP(hipEventSynchronize(p->ev_stop));
    OCH_HIP(hipEventElapsedTime(ms, p->ev_start, p->ev_stop));
    return OCH_OK;
}

OCH_API int och_gpu_trace_batch_dev(och_gpu_pool *p, const float *origin, int origin_stride, const float *dirs,
                                    uint32_t n, int32_t *hit_dir, uint32_t *hit_voxel, float *hit_time,
                                    uint32_t *push_count)
{
    OCH_ENTRY();
    if (!p || (n && (!origin || !dirs || !hit_dir || !hit_voxel || !hit_time)))
        return fail(OCH_E_INVALID, "NULL argument");
    if (origin_stride != 0 && origin_stride != 3) return fail(OCH_E_INVALID, "origin_stride must be 0 or 3");
    if (int rs = check_ready(p)) return rs;
    DeviceGuard g(p->device);
    int ts;
    const och::Schedule sc = timed_schedule(p, ts);
    if (ts) return ts;
    OCH_HIP(och::launch_trace_batch(p->dev(), origin, origin_stride, dirs, n, hit_dir, hit_voxel,
                                    reinterpret_cast<uint32_t *>(hit_time), push_count, sc, p->stream()));
    return timed_done(p, sc, n > 0);
}

OCH_API int och_gpu_trace_bounce_batch_dev(och_gpu_pool *p, const float *origin, int origin_stride, const float *dirs,
                                           uint32_t n, int32_t *hit_dir, uint32_t *hit_voxel, float *hit_time,
                                           int32_t *bounce_dir, uint32_t *bounce_voxel, float *bounce_time,
                                           uint32_t *push_count)
{
    OCH_ENTRY();
    if (!p || (n && (!origin || !dirs || !hit_dir || !hit_voxel || !hit_time || !bounce_dir || !bounce_voxel ||
                     !bounce_time)))
        return fail(OCH_E_INVALID, "NULL argument");
    if (origin_stride != 0 && origin_stride != 3) return fail(OCH_E_INVALID, "origin_stride must be 0 or 3");
    if (int rs = check_ready(p)) return rs;
    DeviceGuard g(p->device);
    int ts;
    const och::Schedule sc = timed_schedule(p, ts);
    if (ts) return ts;
    OCH_HIP(och::launch_trace_bounce_batch(p->dev(), origin, origin_stride, dirs, n, hit_dir, hit_voxel,
                                           reinterpret_cast<uint32_t *>(hit_time), bounce_dir, bounce_voxel,
                                           reinterpret_cast<uint32_t *>(bounce_time), push_count, sc, p->stream()));
    return timed_done(p, sc, n > 0);
}

namespace {

int tiled_args(const och_gpu_pool *p, const float *origin, int origin_stride, const float *dirs, uint32_t n,
               uint32_t width)
{
    if (!p || (n && (!origin || !dirs))) return fail(OCH_E_INVALID, "NULL argument");
    if (origin_stride != 0 && origin_stride != 3) return fail(OCH_E_INVALID, "origin_stride must be 0 or 3");
    if (width == 0) return fail(OCH_E_INVALID, "width must be positive");
    const uint64_t rows = ((uint64_t)n + width - 1) / width;
    if ((uint64_t)((width + 7) / 8) * ((rows + 7) / 8) * 64 >= (1ull << 32))
        return fail(OCH_E_INVALID, "batch of %u rays %u wide too large", n, width);
    return check_ready(p);
}

// The key of a tiled batch's launch plan: the geometry and the block size.
void batch_key(const och_gpu_pool *p, uint32_t n, uint32_t width, int64_t key[9])
{
    const int64_t k[9] = {n, width, p->opt_block, 0, 0, 0, 0, 0, 0};
    std::memcpy(key, k, sizeof k);
}

}  // namespace

OCH_API int och_gpu_trace_batch_tiled_dev(och_gpu_pool *p, const float *origin, int origin_stride, const float *dirs,
                                          uint32_t n, uint32_t width, int32_t *hit_dir, uint32_t *hit_voxel,
                                          float *hit_time, uint32_t *push_count)
{
    OCH_ENTRY();
    if (int st = tiled_args(p, origin, origin_stride, dirs, n, width)) return st;
    if (n && (!hit_dir || !hit_voxel || !hit_time)) return fail(OCH_E_INVALID, "NULL argument");
    DeviceGuard g(p->device);
    int ts;
    och::Schedule sc = timed_schedule(p, ts);
    if (ts) return ts;
    if (p->opt_tile_order >= 2 && p->d_order[2]) {
        int64_t key[9];
        batch_key(p, n, width, key);
        if (std::memcmp(key, p->plan_key[2], sizeof key) == 0) {
            sc.order = p->d_order[2];
            sc.order_n = p->plan_blocks[2];
        }
    }
    OCH_HIP(och::launch_trace_batch_tiled(p->dev(), origin, origin_stride, dirs, n, width, hit_dir, hit_voxel,
                                          reinterpret_cast<uint32_t *>(hit_time), push_count, sc, p->stream()));
    return timed_done(p, sc, n > 0);
}

OCH_API int och_gpu_plan_batch_tiled(och_gpu_pool *p, const float *origin, int origin_stride, const float *dirs,
                                     uint32_t n, uint32_t width)
{
    OCH_ENTRY();
    if (int st = tiled_args(p, origin, origin_stride, dirs, n, width)) return st;
    if (n == 0) return OCH_OK;
    DeviceGuard g(p->device);
    const uint32_t tiles = ((width + 7) / 8) * (uint32_t)(((n + width - 1) / width + 7) / 8);
    const uint32_t max_blocks = (uint32_t)(((uint64_t)tiles * 64 + p->opt_block - 1) / p->opt_block);
    const size_t out_bytes = (((size_t)n * 4 + 255) & ~(size_t)255);
    int st = ensure_scratch(p, 3 * out_bytes + (size_t)max_blocks * 4);
    if (st != OCH_OK) return st;
    char *base = static_cast<char *>(p->d_scratch);
    uint32_t *cost = reinterpret_cast<uint32_t *>(base + 3 * out_bytes);
    OCH_HIP(hipMemsetAsync(cost, 0xFF, (size_t)max_blocks * 4, p->stream()));
    och::Schedule sc = p->schedule();
    sc.tile_order = 0;
    sc.cost = cost;
    OCH_HIP(och::launch_trace_batch_tiled(p->dev(), origin, origin_stride, dirs, n, width,
                                          reinterpret_cast<int32_t *>(base), reinterpret_cast<uint32_t *>(base + out_bytes),
                                          reinterpret_cast<uint32_t *>(base + 2 * out_bytes), nullptr, sc, p->stream()));
    std::vector<uint32_t> c(max_blocks);
    OCH_HIP(hipMemcpyAsync(c.data(), cost, (size_t)max_blocks * 4, hipMemcpyDeviceToHost, p->stream()));
    OCH_HIP(hipStreamSynchronize(p->stream()));
    std::vector<uint32_t> order(max_blocks);
    for (uint32_t i = 0; i < max_blocks; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return c[a] > c[b]; });
    p->plan_key[2][0] = -1;                   // no plan until the new one is in place (a failure below leaves none)
    if (int ds = och::pool_drain(p)) return ds;   // launches in flight on other streams may read the old order
    if (p->order_blocks[2] < max_blocks) {
        for (uint32_t **o : {&p->d_order[2], &p->d_order_xcd[2]}) {
            if (*o) OCH_HIP(hipFree(*o));
            *o = nullptr;
        }
        p->order_blocks[2] = 0;
        OCH_HIP(hipMalloc(&p->d_order[2], (size_t)max_blocks * 4));
        p->order_blocks[2] = max_blocks;
    }
    OCH_HIP(hipMemcpy(p->d_order[2], order.data(), (size_t)max_blocks * 4, hipMemcpyHostToDevice));
    batch_key(p, n, width, p->plan_key[2]);
    p->plan_blocks[2] = max_blocks;
    return OCH_OK;
}

namespace {

// Host rays in, host records out, synchronous: the rays staged in the pool's
// scratch, traced by the array kernel (width 0) or as a `width`-wide image of
// 8x8 tiles (och_gpu_trace_batch_tiled_dev), the records copied back.
int host_batch(och_gpu_pool *p, const float *origin, int origin_stride, const float *dirs, uint32_t n, uint32_t width,
               int32_t *hit_dir, uint32_t *hit_voxel, float *hit_time)
{
    if (!p || (n && (!origin || !dirs || !hit_dir || !hit_voxel || !hit_time)))
        return fail(OCH_E_INVALID, "NULL argument");
    if (origin_stride != 0 && origin_stride != 3) return fail(OCH_E_INVALID, "origin_stride must be 0 or 3");
    if (n == 0) return OCH_OK;
    DeviceGuard g(p->device);
    const size_t n_orig = origin_stride ? (size_t)n * 3 : 3;
    const size_t b_orig = (n_orig * 4 + 255) & ~(size_t)255;
    const size_t b_dirs = ((size_t)n * 12 + 255) & ~(size_t)255;
    const size_t b_out = ((size_t)n * 4 + 255) & ~(size_t)255;
    int st = ensure_scratch(p, b_orig + b_dirs + 3 * b_out);
    if (st != OCH_OK) return st;
    char *base = static_cast<char *>(p->d_scratch);
    float *d_orig = reinterpret_cast<float *>(base);
    float *d_dirs = reinterpret_cast<float *>(base + b_orig);
    int32_t *d_dir = reinterpret_cast<int32_t *>(base + b_orig + b_dirs);
    uint32_t *d_vox = reinterpret_cast<uint32_t *>(base + b_orig + b_dirs + b_out);
    float *d_t = reinterpret_cast<float *>(base + b_orig + b_dirs + 2 * b_out);
    hipStream_t s = p->stream();
    OCH_HIP(hipMemcpyAsync(d_orig, origin, n_orig * 4, hipMemcpyHostToDevice, s));
    OCH_HIP(hipMemcpyAsync(d_dirs, dirs, (size_t)n * 12, hipMemcpyHostToDevice, s));
    st = width ? och_gpu_trace_batch_tiled_dev(p, d_orig, origin_stride, d_dirs, n, width, d_dir, d_vox, d_t, nullptr)
               : och_gpu_trace_batch_dev(p, d_orig, origin_stride, d_dirs, n, d_dir, d_vox, d_t, nullptr);
    if (st != OCH_OK) return st;
    OCH_HIP(hipMemcpyAsync(hit_dir, d_dir, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    OCH_HIP(hipMemcpyAsync(hit_voxel, d_vox, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    OCH_HIP(hipMemcpyAsync(hit_time, d_t, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    OCH_HIP(hipStreamSynchronize(s));
    return OCH_OK;
}

}  // namespace

OCH_API int och_gpu_trace_batch(och_gpu_pool *p, const float *origin, int origin_stride, const float *dirs,
                                uint32_t n, int32_t *hit_dir, uint32_t *hit_voxel, float *hit_time)
{
    OCH_ENTRY();
    return host_batch(p, origin, origin_stride, dirs, n, 0, hit_dir, hit_voxel, hit_time);
}

OCH_API int och_gpu_trace_batch_image(och_gpu_pool *p, const float *origin, int origin_stride, const float *dirs,
                                      uint32_t n, uint32_t width, int32_t *hit_dir, uint32_t *hit_voxel,
                                      float *hit_time)
{
    OCH_ENTRY();
    if (width == 0) return fail(OCH_E_INVALID, "width must be positive");
    return host_batch(p, origin, origin_stride, dirs, n, width, hit_dir, hit_voxel, hit_time);
}

OCH_API int och_gpu_trace(och_gpu_pool *p, float ox, float oy, float oz, float dx, float dy, float dz,
                          int32_t *hit_direction, uint32_t *hit_voxel, float *hit_time)
{
    OCH_ENTRY();
    if (!hit_direction || !hit_voxel || !hit_time) return fail(OCH_E_INVALID, "NULL output");
    const float o[3] = {ox, oy, oz}, d[3] = {dx, dy, dz};
    return och_gpu_trace_batch(p, o, 0, d, 1, hit_direction, hit_voxel, hit_time);
}

OCH_API int och_camera_setup(float px, float py, float pz, float yaw, float pitch, float fov, int width, int height,
                             och_camera *cam)
{
    if (!cam || width <= 0 || height <= 0) return fail(OCH_E_INVALID, "bad camera arguments");
    // ORT/test_och_h_octree.cpp:89-115, evaluated in float exactly as written.
    cam->pos[0] = px;
    cam->pos[1] = py;
    cam->pos[2] = pz;
    cam->aspect = (float)width / (float)height;
    cam->view_x = 2.0F / (float)width;
    cam->view_y = 2.0F / (float)height;
    cam->fov_factor = 1 / tanf(fov / 2);
    const float sin_a = 0, cos_a = 1;
    const float sin_b = sinf(yaw), cos_b = cosf(yaw);
    const float sin_c = sinf(pitch), cos_c = cosf(pitch);
    cam->rot[0] = cos_a * cos_b;
    cam->rot[1] = cos_a * sin_b * sin_c - sin_a * cos_c;
    cam->rot[2] = cos_a * sin_b * cos_c + sin_a * sin_c;
    cam->rot[3] = sin_a * cos_b;
    cam->rot[4] = sin_a * sin_b * sin_c + cos_a * cos_c;
    cam->rot[5] = sin_a * sin_b * cos_c - cos_a * sin_c;
    cam->rot[6] = -sin_b;
    cam->rot[7] = cos_b * sin_c;
    cam->rot[8] = cos_b * cos_c;
    cam->width = width;
    cam->height = height;
    return OCH_OK;
}

OCH_API int och_gpu_raygen_dev(och_gpu_pool *p, const och_camera *cam, float *dirs)
{
    OCH_ENTRY();
    if (!p || !cam || !dirs) return fail(OCH_E_INVALID, "NULL argument");
    DeviceGuard g(p->device);
    OCH_HIP(och::launch_raygen(*cam, dirs, p->stream()));
    return OCH_OK;
}

OCH_API int och_shard_rows(int height, int row_chunk, int n_shards)
{
    if (height <= 0 || row_chunk <= 0 || n_shards <= 0) return 0;
    const int chunks = (height + row_chunk - 1) / row_chunk;
    return ((chunks + n_shards - 1) / n_shards) * row_chunk;
}

namespace {

int render_views(och_gpu_pool *p, const och_camera *cams, int n_views, uint32_t *rgba_slices, int row_chunk, int shard,
                 int n_shards, bool bounce, uint8_t *code_slices = nullptr)
{
    if (!p || !cams || (!rgba_slices && !code_slices)) return fail(OCH_E_INVALID, "NULL argument");
    if (code_slices && (p->n_voxels > OCH_CODE_MAX_VOXELS || !p->d_code_table))
        return fail(OCH_E_INVALID, "indexed-colour frames need a palette (och_gpu_set_palette) of at most %d voxel ids",
                    OCH_CODE_MAX_VOXELS);
    if (n_views < 1 || n_views > OCH_MAX_VIEWS) return fail(OCH_E_INVALID, "n_views %d outside 1..%d", n_views, OCH_MAX_VIEWS);
    if (row_chunk <= 0 || n_shards <= 0 || shard < 0 || shard >= n_shards)
        return fail(OCH_E_INVALID, "bad sharding (%d, %d, %d)", row_chunk, shard, n_shards);
    for (int v = 0; v < n_views; ++v)
        if (cams[v].width != cams[0].width || cams[v].height != cams[0].height || cams[v].width <= 0 || cams[v].height <= 0)
            return fail(OCH_E_INVALID, "views must share one positive width and height");
    if ((uint64_t)cams[0].width * cams[0].height * n_views >= (1ull << 32))
        return fail(OCH_E_INVALID, "frame too large");
    if (int rs = check_ready(p)) return rs;
    DeviceGuard g(p->device);
    och::DevFrame f;
    for (int v = 0; v < n_views; ++v) f.cams[v] = cams[v];
    f.n_views = n_views;
    f.palette = p->d_palette;
    f.n_voxels = p->n_voxels;
    f.out = rgba_slices;
    f.codes = code_slices;
    f.row_chunk = row_chunk;
    f.shard = shard;
    f.n_shards = n_shards;
    f.slice_rows = p->slice_rows(cams[0].height, row_chunk, n_shards);
    const bool dealt = p->deal_for(cams[0].height, row_chunk, n_shards);
    f.chunk_map = dealt ? p->d_chunk_map + (size_t)shard * p->deal_max : nullptr;
    int ts;
    och::Schedule sc = timed_schedule(p, ts);
    if (ts) return ts;
    const int which = bounce ? 1 : 0;
    if (p->opt_tile_order >= 2 && p->d_order[which]) {
        const int64_t key[9] = {cams[0].width, cams[0].height, n_views, row_chunk, shard, n_shards, p->opt_block,
                                bounce ? p->opt_bounce_compact : 0, dealt ? (int64_t)p->deal_serial : 0};
        if (std::memcmp(key, p->plan_key[which], sizeof key) == 0) {
            sc.order = p->opt_tile_order == 3 ? p->d_order_xcd[which] : p->d_order[which];
            sc.order_n = p->plan_blocks[which];
            // the plan's split form, while the options it was made with hold
            if (!bounce && p->opt_tile_order == 2 && p->split_n && p->dev().packed && p->opt_split == p->split_params[0] &&
                p->opt_split_segs == p->split_params[1] && p->opt_split_level == p->split_params[2]) {
                sc.order = p->d_order_split;
                sc.order_n = p->split_n;
                sc.split_extra = p->split_extra;
                sc.split_tasks = p->d_split_tasks;
                sc.split_level = (uint32_t)p->opt_split_level;
            }
        }
    }
    if (code_slices)
        OCH_HIP(och::launch_render_codes(p->dev(), f, sc, bounce, p->stream()));
    else if (bounce)
        OCH_HIP(och::launch_render_bounce(p->dev(), f, sc, p->stream()));
    else
        OCH_HIP(och::launch_render(p->dev(), f, sc, p->stream()));
    return timed_done(p, sc, true);
}

}  // namespace

namespace {

// The launch order from the costliest-first list (OCH_OPT_PLAN): 0 = all
// workgroups costliest first; P in 1..99 = the costliest P % first, then the
// rest in natural order (the tails a frame ends on start early, while the bulk
// keeps the raster order's mix of sky and terrain tiles); 100 = alternate the
// costliest and the cheapest left.  Default 10: with frames in flight, every
// frame starting all its costly tiles at once cost 3.5 % over long runs
// (profiles/r03/ab/plan_*).
void plan_shape(std::vector<uint32_t> &order, int mode)
{
    const size_t n = order.size();
    if (mode <= 0 || n < 2) return;
    std::vector<uint32_t> out;
    out.reserve(n);
    if (mode >= 100) {
        for (size_t i = 0, j = n - 1; i <= j && j < n; ++i, --j) {
            out.push_back(order[i]);
            if (j != i) out.push_back(order[j]);
            if (j == 0) break;
        }
    } else {
        const size_t head = n * (size_t)mode / 100;
        std::vector<uint8_t> taken(n, 0);
        for (size_t i = 0; i < head; ++i) {
            out.push_back(order[i]);
            taken[order[i]] = 1;
        }
        for (uint32_t b = 0; b < n; ++b)
            if (!taken[b]) out.push_back(b);
    }
    order.swap(out);
}

// A split tile's rays longer than this % of its longest walk over
// OCH_OPT_SPLIT_SEGS lanes; the others take one lane and walk whole
// (tools/split_model.c: 30 % keeps the critical path of splitting every ray
// and adds almost no work).
constexpr int kSplitRayPct = 30;

// The split form of a primary plan (OCH_OPT_SPLIT).  The tiles
// whose planning cost reaches opt_split % of the costliest one's are split:
// one counting render gives every pixel's walked PUSHes, a tile's rays longer
// than kSplitRayPct % of its longest get opt_split_segs lanes each (segment
// lanes), the others one, and its rays are packed, costliest first, into
// waves of 64 lanes with every lane of a ray in one wave (their records merge
// through that wave's LDS).  Rows of d_split_tasks: the tile, then 64 lane
// tasks (pixel | seg << 6 | log2(S) << 10, ~0 idle).  The order: the split
// waves (1 << 31 | row), then the plan's other workgroups in its order.
// Block 64 only (workgroup = tile), packed layout, tiles < 2^24, and a split
// level above the leaves; otherwise no split plan.
int plan_split(och_gpu_pool *p, const och::DevFrame &f, const std::vector<uint32_t> &by_cost,
               const std::vector<uint32_t> &order, const std::vector<uint32_t> &c)
{
    p->split_n = p->split_extra = p->split_tiles = 0;
    p->split_params[0] = p->split_params[1] = p->split_params[2] = 0;
    const uint32_t n = (uint32_t)order.size();
    const int S = p->opt_split_segs, log2s = __builtin_ctz((unsigned)S);
    if (p->opt_split <= 0 || p->opt_block != 64 || !p->dev().packed || p->opt_split_level >= p->depth || n == 0 ||
        n >= (1u << 24))
        return OCH_OK;
    const double thr = (double)c[by_cost[0]] * p->opt_split / 100.0;
    std::vector<uint32_t> heavy_tiles;
    const uint32_t cap = std::max(1u, n / 16);                  // a bound on the planner's work
    for (uint32_t k = 0; k < n && k < cap && (double)c[by_cost[k]] >= thr; ++k) heavy_tiles.push_back(by_cost[k]);
    // every pixel's walked PUSHes (one counting render of the planned frame)
    const int W = f.cams[0].width, rows = f.slice_rows;
    const size_t px = (size_t)f.n_views * rows * W;
    uint16_t *d_push = nullptr;
    OCH_HIP(hipMalloc(&d_push, px * 2));
    std::vector<uint16_t> push(px);
    och::Schedule sc = p->schedule();
    sc.tile_order = 0;
    hipError_t e = och::launch_render_push(p->dev(), f, sc, d_push, p->stream());
    if (e == hipSuccess) e = hipMemcpyAsync(push.data(), d_push, px * 2, hipMemcpyDeviceToHost, p->stream());
    if (e == hipSuccess) e = hipStreamSynchronize(p->stream());
    (void)hipFree(d_push);
    if (e != hipSuccess) return fail(OCH_E_HIP, "split plan: counting render: %s", hipGetErrorString(e));
    const uint32_t tiles_x = (uint32_t)(W + 7) / 8, per_view = tiles_x * (uint32_t)((rows + 7) / 8);
    std::vector<uint32_t> rowsv, split;                         // task rows (65 words each), order
    std::vector<uint8_t> heavy(n, 0);
    for (uint32_t t : heavy_tiles) {
        heavy[t] = 1;
        const uint32_t view = t / per_view, tt = t % per_view, ty = tt / tiles_x, tx = tt % tiles_x;
        int cnt[64], mx = 0;
        for (int l = 0; l < 64; ++l) {
            const uint32_t col = tx * 8 + (uint32_t)(l % 8), srow = ty * 8 + (uint32_t)(l / 8);
            cnt[l] = col < (uint32_t)W && srow < (uint32_t)rows ? push[((size_t)view * rows + srow) * W + col] : -1;
            mx = std::max(mx, cnt[l]);
        }
        // rays costliest first (a long ray by its segments' share), first fit into waves
        std::vector<std::pair<int, int>> rays;                  // (estimated lane cost, pixel)
        for (int l = 0; l < 64; ++l)
            if (cnt[l] >= 0) rays.push_back({cnt[l] * 100 > kSplitRayPct * mx ? cnt[l] / S : cnt[l], l});
        std::stable_sort(rays.begin(), rays.end(), [](const auto &a, const auto &b) { return a.first > b.first; });
        std::vector<std::vector<uint32_t>> waves;
        for (const auto &r : rays) {
            const int l = r.second;
            const bool long_ray = cnt[l] * 100 > kSplitRayPct * mx;
            const size_t lanes = long_ray ? (size_t)S : 1;
            size_t w = 0;
            while (w < waves.size() && waves[w].size() + lanes > 64) ++w;
            if (w == waves.size()) waves.emplace_back();
            for (size_t s_ = 0; s_ < lanes; ++s_)
                waves[w].push_back((uint32_t)l | (uint32_t)s_ << 6 | (uint32_t)(long_ray ? log2s : 0) << 10);
        }
        for (auto &w : waves) {
            split.push_back(0x80000000u | (uint32_t)(rowsv.size() / 65));
            rowsv.push_back(t);
            for (size_t l = 0; l < 64; ++l) rowsv.push_back(l < w.size() ? w[l] : ~0u);
        }
    }
    if (heavy_tiles.empty()) return OCH_OK;
    const uint32_t n_waves = (uint32_t)split.size();
    for (uint32_t b : order)
        if (!heavy[b]) split.push_back(b);
    auto upload = [&](uint32_t *&d, uint32_t &alloc, const std::vector<uint32_t> &v) -> hipError_t {
        if (alloc < v.size()) {
            if (d) (void)hipFree(d);
            d = nullptr;
            alloc = 0;
            const hipError_t me = hipMalloc(&d, v.size() * 4);
            if (me != hipSuccess) return me;
            alloc = (uint32_t)v.size();
        }
        return hipMemcpy(d, v.data(), v.size() * 4, hipMemcpyHostToDevice);
    };
    OCH_HIP(upload(p->d_order_split, p->split_alloc, split));
    OCH_HIP(upload(p->d_split_tasks, p->task_alloc, rowsv));
    p->split_n = (uint32_t)split.size();
    p->split_extra = n_waves - (uint32_t)heavy_tiles.size();
    p->split_tiles = (uint32_t)heavy_tiles.size();
    p->split_params[0] = p->opt_split;
    p->split_params[1] = S;
    p->split_params[2] = p->opt_split_level;
    return OCH_OK;
}

}  // namespace

OCH_API int och_gpu_plan_views(och_gpu_pool *p, const och_camera *cams, int n_views, int row_chunk, int shard,
                               int n_shards)
{
    OCH_ENTRY();
    if (!p || !cams) return fail(OCH_E_INVALID, "NULL argument");
    if (n_views < 1 || n_views > OCH_MAX_VIEWS || row_chunk <= 0 || n_shards <= 0 || shard < 0 || shard >= n_shards)
        return fail(OCH_E_INVALID, "bad plan arguments");
    if (int rs = check_ready(p)) return rs;
    DeviceGuard g(p->device);
    // One planning render per kernel (primary grid, config-5 bounce) into
    // scratch in natural order, timing every workgroup.
    const int W = cams[0].width, H = cams[0].height;
    const int rows = p->slice_rows(H, row_chunk, n_shards);
    const bool dealt = p->deal_for(H, row_chunk, n_shards);
    const size_t frame_bytes = (size_t)n_views * rows * W * 4;
    const uint32_t max_blocks = (uint32_t)((size_t)n_views * ((rows + 7) / 8) * ((W + 7) / 8)) + 1024;
    int st = ensure_scratch(p, frame_bytes + (size_t)max_blocks * 4);
    if (st != OCH_OK) return st;
    uint32_t *cost = reinterpret_cast<uint32_t *>(static_cast<char *>(p->d_scratch) + frame_bytes);
    och::DevFrame f;
    for (int v = 0; v < n_views; ++v) f.cams[v] = cams[v];
    f.n_views = n_views;
    f.palette = p->d_palette;
    f.n_voxels = p->n_voxels;
    f.out = static_cast<uint32_t *>(p->d_scratch);
    f.codes = nullptr;
    f.row_chunk = row_chunk;
    f.shard = shard;
    f.n_shards = n_shards;
    f.slice_rows = rows;
    f.chunk_map = dealt ? p->d_chunk_map + (size_t)shard * p->deal_max : nullptr;
    for (int which = 0; which < 2; ++which) {
        OCH_HIP(hipMemsetAsync(cost, 0xFF, (size_t)max_blocks * 4, p->stream()));
        och::Schedule sc = p->schedule();
        sc.tile_order = 0;
        sc.cost = cost;
        if (which == 0)
            OCH_HIP(och::launch_render(p->dev(), f, sc, p->stream()));
        else
            OCH_HIP(och::launch_render_bounce(p->dev(), f, sc, p->stream()));
        std::vector<uint32_t> c(max_blocks);
        OCH_HIP(hipMemcpyAsync(c.data(), cost, (size_t)max_blocks * 4, hipMemcpyDeviceToHost, p->stream()));
        OCH_HIP(hipStreamSynchronize(p->stream()));
        uint32_t n_blocks = 0;
        while (n_blocks < max_blocks && c[n_blocks] != 0xFFFFFFFFu) ++n_blocks;   // launched blocks wrote a cost
        if (n_blocks == 0) {
            p->plan_key[which][0] = -1;          // no plan: later launches run in natural order
            return fail(OCH_E_INVALID, "planning render wrote no workgroup costs (kernel without cost output?)");
        }
        std::vector<uint32_t> order(n_blocks);
        for (uint32_t i = 0; i < n_blocks; ++i) order[i] = i;
        std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return c[a] > c[b]; });
        const std::vector<uint32_t> by_cost = order;
        plan_shape(order, p->opt_plan);
        // Grouped per XCD (OCH_OPT_TILE_ORDER = 3): workgroup slot i runs on XCD
        // i % 8, so deal 64x64-pixel supertiles over the XCDs (each XCD's L2 then
        // holds the nodes of its own neighbouring tiles) and keep the costliest-
        // first order within each XCD's list.
        const uint32_t block = (uint32_t)(which ? std::max(och::kBounceBlock, p->opt_block) : p->opt_block);
        const uint32_t tiles_x = (uint32_t)(W + 7) / 8, tiles_y = (uint32_t)(rows + 7) / 8;
        const uint32_t stx = (tiles_x + 7) / 8, sty = (tiles_y + 7) / 8;
        std::vector<std::vector<uint32_t>> lists(8);
        for (uint32_t b : order) {
            const uint32_t tile = b * (block / 64), view = tile / (tiles_x * tiles_y), t = tile % (tiles_x * tiles_y);
            const uint32_t st = (view * sty + (t / tiles_x) / 8) * stx + (t % tiles_x) / 8;
            lists[st % 8].push_back(b);
        }
        std::vector<uint32_t> grouped;
        grouped.reserve(n_blocks);
        std::vector<size_t> at(8, 0);
        while (grouped.size() < n_blocks)
            for (uint32_t x = 0; x < 8 && grouped.size() < n_blocks; ++x) {
                uint32_t from = x;
                if (at[x] == lists[x].size())       // this XCD's list ran dry: the fullest other list
                    for (uint32_t y = 0; y < 8; ++y)
                        if (lists[y].size() - at[y] > lists[from].size() - at[from]) from = y;
                grouped.push_back(lists[from][at[from]++]);
            }
        p->plan_key[which][0] = -1;           // no plan until the new one is in place (a failure below leaves none)
        if (int ds = och::pool_drain(p)) return ds;   // launches in flight on other streams may read the old order
        if (p->order_blocks[which] < n_blocks) {
            for (uint32_t **o : {&p->d_order[which], &p->d_order_xcd[which]}) {
                if (*o) OCH_HIP(hipFree(*o));
                *o = nullptr;
            }
            p->order_blocks[which] = 0;
            OCH_HIP(hipMalloc(&p->d_order[which], (size_t)n_blocks * 4));
            OCH_HIP(hipMalloc(&p->d_order_xcd[which], (size_t)n_blocks * 4));
            p->order_blocks[which] = n_blocks;
        }
        OCH_HIP(hipMemcpy(p->d_order[which], order.data(), (size_t)n_blocks * 4, hipMemcpyHostToDevice));
        OCH_HIP(hipMemcpy(p->d_order_xcd[which], grouped.data(), (size_t)n_blocks * 4, hipMemcpyHostToDevice));
        if (which == 0)
            if (int ss = plan_split(p, f, by_cost, order, c)) return ss;
        const int64_t key[9] = {W, H, n_views, row_chunk, shard, n_shards, p->opt_block,
                                which ? p->opt_bounce_compact : 0, dealt ? (int64_t)p->deal_serial : 0};
        std::memcpy(p->plan_key[which], key, sizeof key);
        p->plan_blocks[which] = n_blocks;
    }
    return OCH_OK;
}

OCH_API int och_gpu_set_row_deal(och_gpu_pool *p, int height, int row_chunk, int n_shards, const int32_t *chunk_shard)
{
    if (!p) return fail(OCH_E_INVALID, "pool is NULL");
    if (!chunk_shard && !p->deal_n) return OCH_OK;                      // round-robin already
    if (chunk_shard && p->deal_for(height, row_chunk, n_shards) && row_chunk > 0 &&
        std::equal(p->deal_table.begin(), p->deal_table.end(), chunk_shard))
        return OCH_OK;                                                  // this deal already (plans stay valid)
    // Validate the new deal and build its tables on the host first: a bad
    // call leaves the pool's current deal in place.
    std::vector<int32_t> map, owner;
    int n_chunks = 0, max_chunks = 1;
    if (chunk_shard) {
        if (height <= 0 || row_chunk <= 0 || n_shards <= 0 || n_shards > 32767)
            return fail(OCH_E_INVALID, "bad row deal geometry (%d, %d, %d)", height, row_chunk, n_shards);
        n_chunks = (height + row_chunk - 1) / row_chunk;
        std::vector<std::vector<int32_t>> mine(n_shards);
        for (int c = 0; c < n_chunks; ++c) {
            if (chunk_shard[c] < 0 || chunk_shard[c] >= n_shards)
                return fail(OCH_E_INVALID, "chunk %d dealt to shard %d of %d", c, chunk_shard[c], n_shards);
            mine[chunk_shard[c]].push_back(c);
        }
        for (const auto &m : mine) max_chunks = std::max(max_chunks, (int)m.size());
        if (max_chunks > 65535) return fail(OCH_E_INVALID, "more than 65535 chunks for one shard");
        map.assign((size_t)n_shards * max_chunks, -1);
        owner.assign(n_chunks, 0);
        for (int sh = 0; sh < n_shards; ++sh)
            for (size_t l = 0; l < mine[sh].size(); ++l) {
                map[(size_t)sh * max_chunks + l] = mine[sh][l];
                owner[mine[sh][l]] = (sh << 16) | (int32_t)l;
            }
    }
    DeviceGuard g(p->device);
    int32_t *d_map = nullptr, *d_own = nullptr;
    if (chunk_shard) {
        hipError_t e = hipMalloc(&d_map, map.size() * 4);
        if (e == hipSuccess) e = hipMalloc(&d_own, owner.size() * 4);
        if (e == hipSuccess) e = hipMemcpy(d_map, map.data(), map.size() * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(d_own, owner.data(), owner.size() * 4, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            if (d_map) (void)hipFree(d_map);
            if (d_own) (void)hipFree(d_own);
            return fail(OCH_E_HIP, "row deal tables: %s", hipGetErrorString(e));
        }
    }
    // frames in flight may still read the old tables; on failure the new ones
    // are freed and the old deal stays
    const hipError_t se = hipDeviceSynchronize();
    if (se != hipSuccess) {
        if (d_map) (void)hipFree(d_map);
        if (d_own) (void)hipFree(d_own);
        return fail(OCH_E_HIP, "row deal: hipDeviceSynchronize: %s", hipGetErrorString(se));
    }
    if (p->d_chunk_map) (void)hipFree(p->d_chunk_map);
    if (p->d_owner) (void)hipFree(p->d_owner);
    p->d_chunk_map = d_map;
    p->d_owner = d_own;
    ++p->deal_serial;
    if (!chunk_shard) {                        // back to round-robin
        p->deal_n = p->deal_h = p->deal_chunk = p->deal_max = 0;
        p->deal_table.clear();
        return OCH_OK;
    }
    p->deal_h = height;
    p->deal_chunk = row_chunk;
    p->deal_n = n_shards;
    p->deal_max = max_chunks;
    p->deal_table.assign(chunk_shard, chunk_shard + n_chunks);
    return OCH_OK;
}

OCH_API int och_gpu_slice_rows(const och_gpu_pool *p, int height, int row_chunk, int n_shards, int *rows)
{
    if (!p || !rows) return fail(OCH_E_INVALID, "NULL argument");
    *rows = p->slice_rows(height, row_chunk, n_shards);
    return OCH_OK;
}

OCH_API int och_gpu_chunk_costs(och_gpu_pool *p, const och_camera *cams, int n_views, int row_chunk, float *costs)
{
    OCH_ENTRY();
    if (!p || !cams || !costs || row_chunk <= 0) return fail(OCH_E_INVALID, "bad chunk-cost arguments");
    if (n_views < 1 || n_views > OCH_MAX_VIEWS) return fail(OCH_E_INVALID, "n_views %d outside 1..%d", n_views, OCH_MAX_VIEWS);
    for (int v = 0; v < n_views; ++v)
        if (cams[v].width != cams[0].width || cams[v].height != cams[0].height || cams[v].width <= 0 || cams[v].height <= 0)
            return fail(OCH_E_INVALID, "views must share one positive width and height");
    if (int rs = check_ready(p)) return rs;
    DeviceGuard g(p->device);
    // one whole-frame render, natural 8x8-tile order, every workgroup timed
    const int W = cams[0].width, H = cams[0].height;
    const uint32_t tiles_x = (uint32_t)(W + 7) / 8, tiles_y = (uint32_t)(H + 7) / 8;
    // tiles per workgroup exactly as launch_as sizes the grid kernel's grid
    const uint32_t tiles = (uint32_t)n_views * tiles_x * tiles_y,
                   per_block = (uint32_t)p->opt_block / 64;
    const uint32_t n_blocks = (tiles + per_block - 1) / per_block;
    const size_t frame_bytes = ((size_t)n_views * H * W * 4 + 255) & ~(size_t)255;
    int st = ensure_scratch(p, frame_bytes + (size_t)n_blocks * 4);
    if (st != OCH_OK) return st;
    uint32_t *cost = reinterpret_cast<uint32_t *>(static_cast<char *>(p->d_scratch) + frame_bytes);
    och::DevFrame f;
    for (int v = 0; v < n_views; ++v) f.cams[v] = cams[v];
    f.n_views = n_views;
    f.palette = p->d_palette;
    f.n_voxels = p->n_voxels;
    f.out = static_cast<uint32_t *>(p->d_scratch);
    f.codes = nullptr;
    f.row_chunk = H;
    f.shard = 0;
    f.n_shards = 1;
    f.slice_rows = H;
    f.chunk_map = nullptr;
    // The grid kernel writes the costs: every launched workgroup overwrites its 0xFFFFFFFF, so a
    // block the launch did not cover is caught below instead of being read as
    // uninitialised scratch.
    och::Schedule sc = p->schedule();
    sc.tile_order = 0;
    sc.cost = cost;
    OCH_HIP(hipMemsetAsync(cost, 0xFF, (size_t)n_blocks * 4, p->stream()));
    OCH_HIP(och::launch_render(p->dev(), f, sc, p->stream()));
    std::vector<uint32_t> c(n_blocks);
    OCH_HIP(hipMemcpyAsync(c.data(), cost, (size_t)n_blocks * 4, hipMemcpyDeviceToHost, p->stream()));
    OCH_HIP(hipStreamSynchronize(p->stream()));
    for (uint32_t b = 0; b < n_blocks; ++b)
        if (c[b] == 0xFFFFFFFFu) return fail(OCH_E_INVALID, "chunk-cost render left workgroup %u untimed", b);
    // a workgroup's time spread over its tiles, a tile's over its 8 rows
    const int n_chunks = (H + row_chunk - 1) / row_chunk;
    std::vector<double> acc(n_chunks, 0.0);
    for (uint32_t b = 0; b < n_blocks; ++b)
        for (uint32_t t = b * per_block; t < std::min(tiles, (b + 1) * per_block); ++t) {
            const uint32_t ty = (t % (tiles_x * tiles_y)) / tiles_x;
            const int r0 = (int)ty * 8, r1 = std::min(H, r0 + 8);
            for (int r = r0; r < r1; ++r) acc[r / row_chunk] += (double)c[b] / per_block / (r1 - r0);
        }
    for (int k = 0; k < n_chunks; ++k) costs[k] = (float)acc[k];
    return OCH_OK;
}

OCH_API int och_deal_chunks(const float *costs, int n_chunks, int n_shards, const float *weights, int32_t *chunk_shard)
{
    if (!costs || !chunk_shard || n_chunks <= 0 || n_shards <= 0) return fail(OCH_E_INVALID, "bad deal arguments");
    std::vector<double> w(n_shards, 1.0);
    double w_sum = 0.0, w_max = 0.0;
    for (int s = 0; s < n_shards; ++s) {
        if (weights) w[s] = weights[s];
        if (!(w[s] > 0.0)) return fail(OCH_E_INVALID, "shard %d weight %g is not positive", s, w[s]);
        w_sum += w[s];
        w_max = std::max(w_max, w[s]);
    }
    // a shard holds at most its weighted share of the chunks plus two, which
    // bounds the padding of the equal-size slices an all-gather needs
    const int cap = (int)std::ceil(n_chunks * w_max / w_sum) + 2;
    std::vector<int> order(n_chunks);
    for (int k = 0; k < n_chunks; ++k) order[k] = k;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return costs[a] > costs[b]; });
    std::vector<double> load(n_shards, 0.0);
    std::vector<int> count(n_shards, 0);
    for (int k : order) {             // longest processing time first, onto the least loaded shard (per weight)
        int best = -1;
        double best_score = 0.0;
        for (int s = 0; s < n_shards; ++s) {
            if (count[s] >= cap) continue;
            const double score = (load[s] + std::max(0.0f, costs[k])) / w[s];
            if (best < 0 || score < best_score || (score == best_score && count[s] < count[best])) {
                best = s;
                best_score = score;
            }
        }
        chunk_shard[k] = best;
        load[best] += std::max(0.0f, costs[k]);
        ++count[best];
    }
    return OCH_OK;
}

OCH_API int och_gpu_render_views_dev(och_gpu_pool *p, const och_camera *cams, int n_views, uint32_t *rgba_slices,
                                     int row_chunk, int shard, int n_shards)
{
    OCH_ENTRY();
    return render_views(p, cams, n_views, rgba_slices, row_chunk, shard, n_shards, false);
}

OCH_API int och_gpu_render_bounce_views_dev(och_gpu_pool *p, const och_camera *cams, int n_views, uint32_t *rgba_slices,
                                            int row_chunk, int shard, int n_shards)
{
    OCH_ENTRY();
    return render_views(p, cams, n_views, rgba_slices, row_chunk, shard, n_shards, true);
}

OCH_API int och_gpu_render_steps_dev(och_gpu_pool *p, const och_camera *cams, int n_views, int n_steps,
                                     void *const *streams, uint32_t *const *frames, int n_buffers,
                                     void *const *start_events, void *const *stop_events, int row_chunk, int bounce)
{
    OCH_ENTRY();
    if (!p || !cams || !streams || !frames) return fail(OCH_E_INVALID, "NULL argument");
    if (n_steps < 0 || n_buffers < 1) return fail(OCH_E_INVALID, "n_steps %d / n_buffers %d", n_steps, n_buffers);
    if ((start_events == nullptr) != (stop_events == nullptr))
        return fail(OCH_E_INVALID, "start_events and stop_events: both or neither");
    for (int b = 0; b < n_buffers; ++b)
        if (!frames[b]) return fail(OCH_E_INVALID, "frames[%d] is NULL", b);
    // The frame loop of update_image (ORT/test_och_h_octree.cpp:437-457), one
    // launch per frame, issued here rather than by the caller's interpreter.
    // The pool's stream is restored afterwards, also after a failure.
    const bool had_ext = p->use_ext;
    const hipStream_t prev = p->ext_stream;
    int st = OCH_OK;
    for (int k = 0; k < n_steps && st == OCH_OK; ++k) {
        const int b = k % n_buffers;
        p->ext_stream = static_cast<hipStream_t>(streams[b]);
        p->use_ext = true;
        if (start_events) {
            p->next_ev_start = static_cast<hipEvent_t>(start_events[k]);
            p->next_ev_stop = static_cast<hipEvent_t>(stop_events[k]);
        }
        st = render_views(p, cams, n_views, frames[b], row_chunk, 0, 1, bounce != 0);
    }
    p->next_ev_start = p->next_ev_stop = nullptr;
    p->ext_stream = prev;
    p->use_ext = had_ext;
    return st;
}

OCH_API int och_gpu_render_sharded_steps_dev(och_gpu_pool *p, och_comm *comm, const och_camera *cams, int n_views,
                                             int n_steps, void *const *streams, uint8_t *const *slices,
                                             uint8_t *const *gathered, uint32_t *const *frames, int n_buffers,
                                             void *const *start_events, void *const *stop_events, int row_chunk,
                                             int bounce, int exchange)
{
    OCH_ENTRY();
    if (!p || !comm || !cams || !streams || !slices) return fail(OCH_E_INVALID, "NULL argument");
    if (n_steps < 0 || n_buffers < 1) return fail(OCH_E_INVALID, "n_steps %d / n_buffers %d", n_steps, n_buffers);
    if (n_views < 1 || n_views > OCH_MAX_VIEWS || row_chunk <= 0) return fail(OCH_E_INVALID, "bad views / row_chunk");
    if (exchange < OCH_EXCHANGE_ALL_GATHER || exchange > OCH_EXCHANGE_GATHER)
        return fail(OCH_E_INVALID, "unknown exchange %d", exchange);
    if ((start_events == nullptr) != (stop_events == nullptr))
        return fail(OCH_E_INVALID, "start_events and stop_events: both or neither");
    int n_ranks = 0, rank = 0, device = -1;
    if (int cs = och::comm_ranks(comm, &n_ranks, &rank, &device)) return cs;
    if (device != p->device) return fail(OCH_E_INVALID, "communicator on device %d, pool on device %d", device, p->device);
    const bool receives = exchange != OCH_EXCHANGE_GATHER || rank == 0;
    const bool shades = exchange == OCH_EXCHANGE_ALL_GATHER || rank == 0;
    // Everything a frame needs is checked before the first is queued: a rank
    // that stops part way leaves its peers' collectives without a partner.
    for (int b = 0; b < n_buffers; ++b) {
        if (!slices[b]) return fail(OCH_E_INVALID, "slices[%d] is NULL", b);
        if (receives && (!gathered || !gathered[b])) return fail(OCH_E_INVALID, "rank %d needs gathered[%d]", rank, b);
        if (shades && (!frames || !frames[b])) return fail(OCH_E_INVALID, "rank %d needs frames[%d]", rank, b);
    }
    for (int v = 0; v < n_views; ++v)
        if (cams[v].width != cams[0].width || cams[v].height != cams[0].height || cams[v].width <= 0 ||
            cams[v].height <= 0)
            return fail(OCH_E_INVALID, "views must share one positive width and height");
    if (shades && !p->d_code_table)
        return fail(OCH_E_INVALID, "no code table: set a palette of at most %d voxel ids", OCH_CODE_MAX_VOXELS);
    const int W = cams[0].width, H = cams[0].height;
    const size_t count = (size_t)n_views * p->slice_rows(H, row_chunk, n_ranks) * W;
    DeviceGuard g(p->device);
    // Per frame: render -> exchange -> shade, all on the frame's stream, so
    // the three are ordered on the device and the host never waits.  A
    // buffer set is reused only behind the previous frame on its stream.
    const bool had_ext = p->use_ext;
    const hipStream_t prev = p->ext_stream;
    int st = OCH_OK;
    bool issued = false;                     // a collective of this window is queued
    for (int k = 0; k < n_steps && st == OCH_OK; ++k) {
        const int b = k % n_buffers;
        const hipStream_t s = static_cast<hipStream_t>(streams[b]);
        p->ext_stream = s;
        p->use_ext = true;
        if (start_events) {
            p->next_ev_start = static_cast<hipEvent_t>(start_events[k]);
            p->next_ev_stop = static_cast<hipEvent_t>(stop_events[k]);
        }
        st = render_views(p, cams, n_views, nullptr, row_chunk, rank, n_ranks, bounce != 0, slices[b]);
        if (st == OCH_OK) {
            st = exchange == OCH_EXCHANGE_GATHER
                     ? och::comm_gather(comm, slices[b], receives ? gathered[b] : nullptr, count, 0, s)
                     : och::comm_all_gather(comm, slices[b], gathered[b], count, s);
            issued = issued || st == OCH_OK;
        }
        if (st == OCH_OK && shades)
            st = och_gpu_shade_unshard_views_dev(p, gathered[b], frames[b], W, H, row_chunk, n_ranks, n_views);
    }
    p->next_ev_start = p->next_ev_stop = nullptr;
    p->ext_stream = prev;
    p->use_ext = had_ext;
    if (st != OCH_OK && issued) {
        // The peers' collectives of this window can no longer all complete.
        // Aborting here does not unblock the peers: their callers must abort
        // theirs (bench.py's watchdog, or the process exiting).  A failure
        // before this rank queued any collective leaves the communicator as
        // it was (every rank failing alike keeps a consistent one).
        const std::string msg = och_last_error();
        och::comm_abort(comm);
        return fail(st, "%s (communicator aborted: the window stopped part way)", msg.c_str());
    }
    return st;
}

OCH_API int och_gpu_render_codes_views_dev(och_gpu_pool *p, const och_camera *cams, int n_views, uint8_t *code_slices,
                                           int row_chunk, int shard, int n_shards, int bounce)
{
    OCH_ENTRY();
    if (!code_slices) return fail(OCH_E_INVALID, "NULL argument");
    return render_views(p, cams, n_views, nullptr, row_chunk, shard, n_shards, bounce != 0, code_slices);
}

OCH_API int och_gpu_shade_unshard_views_dev(och_gpu_pool *p, const uint8_t *gathered, uint32_t *frames, int width,
                                            int height, int row_chunk, int n_shards, int n_views)
{
    OCH_ENTRY();
    if (!p || !gathered || !frames || width <= 0 || height <= 0 || row_chunk <= 0 || n_shards <= 0 || n_views < 1)
        return fail(OCH_E_INVALID, "bad unshard arguments");
    if (!p->d_code_table)
        return fail(OCH_E_INVALID, "no code table: set a palette of at most %d voxel ids", OCH_CODE_MAX_VOXELS);
    DeviceGuard g(p->device);
    OCH_HIP(och::launch_shade_unshard(gathered, frames, p->d_code_table, width, height, row_chunk, n_shards,
                                      p->slice_rows(height, row_chunk, n_shards), n_views,
                                      p->deal_for(height, row_chunk, n_shards) ? p->d_owner : nullptr, p->stream()));
    return OCH_OK;
}

OCH_API int och_gpu_render_dev(och_gpu_pool *p, const och_camera *cam, uint32_t *rgba_slice, int row_chunk, int shard,
                               int n_shards)
{
    OCH_ENTRY();
    if (!cam) return fail(OCH_E_INVALID, "NULL camera");
    return och_gpu_render_views_dev(p, cam, 1, rgba_slice, row_chunk, shard, n_shards);
}

OCH_API int och_gpu_unshard_views_dev(och_gpu_pool *p, const uint32_t *gathered, uint32_t *frames, int width,
                                      int height, int row_chunk, int n_shards, int n_views)
{
    OCH_ENTRY();
    if (!p || !gathered || !frames || width <= 0 || height <= 0 || row_chunk <= 0 || n_shards <= 0 || n_views < 1)
        return fail(OCH_E_INVALID, "bad unshard arguments");
    DeviceGuard g(p->device);
    OCH_HIP(och::launch_unshard(gathered, frames, width, height, row_chunk, n_shards,
                                p->slice_rows(height, row_chunk, n_shards), n_views,
                                p->deal_for(height, row_chunk, n_shards) ? p->d_owner : nullptr, p->stream()));
    return OCH_OK;
}

OCH_API int och_gpu_unshard_dev(och_gpu_pool *p, const uint32_t *gathered, uint32_t *frame, int width, int height,
                                int row_chunk, int n_shards)
{
    OCH_ENTRY();
    return och_gpu_unshard_views_dev(p, gathered, frame, width, height, row_chunk, n_shards, 1);
}

OCH_API int och_gpu_render(och_gpu_pool *p, const och_camera *cam, uint32_t *rgba)
{
    OCH_ENTRY();
    if (!p || !cam || !rgba) return fail(OCH_E_INVALID, "NULL argument");
    DeviceGuard g(p->device);
    const size_t bytes = (size_t)cam->width * cam->height * 4;
    int st = ensure_scratch(p, bytes);
    if (st != OCH_OK) return st;
    st = och_gpu_render_dev(p, cam, static_cast<uint32_t *>(p->d_scratch), cam->height, 0, 1);
    if (st != OCH_OK) return st;
    OCH_HIP(hipMemcpyAsync(rgba, p->d_scratch, bytes, hipMemcpyDeviceToHost, p->stream()));
    OCH_HIP(hipStreamSynchronize(p->stream()));
    return OCH_OK;
}

OCH_API int och_pool_pack(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth, int index_base,
                          uint32_t *out, uint32_t out_capacity, uint32_t *out_nodes, uint32_t *out_root)
{
    if (!nodes || !out_nodes || !out_root) return fail(OCH_E_INVALID, "NULL argument");
    int st = validate_pool(nodes, n_nodes, root, depth, index_base);
    if (st != OCH_OK) return st;
    std::vector<uint32_t> packed;
    uint32_t proot = 0;
    if (!pack_pool(nodes, n_nodes, root, depth, index_base, packed, proot))
        return fail(OCH_E_CAPACITY, "more than 2^24 - 1 (node, level) pairs");
    *out_nodes = (uint32_t)(packed.size() / 8);
    *out_root = proot;
    if (out) {
        if (out_capacity < *out_nodes) return fail(OCH_E_CAPACITY, "output holds %u nodes, %u needed", out_capacity, *out_nodes);
        std::memcpy(out, packed.data(), packed.size() * 4);
    }
    return OCH_OK;
}

OCH_API int och_pool_occupied_box(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth, int index_base,
                                  int32_t lo[3], int32_t hi[3])
{
    if (!nodes || !lo || !hi) return fail(OCH_E_INVALID, "NULL argument");
    if (index_base != 0 && index_base != 1) return fail(OCH_E_INVALID, "index_base must be 0 or 1");
    const int st = validate_pool(nodes, n_nodes, root, depth, index_base);
    if (st != OCH_OK) return st;
    if (!och::occupied_box(nodes, n_nodes, root, depth, index_base, lo, hi))
        for (int a = 0; a < 3; ++a) lo[a] = hi[a] = 0;
    return OCH_OK;
}

OCH_API uint32_t och_pool_at(const uint32_t *nodes, uint32_t root, int depth, int index_base, int x, int y, int z)
{
    // h_octree::at (ORT/och_h_octree.h:239-258) with the child digit of z_encode_16.
    if (!nodes || (index_base == 1 && root == 0)) return 0;
    uint32_t cur = root;
    for (int l = depth - 1; l >= 0; --l) {
        const int c = ((x >> l) & 1) | (((y >> l) & 1) << 1) | (((z >> l) & 1) << 2);
        const uint32_t nx = nodes[(size_t)(cur - index_base) * 8 + c];
        if (l == 0 || !nx) return nx;
        cur = nx;
    }
    return 0;
}

}  // extern "C"
