// och_builder.cpp -- parallel bottom-up builder of the demo terrain DAG.
//
// The reference builds its tree by recursive create_volume + per-voxel
// h_octree::set edits (ORT/test_och_h_octree.cpp:651-695, :767-787;
// ORT/och_h_octree.h:110-237): single-threaded, ~100 s at depth 10.  Because
// the final content is a pure per-voxel function (och_terrain.h), the same
// canonical DAG (identical subtrees shared, empty subtrees 0) is built here
// brick by brick on all host threads: each 32^3 brick is voxelised, reduced
// bottom-up and hash-consed into one lock-free table; the levels above the
// bricks follow; finally the pool is renumbered breadth-first so the top of
// the DAG is contiguous at the front of the pool.
//
// Unlike the reference's table, a node belongs to exactly one level here
// (the level is part of the key): the reference may share one slot between a
// leaf-level node and an interior node whose child indices happen to spell
// the same 8 words -- harmless for tracing, impossible to renumber.
//
// use_gpu: the voxel function -- simplex noise for every voxel below the
// surface, 2 * 10^10 evaluations at depth 12 -- runs on the GPU instead
// (k_brick_codes): one workgroup per 32^3 brick writes the brick's 4096
// leaf-level nodes as 24-bit codes (3 bits per child voxel), its voxel
// histogram and whether all its leaves are equal.  Host threads hash-cons the
// codes bottom-up exactly as they do their own voxels, batch after batch,
// while the GPU computes the next batch; bricks of one repeated leaf (solid
// stone away from the tunnels) reuse one reduction.  Same DAG, same numbering.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "och_internal.h"
#include "och_terrain.h"

namespace {

using och_terrain::Tables;

const Tables kTables = {OCH_PERM_TABLE, OCH_GRAD_TABLE};

int default_threads()
{
    if (const char *e = std::getenv("OMP_NUM_THREADS")) {
        const int v = std::atoi(e);
        if (v > 0) return std::min(v, 256);
    }
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) return std::max(1, std::min(CPU_COUNT(&set), 256));
    return std::max(1u, std::min(std::thread::hardware_concurrency(), 256u));
}

template <class T>
T *map_zeroed(size_t count)
{
    void *p = mmap(nullptr, count * sizeof(T), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    return p == MAP_FAILED ? nullptr : static_cast<T *>(p);
}

template <class T>
void unmap(T *p, size_t count)
{
    if (p) munmap(p, count * sizeof(T));
}

inline uint64_t mix64(uint64_t h)
{
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    h *= 0xC4CEB9FE1A85EC53ull;
    h ^= h >> 33;
    return h;
}

// Lock-free interning of (level, 8 child words) -> node id.  Ids are handed
// out by one atomic counter; a lost insert race leaves an unused id behind
// (dropped by the breadth-first renumbering).
struct NodeStore {
    uint32_t cap = 0;
    uint32_t *nodes = nullptr;             // cap x 8
    uint8_t *level = nullptr;              // height above the voxels of each id
    std::atomic<uint32_t> next{1};         // id 0 = empty
    std::atomic<uint32_t> *table = nullptr;
    uint64_t table_mask = 0;
    std::atomic<uint32_t> *leaf_ids = nullptr;   // direct map of 3-bit-per-voxel leaf codes
    std::atomic<bool> full{false};
    bool dedup = true;

    bool init(uint32_t capacity, bool dd)
    {
        cap = capacity;
        dedup = dd;
        nodes = map_zeroed<uint32_t>((size_t)cap * 8);
        level = map_zeroed<uint8_t>(cap);
        if (!nodes || !level) return false;
        if (dedup) {
            uint64_t ts = 1;
            while (ts < (uint64_t)cap * 2) ts <<= 1;
            table_mask = ts - 1;
            table = map_zeroed<std::atomic<uint32_t>>(ts);
            leaf_ids = map_zeroed<std::atomic<uint32_t>>(1u << 24);
            if (!table || !leaf_ids) return false;
        }
        return true;
    }
    void release()
    {
        unmap(nodes, (size_t)cap * 8);
        unmap(level, cap);
        unmap(table, table_mask + 1);
        unmap(leaf_ids, (size_t)1 << 24);
        nodes = nullptr;
        level = nullptr;
        table = nullptr;
        leaf_ids = nullptr;
    }

    uint32_t alloc(const uint32_t *c, int h)
    {
        const uint32_t id = next.fetch_add(1, std::memory_order_relaxed);
        if (id >= cap) {
            full.store(true, std::memory_order_relaxed);
            return 0;
        }
        std::memcpy(nodes + (size_t)id * 8, c, 32);
        level[id] = (uint8_t)h;
        return id;
    }

    // A leaf-level node given as its code (3 bits per child, child k at bits 3k).
    uint32_t intern_code(uint32_t code)
    {
        uint32_t c[8];
        for (int k = 0; k < 8; ++k) c[k] = (code >> (3 * k)) & 7u;
        if (!dedup) return alloc(c, 0);
        std::atomic<uint32_t> &slot = leaf_ids[code];
        uint32_t id = slot.load(std::memory_order_acquire);
        if (id) return id;
        const uint32_t mine = alloc(c, 0);
        if (!mine) return 0;
        if (slot.compare_exchange_strong(id, mine, std::memory_order_acq_rel)) return mine;
        return id;
    }

    uint32_t intern(const uint32_t *c, int h)
    {
        if (!dedup) return alloc(c, h);
        if (h == 0) {
            uint32_t code = 0;
            bool small = true;
            for (int k = 0; k < 8; ++k) {
                small &= c[k] < 8;
                code |= (c[k] & 7u) << (3 * k);
            }
            if (small) {
                std::atomic<uint32_t> &slot = leaf_ids[code];
                uint32_t id = slot.load(std::memory_order_acquire);
                if (id) return id;
                const uint32_t mine = alloc(c, h);
                if (!mine) return 0;
                if (slot.compare_exchange_strong(id, mine, std::memory_order_acq_rel)) return mine;
                return id;
            }
        }
        uint64_t w[4];
        std::memcpy(w, c, 32);
        uint64_t hs = mix64((uint64_t)h * 0x9E3779B97F4A7C15ull ^ w[0]);
        hs = mix64(hs ^ w[1]);
        hs = mix64(hs ^ w[2]);
        hs = mix64(hs ^ w[3]);
        uint64_t i = hs & table_mask;
        uint32_t mine = 0;
        for (;;) {
            uint32_t id = table[i].load(std::memory_order_acquire);
            if (!id) {
                if (!mine) {
                    mine = alloc(c, h);
                    if (!mine) return 0;
                }
                if (table[i].compare_exchange_strong(id, mine, std::memory_order_acq_rel)) return mine;
            }
            if (level[id] == h && std::memcmp(nodes + (size_t)id * 8, c, 32) == 0) return id;
            i = (i + 1) & table_mask;
        }
    }
};

struct Terrain {
    int depth = 0, dim = 0;
    bool tunnels = true;
    std::vector<int32_t> heights;
    std::vector<uint8_t> tops;
    std::vector<int32_t> brick_hmax;   // max column height per brick column
};

void parallel_for(int threads, uint64_t n, const std::function<void(uint64_t, int)> &fn)
{
    std::atomic<uint64_t> next{0};
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
        pool.emplace_back([&, t] {
            for (;;) {
                const uint64_t i = next.fetch_add(1, std::memory_order_relaxed);
                if (i >= n) break;
                fn(i, t);
            }
        });
    for (auto &th : pool) th.join();
}

struct BrickStats {
    uint64_t hist[8] = {0};
    uint64_t tree_nodes = 0;
};

// Reduce a brick's leaf-level ids (n^3, n = S/2, (z*n+y)*n+x) to its subtree
// root: levels h = 1 .. s_log2 - 1, in place.
uint32_t reduce_brick(NodeStore &ns, int s_log2, std::vector<uint32_t> &ids, BrickStats &st)
{
    int n = (1 << s_log2) / 2;
    for (int h = 1; h < s_log2; ++h) {
        const int m = n / 2;
        // nodes of eight equal children (solid stone) repeat: the last one per
        // level skips the hash table (a DAG only; an expanded tree shares nothing)
        uint32_t last_child = 0, last_id = 0;
        for (int z = 0; z < m; ++z)
            for (int y = 0; y < m; ++y)
                for (int x = 0; x < m; ++x) {
                    uint32_t c[8];
                    bool any = false, same = true;
                    for (int k = 0; k < 8; ++k) {
                        const int cx = 2 * x + (k & 1), cy = 2 * y + ((k >> 1) & 1), cz = 2 * z + ((k >> 2) & 1);
                        c[k] = ids[((size_t)cz * n + cy) * n + cx];
                        any |= c[k] != 0;
                        same &= c[k] == c[0];
                    }
                    uint32_t id = 0;
                    if (any) {
                        if (same && ns.dedup && c[0] == last_child) {
                            id = last_id;
                        } else {
                            id = ns.intern(c, h);
                            if (same) last_child = c[0], last_id = id;
                        }
                        ++st.tree_nodes;
                    }
                    ids[((size_t)z * m + y) * m + x] = id;   // safe: writes trail reads
                }
        n = m;
    }
    return ids[0];
}

// Voxelise one brick of side S at (bx, by, bz) (brick units) and reduce it to
// its subtree root.  vox: S^3 scratch, ids: (S/2)^3 scratch.
uint32_t build_brick(const Terrain &tr, NodeStore &ns, int s_log2, int bx, int by, int bz, std::vector<uint8_t> &vox,
                     std::vector<uint32_t> &ids, BrickStats &st)
{
    const int S = 1 << s_log2;
    const int x0 = bx * S, y0 = by * S, z0 = bz * S;
    for (int y = 0; y < S; ++y)
        for (int x = 0; x < S; ++x) {
            const size_t col = (size_t)(y0 + y) * tr.dim + (x0 + x);
            const int h = tr.heights[col], top = tr.tops[col];
            uint8_t *v = &vox[((size_t)y * S + x) * S];   // z fastest
            for (int z = 0; z < S; ++z) {
                const uint32_t val = och_terrain::voxel_value(kTables, x0 + x, y0 + y, z0 + z, h, top, tr.tunnels);
                v[z] = (uint8_t)val;
                st.hist[val & 7]++;
            }
        }
    // h = 0: children are voxels, child index c = x | y << 1 | z << 2
    const int n = S / 2;
    for (int z = 0; z < n; ++z)
        for (int y = 0; y < n; ++y)
            for (int x = 0; x < n; ++x) {
                uint32_t c[8];
                bool any = false;
                for (int k = 0; k < 8; ++k) {
                    const int vx = 2 * x + (k & 1), vy = 2 * y + ((k >> 1) & 1), vz = 2 * z + ((k >> 2) & 1);
                    c[k] = vox[((size_t)vy * S + vx) * S + vz];
                    any |= c[k] != 0;
                }
                uint32_t id = 0;
                if (any) {
                    id = ns.intern(c, 0);
                    ++st.tree_nodes;
                }
                ids[((size_t)z * n + y) * n + x] = id;
            }
    return reduce_brick(ns, s_log2, ids, st);
}

// ------------------------------------------------------------ GPU voxelisation

constexpr int kBrickLog2 = 5, kBrick = 32, kLeaves = 4096;   // 32^3 voxels, 16^3 leaf-level nodes
constexpr uint32_t kMixed = 0xFFFFFFFFu;

__constant__ och_terrain::Tables c_tables = {OCH_PERM_TABLE, OCH_GRAD_TABLE};

// One workgroup per brick (bricks[i] = bx | by << 10 | bz << 20): the 4096
// leaf codes, (z * 16 + y) * 16 + x order; info[i] = {the common code when
// every leaf is equal, else kMixed; voxel counts of ids 0..7}.
__global__ __launch_bounds__(256) void k_brick_codes(const int32_t *__restrict__ heights, const uint8_t *__restrict__ tops,
                                                     int dim, int tunnels, const uint32_t *__restrict__ bricks,
                                                     uint32_t *__restrict__ codes, uint32_t *__restrict__ info)
{
    __shared__ och_terrain::Tables T;
    __shared__ uint32_t hist[8], firsts[256];
    __shared__ int mixed;
    for (int i = threadIdx.x; i < (int)sizeof(T); i += blockDim.x)
        reinterpret_cast<uint8_t *>(&T)[i] = reinterpret_cast<const uint8_t *>(&c_tables)[i];
    if (threadIdx.x < 8) hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) mixed = 0;
    __syncthreads();
    const uint32_t b = bricks[blockIdx.x];
    const int x0 = (int)(b & 1023u) * kBrick, y0 = (int)((b >> 10) & 1023u) * kBrick, z0 = (int)(b >> 20) * kBrick;
    uint32_t cnt[5] = {0, 0, 0, 0, 0}, other = 0;
    uint32_t first = 0;
    bool same = true;
    for (int leaf = threadIdx.x; leaf < kLeaves; leaf += blockDim.x) {
        const int lx = leaf & 15, ly = (leaf >> 4) & 15, lz = leaf >> 8;
        uint32_t code = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int x = x0 + 2 * lx + (k & 1), y = y0 + 2 * ly + ((k >> 1) & 1), z = z0 + 2 * lz + ((k >> 2) & 1);
            const size_t col = (size_t)y * dim + x;
            const uint32_t v = och_terrain::voxel_value(T, x, y, z, heights[col], tops[col], tunnels != 0);
            code |= (v & 7u) << (3 * k);
            if (v < 5) ++cnt[v];
            else ++other;
        }
        codes[(size_t)blockIdx.x * kLeaves + leaf] = code;
        if (leaf == (int)threadIdx.x) first = code;
        same &= code == first;
    }
    for (int v = 0; v < 5; ++v)
        if (cnt[v]) atomicAdd(&hist[v], cnt[v]);
    if (other) atomicAdd(&hist[5], other);        // ids above 4 do not occur in this terrain
    firsts[threadIdx.x] = first;
    if (!same) mixed = 1;
    __syncthreads();
    if (firsts[threadIdx.x] != firsts[0]) mixed = 1;
    __syncthreads();
    if (threadIdx.x == 0) info[(size_t)blockIdx.x * 8] = mixed ? kMixed : firsts[0];
    if (threadIdx.x < 6) info[(size_t)blockIdx.x * 8 + 1 + threadIdx.x] = hist[threadIdx.x];
}

#define BUILD_HIP(expr)                       \
    do {                                      \
        if ((expr) != hipSuccess) return false; \
    } while (0)

// Voxelise `work` on the current GPU in batches and hash-cons the codes on
// `threads` host threads, overlapping batch k + 1 on the GPU with batch k on
// the host.  Returns false when no GPU could run the voxel kernel; the caller
// then fails the build with OCH_E_NODEV (no host fallback).
bool build_bricks_gpu(const Terrain &tr, NodeStore &ns, int threads, const std::vector<uint32_t> &work, int G,
                      std::vector<uint32_t> &brick_root, std::vector<BrickStats> &stats, double *gpu_seconds)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return false;
    const size_t n_work = work.size();
    const size_t B = 4096;                        // bricks per batch: 64 MiB of codes
    int32_t *d_heights = nullptr;
    uint8_t *d_tops = nullptr;
    uint32_t *d_bricks[2] = {nullptr, nullptr}, *d_codes[2] = {nullptr, nullptr}, *d_info[2] = {nullptr, nullptr};
    uint32_t *h_codes[2] = {nullptr, nullptr}, *h_info[2] = {nullptr, nullptr}, *h_bricks[2] = {nullptr, nullptr};
    hipStream_t st[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    auto cleanup = [&] {
        for (int k = 0; k < 2; ++k) {
            if (st[k]) (void)hipStreamSynchronize(st[k]);
            if (d_bricks[k]) (void)hipFree(d_bricks[k]);
            if (d_codes[k]) (void)hipFree(d_codes[k]);
            if (d_info[k]) (void)hipFree(d_info[k]);
            if (h_codes[k]) (void)hipHostFree(h_codes[k]);
            if (h_info[k]) (void)hipHostFree(h_info[k]);
            if (h_bricks[k]) (void)hipHostFree(h_bricks[k]);
            if (done[k]) (void)hipEventDestroy(done[k]);
            if (st[k]) (void)hipStreamDestroy(st[k]);
        }
        if (d_heights) (void)hipFree(d_heights);
        if (d_tops) (void)hipFree(d_tops);
    };
    auto run = [&]() -> bool {
        const size_t cols = (size_t)tr.dim * tr.dim;
        BUILD_HIP(hipMalloc(&d_heights, cols * 4));
        BUILD_HIP(hipMalloc(&d_tops, cols));
        BUILD_HIP(hipMemcpy(d_heights, tr.heights.data(), cols * 4, hipMemcpyHostToDevice));
        BUILD_HIP(hipMemcpy(d_tops, tr.tops.data(), cols, hipMemcpyHostToDevice));
        for (int k = 0; k < 2; ++k) {
            BUILD_HIP(hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking));
            BUILD_HIP(hipEventCreateWithFlags(&done[k], hipEventDisableTiming));
            BUILD_HIP(hipMalloc(&d_bricks[k], B * 4));
            BUILD_HIP(hipMalloc(&d_codes[k], B * kLeaves * 4));
            BUILD_HIP(hipMalloc(&d_info[k], B * 8 * 4));
            BUILD_HIP(hipHostMalloc(&h_codes[k], B * kLeaves * 4, hipHostMallocDefault));
            BUILD_HIP(hipHostMalloc(&h_info[k], B * 8 * 4, hipHostMallocDefault));
            BUILD_HIP(hipHostMalloc(&h_bricks[k], B * 4, hipHostMallocDefault));
        }
        const size_t n_batches = (n_work + B - 1) / B;
        auto launch = [&](size_t batch) -> bool {
            const int k = (int)(batch & 1);
            const size_t lo = batch * B, n = std::min(B, n_work - lo);
            for (size_t i = 0; i < n; ++i) {
                const uint32_t w = work[lo + i];
                const uint32_t bx = w % G, by = (w / G) % G, bz = w / (G * G);
                h_bricks[k][i] = bx | by << 10 | bz << 20;
            }
            BUILD_HIP(hipMemcpyAsync(d_bricks[k], h_bricks[k], n * 4, hipMemcpyHostToDevice, st[k]));
            hipLaunchKernelGGL(k_brick_codes, dim3((unsigned)n), dim3(256), 0, st[k], d_heights, d_tops, tr.dim,
                               tr.tunnels ? 1 : 0, d_bricks[k], d_codes[k], d_info[k]);
            BUILD_HIP(hipGetLastError());
            BUILD_HIP(hipMemcpyAsync(h_codes[k], d_codes[k], n * kLeaves * 4, hipMemcpyDeviceToHost, st[k]));
            BUILD_HIP(hipMemcpyAsync(h_info[k], d_info[k], n * 8 * 4, hipMemcpyDeviceToHost, st[k]));
            BUILD_HIP(hipEventRecord(done[k], st[k]));
            return true;
        };
        // Bricks whose 4096 leaves are one repeated code reduce to the same root.
        std::mutex memo_mu;
        std::unordered_map<uint32_t, std::pair<uint32_t, uint64_t>> memo;   // code -> (root, tree nodes)
        std::vector<std::vector<uint32_t>> ids(threads, std::vector<uint32_t>(kLeaves));
        const auto t0 = std::chrono::steady_clock::now();
        if (n_batches && !launch(0)) return false;
        for (size_t batch = 0; batch < n_batches; ++batch) {
            const int k = (int)(batch & 1);
            BUILD_HIP(hipEventSynchronize(done[k]));
            // the other buffer is free: its batch was consumed in the previous round
            if (batch + 1 < n_batches && !launch(batch + 1)) return false;
            const size_t lo = batch * B, n = std::min(B, n_work - lo);
            const uint32_t *codes = h_codes[k], *info = h_info[k];
            parallel_for(threads, n, [&](uint64_t i, int t) {
                BrickStats &bs = stats[t];
                const uint32_t *inf = info + i * 8;
                for (int v = 0; v < 6; ++v) bs.hist[v] += inf[1 + v];
                // an expanded tree (dedup = 0) shares nothing: every brick reduced on its own
                const uint32_t uni = ns.dedup ? inf[0] : kMixed;
                uint32_t root = 0;
                if (uni != kMixed) {
                    {
                        std::lock_guard<std::mutex> g(memo_mu);
                        auto it = memo.find(uni);
                        if (it != memo.end()) {
                            bs.tree_nodes += it->second.second;
                            brick_root[work[lo + i]] = it->second.first;
                            return;
                        }
                    }
                    BrickStats one;
                    std::vector<uint32_t> &id = ids[t];
                    const uint32_t leaf = uni ? ns.intern_code(uni) : 0;
                    std::fill(id.begin(), id.end(), leaf);
                    one.tree_nodes = uni ? (uint64_t)kLeaves : 0;
                    root = reduce_brick(ns, kBrickLog2, id, one);
                    bs.tree_nodes += one.tree_nodes;
                    std::lock_guard<std::mutex> g(memo_mu);
                    memo.emplace(uni, std::make_pair(root, one.tree_nodes));
                } else {
                    std::vector<uint32_t> &id = ids[t];
                    const uint32_t *c = codes + i * kLeaves;
                    uint32_t last_code = 0, last_id = 0;
                    for (int l = 0; l < kLeaves; ++l) {
                        const uint32_t code = c[l];
                        if (code != last_code || !ns.dedup) {
                            last_code = code;
                            last_id = code ? ns.intern_code(code) : 0;
                        }
                        id[l] = last_id;
                        bs.tree_nodes += code != 0;
                    }
                    root = reduce_brick(ns, kBrickLog2, id, bs);
                }
                brick_root[work[lo + i]] = root;
            });
        }
        if (gpu_seconds) *gpu_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return true;
    };
    const bool ok = run();
    cleanup();
    return ok;
}

}  // namespace

extern "C" {

OCH_API void och_host_pool_free(och_host_pool *p)
{
    if (!p) return;
    std::free(p->nodes);
    p->nodes = nullptr;
    p->n_nodes = 0;
}

OCH_API int och_build_terrain(const och_terrain_params *params, och_host_pool *out)
{
    if (!params || !out) return OCH_E_INVALID;
    const int depth = params->depth;
    if (depth < 1 || depth > 12) return OCH_E_INVALID;
    if (!params->dedup && depth > 10) return OCH_E_INVALID;   // expanded tree would exceed 1 GB
    const auto t_start = std::chrono::steady_clock::now();
    std::memset(out, 0, sizeof *out);
    const int threads = params->threads > 0 ? params->threads : default_threads();

    Terrain tr;
    tr.depth = depth;
    tr.dim = 1 << depth;
    tr.tunnels = params->tunnels != 0;
    const int dim = tr.dim;
    tr.heights.resize((size_t)dim * dim);
    tr.tops.resize((size_t)dim * dim);
    parallel_for(threads, (uint64_t)dim, [&](uint64_t y, int) {
        for (int x = 0; x < dim; ++x)
            tr.heights[y * dim + x] = och_terrain::column_height(kTables, x, (int)y, dim);
    });
    // Column tops: one rand() per column, y outer, x inner (ORT/test_och_h_octree.cpp:776-780).
    if (params->rand_kind == 1) {
        och_terrain::MsvcRand r;
        for (size_t i = 0; i < tr.tops.size(); ++i) tr.tops[i] = (uint8_t)(2 + (r.next() > 0x7FFF / 2));
    } else {
        och_terrain::GlibcRand r;
        r.seed(1);
        for (size_t i = 0; i < tr.tops.size(); ++i) tr.tops[i] = (uint8_t)(2 + (r.next() > 0x7FFFFFFF / 2));
    }

    const int s_log2 = std::min(depth, 5);
    const int S = 1 << s_log2, G = dim / S;
    tr.brick_hmax.assign((size_t)G * G, -1);
    for (int by = 0; by < G; ++by)
        for (int bx = 0; bx < G; ++bx) {
            int hm = -1;
            for (int y = by * S; y < (by + 1) * S; ++y)
                for (int x = bx * S; x < (bx + 1) * S; ++x) hm = std::max(hm, tr.heights[(size_t)y * dim + x]);
            tr.brick_hmax[(size_t)by * G + bx] = hm;
        }

    NodeStore ns;
    const uint32_t cap = params->dedup ? (depth <= 8 ? (1u << 20) : depth <= 10 ? (1u << 23) : (1u << 28))
                                       : (uint32_t)std::min<uint64_t>(1ull << 28, 48ull << (2 * depth));
    if (!ns.init(cap, params->dedup != 0)) {
        ns.release();
        return OCH_E_NOMEM;
    }

    // Bricks that reach below the highest surface of their columns.
    std::vector<uint32_t> work;
    for (int bz = 0; bz < G; ++bz)
        for (int by = 0; by < G; ++by)
            for (int bx = 0; bx < G; ++bx)
                if (bz * S <= tr.brick_hmax[(size_t)by * G + bx]) work.push_back(((uint32_t)bz * G + by) * G + bx);
    std::vector<uint32_t> brick_root((size_t)G * G * G, 0);
    std::vector<BrickStats> stats(threads);
    double gpu_s = 0.0;
    if (params->use_gpu && s_log2 == kBrickLog2) {
        if (!build_bricks_gpu(tr, ns, threads, work, G, brick_root, stats, &gpu_s)) {
            ns.release();
            return OCH_E_NODEV;   // asked for the GPU and none could run the voxel kernel
        }
    } else {
        std::vector<std::vector<uint8_t>> vox(threads, std::vector<uint8_t>((size_t)S * S * S));
        std::vector<std::vector<uint32_t>> ids(threads, std::vector<uint32_t>((size_t)S * S * S / 8));
        parallel_for(threads, work.size(), [&](uint64_t i, int t) {
            const uint32_t b = work[i];
            const int bx = b % G, by = (b / G) % G, bz = b / (G * G);
            brick_root[b] = build_brick(tr, ns, s_log2, bx, by, bz, vox[t], ids[t], stats[t]);
        });
    }
    BrickStats total;
    for (auto &s : stats) {
        for (int k = 0; k < 8; ++k) total.hist[k] += s.hist[k];
        total.tree_nodes += s.tree_nodes;
    }
    // Levels above the bricks.
    uint32_t root = 0;
    {
        std::vector<uint32_t> cur = brick_root, nxt;
        int n = G;
        for (int h = s_log2; h < depth; ++h) {
            const int m = n / 2;
            nxt.assign((size_t)m * m * m, 0);
            for (int z = 0; z < m; ++z)
                for (int y = 0; y < m; ++y)
                    for (int x = 0; x < m; ++x) {
                        uint32_t c[8];
                        bool any = false;
                        for (int k = 0; k < 8; ++k) {
                            const int cx = 2 * x + (k & 1), cy = 2 * y + ((k >> 1) & 1), cz = 2 * z + ((k >> 2) & 1);
                            c[k] = cur[((size_t)cz * n + cy) * n + cx];
                            any |= c[k] != 0;
                        }
                        if (any) {
                            nxt[((size_t)z * m + y) * m + x] = ns.intern(c, h);
                            ++total.tree_nodes;
                        }
                    }
            cur.swap(nxt);
            n = m;
        }
        root = cur[0];
    }
    if (ns.full.load()) {
        ns.release();
        return OCH_E_CAPACITY;
    }

    // Breadth-first renumbering: level by level from the root, children in
    // slot order.  1-based (h_octree, slot 0 never used) or 0-based octree.
    const uint32_t used = std::min(ns.next.load(), ns.cap);
    const int base = params->dedup ? 1 : 0;
    std::vector<uint32_t> newid(used, 0);
    std::vector<uint32_t> order;
    if (root) {
        order.reserve(1024);
        std::vector<uint32_t> level{root};
        newid[root] = (uint32_t)base;
        order.push_back(root);
        for (int l = 1; l < depth; ++l) {
            std::vector<uint32_t> nxt;
            for (uint32_t v : level) {
                const uint32_t *c = ns.nodes + (size_t)v * 8;
                for (int k = 0; k < 8; ++k)
                    if (c[k] && !(newid[c[k]] || c[k] == root)) {
                        newid[c[k]] = (uint32_t)(order.size() + base);
                        order.push_back(c[k]);
                        nxt.push_back(c[k]);
                    }
            }
            level.swap(nxt);
        }
    }
    const uint32_t n_out = (uint32_t)std::max<size_t>(order.size(), 1);
    uint32_t *nodes = static_cast<uint32_t *>(std::calloc((size_t)n_out * 8, 4));
    if (!nodes) {
        ns.release();
        return OCH_E_NOMEM;
    }
    for (size_t i = 0; i < order.size(); ++i) {
        const uint32_t v = order[i];
        const uint32_t *c = ns.nodes + (size_t)v * 8;
        const bool leaf = ns.level[v] == 0;
        for (int k = 0; k < 8; ++k) nodes[i * 8 + k] = (leaf || !c[k]) ? c[k] : newid[c[k]];
    }
    ns.release();

    out->nodes = nodes;
    out->n_nodes = n_out;
    out->root = root ? (uint32_t)base : 0;
    out->depth = depth;
    out->index_base = base;
    out->tree_nodes = total.tree_nodes;
    for (int k = 0; k < 8; ++k) out->voxel_hist[k] = total.hist[k];
    out->solid_voxels = 0;
    for (int k = 1; k < 8; ++k) out->solid_voxels += total.hist[k];
    out->build_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    return OCH_OK;
}

}  // extern "C"
