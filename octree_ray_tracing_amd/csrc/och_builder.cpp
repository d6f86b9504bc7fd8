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
// histogram and whether all its leaves are equal.  A DAG is then hash-consed
// on the GPU too (build_dag_gpu, below) and only renumbered on the host; an
// expanded tree's nodes are allocated by host threads from the codes, batch
// after batch, while the GPU computes the next batch.  Same pool either way.
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

#include <hipcub/hipcub.hpp>

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

// Zeroed, lazily backed; transparent huge pages where the kernel allows them
// (the hash table and the leaf map are probed at random: fewer TLB misses).
template <class T>
T *map_zeroed(size_t count)
{
    void *p = mmap(nullptr, count * sizeof(T), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (p == MAP_FAILED) return nullptr;
    (void)madvise(p, count * sizeof(T), MADV_HUGEPAGE);
    return static_cast<T *>(p);
}

template <class T>
void unmap(T *p, size_t count)
{
    if (p) munmap(p, count * sizeof(T));
}

__host__ __device__ inline uint64_t mix64(uint64_t h)
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
// every leaf is equal, else kMixed; voxel counts of ids 0..5; non-empty leaf codes}.
__global__ __launch_bounds__(256) void k_brick_codes(const int32_t *__restrict__ heights, const uint8_t *__restrict__ tops,
                                                     int dim, int tunnels, const uint32_t *__restrict__ bricks,
                                                     uint32_t *__restrict__ codes, uint32_t *__restrict__ info)
{
    __shared__ och_terrain::Tables T;
    __shared__ uint32_t hist[8], firsts[256];
    __shared__ uint32_t leaves;   // non-empty leaf-level nodes of the brick
    __shared__ int mixed;
    for (int i = threadIdx.x; i < (int)sizeof(T); i += blockDim.x)
        reinterpret_cast<uint8_t *>(&T)[i] = reinterpret_cast<const uint8_t *>(&c_tables)[i];
    if (threadIdx.x < 8) hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) mixed = 0, leaves = 0;
    __syncthreads();
    const uint32_t b = bricks[blockIdx.x];
    const int x0 = (int)(b & 1023u) * kBrick, y0 = (int)((b >> 10) & 1023u) * kBrick, z0 = (int)(b >> 20) * kBrick;
    uint32_t cnt[5] = {0, 0, 0, 0, 0}, other = 0;
    uint32_t first = 0, nonempty = 0;
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
        nonempty += code != 0;
        if (leaf == (int)threadIdx.x) first = code;
        same &= code == first;
    }
    for (int v = 0; v < 5; ++v)
        if (cnt[v]) atomicAdd(&hist[v], cnt[v]);
    if (other) atomicAdd(&hist[5], other);        // ids above 4 do not occur in this terrain
    if (nonempty) atomicAdd(&leaves, nonempty);
    firsts[threadIdx.x] = first;
    if (!same) mixed = 1;
    __syncthreads();
    if (firsts[threadIdx.x] != firsts[0]) mixed = 1;
    __syncthreads();
    if (threadIdx.x == 0) info[(size_t)blockIdx.x * 8] = mixed ? kMixed : firsts[0];
    if (threadIdx.x < 6) info[(size_t)blockIdx.x * 8 + 1 + threadIdx.x] = hist[threadIdx.x];
    if (threadIdx.x == 6) info[(size_t)blockIdx.x * 8 + 7] = leaves;
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
    (void)hipGetLastError();        // a stale error of an earlier HIP call (another library's) is not this build's
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
        double wait_s = 0.0, host_s = 0.0;
        size_t mixed = 0;
        for (size_t batch = 0; batch < n_batches; ++batch) {
            const int k = (int)(batch & 1);
            const auto w0 = std::chrono::steady_clock::now();
            BUILD_HIP(hipEventSynchronize(done[k]));
            const auto w1 = std::chrono::steady_clock::now();
            wait_s += std::chrono::duration<double>(w1 - w0).count();
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
            for (size_t i = 0; i < n; ++i) mixed += h_info[k][i * 8] == kMixed;
            host_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - w1).count();
        }
        if (std::getenv("OCH_BUILD_TRACE"))
            std::fprintf(stderr, "[och_build] bricks: %zu (%zu mixed), %zu batches, waited %.3f s, host %.3f s\n", n_work,
                         mixed, (size_t)n_batches, wait_s, host_s);
        if (gpu_seconds) *gpu_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return true;
    };
    const bool ok = run();
    cleanup();
    return ok;
}

// ------------------------------------------------------------ GPU hash-consing
//
// A DAG build (dedup) with use_gpu interns on the GPU as well; the host only
// renumbers.  Leaf-level nodes are interned by their 24-bit code through a
// direct map (k_intern_codes).  Every level above is one pair of dispatches
// over all its nodes:
//   k_intern -- each node gathers its eight child ids (written by an earlier
//               dispatch); empty nodes stop there.  The rest probe one open-
//               addressing table shared by all levels.  An empty slot is
//               claimed by compare-and-swap with the node's own index (kCand |
//               index) and the claimant allocates the node's id and writes its
//               record.  A node meeting a claimed slot compares its children
//               with the claimant's, gathered again from the same earlier
//               dispatch's ids; a slot holding a finished id is compared with
//               that node's record, written by an earlier dispatch.
//   k_settle -- each node takes its id (its own or its claimant's) and each
//               claimant turns its slot into the finished id.
// No dispatch reads what another workgroup writes in the same dispatch except
// through the atomics, so the per-XCD L2s need no coherence beyond dispatch
// boundaries.  Ids come from one counter in claim order and differ from run to
// run; the breadth-first renumbering makes the pool identical to the host
// build's, slot for slot.

constexpr uint32_t kCand = 0x80000000u;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

struct GpuStore {
    uint32_t *nodes;                 // cap x 8 child words
    uint8_t *level;                  // height above the voxels of each id
    uint32_t *next;                  // id counter, starts at 1 (0 = empty)
    uint32_t *table;                 // tmask + 1 slots: 0, kCand | node index (this level), or an id
    uint32_t *leaf_id;               // 2^24 leaf codes -> id
    uint32_t *overflow;              // 1: capacity exhausted, 2: table exhausted
    unsigned long long *tree_nodes;  // kCounters partial counts of expanded-tree nodes, 128 B apart
    uint32_t cap, tmask;
};

// One level: nb grids of side n (node index = grid * n^3 + (z * n + y) * n + x),
// children in the previous level's grids of side 2n.
struct GpuLevel {
    const uint32_t *src;   // child ids, or leaf codes (codes = 1: the child id is leaf_id[code])
    int codes;
    int log2n;
    uint32_t count;        // nb * n^3
    int h;
};

constexpr int kCounters = 64;

// Block-wide count, then one atomic per block on one of kCounters addresses.
__device__ inline void count_nodes(const GpuStore &S, bool nz)
{
    __shared__ uint32_t block_count;
    if (threadIdx.x == 0) block_count = 0;
    __syncthreads();
    const uint64_t b = __ballot(nz);
    if ((threadIdx.x & 63u) == 0 && b) atomicAdd(&block_count, (uint32_t)__popcll(b));
    __syncthreads();
    if (threadIdx.x == 0 && block_count)
        atomicAdd(S.tree_nodes + 16 * (blockIdx.x % kCounters), (unsigned long long)block_count);
}

__device__ inline uint32_t alloc_node(const GpuStore &S, const uint32_t c[8], int h)
{
    const uint32_t id = atomicAdd(S.next, 1u);
    if (id >= S.cap) {
        atomicOr(S.overflow, 1u);
        return 0;
    }
    uint4 *dst = reinterpret_cast<uint4 *>(S.nodes + (size_t)id * 8);
    dst[0] = make_uint4(c[0], c[1], c[2], c[3]);
    dst[1] = make_uint4(c[4], c[5], c[6], c[7]);
    S.level[id] = (uint8_t)h;
    return id;
}

__device__ inline bool gather(const GpuStore &S, const GpuLevel &L, uint32_t idx, uint32_t c[8])
{
    const uint32_t n = 1u << L.log2n, m = 2u * n;
    const uint32_t g = idx >> (3 * L.log2n), r = idx & ((1u << (3 * L.log2n)) - 1u);
    const uint32_t x = r & (n - 1u), y = (r >> L.log2n) & (n - 1u), z = r >> (2 * L.log2n);
    const size_t base = (size_t)g * m * m * m;
    bool any = false;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t cx = 2u * x + (k & 1), cy = 2u * y + ((k >> 1) & 1), cz = 2u * z + ((k >> 2) & 1);
        uint32_t v = L.src[base + ((size_t)cz * m + cy) * m + cx];
        if (L.codes && v) v = S.leaf_id[v];
        c[k] = v;
        any |= v != 0;
    }
    return any;
}

__device__ inline uint32_t node_slot(const uint32_t c[8], int h, uint32_t mask)
{
    uint64_t hs = mix64((uint64_t)h * 0x9E3779B97F4A7C15ull ^ ((uint64_t)c[1] << 32 | c[0]));
    hs = mix64(hs ^ ((uint64_t)c[3] << 32 | c[2]));
    hs = mix64(hs ^ ((uint64_t)c[5] << 32 | c[4]));
    hs = mix64(hs ^ ((uint64_t)c[7] << 32 | c[6]));
    return (uint32_t)hs & mask;
}

__global__ __launch_bounds__(256) void k_intern_codes(GpuStore S, const uint32_t *__restrict__ codes, uint32_t count)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t code = i < count ? codes[i] : 0u;   // counted by k_brick_codes (info[7])
    if (!code) return;
    // A plain (cached) load: a stale 0 only sends the thread to the CAS, which
    // sees the truth; most codes were interned by an earlier batch.
    if (S.leaf_id[code] != 0 || atomicCAS(&S.leaf_id[code], 0u, kCand) != 0u) return;
    uint32_t c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = (code >> (3 * k)) & 7u;
    __hip_atomic_store(&S.leaf_id[code], alloc_node(S, c, 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void k_intern(GpuStore S, GpuLevel L, uint32_t *__restrict__ rep,
                                                uint32_t *__restrict__ slot)
{
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t c[8];
    const bool any = idx < L.count && gather(S, L, idx, c);
    count_nodes(S, any);
    if (idx >= L.count) return;
    slot[idx] = kNoSlot;
    if (!any) {
        rep[idx] = 0;
        return;
    }
    uint32_t i = node_slot(c, L.h, S.tmask);
    for (uint32_t probe = 0; probe <= S.tmask; ++probe, i = (i + 1u) & S.tmask) {
        uint32_t v = S.table[i];   // a stale 0 is corrected by the CAS; claims and ids are never stale
        if (v == 0) {
            v = atomicCAS(&S.table[i], 0u, kCand | idx);
            if (v == 0) {
                rep[idx] = alloc_node(S, c, L.h);
                slot[idx] = i;
                return;
            }
        }
        bool same = true;
        if (v & kCand) {
            uint32_t d[8];
            gather(S, L, v & ~kCand, d);
#pragma unroll
            for (int k = 0; k < 8; ++k) same &= d[k] == c[k];
        } else {
            const uint4 *rec = reinterpret_cast<const uint4 *>(S.nodes + (size_t)v * 8);
            const uint4 a = rec[0], b = rec[1];
            same = S.level[v] == (uint8_t)L.h && a.x == c[0] && a.y == c[1] && a.z == c[2] && a.w == c[3] &&
                   b.x == c[4] && b.y == c[5] && b.z == c[6] && b.w == c[7];
        }
        if (same) {
            rep[idx] = v;
            return;
        }
    }
    atomicOr(S.overflow, 2u);
    rep[idx] = 0;
}

// dst[dst_index ? dst_index[idx] : idx] = the node's id.
__global__ __launch_bounds__(256) void k_settle(GpuStore S, uint32_t count, const uint32_t *__restrict__ rep,
                                                const uint32_t *__restrict__ slot, uint32_t *__restrict__ dst,
                                                const uint32_t *__restrict__ dst_index)
{
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= count) return;
    uint32_t r = rep[idx];
    if (r & kCand) r = rep[r & ~kCand];
    dst[dst_index ? dst_index[idx] : idx] = r;
    const uint32_t s = slot[idx];
    if (s != kNoSlot) S.table[s] = r;
}

// Breadth-first renumbering on the device, one BFS level at a time (ids of
// one height are reachable at one depth only: the height is part of every
// node's key).  The frontier is order[off, off + f), in BFS order; its
// children, in (parent, slot) order, are the candidates q = 8 i + k, and a
// child's first candidate (k_bfs_first, atomicMin) places it (k_bfs_place,
// after an exclusive scan of k_bfs_mark's flags) -- the host renumbering's
// first-occurrence order.
__global__ __launch_bounds__(256) void k_bfs_first(const uint32_t *__restrict__ store, const uint32_t *__restrict__ front,
                                                   uint32_t f, uint32_t *__restrict__ first)
{
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= 8u * f) return;
    const uint32_t c = store[(size_t)front[q >> 3] * 8 + (q & 7u)];
    // first[] only decreases: a cached value at or below q (stale ones are
    // only larger) makes the atomic unnecessary -- shared children (solid
    // stone) are named by millions of slots, and one address's atomics serialise
    if (c && q < first[c]) atomicMin(&first[c], q);
}

__global__ __launch_bounds__(256) void k_bfs_mark(const uint32_t *__restrict__ store, const uint32_t *__restrict__ front,
                                                  uint32_t f, const uint32_t *__restrict__ first, uint32_t *__restrict__ mark)
{
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= 8u * f) return;
    const uint32_t c = store[(size_t)front[q >> 3] * 8 + (q & 7u)];
    mark[q] = (c && first[c] == q) ? 1u : 0u;
}

// order[next + pos[q]] = child, newid[child] = base + next + pos[q]
__global__ __launch_bounds__(256) void k_bfs_place(const uint32_t *__restrict__ store, const uint32_t *__restrict__ front,
                                                   uint32_t f, const uint32_t *__restrict__ mark,
                                                   const uint32_t *__restrict__ pos, uint32_t *__restrict__ order,
                                                   uint32_t next, uint32_t *__restrict__ newid, uint32_t base)
{
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= 8u * f || !mark[q]) return;
    const uint32_t c = store[(size_t)front[q >> 3] * 8 + (q & 7u)];
    order[next + pos[q]] = c;
    newid[c] = base + next + pos[q];
}

__global__ __launch_bounds__(256) void k_bfs_output(const uint32_t *__restrict__ store, const uint8_t *__restrict__ level,
                                                    const uint32_t *__restrict__ order, const uint32_t *__restrict__ newid,
                                                    uint32_t n, uint32_t *__restrict__ out)
{
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= 8u * n) return;
    const uint32_t v = order[q >> 3];
    const uint32_t c = store[(size_t)v * 8 + (q & 7u)];
    out[q] = (level[v] == 0 || !c) ? c : newid[c];
}

// The whole DAG on the current GPU: bricks voxelised (k_brick_codes) and
// interned batch by batch, then the levels above the bricks, then renumbered
// breadth-first (1-based).  *out: malloc'd n_out x 8 words, as renumber().
// Returns a status.
int build_dag_gpu(const Terrain &tr, uint32_t cap, const std::vector<uint32_t> &work, int G, uint32_t **out,
                  uint32_t *n_out, uint32_t &root, BrickStats &total, bool trace)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return OCH_E_NODEV;
    (void)hipGetLastError();        // a stale error of an earlier HIP call (another library's) is not this build's
    const size_t n_work = work.size();
    const size_t B = 8192;                                    // bricks per batch
    const size_t cols = (size_t)tr.dim * tr.dim, grid_cells = (size_t)G * G * G;
    uint32_t tsize = 1;
    while (tsize < 2 * cap) tsize <<= 1;
    const size_t rep_cap = std::max(B * 512, grid_cells / 8);
    std::vector<void *> bufs;
    hipStream_t st = nullptr;
    auto dalloc = [&](void **p, size_t bytes) {
        if (hipMalloc(p, bytes) != hipSuccess) return false;
        bufs.push_back(*p);
        return true;
    };
    int status = OCH_OK;
    auto run = [&]() -> int {
        int32_t *d_heights;
        uint8_t *d_tops;
        uint32_t *d_enc, *d_work, *d_codes, *d_info, *d_rep, *d_slot, *d_a, *d_b, *d_grid[2];
        GpuStore S{};
        S.cap = cap;
        S.tmask = tsize - 1;
        bool ok = dalloc((void **)&d_heights, cols * 4) && dalloc((void **)&d_tops, cols) &&
                  dalloc((void **)&d_enc, std::max<size_t>(n_work, 1) * 4) &&
                  dalloc((void **)&d_work, std::max<size_t>(n_work, 1) * 4) && dalloc((void **)&d_codes, B * kLeaves * 4) &&
                  dalloc((void **)&d_info, std::max<size_t>(n_work, 1) * 32) && dalloc((void **)&d_rep, rep_cap * 4) &&
                  dalloc((void **)&d_slot, rep_cap * 4) && dalloc((void **)&d_a, B * 512 * 4) &&
                  dalloc((void **)&d_b, B * 64 * 4) && dalloc((void **)&d_grid[0], grid_cells * 4) &&
                  dalloc((void **)&d_grid[1], grid_cells * 4) && dalloc((void **)&S.nodes, (size_t)cap * 32) &&
                  dalloc((void **)&S.level, cap) && dalloc((void **)&S.next, 256 + 128 * kCounters) &&
                  dalloc((void **)&S.table, (size_t)tsize * 4) && dalloc((void **)&S.leaf_id, (size_t)4 << 24);
        if (!ok) return OCH_E_NOMEM;
        S.overflow = S.next + 1;
        S.tree_nodes = reinterpret_cast<unsigned long long *>(S.next + 64);
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return OCH_E_HIP;
        std::vector<uint32_t> enc(n_work);
        for (size_t i = 0; i < n_work; ++i) {
            const uint32_t w = work[i];
            enc[i] = (w % G) | ((w / G) % G) << 10 | (w / (G * G)) << 20;
        }
        const uint32_t one = 1;
#define DAG_HIP(expr)                          \
    do {                                       \
        if ((expr) != hipSuccess) return OCH_E_HIP; \
    } while (0)
        DAG_HIP(hipMemcpyAsync(d_heights, tr.heights.data(), cols * 4, hipMemcpyHostToDevice, st));
        DAG_HIP(hipMemcpyAsync(d_tops, tr.tops.data(), cols, hipMemcpyHostToDevice, st));
        DAG_HIP(hipMemcpyAsync(d_enc, enc.data(), n_work * 4, hipMemcpyHostToDevice, st));
        DAG_HIP(hipMemcpyAsync(d_work, work.data(), n_work * 4, hipMemcpyHostToDevice, st));
        DAG_HIP(hipMemsetAsync(S.next, 0, 256 + 128 * kCounters, st));
        DAG_HIP(hipMemcpyAsync(S.next, &one, 4, hipMemcpyHostToDevice, st));
        DAG_HIP(hipMemsetAsync(S.table, 0, (size_t)tsize * 4, st));
        DAG_HIP(hipMemsetAsync(S.leaf_id, 0, (size_t)4 << 24, st));
        DAG_HIP(hipMemsetAsync(S.nodes, 0, 32, st));
        DAG_HIP(hipMemsetAsync(d_grid[0], 0, grid_cells * 4, st));
        auto blocks = [](size_t n) { return dim3((unsigned)((n + 255) / 256)); };
        auto level_pass = [&](const GpuLevel &L, uint32_t *dst, const uint32_t *dst_index) -> bool {
            if (L.count == 0) return true;
            hipLaunchKernelGGL(k_intern, blocks(L.count), dim3(256), 0, st, S, L, d_rep, d_slot);
            hipLaunchKernelGGL(k_settle, blocks(L.count), dim3(256), 0, st, S, L.count, d_rep, d_slot, dst, dst_index);
            return hipGetLastError() == hipSuccess;
        };
        for (size_t lo = 0; lo < n_work; lo += B) {
            const uint32_t n = (uint32_t)std::min(B, n_work - lo);
            hipLaunchKernelGGL(k_brick_codes, dim3(n), dim3(256), 0, st, d_heights, d_tops, tr.dim, tr.tunnels ? 1 : 0,
                               d_enc + lo, d_codes, d_info + lo * 8);
            hipLaunchKernelGGL(k_intern_codes, blocks((size_t)n * kLeaves), dim3(256), 0, st, S, d_codes,
                               n * (uint32_t)kLeaves);
            DAG_HIP(hipGetLastError());
            // brick levels 1..4: 8^3, 4^3, 2^3, 1 node per brick; the roots land in the grid
            if (!level_pass({d_codes, 1, 3, n * 512u, 1}, d_a, nullptr) ||
                !level_pass({d_a, 0, 2, n * 64u, 2}, d_b, nullptr) || !level_pass({d_b, 0, 1, n * 8u, 3}, d_a, nullptr) ||
                !level_pass({d_a, 0, 0, n, 4}, d_grid[0], d_work + lo))
                return OCH_E_HIP;
        }
        // levels above the bricks, one grid of side G / 2, G / 4, ... 1
        int cur = 0, log2n = 0;
        while ((1 << (log2n + 1)) < G) ++log2n;   // G = 2^(log2n + 1)
        for (int h = kBrickLog2; h < tr.depth; ++h, --log2n) {
            if (!level_pass({d_grid[cur], 0, log2n, 1u << (3 * log2n), h}, d_grid[cur ^ 1], nullptr)) return OCH_E_HIP;
            cur ^= 1;
        }
        uint32_t head[4] = {0, 0, 0, 0};
        std::vector<unsigned long long> counts((size_t)16 * kCounters);
        DAG_HIP(hipMemcpyAsync(head, S.next, 16, hipMemcpyDeviceToHost, st));
        DAG_HIP(hipMemcpyAsync(counts.data(), S.tree_nodes, counts.size() * 8, hipMemcpyDeviceToHost, st));
        DAG_HIP(hipMemcpyAsync(&root, d_grid[cur], 4, hipMemcpyDeviceToHost, st));
        std::vector<uint32_t> info(n_work * 8);
        DAG_HIP(hipMemcpyAsync(info.data(), d_info, n_work * 32, hipMemcpyDeviceToHost, st));
        DAG_HIP(hipStreamSynchronize(st));
        if (head[1]) return OCH_E_CAPACITY;
        const uint32_t used = std::min(head[0], cap);
        total.tree_nodes = 0;
        for (int k = 0; k < kCounters; ++k) total.tree_nodes += counts[(size_t)16 * k];
        for (size_t i = 0; i < n_work; ++i) {
            for (int v = 0; v < 6; ++v) total.hist[v] += info[i * 8 + 1 + v];
            total.tree_nodes += info[i * 8 + 7];
        }
        const auto t_bfs = std::chrono::steady_clock::now();
        if (!root) {   // empty world: one zero node
            *n_out = 1;
            *out = static_cast<uint32_t *>(std::calloc(8, 4));
            return *out ? OCH_OK : OCH_E_NOMEM;
        }
        // renumbering: first / newid / order over the ids, mark / pos over one level's candidates
        uint32_t *d_first, *d_newid, *d_order, *d_mark, *d_pos, *d_out;
        const size_t max_cand = (size_t)used * 8;
        if (!dalloc((void **)&d_first, (size_t)used * 4) || !dalloc((void **)&d_newid, (size_t)used * 4) ||
            !dalloc((void **)&d_order, (size_t)used * 4) || !dalloc((void **)&d_mark, max_cand * 4) ||
            !dalloc((void **)&d_pos, max_cand * 4) || !dalloc((void **)&d_out, max_cand * 4))
            return OCH_E_NOMEM;
        size_t scan_bytes = 0;
        DAG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, d_mark, d_pos, (int)max_cand, st));
        void *d_scan = nullptr;
        if (!dalloc(&d_scan, std::max<size_t>(scan_bytes, 4))) return OCH_E_NOMEM;
        const uint32_t base = 1;
        DAG_HIP(hipMemsetAsync(d_first, 0xFF, (size_t)used * 4, st));
        DAG_HIP(hipMemcpyAsync(d_order, &root, 4, hipMemcpyHostToDevice, st));
        DAG_HIP(hipMemcpyAsync(d_newid + root, &base, 4, hipMemcpyHostToDevice, st));
        uint32_t off = 0, f = 1;
        for (int l = 1; l < tr.depth && f; ++l) {
            const uint32_t nc = 8 * f, next = off + f;
            hipLaunchKernelGGL(k_bfs_first, blocks(nc), dim3(256), 0, st, S.nodes, d_order + off, f, d_first);
            hipLaunchKernelGGL(k_bfs_mark, blocks(nc), dim3(256), 0, st, S.nodes, d_order + off, f, d_first, d_mark);
            DAG_HIP(hipGetLastError());
            DAG_HIP(hipcub::DeviceScan::ExclusiveSum(d_scan, scan_bytes, d_mark, d_pos, (int)nc, st));
            hipLaunchKernelGGL(k_bfs_place, blocks(nc), dim3(256), 0, st, S.nodes, d_order + off, f, d_mark, d_pos, d_order,
                               next, d_newid, base);
            DAG_HIP(hipGetLastError());
            uint32_t tail[2];
            DAG_HIP(hipMemcpyAsync(&tail[0], d_pos + nc - 1, 4, hipMemcpyDeviceToHost, st));
            DAG_HIP(hipMemcpyAsync(&tail[1], d_mark + nc - 1, 4, hipMemcpyDeviceToHost, st));
            DAG_HIP(hipStreamSynchronize(st));
            off = next;
            f = tail[0] + tail[1];
        }
        const uint32_t n = off + f;
        hipLaunchKernelGGL(k_bfs_output, blocks((size_t)n * 8), dim3(256), 0, st, S.nodes, S.level, d_order, d_newid, n, d_out);
        DAG_HIP(hipGetLastError());
        uint32_t *nodes = static_cast<uint32_t *>(std::malloc((size_t)n * 32));
        if (!nodes) return OCH_E_NOMEM;
        if (hipMemcpyAsync(nodes, d_out, (size_t)n * 32, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            std::free(nodes);
            return OCH_E_HIP;
        }
        *out = nodes;
        *n_out = n;
        if (trace)
            std::fprintf(stderr, "[och_build] gpu renumbering %.3f s\n",
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - t_bfs).count());
#undef DAG_HIP
        if (trace) std::fprintf(stderr, "[och_build] gpu dag: %zu bricks, %u ids\n", n_work, used);
        return OCH_OK;
    };
    status = run();
    if (st) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
    }
    for (void *p : bufs) (void)hipFree(p);
    return status;
}

// Breadth-first renumbering of a node store (ids 1 .. used - 1, records of 8
// child words, level[id] = height above the voxels): level by level from the
// root, children in slot order; 1-based (h_octree, slot 0 never used) or
// 0-based octree.  *out: malloc'd n_out x 8 words (one zero node when empty).
int renumber(const uint32_t *store, const uint8_t *level, uint32_t used, uint32_t root, int depth, int base,
             uint32_t **out, uint32_t *n_out)
{
    std::vector<uint32_t> newid(used, 0);
    std::vector<uint32_t> order;
    if (root) {
        order.reserve(1024);
        std::vector<uint32_t> lv{root};
        newid[root] = (uint32_t)base;
        order.push_back(root);
        for (int l = 1; l < depth; ++l) {
            std::vector<uint32_t> nxt;
            for (uint32_t v : lv) {
                const uint32_t *c = store + (size_t)v * 8;
                for (int k = 0; k < 8; ++k)
                    if (c[k] && !(newid[c[k]] || c[k] == root)) {
                        newid[c[k]] = (uint32_t)(order.size() + base);
                        order.push_back(c[k]);
                        nxt.push_back(c[k]);
                    }
            }
            lv.swap(nxt);
        }
    }
    *n_out = (uint32_t)std::max<size_t>(order.size(), 1);
    uint32_t *nodes = static_cast<uint32_t *>(std::calloc((size_t)*n_out * 8, 4));
    if (!nodes) return OCH_E_NOMEM;
    for (size_t i = 0; i < order.size(); ++i) {
        const uint32_t v = order[i];
        const uint32_t *c = store + (size_t)v * 8;
        const bool leaf = level[v] == 0;
        for (int k = 0; k < 8; ++k) nodes[i * 8 + k] = (leaf || !c[k]) ? c[k] : newid[c[k]];
    }
    *out = nodes;
    return OCH_OK;
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
    // OCH_BUILD_TRACE=1: phase times on stderr
    const bool trace = std::getenv("OCH_BUILD_TRACE") != nullptr;
    auto phase = [&, t_last = t_start](const char *name) mutable {
        if (!trace) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[och_build] %-10s %8.3f s\n", name, std::chrono::duration<double>(now - t_last).count());
        t_last = now;
    };
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

    phase("columns");
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

    // DAG capacity: 3x the unique nodes of the default terrain (19 318 / 334 025 /
    // 4 980 409 at depth 8 / 10 / 12); the hash table is twice the capacity
    const uint32_t cap = params->dedup ? (depth <= 8 ? (1u << 20) : depth <= 10 ? (1u << 23) : (1u << 24))
                                       : (uint32_t)std::min<uint64_t>(1ull << 28, 48ull << (2 * depth));
    phase("init");
    // Bricks that reach below the highest surface of their columns.
    std::vector<uint32_t> work;
    for (int bz = 0; bz < G; ++bz)
        for (int by = 0; by < G; ++by)
            for (int bx = 0; bx < G; ++bx)
                if (bz * S <= tr.brick_hmax[(size_t)by * G + bx]) work.push_back(((uint32_t)bz * G + by) * G + bx);
    const int base = params->dedup ? 1 : 0;
    BrickStats total;
    uint32_t root = 0, n_out = 0;
    uint32_t *nodes = nullptr;
    if (params->use_gpu && params->dedup && s_log2 == kBrickLog2) {
        // the whole DAG on the GPU, renumbering included
        const int st = build_dag_gpu(tr, cap, work, G, &nodes, &n_out, root, total, trace);
        if (st != OCH_OK)
            return och::report(st, st == OCH_E_NODEV    ? "use_gpu: no HIP device"
                                   : st == OCH_E_CAPACITY ? "GPU builder: node capacity exhausted"
                                   : st == OCH_E_NOMEM    ? "GPU builder: device allocation failed"
                                                          : "GPU builder: HIP error");
        phase("gpu dag");
    } else {
        NodeStore ns;
        if (!ns.init(cap, params->dedup != 0)) {
            ns.release();
            return OCH_E_NOMEM;
        }
        std::vector<uint32_t> brick_root((size_t)G * G * G, 0);
        std::vector<BrickStats> stats(threads);
        double gpu_s = 0.0;
        if (params->use_gpu && s_log2 == kBrickLog2) {
            // an expanded tree: voxels from the GPU, one node per tree node on the host
            if (!build_bricks_gpu(tr, ns, threads, work, G, brick_root, stats, &gpu_s)) {
                ns.release();
                return och::report(OCH_E_NODEV, "use_gpu: no HIP device could run the voxel kernel");
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
        phase("bricks");
        for (auto &s : stats) {
            for (int k = 0; k < 8; ++k) total.hist[k] += s.hist[k];
            total.tree_nodes += s.tree_nodes;
        }
        // Levels above the bricks.
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
        phase("upper");
        if (ns.full.load()) {
            ns.release();
            return OCH_E_CAPACITY;
        }
        const int rs = renumber(ns.nodes, ns.level, std::min(ns.next.load(), ns.cap), root, depth, base, &nodes, &n_out);
        ns.release();
        if (rs != OCH_OK) return rs;
    }
    phase("renumber");

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
