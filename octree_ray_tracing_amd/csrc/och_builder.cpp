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
#include <sched.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
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
    int n = S / 2;
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
    // h >= 1: reduce in place ((z*n+y)*n+x indexing, n halves each level)
    for (int h = 1; h < s_log2; ++h) {
        const int m = n / 2;
        for (int z = 0; z < m; ++z)
            for (int y = 0; y < m; ++y)
                for (int x = 0; x < m; ++x) {
                    uint32_t c[8];
                    bool any = false;
                    for (int k = 0; k < 8; ++k) {
                        const int cx = 2 * x + (k & 1), cy = 2 * y + ((k >> 1) & 1), cz = 2 * z + ((k >> 2) & 1);
                        c[k] = ids[((size_t)cz * n + cy) * n + cx];
                        any |= c[k] != 0;
                    }
                    uint32_t id = 0;
                    if (any) {
                        id = ns.intern(c, h);
                        ++st.tree_nodes;
                    }
                    ids[((size_t)z * m + y) * m + x] = id;   // safe: writes trail reads
                }
        n = m;
    }
    return ids[0];
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
    {
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
