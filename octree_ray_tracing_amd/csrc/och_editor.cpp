// Host-side DAG editor: h_octree::set / at (ORT/och_h_octree.h:176-258) over a
// compact, capacity-bounded slot pool that a device pool mirrors slot for slot.
//
// The reference edits its node_hashtable in place: set() walks root -> voxel,
// then path-copies bottom-up, remove_node()-ing each old path node and
// register_node()-ing the new one (hash-consed, refcounted; :110-174).  Slot
// placement follows the FNV hash, so an edit touches slots scattered over the
// whole 2^L table.  Here a node keeps its slot until it dies, new nodes take
// the lowest free slots, and every written slot is recorded, so
// och_editor_flush re-uploads only the dirty slots (staged in one copy and
// scattered by one kernel, och::pool_scatter_slots) instead of the pool.
//
// Differences from the reference that do not change any traced record (the
// tracer reads children only, never slot positions or counts):
//  * nodes are interned per level (content + level key), so refcounts are
//    exact parent counts and a dead node releases its children recursively;
//    the reference's per-registration counts (:144, :166) never release a
//    dead node's children and can share one slot between levels.
//  * a full pool is reported (OCH_E_CAPACITY) before the edit starts and the
//    tree is left unchanged; the reference exit(0)s mid-edit (:112-116).
#include "och_internal.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <new>
#include <unordered_map>
#include <vector>

namespace {

inline int child_of(int x, int y, int z, int level)   // z_encode_16 digit, ORT/och_z_order.cpp
{
    return ((x >> level) & 1) | (((y >> level) & 1) << 1) | (((z >> level) & 1) << 2);
}

}  // namespace

struct och_editor {
    int depth = 0;
    uint32_t capacity = 0;                // slots 1..capacity
    uint32_t root = 0;
    uint32_t next_unused = 1;             // slots >= next_unused were never handed out
    uint32_t live = 0;
    std::vector<uint32_t> nodes;          // capacity x 8, slot s at (s-1)*8
    // The kernels' packed layout numbered like the slots ((capacity+1) x 8, slot
    // s at s*8, 0 = padding): interior words child | child_mask << 24.  A node
    // is immutable while it lives, so its word is written once, at intern.
    std::vector<uint32_t> packed;
    bool packed_ok = false;               // capacity < 2^24
    uint64_t id = 0;                      // process-unique editor id (the pools' last_writer)
    uint64_t synced = 0;                  // och::pool_serial of the pool the last flush wrote
    std::vector<uint32_t> refs;           // parent count (+1 for the root)
    std::vector<uint8_t> level;
    std::vector<uint32_t> free_slots;
    // Hash-cons index (the reference's node_hashtable role, :70-83, :110-160):
    // open addressing over slot ids (0 = empty, kTomb = removed), keyed by the
    // slot's 8 words + level and compared in place in `nodes`.
    static constexpr uint32_t kTomb = UINT32_MAX;
    std::vector<uint32_t> table;
    size_t table_mask = 0;
    size_t table_used = 0;                // entries + tombstones
    std::vector<uint32_t> dirty;          // slots written since the last flush (repeats allowed)
    bool root_dirty = false;
    // A bounding box of the voxels (voxel units, [lo, hi)), handed to the pool
    // at flush for its cull (OCH_OPT_CULL): exact after adoption, grown by
    // every set() of a voxel, never shrunk by a removal (a superset is valid).
    bool box_any = false;
    int32_t box_lo[3] = {0, 0, 0}, box_hi[3] = {0, 0, 0};
    void box_add(int x, int y, int z)
    {
        const int32_t v[3] = {x, y, z};
        for (int a = 0; a < 3; ++a) {
            box_lo[a] = box_any ? std::min(box_lo[a], v[a]) : v[a];
            box_hi[a] = box_any ? std::max(box_hi[a], v[a] + 1) : v[a] + 1;
        }
        box_any = true;
    }

    uint32_t *slot(uint32_t s) { return nodes.data() + (size_t)(s - 1) * 8; }
    const uint32_t *slot(uint32_t s) const { return nodes.data() + (size_t)(s - 1) * 8; }
    void mark(uint32_t s) { dirty.push_back(s); }
    uint32_t mask_of(uint32_t s) const
    {
        uint32_t m = 0;
        for (int c = 0; c < 8; ++c) m |= (uint32_t)(slot(s)[c] != 0) << c;
        return m;
    }
    uint32_t packed_root() const { return root ? root | mask_of(root) << 24 : 0; }
    static size_t hash_of(const uint32_t *n, int lvl)
    {
        uint64_t h = 0x9E3779B97F4A7C15ull * (uint64_t)(lvl + 1);
        for (int c = 0; c < 8; ++c) {
            h = (h ^ n[c]) * 0xFF51AFD7ED558CCDull;
            h ^= h >> 29;
        }
        return (size_t)h;
    }
    // The slot holding (n, lvl), or 0 with *ins = where to insert it.
    uint32_t lookup(const uint32_t *n, int lvl, size_t *ins) const
    {
        size_t i = hash_of(n, lvl) & table_mask, tomb = SIZE_MAX;
        for (;; i = (i + 1) & table_mask) {
            const uint32_t e = table[i];
            if (e == 0) {
                *ins = tomb != SIZE_MAX ? tomb : i;
                return 0;
            }
            if (e == kTomb) {
                if (tomb == SIZE_MAX) tomb = i;
            } else if (level[e] == lvl && !std::memcmp(slot(e), n, 32)) {
                return e;
            }
        }
    }
    void unindex(uint32_t s)              // while the slot still holds its node
    {
        size_t i = hash_of(slot(s), level[s]) & table_mask;
        while (table[i] != s) i = (i + 1) & table_mask;
        table[i] = kTomb;
    }
    // Rebuild without tombstones from the live slots (refs > 0 between edits).
    void reindex()
    {
        std::fill(table.begin(), table.end(), 0u);
        table_used = 0;
        for (uint32_t s = 1; s < next_unused; ++s) {
            if (!refs[s]) continue;
            size_t ins;
            lookup(slot(s), level[s], &ins);
            table[ins] = s;
            ++table_used;
        }
    }
    uint32_t headroom() const { return (uint32_t)free_slots.size() + (capacity + 1 - next_unused); }

    // register_node (:110-160): find the node or give it a slot; a new node
    // takes one reference on each of its children.
    uint32_t intern(const uint32_t *n, int lvl)
    {
        size_t ins;
        if (const uint32_t found = lookup(n, lvl, &ins)) return found;
        uint32_t s;
        if (!free_slots.empty()) {
            s = free_slots.back();
            free_slots.pop_back();
        } else {
            s = next_unused++;
        }
        std::memcpy(slot(s), n, 32);
        if (packed_ok)
            for (int c = 0; c < 8; ++c)
                packed[(size_t)s * 8 + c] = lvl > 0 && n[c] ? n[c] | mask_of(n[c]) << 24 : n[c];
        refs[s] = 0;
        level[s] = (uint8_t)lvl;
        if (table[ins] == 0) ++table_used;
        table[ins] = s;
        ++live;
        mark(s);
        if (lvl > 0)
            for (int c = 0; c < 8; ++c)
                if (n[c]) ++refs[n[c]];
        return s;
    }

    // remove_node (:162-174), completed: a dead node is unindexed, zeroed and
    // releases its children.
    void release(uint32_t s)
    {
        if (--refs[s]) return;
        unindex(s);
        const int lvl = level[s];
        uint32_t n[8];
        std::memcpy(n, slot(s), 32);
        std::memset(slot(s), 0, 32);
        if (packed_ok) std::memset(packed.data() + (size_t)s * 8, 0, 32);
        free_slots.push_back(s);
        --live;
        mark(s);
        if (lvl > 0)
            for (int c = 0; c < 8; ++c)
                if (n[c]) release(n[c]);
    }

    // Renumber the live slots breadth-first from the root (levels contiguous,
    // siblings adjacent): the builder's order, which the traversal's cache
    // locality depends on.  Adoption hands out slots in post-order.
    void renumber_breadth_first()
    {
        if (!root) return;
        std::vector<uint32_t> order{root};
        std::vector<uint32_t> to(capacity + 1, 0);
        to[root] = 1;
        for (size_t q = 0; q < order.size(); ++q) {
            const uint32_t s = order[q];
            if (level[s] == 0) continue;
            for (int c = 0; c < 8; ++c) {
                const uint32_t ch = slot(s)[c];
                if (ch && !to[ch]) {
                    to[ch] = (uint32_t)order.size() + 1;
                    order.push_back(ch);
                }
            }
        }
        std::vector<uint32_t> nn((size_t)capacity * 8, 0u), nr(capacity + 1, 0u);
        std::vector<uint8_t> nl(capacity + 1, 0);
        for (size_t q = 0; q < order.size(); ++q) {
            const uint32_t s = order[q], d = (uint32_t)q + 1;
            uint32_t *o = nn.data() + (size_t)q * 8;
            for (int c = 0; c < 8; ++c) {
                const uint32_t ch = slot(s)[c];
                o[c] = level[s] > 0 && ch ? to[ch] : ch;
            }
            nr[d] = refs[s];
            nl[d] = level[s];
        }
        nodes.swap(nn);
        refs.swap(nr);
        level.swap(nl);
        free_slots.clear();
        next_unused = (uint32_t)order.size() + 1;
        live = (uint32_t)order.size();
        root = 1;
        reindex();
        if (packed_ok) std::fill(packed.begin(), packed.end(), 0u);
        for (uint32_t d = 1; d < next_unused; ++d) {
            if (packed_ok)
                for (int c = 0; c < 8; ++c) {
                    const uint32_t ch = slot(d)[c];
                    packed[(size_t)d * 8 + c] = level[d] > 0 && ch ? ch | mask_of(ch) << 24 : ch;
                }
        }
        dirty.clear();
    }

    // Adoption of a pool that is already a canonical DAG -- every reachable node
    // at one level only, no two equal (content, level), none empty -- such as
    // och_build_terrain's: the result of adopt() + renumber_breadth_first() is
    // then the input renumbered breadth-first, built here in O(n) without the
    // recursive walk.  False (editor untouched) when the input is not canonical
    // or does not fit; the caller then takes the general path.
    bool adopt_canonical(const uint32_t *in, uint32_t n_in, uint32_t in_root)
    {
        if (in_root == 0 || in_root > n_in) return false;
        std::vector<uint32_t> to((size_t)n_in + 1, 0), order{in_root};
        std::vector<uint8_t> lv((size_t)n_in + 1, 0);
        to[in_root] = 1;
        lv[in_root] = (uint8_t)(depth - 1);
        for (size_t q = 0; q < order.size(); ++q) {
            const uint32_t v = order[q];
            const int l = lv[v];
            const uint32_t *c = in + (size_t)(v - 1) * 8;
            bool zero = true;
            for (int k = 0; k < 8; ++k) zero &= c[k] == 0;
            if (zero) return false;
            if (l == 0) continue;
            for (int k = 0; k < 8; ++k) {
                const uint32_t ch = c[k];
                if (!ch) continue;
                if (ch > n_in) return false;
                if (to[ch]) {
                    if (lv[ch] != l - 1) return false;   // one slot at two levels
                    continue;
                }
                if (order.size() >= capacity) return false;
                to[ch] = (uint32_t)order.size() + 1;
                lv[ch] = (uint8_t)(l - 1);
                order.push_back(ch);
            }
        }
        const uint32_t n = (uint32_t)order.size();
        for (uint32_t q = 0; q < n; ++q) {
            const uint32_t v = order[q], d = q + 1;
            const uint32_t *c = in + (size_t)(v - 1) * 8;
            uint32_t *o = slot(d);
            for (int k = 0; k < 8; ++k) o[k] = lv[v] > 0 && c[k] ? to[c[k]] : c[k];
            level[d] = lv[v];
        }
        // the index, and the uniqueness check: an equal node already indexed
        // means the input is not canonical
        for (uint32_t d = 1; d <= n; ++d) {
            size_t ins;
            if (lookup(slot(d), level[d], &ins)) {
                std::fill(table.begin(), table.end(), 0u);
                std::fill(nodes.begin(), nodes.begin() + (size_t)n * 8, 0u);
                std::fill(level.begin(), level.begin() + n + 1, 0);
                return false;
            }
            table[ins] = d;
        }
        table_used = n;
        for (uint32_t d = 1; d <= n; ++d)
            if (level[d] > 0)
                for (int k = 0; k < 8; ++k)
                    if (slot(d)[k]) ++refs[slot(d)[k]];
        root = 1;
        ++refs[1];
        next_unused = n + 1;
        live = n;
        if (packed_ok)
            for (uint32_t d = 1; d <= n; ++d)
                for (int c = 0; c < 8; ++c) {
                    const uint32_t ch = slot(d)[c];
                    packed[(size_t)d * 8 + c] = level[d] > 0 && ch ? ch | mask_of(ch) << 24 : ch;
                }
        dirty.clear();
        return true;
    }

    // Copy an input pool in, level by level; memo maps (input id, level) to slots.
    int adopt(const uint32_t *in, uint32_t n_in, uint32_t id, int lvl,
              std::unordered_map<uint64_t, uint32_t> &memo, uint32_t *out)
    {
        if (id == 0 || id > n_in) return OCH_E_INVALID;
        auto it = memo.find((uint64_t)id << 8 | (uint64_t)lvl);
        if (it != memo.end()) {
            *out = it->second;
            return OCH_OK;
        }
        uint32_t n[8];
        std::memcpy(n, in + (size_t)(id - 1) * 8, 32);
        if (lvl > 0)
            for (int c = 0; c < 8; ++c)
                if (n[c]) {
                    const int st = adopt(in, n_in, n[c], lvl - 1, memo, &n[c]);
                    if (st != OCH_OK) return st;
                }
        bool zero = true;
        for (int c = 0; c < 8; ++c) zero &= n[c] == 0;
        if (zero) return OCH_E_INVALID;   // an empty node is never registered (:226-229)
        if (headroom() == 0) return OCH_E_CAPACITY;
        *out = intern(n, lvl);
        memo.emplace((uint64_t)id << 8 | (uint64_t)lvl, *out);
        return OCH_OK;
    }
};

extern "C" {

OCH_API int och_editor_create(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth, uint32_t capacity,
                              och_editor **out)
{
    if (!out || (n_nodes && !nodes) || depth < 1 || depth > 16 || capacity == 0 || capacity > (1u << 28))
        return och::report(OCH_E_INVALID, "och_editor_create: bad argument (depth 1..16, capacity 1..2^28)");
    *out = nullptr;
    och_editor *e = new (std::nothrow) och_editor;
    if (!e) return och::report(OCH_E_NOMEM, "och_editor_create: out of host memory");
    static std::atomic<uint64_t> next_id{1};
    e->id = next_id.fetch_add(1);
    try {
        e->depth = depth;
        e->capacity = capacity;
        e->nodes.assign((size_t)capacity * 8, 0u);
        e->packed_ok = capacity < (1u << 24);
        if (e->packed_ok) e->packed.assign((size_t)(capacity + 1) * 8, 0u);
        e->refs.assign((size_t)capacity + 1, 0u);
        e->level.assign((size_t)capacity + 1, 0);
        size_t tsize = 64;
        while (tsize < 2 * (size_t)capacity) tsize <<= 1;
        e->table.assign(tsize, 0u);
        e->table_mask = tsize - 1;
    } catch (const std::bad_alloc &) {
        delete e;
        return och::report(OCH_E_NOMEM, "och_editor_create: out of host memory");
    }
    if (root && !e->adopt_canonical(nodes, n_nodes, root)) {
        std::unordered_map<uint64_t, uint32_t> memo;
        const int st = e->adopt(nodes, n_nodes, root, depth - 1, memo, &e->root);
        if (st != OCH_OK) {
            delete e;
            return och::report(st, st == OCH_E_CAPACITY ? "och_editor_create: the pool does not fit in capacity slots"
                                                        : "och_editor_create: a child names a slot outside the pool "
                                                          "or an empty node");
        }
        ++e->refs[e->root];
        e->renumber_breadth_first();
    }
    e->root_dirty = true;
    e->box_any = och::occupied_box(e->nodes.data(), e->capacity, e->root, depth, 1, e->box_lo, e->box_hi);
    *out = e;
    return OCH_OK;
}

OCH_API int och_editor_destroy(och_editor *e)
{
    delete e;
    return OCH_OK;
}

OCH_API int och_editor_set(och_editor *e, int xi, int yi, int zi, uint32_t v)
{
    if (!e) return OCH_E_INVALID;
    const int dim = 1 << e->depth;
    if (xi < 0 || yi < 0 || zi < 0 || xi >= dim || yi >= dim || zi >= dim) return OCH_OK;   // :180 ignores
    if (e->headroom() < (uint32_t)e->depth)
        return och::report(OCH_E_CAPACITY, "och_editor_set: fewer free slots than depth (tree unchanged)");
    if (e->table_used + (size_t)e->depth > (e->table_mask + 1) / 4 * 3) e->reindex();   // tombstones
    uint32_t path[32];
    uint32_t cur = e->root;
    for (int l = e->depth - 1; l >= 0; --l) {
        path[l] = cur;
        cur = cur ? e->slot(cur)[child_of(xi, yi, zi, l)] : 0;
    }
    if (cur == v) return OCH_OK;   // unchanged voxel: the path re-registers to itself
    if (v) e->box_add(xi, yi, zi);
    uint32_t child = v;
    for (int l = 0; l < e->depth; ++l) {
        uint32_t n[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (path[l]) std::memcpy(n, e->slot(path[l]), 32);
        n[child_of(xi, yi, zi, l)] = child;
        bool zero = true;
        for (int c = 0; c < 8; ++c) zero &= n[c] == 0;
        child = zero ? 0 : e->intern(n, l);
    }
    if (child) ++e->refs[child];
    if (e->root) e->release(e->root);
    e->root = child;
    e->root_dirty = true;
    return OCH_OK;
}

OCH_API uint32_t och_editor_at(const och_editor *e, int x, int y, int z)
{
    if (!e || !e->root) return 0;
    uint32_t cur = e->root;
    for (int l = e->depth - 1; l >= 0; --l) {
        const uint32_t nx = e->slot(cur)[child_of(x, y, z, l)];
        if (l == 0 || !nx) return nx;
        cur = nx;
    }
    return 0;
}

OCH_API int och_editor_info(const och_editor *e, och_editor_stats *info)
{
    if (!e || !info) return OCH_E_INVALID;
    info->capacity = e->capacity;
    info->live_nodes = e->live;
    info->high_water = e->next_unused - 1;
    info->root = e->root;
    info->depth = e->depth;
    std::vector<uint32_t> d(e->dirty);
    std::sort(d.begin(), d.end());
    d.erase(std::unique(d.begin(), d.end()), d.end());
    info->dirty_first = d.empty() ? 0 : d.front();
    info->dirty_count = (uint32_t)d.size();
    return OCH_OK;
}

OCH_API int och_editor_nodes(const och_editor *e, const uint32_t **nodes, uint32_t *n_slots, uint32_t *root)
{
    if (!e || !nodes || !n_slots || !root) return OCH_E_INVALID;
    *nodes = e->nodes.data();
    *n_slots = e->capacity;
    *root = e->root;
    return OCH_OK;
}

OCH_API int och_editor_flush(och_editor *e, och_gpu_pool *pool)
{
    OCH_ENTRY();
    if (!e || !pool) return OCH_E_INVALID;
    och_pool_info pi;
    int st = och_gpu_pool_info(pool, &pi);
    if (st != OCH_OK) return st;
    if (pi.index_base != 1 || pi.depth != e->depth || pi.n_nodes != e->capacity + 1)
        return och::report(OCH_E_INVALID, "och_editor_flush: the pool was not made from this editor's slots");
    const uint32_t *pk = e->packed_ok ? e->packed.data() : nullptr;
    // Windowed only when this pool holds exactly what this editor's last flush
    // wrote: same pool (by serial -- a new pool can reuse a freed address) and
    // nobody (another editor, och_gpu_pool_update) wrote it since.
    const bool windowed = e->synced == och::pool_serial(pool) && och::pool_last_writer(pool) == e->id;
    if (windowed && e->dirty.empty() && !e->root_dirty) return OCH_OK;
    st = och::pool_drain(pool);
    const bool drained = st == OCH_OK;
    if (st == OCH_OK && !windowed) {
        // both layouts whole, packed in slot numbering
        std::vector<uint32_t> raw((size_t)(e->capacity + 1) * 8, 0u);
        std::memcpy(raw.data() + 8, e->nodes.data(), e->nodes.size() * 4);
        st = och::pool_write_slots(pool, 0, e->capacity + 1, raw.data(), pk, true);
    } else if (st == OCH_OK) {
        // the dirty slots, staged in one buffer and scattered by one kernel
        std::sort(e->dirty.begin(), e->dirty.end());
        e->dirty.erase(std::unique(e->dirty.begin(), e->dirty.end()), e->dirty.end());
        const uint32_t n = (uint32_t)e->dirty.size();
        std::vector<uint32_t> raw((size_t)n * 8), packed(pk ? (size_t)n * 8 : 0);
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t sl = e->dirty[i];
            std::memcpy(raw.data() + (size_t)i * 8, e->slot(sl), 32);
            if (pk) std::memcpy(packed.data() + (size_t)i * 8, pk + (size_t)sl * 8, 32);
        }
        st = och::pool_scatter_slots(pool, e->dirty.data(), n, raw.data(), pk ? packed.data() : nullptr);
    }
    // The roots go out last, once every slot they reach is on the device.
    if (st == OCH_OK)
        st = och::pool_commit(pool, e->root, e->packed_root(), pk != nullptr, e->id, e->box_any ? e->box_lo : nullptr,
                              e->box_any ? e->box_hi : nullptr);
    if (st != OCH_OK) {
        e->synced = 0;   // the next flush rewrites the pool whole
        // slots may be half written: no launch may walk the pool until then
        if (drained) (void)och::pool_mark_torn(pool);
        return st;
    }
    e->synced = och::pool_serial(pool);
    e->dirty.clear();
    e->root_dirty = false;
    return OCH_OK;
}

}  // extern "C"
