// och_internal.h -- shared between the C-ABI layer (och_api.cpp) and the
// gfx950 kernels (och_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/och_gpu.h"

namespace och {

// What a kernel needs to walk one pool: all device pointers.
// Two device layouts of the same DAG:
//   raw    -- the caller's nodes, nodes[8 * v + c] = child c of the node the
//             reference calls v (1-based pools get one zero padding node at 0);
//   packed -- re-linearised breadth-first per level; an interior slot holds
//             child_id | child_mask << 24 (child_mask = which of the child's
//             eight slots are non-empty), leaf-level slots hold voxel ids.
//             An empty child is rejected from the held mask and a POP
//             restores (node | mask << 24) from the LDS stack, so only a
//             descent or a hit touches memory.
struct DevPool {
    const uint32_t *nodes;  // raw or packed, per `packed`
    uint32_t n_slots;       // 8 x the nodes in `nodes`: the descent's buffer loads are bounds-checked against it
    const uint32_t *lut;    // RCPPS table, 1 << (23 - lut_shift) entries, each + (127 << 23) (upload_lut)
    uint32_t rcp_xlo;       // exponent bits of the smallest x the one-subtraction RCPPS serves (rcpps)
    uint32_t rcp_xspan;     // and the span of that range (0: the model for every x)
    uint32_t root;          // raw: root index; packed: root_id | root_mask << 24
    int32_t packed;
    int32_t depth;
    int32_t lut_shift;
    uint32_t miss_bits;     // hit_time bits of a miss (+INF or +0.0)
    float half_voxel;       // voxel_dim / 2 = 2^-(depth+1) (ORT/och_h_octree.h:28), bounce origins
    uint32_t dim_lo;        // child-size bit at the leaf level, 1 << (23 - depth)
    uint32_t dim_span;      // (1 << 22) - dim_lo: a walk is active while dim - dim_lo <= dim_span
    // Occupied-box cull (OCH_OPT_CULL, och_kernels.hip ray_cull): the bounding
    // box of the pool's voxels, world coordinates (1 + voxel / 2^depth).
    int32_t cull;           // 0 off, 1 launches without PUSH counts, 2 all launches
    float cull_lo[3], cull_hi[3];
    // camera_proven_miss (the cull's cheaper test before a camera ray's setup)
    // budgets the RCPPS table's relative error: 1 only when the uploaded
    // table's maximum error is within kCameraCullRcpError (och_api.cpp).
    int32_t cam_cull;
};

// Largest RCPPS-table relative error for which camera_proven_miss is sound
// (och_kernels.hip has the budget: per-axis factors within 2^-9 of 1 against
// its 2^-7 margin); x86 RCPPS is specified within 1.5 * 2^-12.
constexpr double kCameraCullRcpError = 0x1p-10;

// Bounding box of the reachable non-empty leaf voxels, voxel units, [lo, hi)
// per axis; false when there are none (och_pool_occupied_box).
bool occupied_box(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth, int base, int32_t lo[3],
                  int32_t hi[3]);

// The editor's flush (och_editor.cpp) writes a 1-based pool in three steps:
//   pool_drain       -- waits for all work on the pool's device (kernels on any
//                       stream may still be walking the slots about to change);
//   pool_write_slots -- copies slots [first, first + count) of the raw layout
//                       and, when `packed` is given, of a packed layout
//                       numbered like the raw one (id = slot; the editor keeps
//                       one level per slot and ids below 2^24).  `full`
//                       replaces the packed buffer (count must then cover
//                       slots 0..n_nodes-1 and raw/packed start at slot 0).
//                       Roots are not touched; a failed write may leave
//                       slots half written, so the flush then marks the
//                       pool torn (pool_mark_torn);
//   pool_commit      -- publishes both roots (packed == false drops the packed
//                       layout) and the editor's voxel bounding box (the cull
//                       box, OCH_OPT_CULL), and records `writer` as the pool's
//                       last writer.
// No re-validation: the editor only writes ids it handed out.
// pool_serial: a process-unique id of the pool (never reused, unlike its
// address); pool_last_writer: the editor id of the last commit, 0 after
// och_gpu_pool_create / och_gpu_pool_update / a failed write.
// report: record `msg` as och_last_error's text and return status.
int report(int status, const char *msg);

// Launch hygiene (och_kernels.hip): a launcher clears the thread's pending HIP
// error before it launches, because hipGetLastError() after the launch also
// returns an error that an earlier HIP call of the thread left behind (another
// library's -- RCCL's communicator init, say) and would fail a correct launch.
// What it clears is kept, not dropped: the first such error since the last
// reset, the C-ABI entry the thread was in (EntryScope) and the launcher, read
// by och_discarded_error.
void clear_pending_error(const char *launcher);
// The outermost C-ABI entry of this thread, by name, while it runs (OCH_ENTRY).
struct EntryScope {
    const char *prev;
    explicit EntryScope(const char *name);
    ~EntryScope();
};
#define OCH_ENTRY() const och::EntryScope och_entry_scope_(__func__)

int pool_drain(och_gpu_pool *pool);
int pool_write_slots(och_gpu_pool *pool, uint32_t first, uint32_t count, const uint32_t *raw,
                     const uint32_t *packed, bool full);
// box: the editor's bounding box of its voxels (a superset is fine), or
// nullptr when it holds none.
int pool_commit(och_gpu_pool *pool, uint32_t root, uint32_t packed_root, bool packed, uint64_t writer,
                const int32_t *box_lo, const int32_t *box_hi);
// After a failed pool_write_slots / pool_scatter_slots: the slots may be half
// written (a freed-and-reused slot rewritten in place, or the packed buffer
// reallocated before its copy failed).  Drops the packed layout, sets root 0,
// clears the cull box and marks the pool torn: trace / render launches and
// och_gpu_pool_update refuse it until a pool_commit (a successful flush).
int pool_mark_torn(och_gpu_pool *pool);
// pool_write_slots for scattered slots: ids[count] (1..n_nodes-1, distinct),
// raw / packed = count x 8 words; one staged copy and one scatter kernel,
// complete on return.
int pool_scatter_slots(och_gpu_pool *pool, const uint32_t *ids, uint32_t count, const uint32_t *raw,
                       const uint32_t *packed);
hipError_t launch_scatter_slots(const uint32_t *ids, const uint32_t *raw, const uint32_t *packed, uint32_t count,
                                uint32_t *d_raw, uint32_t *d_packed, hipStream_t stream);
uint64_t pool_serial(const och_gpu_pool *pool);
// The stream the pool enqueues on (hipStream_t) and its palette size
// (och_group.cpp drives several pools from one thread).
void *pool_stream(const och_gpu_pool *pool);
int pool_palette_size(const och_gpu_pool *pool, int *n_voxels);
uint64_t pool_last_writer(const och_gpu_pool *pool);

// The library's RCCL communicator (och_comm.cpp), for the sharded frame loop
// in och_api.cpp.  comm_all_gather: recv = [n_ranks][bytes]; comm_gather:
// only rank `root` receives (recv may be null elsewhere).  Both enqueue on
// `stream`; the caller has the communicator's device current.
int comm_ranks(const och_comm *comm, int *n_ranks, int *rank, int *device);
int comm_all_gather(och_comm *comm, const void *send, void *recv, size_t bytes, hipStream_t stream);
int comm_gather(och_comm *comm, const void *send, void *recv, size_t bytes, int root, hipStream_t stream);
// ncclCommAbort after a failure that followed an issued collective; the
// communicator then reports itself destroyed.
void comm_abort(och_comm *comm);

struct DevFrame {
    och_camera cams[OCH_MAX_VIEWS];   // equal width / height
    int32_t n_views;
    const uint32_t *palette;  // 6 * n_voxels RGBA8
    uint32_t n_voxels;
    uint32_t *out;            // n_views compact slices, each slice_rows x width (RGBA8)
    uint8_t *codes;           // or the same slices as indexed colour (launch_render_codes)
    int32_t row_chunk, shard, n_shards, slice_rows;
    const int32_t *chunk_map; // row deal: this shard's global chunk per local chunk (-1 = padding), or null
};

// Threads per workgroup of the config-5 (bounce) kernels: compaction spans
// the block's 4 waves.
constexpr int kBounceBlock = 256;

// How trace/render launches are scheduled (och_gpu_set_option).
struct Schedule {
    int block;              // threads per workgroup (multiple of 64)
    int tile_order;         // camera rays: 0 row-major 8x8 tiles, 1 supertiles grouped per XCD, 2 planned order
    int bounce_compact;     // config 5: compact the block's secondary rays into its first lanes
    uint64_t *stamps;       // optional per-wave residency records
    uint32_t stamp_cap;
    const uint32_t *order;  // optional workgroup permutation (och_gpu_plan_views)
    uint32_t order_n;       // entries in *order: a launch whose grid differs runs in natural order
    uint32_t *cost;         // optional per-workgroup duration output (the planning launch)
    // A split plan (OCH_OPT_SPLIT; camera renders, packed layout, block 64):
    // order lists the grid's workgroups with the heavy tiles replaced by split
    // waves (1 << 31 | row of split_tasks), order_n = grid + split_extra;
    // split_tasks rows: the tile, then 64 lane tasks (och_kernels.hip
    // split_tile).  split_tasks = null: no split.
    const uint32_t *split_tasks;
    uint32_t split_level;
    uint32_t split_extra;
    hipEvent_t ev_start;    // optional: recorded by the traversal kernel's own dispatch (hipExtLaunchKernel)
    hipEvent_t ev_stop;
};

hipError_t launch_trace_batch(const DevPool &p, const float *origin, int origin_stride, const float *dirs,
                              uint32_t n, int32_t *hit_dir, uint32_t *hit_voxel, uint32_t *hit_time,
                              uint32_t *push_count, const Schedule &sc, hipStream_t stream);
// The same rays as a row-major image `width` rays wide, one 8x8 tile per
// wave (TiledArraySource); records in the caller's order.
hipError_t launch_trace_batch_tiled(const DevPool &p, const float *origin, int origin_stride, const float *dirs,
                                    uint32_t n, uint32_t width, int32_t *hit_dir, uint32_t *hit_voxel,
                                    uint32_t *hit_time, uint32_t *push_count, const Schedule &sc, hipStream_t stream);
// hipOccupancyMaxActiveBlocksPerMultiprocessor of kind 0 render grid or
// 2 trace grid, at this block size and stack depth.
hipError_t occupancy_blocks_per_cu(int kind, int block, int depth, int *blocks);
// Config 5: primary ray, then one mirrored secondary ray per hit (see
// bounce_ray in och_kernels.hip); secondary records get direction -1 when the
// primary ray did not hit.
hipError_t launch_trace_bounce_batch(const DevPool &p, const float *origin, int origin_stride, const float *dirs,
                                     uint32_t n, int32_t *hit_dir, uint32_t *hit_voxel, uint32_t *hit_time,
                                     int32_t *bounce_dir, uint32_t *bounce_voxel, uint32_t *bounce_time,
                                     uint32_t *push_count, const Schedule &sc, hipStream_t stream);
hipError_t launch_render_bounce(const DevPool &p, const DevFrame &f, const Schedule &sc, hipStream_t stream);
hipError_t launch_raygen(const och_camera &cam, float *dirs, hipStream_t stream);
hipError_t launch_render(const DevPool &p, const DevFrame &f, const Schedule &sc, hipStream_t stream);
// The split planner's counting render: each pixel's walked PUSH count (16 bits)
// into push, indexed as the frame's slices.
hipError_t launch_render_push(const DevPool &p, const DevFrame &f, const Schedule &sc, uint16_t *push, hipStream_t stream);
// Indexed-colour frames (OCH_CODE_*): render into f.codes, and turn gathered
// code slices into RGBA8 frames through a 256-entry table.
hipError_t launch_render_codes(const DevPool &p, const DevFrame &f, const Schedule &sc, bool bounce, hipStream_t stream);
// owner: the row deal's table (global chunk -> shard << 16 | local chunk), or
// null for round-robin chunks.
hipError_t launch_shade_unshard(const uint8_t *gathered, uint32_t *frames, const uint32_t *table, int width, int height,
                                int row_chunk, int n_shards, int slice_rows, int n_views, const int32_t *owner,
                                hipStream_t stream);
hipError_t launch_unshard(const uint32_t *gathered, uint32_t *frames, int width, int height, int row_chunk,
                          int n_shards, int slice_rows, int n_views, const int32_t *owner, hipStream_t stream);

}  // namespace och
