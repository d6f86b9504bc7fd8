/*
 * och_gpu.h -- C ABI of the MI355X (gfx950) sparse-voxel-octree ray caster.
 *
 * Drop-in boundary for the reference's hot path (ORT/ = Octree_Ray_Tracing/):
 *
 *   void h_octree<L,D>::sse_trace(float ox, float oy, float oz,
 *                                 float dx, float dy, float dz,
 *                                 och::direction& hit_direction,
 *                                 uint32_t& hit_voxel, float& hit_time) const;
 *                                                   ORT/och_h_octree.h:292, :449
 *   void octree::sse_trace(...)                     ORT/och_octree.h:56-58, ORT/och_octree.cpp:167
 *   tree_camera::update_position()  (ray generator) ORT/test_och_h_octree.cpp:87-138
 *   tree_window::update_image() + trace_pixel()     ORT/test_och_h_octree.cpp:437-457, :64-85
 *
 * Every entry point returns an och_status (0 = OK).  Host buffers belong to
 * the caller; device memory belongs to the pool.  Functions suffixed _dev take
 * device pointers and enqueue on the pool's HIP stream without synchronising.
 * Results are bit-identical to the reference CPU tracer run with the same
 * RCPPS table (och_gpu_set_rcp_lut / och_host_rcp_lut).
 */
#ifndef OCH_GPU_H
#define OCH_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OCH_GPU_ABI_VERSION 1
#define OCH_MAX_VIEWS 8

#if defined(__GNUC__)
#define OCH_API __attribute__((visibility("default")))
#else
#define OCH_API
#endif

typedef enum och_status {
    OCH_OK = 0,
    OCH_E_INVALID = -1,     /* bad argument / precondition */
    OCH_E_HIP = -2,         /* HIP runtime error (see och_last_error) */
    OCH_E_NODEV = -3,       /* no gfx950 device visible */
    OCH_E_RCP_MODEL = -4,   /* host RCPPS is not representable as a mantissa table */
    OCH_E_NOMEM = -5,
    OCH_E_CAPACITY = -6     /* builder: node table full (reference: exit(0), ORT/och_h_octree.h:112-116) */
} och_status;

/* och::direction, ORT/och_tree_helper.h:7-18: the ray-travel sign on the
 * axis whose face was crossed last; exit = miss, inside = origin in a voxel. */
typedef enum och_direction {
    OCH_X_POS = 0, OCH_Y_POS = 1, OCH_Z_POS = 2,
    OCH_X_NEG = 3, OCH_Y_NEG = 4, OCH_Z_NEG = 5,
    OCH_EXIT = 6, OCH_INSIDE = 7, OCH_ERROR = 8
} och_direction;

/* Indexed-colour frame codes (1 byte per pixel, the multi-GPU exchange format
 * of och_gpu_render_codes_views_dev): 6 * (voxel - 1) + direction for a hit
 * face with a palette entry, the three fixed colours of trace_pixel
 * (ORT/test_och_h_octree.cpp:76-84, magenta for an id without a palette
 * entry), | OCH_CODE_BLOCKED when a config-5 secondary ray was blocked.
 * Needs a palette of at most OCH_CODE_MAX_VOXELS voxel ids. */
#define OCH_CODE_MAGENTA 125
#define OCH_CODE_INSIDE 126
#define OCH_CODE_SKY 127
#define OCH_CODE_BLOCKED 128
#define OCH_CODE_MAX_VOXELS 20

typedef struct och_gpu_pool och_gpu_pool;

/* Camera uniforms of tree_camera::update_position (ORT/test_och_h_octree.cpp:87-115),
 * computed ONCE per frame on the host (sinf/cosf/tanf of this host's libm)
 * by och_camera_setup; the per-pixel part runs on the GPU. */
typedef struct och_camera {
    float pos[3];        /* ray origin, tree occupies [1,2)^3 (ORT/test_och_h_octree.cpp:55) */
    float rot[9];        /* t_x_fx, t_x_fy, t_x_fz, t_y_fx, ..., t_z_fz (:107-115) */
    float fov_factor;    /* 1 / tanf(fov / 2) (:97) */
    float aspect;        /* (float)W / (float)H (:89) */
    float view_x;        /* 2.0F / (float)W (:91) */
    float view_y;        /* 2.0F / (float)H (:93) */
    int32_t width, height;
} och_camera;

typedef struct och_pool_info {
    uint64_t device_bytes;   /* node pool bytes resident in HBM */
    uint32_t n_nodes;        /* nodes uploaded (incl. the padding slot of 1-based pools) */
    uint32_t root;
    int32_t depth;
    int32_t index_base;
    float miss_t;
    int32_t rcp_log2_entries;
    int32_t device;
} och_pool_info;

/* ------------------------------------------------------------ runtime */
OCH_API int och_abi_version(void);
OCH_API const char *och_last_error(void);      /* thread-local message of the last failure */
/* Every kernel launch first clears its thread's pending HIP error: one left by
 * an earlier HIP call of the thread (another library's, e.g. RCCL's
 * communicator init) would otherwise be reported as the launch's own.  The
 * error is kept, not dropped: the first one cleared since the last reset, in
 * any thread -- its hipError_t in *hip_error (0 = none), the number cleared in
 * *count, and into what (what_cap bytes, may be NULL) its name and the C-ABI
 * entry and launcher that found it.  reset != 0 clears the record after
 * reading.  Any argument may be NULL. */
OCH_API int och_discarded_error(int *hip_error, int *count, char *what, size_t what_cap, int reset);
OCH_API int och_device_count(int *count);       /* visible gfx950 devices */
/* HIP indices of the visible gfx950 devices, in HIP order: up to capacity of
 * them into devices[], their total into *count. */
OCH_API int och_device_list(int *devices, int capacity, int *count);

/* ------------------------------------------------------------ RCPPS model */
/* Capture this host CPU's _mm_rcp_ps (the reference's reciprocal,
 * ORT/och_h_octree.h:316) as a 2^k table over the mantissa of inputs in [-2,-1),
 * after checking that the result depends only on the top k mantissa bits and
 * that other exponents shift the result exponent.  lut must hold 1<<23 entries
 * (worst case); *log2_entries receives k.  Returns OCH_E_RCP_MODEL if the host
 * instruction does not follow the model (then pass an explicit table). */
OCH_API int och_host_rcp_lut(uint32_t *lut, int *log2_entries);
/* Same model evaluated on the host, for a single input bit pattern. */
OCH_API uint32_t och_rcp_from_lut(uint32_t xbits, const uint32_t *lut, int log2_entries);
/* Largest relative error |r * x - 1| of a table over x in [-2, -1).  A pool
 * whose table exceeds 2^-10 (x86 RCPPS: within 1.5 * 2^-12) does not use the
 * cull's approximate camera test, only its exact per-ray test (OCH_OPT_CULL),
 * so records stay the reference's under any table. */
OCH_API int och_rcp_lut_error(const uint32_t *lut, int log2_entries, double *max_rel_error);

/* ------------------------------------------------------------ node pools */
/* Upload a node pool.  nodes = n_nodes x 8 uint32 child slots exactly as the
 * reference lays them out (ORT/och_h_octree.h:38-40): interior slots hold node
 * indices, the leaf level holds voxel ids, 0 = empty.
 *   index_base 1: h_octree -- indices are 1-based into nodes[] (the
 *                 reference's table->nodes with root_idx, ORT/och_h_octree.h:93-95);
 *   index_base 0: octree   -- 0-based, root = 0 (ORT/och_octree.cpp:207).
 * miss_t: hit_time reported for a miss (+INF for h_octree, :429; 0.0F for
 * octree, ORT/och_octree.cpp:302).  depth = number of levels (1..22).
 * The pool starts with this host's RCPPS table (och_host_rcp_lut); override
 * with och_gpu_set_rcp_lut.  device < 0 selects the current HIP device. */
OCH_API int och_gpu_pool_create(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth,
                                int index_base, float miss_t, int device, och_gpu_pool **out);
OCH_API int och_gpu_pool_destroy(och_gpu_pool *pool);
OCH_API int och_gpu_pool_info(const och_gpu_pool *pool, och_pool_info *info);
/* Re-upload nodes [first, first+count) (pool numbering) and set a new root --
 * mirrors h_octree::set's path copy (ORT/och_h_octree.h:176-237) after an edit. */
OCH_API int och_gpu_pool_update(och_gpu_pool *pool, uint32_t first, uint32_t count,
                                const uint32_t *nodes, uint32_t root);
OCH_API int och_gpu_set_rcp_lut(och_gpu_pool *pool, const uint32_t *lut, int log2_entries);
/* Palette: n_voxels x 6 RGBA8 colours (olc::Pixel layout, r in the low byte),
 * ordered x_pos..z_neg per voxel id 1..n (ORT/och_voxel.cpp:195-305). */
OCH_API int och_gpu_set_palette(och_gpu_pool *pool, const uint32_t *rgba, uint32_t n_voxels);
/* Enqueue all later work on a caller-owned HIP stream (hipStream_t); NULL is
 * HIP's null stream (torch's default stream).  Until called, the pool uses a
 * non-blocking stream of its own. */
OCH_API int och_gpu_set_stream(och_gpu_pool *pool, void *hip_stream);
OCH_API int och_gpu_synchronize(och_gpu_pool *pool);
/* Launch options of trace/render kernels.  Every launch is a grid of one ray
 * per thread.  Ids 0, 2, 3, 7, 9, 12 and 13 belonged to arms measured slower
 * on every scene and retired in round 5 (persistent and refill schedules,
 * in-block wave merging, the per-node voxel-box skip, the column cull;
 * DESIGN.md section 8): setting or reading them fails with OCH_E_INVALID. */
typedef enum och_option {
    OCH_OPT_BLOCK = 1,         /* threads per workgroup: 64..1024, multiple of 64 (default 64) */
    OCH_OPT_LAYOUT = 4,        /* 0 = the caller's node layout; 1 = packed (default when the DAG has < 2^24
                                  (node, level) pairs): per-level breadth-first ids, interior slots carry the
                                  child's occupancy mask so only descents and hits touch memory */
    OCH_OPT_TILE_ORDER = 5,    /* camera rays (render): 0 = 8x8-pixel tiles row-major; 1 = 64x64-pixel supertiles,
                                  each handed to one XCD so neighbouring rays share that XCD's L2; 2 = the launch
                                  order planned by och_gpu_plan_views (costliest tiles first) for frames of the
                                  planned geometry, else 0; 3 = that plan grouped per XCD.  Dispatch order only:
                                  frames are identical */
    OCH_OPT_BOUNCE_COMPACT = 6,/* config 5: 1 (default) = compact each block's secondary rays into its first lanes
                                  (wave ballot/popcount + LDS queue) before tracing them; 0 = trace each in place;
                                  2 = per block, compact when that packs the block's secondary rays into fewer
                                  waves than hold them, else in place */
    OCH_OPT_CULL = 8,          /* 1 (default) = a ray whose walk provably never enters the bounding box of the
                                  pool's voxels (och_pool_occupied_box) is recorded as the miss it would end in,
                                  without walking (camera rays: a cheaper conservative test first, before the
                                  ray's setup); exact, for launches that do not count
                                  PUSHes.  0 = every ray walks.  2 = diagnostic: launches that count PUSHes
                                  cull too, a culled ray counting 0 (the PUSHes the culled launch walks) */
    OCH_OPT_TIMING = 10,       /* per-launch timing of trace/render kernels (och_gpu_last_kernel_ms):
                                  1 (default) = recorded by the kernel's own dispatch (hipExtLaunchKernel: no
                                  packets between two launches of a stream); 2 = hipEventRecord before and
                                  after the launch; 0 = not timed */
    OCH_OPT_PLAN = 11,         /* shape of och_gpu_plan_views' launch order (set before planning): 0 =
                                  costliest first; P in 1..99 = the costliest P % first, the rest in natural
                                  order (default 10); 100 = costliest and cheapest alternating */
    OCH_OPT_SPLIT = 14,        /* heavy-tile split (set before och_gpu_plan_views; renders with OCH_OPT_TILE_ORDER
                                  2, block 64, packed layout): the planned tiles whose cost reaches this % of the
                                  costliest one's walk each ray over OCH_OPT_SPLIT_SEGS lanes, a lane entering
                                  only every S-th present cell of level OCH_OPT_SPLIT_LEVEL along the ray, the
                                  lowest one's hit kept -- the same records, a lone
                                  frame no longer waiting on its few longest rays.  0 = off */
    OCH_OPT_SPLIT_SEGS = 15,   /* lanes per ray of a split tile: 2, 4 (default), 8 or 16 */
    OCH_OPT_SPLIT_LEVEL = 16,  /* the level whose cells are the split's segments (default 6) */
    OCH_OPT_SPLIT_TILES = 17   /* read only: tiles split by the current plan */
} och_option;
OCH_API int och_gpu_set_option(och_gpu_pool *pool, int option, int value);
OCH_API int och_gpu_get_option(const och_gpu_pool *pool, int option, int *value);
/* Diagnostics: later trace/render launches write one record per wave into a
 * device buffer of capacity_waves x 4 uint64: {start, end} (s_memrealtime,
 * 100 MHz), HW_ID | XCC_ID << 32, rays finished.  NULL turns it off. */
OCH_API int och_gpu_set_stamp_buffer(och_gpu_pool *pool, uint64_t *stamps, uint32_t capacity_waves);
/* Diagnostics: HIP's occupancy answer (workgroups per CU) for kind 0 = render
 * grid kernel or 2 = trace grid kernel, at the pool's block size and stack
 * depth (kind 1, the retired persistent kernel, fails). */
OCH_API int och_gpu_occupancy(const och_gpu_pool *pool, int kind, int *blocks_per_cu);
/* Duration of the most recent trace/render kernel launched on the pool,
 * measured with HIP events on the stream it ran on (blocks until it ends).
 * OCH_E_INVALID if that launch was not timed (OCH_OPT_TIMING 0, n = 0, or it
 * recorded the caller's events). */
OCH_API int och_gpu_last_kernel_ms(och_gpu_pool *pool, float *ms);
/* The next trace/render launch on the pool records these HIP events
 * (hipEvent_t, created by the caller; either may be NULL) at its kernel's
 * start and end, through the dispatch itself, instead of the pool's own.
 * One launch only; a call that launches nothing (n = 0) leaves them
 * unrecorded.  For frame timers: no event packets between the launches of a
 * stream. */
OCH_API int och_gpu_set_launch_events(och_gpu_pool *pool, void *start_event, void *stop_event);

/* ------------------------------------------------------------ tracing */
/* Reference signature: one ray, synchronous (the pick ray of
 * ORT/test_och_h_octree.cpp:536).  Requires origin in (1,2)^3. */
OCH_API int och_gpu_trace(och_gpu_pool *pool, float ox, float oy, float oz, float dx, float dy, float dz,
                          int32_t *hit_direction, uint32_t *hit_voxel, float *hit_time);
/* Batch of n rays, host buffers, synchronous.  origin_stride 0 = one shared
 * origin (3 floats), 3 = one origin per ray.  dirs: n x 3 floats (och::float3
 * AoS, ORT/test_och_h_octree.cpp:49).  Outputs: n each. */
OCH_API int och_gpu_trace_batch(och_gpu_pool *pool, const float *origin, int origin_stride,
                                const float *dirs, uint32_t n,
                                int32_t *hit_direction, uint32_t *hit_voxel, float *hit_time);
/* Same with device buffers, asynchronous on the pool stream.  push_count
 * (optional, may be NULL) receives the PUSH iterations (child fetches) per ray. */
OCH_API int och_gpu_trace_batch_dev(och_gpu_pool *pool, const float *origin, int origin_stride,
                                    const float *dirs, uint32_t n,
                                    int32_t *hit_direction, uint32_t *hit_voxel, float *hit_time,
                                    uint32_t *push_count);

/* och_gpu_trace_batch_dev for rays laid out as a row-major image `width`
 * rays wide (a camera's rays as update_position stores them, x + y * W,
 * ORT/test_och_h_octree.cpp:135): each wavefront walks an 8x8 tile of
 * neighbouring rays instead of 64 consecutive rays of one row, so its lanes
 * share the DAG's top nodes and finish after similar walks.  n need not be a
 * multiple of width (the last row is partial).  Records in the caller's
 * order, bit-identical to och_gpu_trace_batch_dev.  With OCH_OPT_TILE_ORDER
 * >= 2, batches of the geometry planned by och_gpu_plan_batch_tiled dispatch
 * their costliest tiles first. */
OCH_API int och_gpu_trace_batch_tiled_dev(och_gpu_pool *pool, const float *origin, int origin_stride,
                                          const float *dirs, uint32_t n, uint32_t width,
                                          int32_t *hit_direction, uint32_t *hit_voxel, float *hit_time,
                                          uint32_t *push_count);
/* och_gpu_trace_batch for a camera's rays in the reference's layout, a
 * row-major image `width` rays wide (x + y * W, ORT/test_och_h_octree.cpp:135):
 * host buffers, synchronous, traced as och_gpu_trace_batch_tiled_dev traces
 * them (8x8 tiles per wave; the plan of och_gpu_plan_batch_tiled when one
 * exists for this geometry).  Records in the caller's order, bit-identical to
 * och_gpu_trace_batch. */
OCH_API int och_gpu_trace_batch_image(och_gpu_pool *pool, const float *origin, int origin_stride,
                                      const float *dirs, uint32_t n, uint32_t width,
                                      int32_t *hit_direction, uint32_t *hit_voxel, float *hit_time);
/* Plan the launch order of tiled batches of n rays `width` wide (block size
 * included in the key): one timed trace of these rays, then
 * costliest tiles first.  Synchronous; a plan stays valid while the rays
 * change (it orders dispatch only). */
OCH_API int och_gpu_plan_batch_tiled(och_gpu_pool *pool, const float *origin, int origin_stride,
                                     const float *dirs, uint32_t n, uint32_t width);

/* Config 5 (BASELINE configs[4]): each primary ray that hits a voxel face
 * spawns one secondary ray -- from o + d*t - offset, the point half a voxel in
 * front of the hit face (get_directional_hit_offset, ORT/test_och_h_octree.cpp:
 * 487-502, as the editor's placement point :385), along d mirrored on the hit
 * axis -- traced by the same traversal.  Build-defined: the reference renders
 * primary rays only.  Secondary records: direction -1, voxel 0, t 0 when the
 * primary ray did not hit (exit / inside).  push_count (optional) receives the
 * PUSH iterations of both rays.  Device buffers, asynchronous on the pool stream. */
OCH_API int och_gpu_trace_bounce_batch_dev(och_gpu_pool *pool, const float *origin, int origin_stride,
                                           const float *dirs, uint32_t n,
                                           int32_t *hit_direction, uint32_t *hit_voxel, float *hit_time,
                                           int32_t *bounce_direction, uint32_t *bounce_voxel, float *bounce_time,
                                           uint32_t *push_count);

/* ------------------------------------------------------------ camera / frame */
/* tree_camera::update_position's per-frame constants (ORT/test_och_h_octree.cpp:89-115):
 * yaw = camera.dir.x, pitch = camera.dir.y, fov = 1.25F in the reference. */
OCH_API int och_camera_setup(float px, float py, float pz, float yaw, float pitch, float fov,
                             int width, int height, och_camera *cam);
/* Per-pixel ray directions (row-major, x + y*W) into a device buffer of W*H*3 floats. */
OCH_API int och_gpu_raygen_dev(och_gpu_pool *pool, const och_camera *cam, float *dirs);
/* One frame of update_position + update_image (ORT/test_och_h_octree.cpp:437-457):
 * raygen, trace and shade fused, RGBA8 into a host W*H buffer. */
OCH_API int och_gpu_render(och_gpu_pool *pool, const och_camera *cam, uint32_t *rgba);
/* Sharded device render: rows are dealt in chunks of row_chunk rows round-robin
 * over n_shards; this call renders shard `shard` into `rgba_slice`, a compact
 * buffer of och_shard_rows(H, row_chunk, n_shards) x W pixels. n_shards = 1,
 * row_chunk = H renders the whole frame. */
OCH_API int och_gpu_render_dev(och_gpu_pool *pool, const och_camera *cam, uint32_t *rgba_slice,
                               int row_chunk, int shard, int n_shards);
OCH_API int och_shard_rows(int height, int row_chunk, int n_shards);
/* Several cameras of equal size in one launch (stereo / multi-view frames):
 * view v's slice goes to rgba_slices + v * och_shard_rows(H, row_chunk, n_shards) * W.
 * One launch keeps the GPU busy with other views while a view's slowest rays finish. */
OCH_API int och_gpu_render_views_dev(och_gpu_pool *pool, const och_camera *cams, int n_views, uint32_t *rgba_slices,
                                     int row_chunk, int shard, int n_shards);
/* Plan the launch order of frames of this geometry (size, views, sharding,
 * block, bounce compaction): one render of these cameras per kernel (primary
 * and config-5 bounce frames) times every workgroup, and later renders with
 * OCH_OPT_TILE_ORDER = 2 dispatch the costliest tiles first, so a frame does
 * not end on a few late grazing tiles.  Synchronous.  A plan made from one
 * camera stays valid (and approximately right) while the camera moves;
 * re-plan at will. */
OCH_API int och_gpu_plan_views(och_gpu_pool *pool, const och_camera *cams, int n_views, int row_chunk, int shard,
                               int n_shards);
/* Config 5 frame: och_gpu_render_views_dev with one bounce per hit; a hit
 * pixel keeps its face colour when its secondary ray escapes (exit) and is
 * halved (RGB >> 1, alpha kept) when the secondary ray is blocked. */
OCH_API int och_gpu_render_bounce_views_dev(och_gpu_pool *pool, const och_camera *cams, int n_views,
                                            uint32_t *rgba_slices, int row_chunk, int shard, int n_shards);
/* The frame loop (update_image once per frame, ORT/test_och_h_octree.cpp:
 * 437-457) issued natively: n_steps whole frames of the same cameras
 * (och_gpu_render_views_dev, or _bounce_views_dev with bounce = 1; one shard),
 * frame k on streams[k % n_buffers] into frames[k % n_buffers] (each
 * n_views * H * W RGBA8 words), so up to n_buffers frames are in flight and a
 * frame reuses a buffer only behind the previous frame on that stream.  With
 * start_events / stop_events (n_steps hipEvent_t each, or both NULL) the
 * dispatch of frame k records start_events[k] and stop_events[k].
 * Asynchronous; the pool's stream is left as it was. */
OCH_API int och_gpu_render_steps_dev(och_gpu_pool *pool, const och_camera *cams, int n_views, int n_steps,
                                     void *const *streams, uint32_t *const *frames, int n_buffers,
                                     void *const *start_events, void *const *stop_events, int row_chunk,
                                     int bounce);
/* Row deal: instead of round-robin, row chunk g of frames `height` rows tall
 * (chunks of row_chunk rows over n_shards) belongs to shard chunk_shard[g],
 * for ceil(height / row_chunk) chunks; each shard's chunks keep their order.
 * Render, plan, shade and unshard calls of exactly this geometry use it.  A
 * slice then holds och_gpu_slice_rows rows -- the largest shard's chunks, the
 * others' slices padded -- so slices stay equal for an all-gather.  Every
 * rank must set the same deal.  chunk_shard = NULL restores round-robin.
 * Waits for the device (frames in flight may read the old tables). */
OCH_API int och_gpu_set_row_deal(och_gpu_pool *pool, int height, int row_chunk, int n_shards, const int32_t *chunk_shard);
/* Rows per slice for this geometry under the pool's deal (och_shard_rows without one). */
OCH_API int och_gpu_slice_rows(const och_gpu_pool *pool, int height, int row_chunk, int n_shards, int *rows);
/* The cost of every row chunk of these views: one timed render of the whole
 * frame (every workgroup timed, shader clocks), spread over its tiles' rows.
 * costs: ceil(height / row_chunk) floats.  Synchronous. */
OCH_API int och_gpu_chunk_costs(och_gpu_pool *pool, const och_camera *cams, int n_views, int row_chunk, float *costs);
/* Host only: deal n_chunks chunks of the given costs over n_shards, longest
 * first onto the shard with the least cost per weight (weights NULL = all 1;
 * a shard with other fixed work, e.g. the display rank's shading, gets a
 * smaller weight), at most ceil(n_chunks * max weight / sum) + 2 chunks per
 * shard.  Deterministic: the same costs give the same deal on every rank. */
OCH_API int och_deal_chunks(const float *costs, int n_chunks, int n_shards, const float *weights, int32_t *chunk_shard);
/* Reassemble n_shards gathered slices (slice s at gathered + s*rows*W) into a
 * full W*H frame on the device. */
OCH_API int och_gpu_unshard_dev(och_gpu_pool *pool, const uint32_t *gathered, uint32_t *frame,
                                int width, int height, int row_chunk, int n_shards);
/* Multi-view form: gathered = [n_shards][n_views][rows][W] (each rank's
 * och_gpu_render_views_dev output, all-gathered), frames = [n_views][H][W]. */
OCH_API int och_gpu_unshard_views_dev(och_gpu_pool *pool, const uint32_t *gathered, uint32_t *frames,
                                      int width, int height, int row_chunk, int n_shards, int n_views);

/* Indexed-colour form of och_gpu_render_views_dev / _bounce_views_dev (bounce
 * = 0 / 1): the same pixels as OCH_CODE_* bytes, a quarter of the RGBA8 bytes
 * to all-gather between ranks.  OCH_E_INVALID when the pool's palette has
 * more than OCH_CODE_MAX_VOXELS ids. */
OCH_API int och_gpu_render_codes_views_dev(och_gpu_pool *pool, const och_camera *cams, int n_views,
                                           uint8_t *code_slices, int row_chunk, int shard, int n_shards,
                                           int bounce);
/* och_gpu_unshard_views_dev for gathered code slices, shading each code to
 * the RGBA8 word the RGBA render would have written (bit-identical frames). */
OCH_API int och_gpu_shade_unshard_views_dev(och_gpu_pool *pool, const uint8_t *gathered, uint32_t *frames,
                                            int width, int height, int row_chunk, int n_shards, int n_views);

/* ------------------------------------------------------------ multi-GPU frames, one process */
/* SURVEY §8(e) for a C++ host: one process, one thread, every GPU of the node.
 * Each device holds a replica of the pool; rows are dealt in chunks of
 * row_chunk rows round-robin over the devices (och_shard_rows); every device
 * renders its slice, one RCCL all-gather (ncclCommInitAll over the devices,
 * xGMI) hands every device all slices, and each device shades + unshards them
 * into [n_views][H][W] RGBA8 frames -- the frames och_gpu_render_views_dev
 * would write, bit for bit.  Slices travel as 1-byte colour codes when the
 * palette has at most OCH_CODE_MAX_VOXELS ids, as RGBA8 otherwise.  RCCL is
 * loaded on first use (dlopen; an RCCL already in the process is reused);
 * OCH_E_NODEV when it cannot be.  devices = NULL means the first n_devices gfx950 devices (och_device_list).
 * Replaces the per-pixel loop of ORT/test_och_h_octree.cpp:437-457 across GPUs.
 * och_frame_group_plan also deals the row chunks by cost (och_gpu_chunk_costs,
 * och_deal_chunks) so that every device gets an equal share of the work. */
typedef struct och_frame_group och_frame_group;
OCH_API int och_frame_group_create(const int *devices, int n_devices, const uint32_t *nodes, uint32_t n_nodes,
                                   uint32_t root, int depth, int index_base, float miss_t, och_frame_group **out);
OCH_API int och_frame_group_destroy(och_frame_group *group);
OCH_API int och_frame_group_size(const och_frame_group *group, int *n_devices);
/* The pool replica on device `rank` (RCPPS table, stamps; owned by the group). */
OCH_API int och_frame_group_pool(och_frame_group *group, int rank, och_gpu_pool **pool);
OCH_API int och_frame_group_set_palette(och_frame_group *group, const uint32_t *rgba, uint32_t n_voxels);
OCH_API int och_frame_group_set_option(och_frame_group *group, int option, int value);
/* och_gpu_plan_views on every device for this geometry, then OCH_OPT_TILE_ORDER = 2. */
OCH_API int och_frame_group_plan(och_frame_group *group, const och_camera *cams, int n_views, int row_chunk);
/* Enqueue one frame of n_views equal-size cameras on every device (bounce = 1:
 * config 5's secondary rays).  Asynchronous; frames are valid once the
 * group is synchronised (or downloaded). */
OCH_API int och_frame_group_render(och_frame_group *group, const och_camera *cams, int n_views, int row_chunk,
                                   int bounce);
/* Device pointer of device `rank`'s [n_views][H][W] RGBA8 frames (valid until the next render). */
OCH_API int och_frame_group_frames_dev(och_frame_group *group, int rank, uint32_t **frames);
/* Copy device `rank`'s frames to a host buffer of n_views*H*W words (synchronous). */
OCH_API int och_frame_group_download(och_frame_group *group, int rank, uint32_t *rgba);
OCH_API int och_frame_group_synchronize(och_frame_group *group);
/* n_steps frames of the same cameras issued natively: frame k renders,
 * exchanges and shades into buffer set k % n_buffers of every device, on
 * that set's stream, so up to n_buffers frames are in flight (n_buffers
 * 1..8).  Asynchronous.  och_frame_group_frames_dev / _download then give
 * buffer set (n_steps - 1) % n_buffers: the last frame. */
OCH_API int och_frame_group_render_steps(och_frame_group *group, const och_camera *cams, int n_views, int n_steps,
                                         int n_buffers, int row_chunk, int bounce);

/* ------------------------------------------------------------ multi-GPU frames, one process per GPU */
/* SURVEY §8(e) with one process per GPU (the driver's torch.distributed
 * launch, MPI, ...): the library's own RCCL communicator over the ranks.
 * Rank 0 calls och_comm_unique_id; the caller hands the OCH_COMM_ID_BYTES
 * bytes to every rank by its own means (torch.distributed broadcast, MPI_Bcast,
 * a file); every rank then calls och_comm_create with its device (collective:
 * returns once all ranks joined).  RCCL is loaded on first use, as for the
 * frame group; OCH_E_NODEV when it cannot be. */
#define OCH_COMM_ID_BYTES 128
typedef struct och_comm och_comm;
OCH_API int och_comm_unique_id(uint8_t *id);
OCH_API int och_comm_create(const uint8_t *id, int n_ranks, int rank, int device, och_comm **out);
OCH_API int och_comm_destroy(och_comm *comm);
/* OCH_OK when RCCL can be loaded (no communicator made): lets every rank agree
 * that all can join before any of them blocks in och_comm_create. */
OCH_API int och_comm_available(void);
/* ncclCommAbort, callable from another thread (a watchdog): a collective whose
 * peer never comes stops blocking its stream.  The handle stays valid for
 * och_comm_destroy; later calls on it fail.  Aborting one rank does not
 * unblock the others: each rank's caller aborts its own. */
OCH_API int och_comm_abort(och_comm *comm);
OCH_API int och_comm_info(const och_comm *comm, int *n_ranks, int *rank, int *device);
/* recv = [n_ranks][bytes]: every rank's `bytes` (ncclAllGather), enqueued on stream. */
OCH_API int och_comm_all_gather(och_comm *comm, const void *send, void *recv, size_t bytes, void *stream);
/* Only rank `root` receives recv = [n_ranks][bytes]; the others send (recv may be NULL there).
 * One ncclSend / ncclRecv group per call: the root receives from every rank, its own slice
 * included (a send to itself, skipped when send already sits at recv + root * bytes). */
OCH_API int och_comm_gather(och_comm *comm, const void *send, void *recv, size_t bytes, int root, void *stream);

/* Exchange of a sharded frame (och_gpu_render_sharded_steps_dev). */
enum {
    OCH_EXCHANGE_ALL_GATHER = 0,   /* every rank receives every slice (ncclAllGather), every rank shades */
    OCH_EXCHANGE_DISPLAY = 1,      /* every rank receives every slice, only rank 0 (the display) shades */
    OCH_EXCHANGE_GATHER = 2        /* only rank 0 receives the slices (ncclSend / ncclRecv) and shades */
};
/* The sharded frame loop of update_image (ORT/test_och_h_octree.cpp:437-457)
 * on one rank, issued natively: n_steps frames of the same cameras, frame k on
 * streams[k % n_buffers]:
 *   1. this rank's row chunks of the n_views cameras as colour codes
 *      (och_gpu_render_codes_views_dev, shard = the comm's rank, n_shards = its
 *      size) into slices[b]: [n_views][rows][W] bytes, rows = och_gpu_slice_rows;
 *   2. the exchange into gathered[b]: [n_ranks][n_views][rows][W] bytes;
 *   3. where this rank shades (`exchange` above): shade + unshard into frames[b],
 *      [n_views][H][W] RGBA8 -- the frames och_gpu_render_views_dev writes.
 * gathered / frames may be NULL (or hold NULL entries) on ranks that do not
 * receive / shade.  start_events / stop_events (n_steps each, or both NULL):
 * recorded by frame k's render dispatch.  Every rank must issue the same
 * n_steps.  Asynchronous; the pool's stream is left as it was. */
OCH_API int och_gpu_render_sharded_steps_dev(och_gpu_pool *pool, och_comm *comm, const och_camera *cams, int n_views,
                                             int n_steps, void *const *streams, uint8_t *const *slices,
                                             uint8_t *const *gathered, uint32_t *const *frames, int n_buffers,
                                             void *const *start_events, void *const *stop_events, int row_chunk,
                                             int bounce, int exchange);

/* ------------------------------------------------------------ builder */
/* The demo terrain (ORT/test_och_h_octree.cpp:561-787) built in parallel
 * bottom-up, hash-consed to the same canonical DAG h_octree produces.
 * Output pool is breadth-first (root first, levels contiguous), 1-based with
 * slot 0 unused when dedup = 1 (an h_octree pool), or an expanded 0-based tree
 * with root 0 when dedup = 0 (an och::octree pool). */
typedef struct och_terrain_params {
    int32_t depth;          /* 1..12: dim = 1 << depth */
    int32_t tunnels;        /* apply the remove(tree, tunnels) pass (:786) */
    int32_t dedup;          /* 1 = h_octree DAG, 0 = pointer octree */
    int32_t rand_kind;      /* 0 = glibc rand() default seed, 1 = MSVC rand() */
    int32_t threads;        /* 0 = all hardware threads */
    int32_t use_gpu;        /* 1: voxelise 32^3 bricks on the current GPU (depth >= 5; smaller trees
                               are built on the host); a DAG (dedup = 1) is also hash-consed on
                               the GPU, an expanded tree allocated by host threads;
                               OCH_E_NODEV if no GPU can run the kernels.  0: host threads only.
                               Both give the same pool, slot for slot. */
} och_terrain_params;

typedef struct och_host_pool {
    uint32_t *nodes;        /* n_nodes x 8 */
    uint32_t n_nodes;
    uint32_t root;
    int32_t depth;
    int32_t index_base;
    uint64_t solid_voxels;  /* statistics */
    uint64_t voxel_hist[8]; /* count per voxel id 0..7 (solid ids) */
    uint64_t tree_nodes;    /* nodes of the expanded tree (h_octree nodecnt) */
    double build_seconds;
} och_host_pool;

OCH_API int och_build_terrain(const och_terrain_params *params, och_host_pool *out);
OCH_API void och_host_pool_free(och_host_pool *pool);
/* The packed device layout (OCH_OPT_LAYOUT 1) of a pool, on the host: node 0
 * is zero padding, ids are breadth-first per level, interior slots hold
 * child_id | child_mask << 24, leaf-level slots voxel ids; *out_root =
 * root_id | root_mask << 24.  out = NULL only reports *out_nodes. */
OCH_API int och_pool_pack(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth, int index_base,
                          uint32_t *out, uint32_t out_capacity, uint32_t *out_nodes, uint32_t *out_root);
/* Bounding box of every non-empty leaf voxel reachable from root, in voxel
 * units: voxel (x, y, z) lies in it iff lo <= (x, y, z) < hi per axis.
 * Returns OCH_OK with lo = hi = {0, 0, 0} for a pool without voxels. */
OCH_API int och_pool_occupied_box(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth, int index_base,
                                  int32_t lo[3], int32_t hi[3]);
/* h_octree::at over any pool (ORT/och_h_octree.h:239-258). */
OCH_API uint32_t och_pool_at(const uint32_t *nodes, uint32_t root, int depth, int index_base,
                             int x, int y, int z);

/* ------------------------------------------------------------ editor */
/* Interactive editing (the demo's place/remove, ORT/test_och_h_octree.cpp:
 * 301-435): h_octree::set / at (ORT/och_h_octree.h:176-258) over a host pool of
 * `capacity` slots (1-based, slot s at nodes[(s-1)*8]) that a device pool of
 * the same size mirrors.  An edit path-copies at most `depth` new nodes into
 * freed or never-used slots and frees dead ones; och_editor_flush uploads the
 * runs of slots written since the last flush, raw and packed layouts alike.
 * Traced records equal the reference's after the same edits (slot numbering
 * differs: the reference places nodes by hash, :110-160). */
typedef struct och_editor och_editor;

typedef struct och_editor_stats {
    uint32_t capacity;      /* slots */
    uint32_t live_nodes;    /* distinct nodes reachable from the root */
    uint32_t high_water;    /* highest slot ever handed out */
    uint32_t root;
    int32_t depth;
    uint32_t dirty_first;   /* lowest slot written since the last flush */
    uint32_t dirty_count;   /* distinct slots written since the last flush (0 = none) */
} och_editor_stats;

/* Adopt a 1-based pool (e.g. och_build_terrain's; root 0 = empty tree).
 * OCH_E_INVALID for an out-of-range child or an empty interior node,
 * OCH_E_CAPACITY if its nodes do not fit in capacity slots. */
OCH_API int och_editor_create(const uint32_t *nodes, uint32_t n_nodes, uint32_t root, int depth,
                              uint32_t capacity, och_editor **out);
OCH_API int och_editor_destroy(och_editor *editor);
/* h_octree::set: voxel (x,y,z) := v (0 removes).  Out-of-range coordinates are
 * ignored, as in the reference.  OCH_E_CAPACITY (tree unchanged) when fewer
 * than depth slots are free; the reference exit(0)s (ORT/och_h_octree.h:112-116). */
OCH_API int och_editor_set(och_editor *editor, int x, int y, int z, uint32_t v);
OCH_API uint32_t och_editor_at(const och_editor *editor, int x, int y, int z);
OCH_API int och_editor_info(const och_editor *editor, och_editor_stats *info);
/* The slot array (capacity x 8, valid until the next edit) and root: pass
 * them to och_gpu_pool_create to make the mirroring device pool. */
OCH_API int och_editor_nodes(const och_editor *editor, const uint32_t **nodes, uint32_t *n_slots, uint32_t *root);
/* Upload the dirty slots, then the root, to a pool made from this editor
 * (index_base 1, same depth, capacity slots).  Slots are rewritten in place,
 * so the flush first waits for ALL work on the pool's device (every stream).
 * Only a pool this editor's last flush wrote, untouched since, gets the
 * windowed upload; any other pool (a new one, one another editor or
 * och_gpu_pool_update wrote, or one a failed flush left behind) is written
 * whole, its packed layout replaced by one numbered like the slots.  The root
 * is published after every slot it reaches.  A flush that fails after it
 * began writing leaves slots half written (slots are reused in place), so it
 * marks the pool torn: traces, renders and och_gpu_pool_update on it return
 * OCH_E_INVALID until a later flush of this editor succeeds. */
OCH_API int och_editor_flush(och_editor *editor, och_gpu_pool *pool);

#ifdef __cplusplus
}
#endif
#endif /* OCH_GPU_H */
