// och_internal.h -- shared between the C-ABI layer (och_api.cpp) and the
// gfx950 kernels (och_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/och_gpu.h"

namespace och {

// What a kernel needs to walk one pool: all device pointers.
struct DevPool {
    const uint32_t *nodes;  // nodes[8 * v + c] = child c of the node the reference calls v
    const uint32_t *lut;    // RCPPS table, 1 << (23 - lut_shift) entries
    uint32_t root;
    int32_t depth;
    int32_t lut_shift;
    uint32_t miss_bits;     // hit_time bits of a miss (+INF or +0.0)
};

struct DevFrame {
    och_camera cam;
    const uint32_t *palette;  // 6 * n_voxels RGBA8
    uint32_t n_voxels;
    uint32_t *out;            // compact slice, slice_rows x width
    int32_t row_chunk, shard, n_shards, slice_rows;
};

hipError_t launch_trace_batch(const DevPool &p, const float *origin, int origin_stride, const float *dirs,
                              uint32_t n, int32_t *hit_dir, uint32_t *hit_voxel, uint32_t *hit_time,
                              uint32_t *push_count, hipStream_t stream);
hipError_t launch_raygen(const och_camera &cam, float *dirs, hipStream_t stream);
hipError_t launch_render(const DevPool &p, const DevFrame &f, hipStream_t stream);
hipError_t launch_unshard(const uint32_t *gathered, uint32_t *frame, int width, int height, int row_chunk,
                          int n_shards, int slice_rows, hipStream_t stream);
// Builder: voxel codes of the 2x2x2 leaves of one brick (GPU half of och_build_terrain).
hipError_t launch_terrain_leaves(int depth, int tunnels, const int32_t *heights, const uint8_t *tops,
                                 int bx, int by, int bz, int brick_leaves, uint32_t *codes, hipStream_t stream);

}  // namespace och
