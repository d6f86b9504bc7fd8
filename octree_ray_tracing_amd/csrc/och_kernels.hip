// och_kernels.hip -- gfx950 (CDNA4) kernels of the SVO-DAG ray caster.
//
// One ray per lane of a 64-wide wavefront.  Per-ray state (reflected-frame
// position bits, ray coefficients, child index, level) lives in VGPRs; the
// parent stack lives in LDS, lane-strided so a wave's 64 pushes hit 64
// distinct banks.  Every floating-point step reproduces the reference's SSE
// sequence bit for bit: fused only where the reference calls _mm_fmadd_ps,
// RCPPS emulated from a host-captured table, x86's default NaN restored
// before the unsigned t compare, denormal masks compared as integers.
// Build with -ffp-contract=off and without denormal flushing.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "och_internal.h"

namespace och {
namespace {

constexpr int kBlock = 256;                 // 4 waves
constexpr uint32_t kX86DefaultNaN = 0xFFC00000u;

__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float ffrom(uint32_t u) { return __uint_as_float(u); }

// RCPPS model (ORT/och_h_octree.h:316): the table holds RCPPS(-(1 + m/2^k))
// for exponent-127 inputs; other exponents move the result exponent.
__device__ __forceinline__ uint32_t rcpps(uint32_t x, const uint32_t *__restrict__ lut, int shift)
{
    const uint32_t sign = x & 0x80000000u, e = (x >> 23) & 0xFFu;
    if (e == 0) return sign | 0x7F800000u;                          // +-0, denormal -> inf
    if (e == 0xFFu) return (x & 0x7FFFFFu) ? (x | 0x400000u) : sign;
    const uint32_t ent = lut[(x & 0x7FFFFFu) >> shift];
    const int ne = (int)((ent >> 23) & 0xFFu) + 127 - (int)e;
    return ne <= 0 ? sign : (sign | ((uint32_t)ne << 23) | (ent & 0x7FFFFFu));
}

// The t compare of STEP is on raw bit patterns (ORT/och_h_octree.h:384-406);
// x86 produces 0xFFC00000 for fma(p, -inf, +inf), gfx950 0x7FC00000.
__device__ __forceinline__ uint32_t t_bits(float t)
{
    const uint32_t u = fbits(t);
    return ((u & 0x7FFFFFFFu) > 0x7F800000u) ? kX86DefaultNaN : u;
}

struct Hit {
    int32_t dir;
    uint32_t voxel;
    uint32_t t;
    uint32_t push;
};

// h_octree::sse_trace / octree::sse_trace (ORT/och_h_octree.h:292-447,
// ORT/och_octree.cpp:167-320) for one ray.  stack points at this lane's first
// LDS slot; consecutive levels are kBlock words apart.
template <bool kCount>
__device__ __forceinline__ Hit trace_one(const DevPool &P, float ox, float oy, float oz, float dx, float dy,
                                         float dz, uint32_t *stack)
{
    const float o[3] = {ox, oy, oz};
    const float d[3] = {dx, dy, dz};
    float c[3], b[3];
    uint32_t p[3];
    uint32_t inv = 0, idx = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const uint32_t db = fbits(d[a]);
        const bool positive = (int32_t)db > 0 && db <= 0x7F800000u;          // 0 < d, :310
        inv |= (uint32_t)positive << a;
        const float refl = fabsf(__fsub_rn(positive ? 3.0F : 0.0F, o[a]));   // :314
        c[a] = ffrom(rcpps(db | 0x80000000u, P.lut, P.lut_shift));           // :312, :316
        b[a] = ffrom(fbits(__fmul_rn(c[a], refl)) ^ 0x80000000u);           // :318
        p[a] = fbits(refl) & 0x3FC00000u;                                   // :320
        idx |= (uint32_t)(p[a] == 0x3FC00000u) << a;                        // :324
    }

    const uint32_t *__restrict__ nodes = P.nodes;
    uint32_t dim = 1u << 22;
    uint32_t node = P.root;
    uint32_t t_min = 0;           // +0.0F
    int level = 1;
    uint32_t min_axis = 8;
    uint32_t push = 0;
    bool stepping = false;
    Hit h;
    for (;;) {
        if (!stepping) {                                                    // PUSH :342
            if (kCount) ++push;
            const uint32_t child = nodes[8u * node + ((idx ^ inv) & 7u)];
            if (child) {
                if (level == P.depth) {                                     // HIT :346-355
                    h.voxel = child;
                    h.dir = (int32_t)((min_axis >> 1) + 3u * ((inv & min_axis) == 0));
                    h.t = t_min;
                    break;
                }
                stack[(level - 1) * kBlock] = node;                          // :357
                ++level;
                node = child;
                dim >>= 1;                                                  // :361
                const float tm = ffrom(t_min);
                uint32_t nidx = 0;
#pragma unroll
                for (int a = 0; a < 3; ++a) {                               // :363-373
                    const float t_mid = __builtin_fmaf(ffrom(p[a] | dim), c[a], b[a]);
                    const bool upper = t_mid >= tm;
                    nidx |= (uint32_t)upper << a;
                    p[a] |= upper ? dim : 0u;
                }
                idx = nidx;
                continue;
            }
            stepping = true;
        }
        // STEP :378-419
        const uint32_t tx = t_bits(__builtin_fmaf(ffrom(p[0]), c[0], b[0]));
        const uint32_t ty = t_bits(__builtin_fmaf(ffrom(p[1]), c[1], b[1]));
        const uint32_t tz = t_bits(__builtin_fmaf(ffrom(p[2]), c[2], b[2]));
        const bool sx = tx <= ty && tx <= tz;
        const bool sy = !sx && ty < tx && ty <= tz;
        min_axis = sx ? 1u : (sy ? 2u : 4u);
        t_min = sx ? tx : (sy ? ty : tz);
        if (idx & min_axis) {                                               // advance :413-419
            const int a = sx ? 0 : (sy ? 1 : 2);
            p[a] &= ~dim;
            idx ^= min_axis;
            stepping = false;
            continue;
        }
        // POP :421-446
        if (--level == 0) {
            h.voxel = 0;
            h.dir = OCH_EXIT;
            h.t = P.miss_bits;
            break;
        }
        node = stack[(level - 1) * kBlock];
#pragma unroll
        for (int a = 0; a < 3; ++a) p[a] &= ~dim;
        dim <<= 1;
        idx = (uint32_t)((p[0] & dim) != 0) | ((uint32_t)((p[1] & dim) != 0) << 1) |
              ((uint32_t)((p[2] & dim) != 0) << 2);
    }
    h.push = push;
    return h;
}

template <bool kCount>
__global__ __launch_bounds__(kBlock) void k_trace_batch(DevPool P, const float *__restrict__ origin,
                                                        int origin_stride, const float *__restrict__ dirs,
                                                        uint32_t n, int32_t *__restrict__ hit_dir,
                                                        uint32_t *__restrict__ hit_voxel,
                                                        uint32_t *__restrict__ hit_time,
                                                        uint32_t *__restrict__ push_count)
{
    extern __shared__ uint32_t lds_stack[];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float *o = origin + (size_t)origin_stride * i;
    const float *d = dirs + 3 * (size_t)i;
    const Hit h = trace_one<kCount>(P, o[0], o[1], o[2], d[0], d[1], d[2], lds_stack + threadIdx.x);
    hit_dir[i] = h.dir;
    hit_voxel[i] = h.voxel;
    hit_time[i] = h.t;
    if (kCount) push_count[i] = h.push;
}

// tree_camera::update_position per pixel (ORT/test_och_h_octree.cpp:119-136):
// products rounded, sums left to right, correctly rounded sqrt and divide.
__device__ __forceinline__ void camera_ray(const och_camera &C, int col, int row, float &rx, float &ry, float &rz)
{
    const float u = __fmul_rn(C.aspect, __fsub_rn(__fmul_rn(C.view_x, (float)col), 1.0F));
    const float v = __fsub_rn(__fmul_rn(C.view_y, (float)row), 1.0F);
    const float f = C.fov_factor;
    const float *m = C.rot;
    const float ru = __fadd_rn(__fadd_rn(__fmul_rn(u, m[0]), __fmul_rn(v, m[1])), __fmul_rn(f, m[2]));
    const float rv = __fadd_rn(__fadd_rn(__fmul_rn(u, m[3]), __fmul_rn(v, m[4])), __fmul_rn(f, m[5]));
    const float rw = __fadd_rn(__fadd_rn(__fmul_rn(u, m[6]), __fmul_rn(v, m[7])), __fmul_rn(f, m[8]));
    const float mag2 = __fadd_rn(__fadd_rn(__fmul_rn(ru, ru), __fmul_rn(rv, rv)), __fmul_rn(rw, rw));
    // __builtin_sqrtf lowers to the correctly rounded expansion; __fsqrt_rn is a bare v_sqrt_f32 (1 ulp).
    const float rmag = __fdiv_rn(1.0F, __builtin_sqrtf(mag2));
    rx = __fmul_rn(rw, rmag);
    ry = __fmul_rn(ru, rmag);
    rz = __fmul_rn(-rv, rmag);
}

__global__ __launch_bounds__(kBlock) void k_raygen(och_camera C, float *__restrict__ dirs)
{
    const int col = blockIdx.x * 16 + (threadIdx.x & 15);
    const int row = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (col >= C.width || row >= C.height) return;
    float x, y, z;
    camera_ray(C, col, row, x, y, z);
    const size_t k = 3 * ((size_t)row * C.width + col);
    dirs[k] = x;
    dirs[k + 1] = y;
    dirs[k + 2] = z;
}

// trace_pixel's colour choice (ORT/test_och_h_octree.cpp:76-84) as olc::Pixel RGBA8.
__device__ __forceinline__ uint32_t shade(const Hit &h, const uint32_t *__restrict__ palette, uint32_t n_voxels)
{
    if (h.dir == OCH_EXIT) return 0xFFFEBF00u;      // {0x00, 0xBF, 0xFE}
    if (h.dir == OCH_INSIDE) return 0xFF07193Fu;    // {0x3F, 0x19, 0x07}
    if (h.voxel == 0 || h.voxel > n_voxels) return 0xFFFF00FFu;
    return palette[6u * (h.voxel - 1u) + (uint32_t)h.dir];
}

// One frame of update_image for shard f.shard: each wave shades an 8x8 pixel
// tile (so its 64 rays descend the same top-of-DAG lines), a 256-thread block
// a 16x16 tile of the shard's compact slice.
__global__ __launch_bounds__(kBlock) void k_render(DevPool P, DevFrame F)
{
    extern __shared__ uint32_t lds_stack[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int col = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int srow = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    if (srow >= F.slice_rows || col >= F.cam.width) return;
    const int chunk = srow / F.row_chunk, within = srow - chunk * F.row_chunk;
    const int row = (chunk * F.n_shards + F.shard) * F.row_chunk + within;
    if (row >= F.cam.height) return;
    // An empty h_octree (root 0) walks the all-zero padding node and misses
    // everywhere: the exit colour update_image draws for it (:443-446).
    float dx, dy, dz;
    camera_ray(F.cam, col, row, dx, dy, dz);
    const Hit h = trace_one<false>(P, F.cam.pos[0], F.cam.pos[1], F.cam.pos[2], dx, dy, dz, lds_stack + threadIdx.x);
    F.out[(size_t)srow * F.cam.width + col] = shade(h, F.palette, F.n_voxels);
}

__global__ __launch_bounds__(kBlock) void k_unshard(const uint32_t *__restrict__ gathered, uint32_t *__restrict__ frame,
                                                    int width, int height, int row_chunk, int n_shards,
                                                    int slice_rows)
{
    const int col = blockIdx.x * kBlock + threadIdx.x;
    const int row = blockIdx.y;
    if (col >= width || row >= height) return;
    const int gchunk = row / row_chunk, within = row - gchunk * row_chunk;
    const int shard = gchunk % n_shards, lchunk = gchunk / n_shards;
    const size_t src = ((size_t)shard * slice_rows + (size_t)lchunk * row_chunk + within) * width + col;
    frame[(size_t)row * width + col] = gathered[src];
}

size_t stack_bytes(int depth) { return (size_t)(depth > 1 ? depth - 1 : 1) * kBlock * sizeof(uint32_t); }

}  // namespace

hipError_t launch_trace_batch(const DevPool &p, const float *origin, int origin_stride, const float *dirs,
                              uint32_t n, int32_t *hit_dir, uint32_t *hit_voxel, uint32_t *hit_time,
                              uint32_t *push_count, hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    const dim3 grid((n + kBlock - 1) / kBlock);
    if (push_count)
        hipLaunchKernelGGL(k_trace_batch<true>, grid, dim3(kBlock), stack_bytes(p.depth), stream, p, origin,
                           origin_stride, dirs, n, hit_dir, hit_voxel, hit_time, push_count);
    else
        hipLaunchKernelGGL(k_trace_batch<false>, grid, dim3(kBlock), stack_bytes(p.depth), stream, p, origin,
                           origin_stride, dirs, n, hit_dir, hit_voxel, hit_time, push_count);
    return hipGetLastError();
}

hipError_t launch_raygen(const och_camera &cam, float *dirs, hipStream_t stream)
{
    const dim3 grid((cam.width + 15) / 16, (cam.height + 15) / 16);
    hipLaunchKernelGGL(k_raygen, grid, dim3(kBlock), 0, stream, cam, dirs);
    return hipGetLastError();
}

hipError_t launch_render(const DevPool &p, const DevFrame &f, hipStream_t stream)
{
    const dim3 grid((f.cam.width + 15) / 16, (f.slice_rows + 15) / 16);
    hipLaunchKernelGGL(k_render, grid, dim3(kBlock), stack_bytes(p.depth), stream, p, f);
    return hipGetLastError();
}

hipError_t launch_unshard(const uint32_t *gathered, uint32_t *frame, int width, int height, int row_chunk,
                          int n_shards, int slice_rows, hipStream_t stream)
{
    const dim3 grid((width + kBlock - 1) / kBlock, height);
    hipLaunchKernelGGL(k_unshard, grid, dim3(kBlock), 0, stream, gathered, frame, width, height, row_chunk,
                       n_shards, slice_rows);
    return hipGetLastError();
}

}  // namespace och
