// och_sort.hip -- coherence order for batches of arbitrary rays (OCH_OPT_SORT).
//
// och_gpu_trace_batch_dev takes rays in the caller's order.  A wave of 64
// rays that are neighbours in that order may point anywhere (secondary rays,
// a row of a camera image), and the wave's walk lasts as long as its longest
// ray while its lanes touch unrelated nodes.  Sorting the batch by where the
// rays start and where they point gives each wave rays that walk the same
// nodes and end after similar walks, as the camera path's 8x8 tiles do.  The
// records are unchanged: the kernel walks ray perm[i] as its i-th ray and
// writes the record at perm[i].
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <stdint.h>

#include "och_internal.h"

namespace och {
namespace {

__device__ __forceinline__ uint32_t spread2(uint32_t x)      // 16 bits -> even bits
{
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}

__device__ __forceinline__ uint32_t spread3(uint32_t x)      // 10 bits -> every third bit
{
    x &= 0x3FFu;
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}

__device__ __forceinline__ uint32_t quant(float v, float scale, uint32_t top)   // v in [0, 1] -> 0..top
{
    const float q = v * scale;
    return q > 0.0F ? (q < (float)top ? (uint32_t)q : top) : 0u;   // NaN -> 0
}

// Octahedral map of a direction to [0, 1]^2, 16 bits per coordinate, in
// Morton order: nearby directions get nearby keys.  Zero, denormal or NaN
// directions map somewhere; any key is correct, only the walk's speed changes.
__device__ __forceinline__ uint32_t dir_key(float x, float y, float z)
{
    const float s = fabsf(x) + fabsf(y) + fabsf(z);
    float u = 0.0F, v = 0.0F;
    if (s > 0.0F && s < INFINITY) {
        u = x / s;
        v = y / s;
        if (z < 0.0F) {
            const float uu = (1.0F - fabsf(v)) * (u < 0.0F ? -1.0F : 1.0F);
            v = (1.0F - fabsf(u)) * (v < 0.0F ? -1.0F : 1.0F);
            u = uu;
        }
    }
    return spread2(quant(0.5F * u + 0.5F, 65536.0F, 65535u)) |
           (spread2(quant(0.5F * v + 0.5F, 65536.0F, 65535u)) << 1);
}

__global__ __launch_bounds__(256) void k_ray_keys(const float *__restrict__ origin, int origin_stride,
                                                  const float *__restrict__ dirs, uint32_t n, uint32_t *__restrict__ keys,
                                                  uint32_t *__restrict__ idx)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const float *d = dirs + 3 * (size_t)i;
    uint32_t key = dir_key(d[0], d[1], d[2]);
    if (origin_stride) {
        // origin cell (7 bits per axis over the root's (1, 2)^3) first, then
        // the top 11 bits of the direction key
        const float *o = origin + 3 * (size_t)i;
        const uint32_t cell = spread3(quant(o[0] - 1.0F, 128.0F, 127u)) | (spread3(quant(o[1] - 1.0F, 128.0F, 127u)) << 1) |
                              (spread3(quant(o[2] - 1.0F, 128.0F, 127u)) << 2);
        key = (cell << 11) | (key >> 21);
    }
    keys[i] = key;
    idx[i] = i;
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

size_t sort_temp_bytes(uint32_t n)
{
    size_t bytes = 0;
    uint32_t *k = nullptr, *v = nullptr;
    (void)rocprim::radix_sort_pairs(nullptr, bytes, k, k, v, v, n, 0, 32, 0);
    return align256(bytes);
}

}  // namespace

size_t sort_rays_bytes(uint32_t n)
{
    return 4 * align256((size_t)n * 4) + sort_temp_bytes(n);
}

hipError_t sort_rays(const float *origin, int origin_stride, const float *dirs, uint32_t n, void *scratch,
                     size_t scratch_bytes, const uint32_t **perm, hipStream_t stream)
{
    if (n == 0 || scratch_bytes < sort_rays_bytes(n)) return hipErrorInvalidValue;
    char *b = static_cast<char *>(scratch);
    const size_t a = align256((size_t)n * 4);
    uint32_t *keys_in = reinterpret_cast<uint32_t *>(b), *keys_out = reinterpret_cast<uint32_t *>(b + a);
    uint32_t *idx_in = reinterpret_cast<uint32_t *>(b + 2 * a), *idx_out = reinterpret_cast<uint32_t *>(b + 3 * a);
    size_t temp = scratch_bytes - 4 * a;
    hipLaunchKernelGGL(k_ray_keys, dim3((n + 255) / 256), dim3(256), 0, stream, origin, origin_stride, dirs, n, keys_in,
                       idx_in);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = rocprim::radix_sort_pairs(b + 4 * a, temp, keys_in, keys_out, idx_in, idx_out, n, 0, 32, stream);
    if (e != hipSuccess) return e;
    *perm = idx_out;
    return hipSuccess;
}

}  // namespace och
