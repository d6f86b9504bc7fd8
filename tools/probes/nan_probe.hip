// Does v_fma_f32 propagate an input NaN's payload on gfx950?  fma(p, 0, NaN)
// with NaN = 0xFFC00000 (x86's default NaN) for p in [1,2) bit patterns.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
__global__ void k(const float *p, float c, float b, uint32_t *out, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = __float_as_uint(__builtin_fmaf(p[i], c, b));
}
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void kpk(const float *p, float c, float b, uint32_t *out, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * i + 1 < n) {
        f2 x = {p[2 * i], p[2 * i + 1]}, cc = {c, c}, bb = {b, b};
        f2 r = __builtin_elementwise_fma(x, cc, bb);
        out[2 * i] = __float_as_uint(r.x);
        out[2 * i + 1] = __float_as_uint(r.y);
    }
}
int main()
{
    const int n = 1024;
    float hp[n];
    for (int i = 0; i < n; ++i) hp[i] = 1.0f + i / 1024.0f;
    float *dp; uint32_t *dout; uint32_t hout[n];
    hipMalloc(&dp, sizeof hp); hipMalloc(&dout, sizeof hout);
    hipMemcpy(dp, hp, sizeof hp, hipMemcpyHostToDevice);
    const uint32_t nans[] = {0xFFC00000u, 0x7FC00000u, 0xFFC00001u, 0xFF800001u};
    for (uint32_t nb : nans) {
        float b; std::memcpy(&b, &nb, 4);
        for (float c : {0.0f, -0.0f, 1.0f}) {
            hipLaunchKernelGGL(k, dim3(4), dim3(256), 0, 0, dp, c, b, dout, n);
            hipMemcpy(hout, dout, sizeof hout, hipMemcpyDeviceToHost);
            int same = 0; uint32_t first = hout[0];
            for (int i = 0; i < n; ++i) same += hout[i] == first;
            printf("b=0x%08x c=%g -> 0x%08x (%d/%d identical)\n", nb, c, first, same, n);
        }
    }
    // inf * finite + (-inf) : what the tracer produces today
    float inf = __builtin_inff();
    hipLaunchKernelGGL(k, dim3(4), dim3(256), 0, 0, dp, -inf, inf, dout, n);
    hipMemcpy(hout, dout, sizeof hout, hipMemcpyDeviceToHost);
    printf("fma(p, -inf, +inf) -> 0x%08x\n", hout[0]);
    for (uint32_t nb : {0xFFC00000u, 0x7F800000u}) {
        float b; std::memcpy(&b, &nb, 4);
        const float c = nb == 0xFFC00000u ? 0.0f : -inf;
        hipLaunchKernelGGL(kpk, dim3(4), dim3(256), 0, 0, dp, c, b, dout, n);
        hipMemcpy(hout, dout, sizeof hout, hipMemcpyDeviceToHost);
        int same = 0;
        for (int i = 0; i < n; ++i) same += hout[i] == hout[0];
        printf("pk_fma(p, %g, 0x%08x) -> 0x%08x (%d/%d identical)\n", c, nb, hout[0], same, n);
    }
    return 0;
}
