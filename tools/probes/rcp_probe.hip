// Is one Newton step on v_rcp_f32 a correctly rounded reciprocal on gfx950?
//   r = rcp(s); e = fma(-s, r, 1); q = fma(e, r, r)   vs   __fdiv_rn(1, s)
// Exhaustive over every positive normal s with exponent in [LO, HI) (the
// camera ray's |D| = sqrt(|rot (u, v, f)|^2) lies far inside it), plus the
// sqrt without its small-input scaling against __builtin_sqrtf over the
// squares' range.  Prints the mismatch counts and the first few of each.
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-gpu-flush-denormals-to-zero rcp_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ float fast_rcp(float s)
{
    const float r = __builtin_amdgcn_rcpf(s);
    const float e = __builtin_fmaf(-s, r, 1.0F);
    return __builtin_fmaf(e, r, r);
}

// the compiler's correctly rounded sqrt for inputs it need not scale
__device__ __forceinline__ float fast_sqrt(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x), rp = __builtin_fmaf(-sp, s, x);
    float y = rm <= 0.0F ? sm : s;
    y = rp > 0.0F ? sp : y;
    return y;
}

__global__ void k(uint32_t lo, uint32_t count, int which, unsigned long long *bad, uint32_t *first)
{
    const uint32_t base = (blockIdx.x * blockDim.x + threadIdx.x) * 64u;
    for (uint32_t k = 0; k < 64u; ++k) {
        const uint32_t i = base + k;
        if (i >= count) return;
        const float x = __uint_as_float(lo + i);
        const bool miss = which == 0 ? __float_as_uint(fast_rcp(x)) != __float_as_uint(__fdiv_rn(1.0F, x))
                                     : __float_as_uint(fast_sqrt(x)) != __float_as_uint(__builtin_sqrtf(x));
        if (miss) {
            const unsigned long long n = atomicAdd(bad, 1ull);
            if (n < 8) first[n] = lo + i;
        }
    }
}

int main()
{
    unsigned long long *bad;
    uint32_t *first;
    hipMalloc(&bad, 8);
    hipMalloc(&first, 32);
    struct Case { const char *name; int which; int e_lo, e_hi; };
    const Case cases[] = {{"rcp  s in [2^-60, 2^60)", 0, 127 - 60, 127 + 60},
                          {"sqrt x in [2^-96, 2^96)", 1, 127 - 96, 127 + 96}};
    int fails = 0;
    for (const Case &c : cases) {
        hipMemset(bad, 0, 8);
        const uint32_t lo = (uint32_t)c.e_lo << 23, count = (uint32_t)(c.e_hi - c.e_lo) << 23;
        const uint32_t threads = (count + 63) / 64;
        hipLaunchKernelGGL(k, dim3((threads + 255) / 256), dim3(256), 0, 0, lo, count, c.which, bad, first);
        unsigned long long n = 0;
        uint32_t f[8] = {};
        hipMemcpy(&n, bad, 8, hipMemcpyDeviceToHost);
        hipMemcpy(f, first, 32, hipMemcpyDeviceToHost);
        printf("%s: %u inputs, %llu mismatches", c.name, count, n);
        for (unsigned long long j = 0; j < n && j < 8; ++j) printf(" %08x", f[j]);
        printf("\n");
        fails += n != 0;
    }
    return fails;
}
