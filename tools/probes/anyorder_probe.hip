// Does hipExtLaunchKernel's hipExtAnyOrderLaunch flag let the next kernel of
// the same stream start before the previous one has finished, on gfx950?
// (hip_ext.h says the flag is not supported on GFX9 boards.)  Kernel `slow`
// is one workgroup that spins for ~100 us on s_memrealtime (bounded: it always
// ends); kernel `fast` records when its first workgroup starts.  With the flag
// honoured, fast starts before slow ends.  Also: two frames' worth of
// workgroups, to see whether dispatch of the second launch overlaps the first's
// tail.  Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/anyorder anyorder_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdint>

__global__ void slow(uint64_t *t, uint64_t ticks)
{
    if (threadIdx.x == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint64_t now = t0;
        while (now - t0 < ticks) now = __builtin_amdgcn_s_memrealtime();
        t[0] = t0;
        t[1] = now;
    }
}

__global__ void fast(uint64_t *t)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) t[2] = __builtin_amdgcn_s_memrealtime();
}

int main()
{
    uint64_t *d, h[3];
    if (hipMalloc(&d, 3 * sizeof(uint64_t)) != hipSuccess) return 1;
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    for (int flags : {0, hipExtAnyOrderLaunch, 0, hipExtAnyOrderLaunch}) {
        hipMemset(d, 0, 3 * sizeof(uint64_t));
        hipDeviceSynchronize();
        void *a1[] = {&d, nullptr};
        uint64_t ticks = 10000;   // 100 us at the 100 MHz realtime clock
        a1[1] = &ticks;
        void *a2[] = {&d};
        hipError_t e1 = hipExtLaunchKernel((const void *)slow, dim3(1), dim3(64), a1, 0, s, nullptr, nullptr, flags);
        hipError_t e2 = hipExtLaunchKernel((const void *)fast, dim3(1024), dim3(64), a2, 0, s, nullptr, nullptr, flags);
        hipStreamSynchronize(s);
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        printf("flags=%d launch=%d/%d slow [%llu, %llu] fast start %llu -> fast started %s slow ended (%+lld ticks)\n",
               flags, (int)e1, (int)e2, (unsigned long long)h[0], (unsigned long long)h[1],
               (unsigned long long)h[2], h[2] < h[1] ? "BEFORE" : "after", (long long)(h[2] - h[1]));
    }
    hipStreamDestroy(s);
    hipFree(d);
    return 0;
}
