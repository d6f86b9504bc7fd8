// Does a stream's priority reorder workgroup dispatch on gfx950?  Launch A, a
// grid of one-wave workgroups that each spin for `us` microseconds (40 GPU-fulls),
// then right behind it, on another stream, B (one GPU-full of the same
// workgroups).  If the dispatcher serves B's queue ahead of A's pending
// workgroups, B ends about 2 x `us` after A starts; if it shares dispatch
// round-robin, later; if in order, when A ends.  Arms: B's stream at normal,
// high priority, and A's stream at low with B's at high.
// Build: hipcc --offload-arch=gfx950 -O2 prio_probe.hip -o prio_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void spin(uint64_t ticks, uint32_t *out)
{
    const uint64_t t0 = wall_clock64();                // 100 MHz constant clock
    while (wall_clock64() - t0 < ticks) {
    }
    if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
            return 1;                                                           \
        }                                                                       \
    } while (0)

int main()
{
    int lo = 0, hi = 0, cus = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("priority range: least %d greatest %d; CUs %d\n", lo, hi, cus);
    const uint32_t full = (uint32_t)cus * 32;          // one wave per workgroup, 32 per CU
    const uint32_t na = 40 * full, nb = full;
    const uint64_t ticks = 10 * 100;                    // 10 us
    uint32_t *out;
    CK(hipMalloc(&out, (size_t)na * 4));
    struct Arm { const char *name; int pa, pb; } arms[] = {
        {"both normal", 0, 0}, {"B greatest", 0, hi}, {"A least, B greatest", lo, hi}};
    for (int rep = 0; rep < 3; ++rep)
        for (const Arm &arm : arms) {
            hipStream_t sa, sb;
            CK(hipStreamCreateWithPriority(&sa, hipStreamNonBlocking, arm.pa));
            CK(hipStreamCreateWithPriority(&sb, hipStreamNonBlocking, arm.pb));
            hipEvent_t a0, a1, b0, b1;
            CK(hipEventCreate(&a0));
            CK(hipEventCreate(&a1));
            CK(hipEventCreate(&b0));
            CK(hipEventCreate(&b1));
            // warm both streams
            hipLaunchKernelGGL(spin, dim3(64), dim3(64), 0, sa, (uint64_t)10, out);
            hipLaunchKernelGGL(spin, dim3(64), dim3(64), 0, sb, (uint64_t)10, out);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a0, sa));
            hipLaunchKernelGGL(spin, dim3(na), dim3(64), 0, sa, ticks, out);
            CK(hipEventRecord(a1, sa));
            CK(hipEventRecord(b0, sb));
            hipLaunchKernelGGL(spin, dim3(nb), dim3(64), 0, sb, ticks, out);
            CK(hipEventRecord(b1, sb));
            CK(hipDeviceSynchronize());
            CK(hipGetLastError());
            float ta = 0, tb = 0, tab = 0;
            CK(hipEventElapsedTime(&ta, a0, a1));
            CK(hipEventElapsedTime(&tb, b0, b1));
            CK(hipEventElapsedTime(&tab, a0, b1));
            printf("rep %d %-20s A %.1f us  B %.1f us  B ends %.1f us after A starts\n", rep, arm.name,
                   ta * 1e3, tb * 1e3, tab * 1e3);
            (void)hipEventDestroy(a0);
            (void)hipEventDestroy(a1);
            (void)hipEventDestroy(b0);
            (void)hipEventDestroy(b1);
            (void)hipStreamDestroy(sa);
            (void)hipStreamDestroy(sb);
        }
    (void)hipFree(out);
    return 0;
}
