// icache_probe.hip -- diagnostic (not part of the engine): what does a long
// straight-line kernel body cost when its code is cold?  k_step is a ~96 KB
// single-workgroup kernel run once per Balance() step right after k_scan streamed
// the partition arrays through L2; this times a 1-wave (and a 16-wave) run through
// N KB of s_nop / v_add code, warm (back-to-back launches) and after an 18 MB stream.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/icache_probe tools/icache_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %s\n", hipGetErrorString(e_), #x); return 1; } } while (0)

// 4-byte VALU ops: 1024 per KB/4
#define BODY(KB) asm volatile(".rept %1*256\n v_add_u32 %0, 1, %0\n .endr" : "+v"(x) : "i"(KB))

template <int KB>
__global__ __launch_bounds__(1024) void k_line(unsigned long long* o, int rep) {
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int x = threadIdx.x;
    for (int r = 0; r < rep; r++) BODY(KB);
    __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { o[0] = t1 - t0; o[1] = (unsigned long long)x; }
}

__global__ void k_stream(const double4* a, double4* b, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        double4 v = a[i];
        if (v.x == 12345.0) b[i] = v;
    }
}

template <int KB>
static int probe(int threads, const double4* a, double4* b, long n, unsigned long long* d) {
    unsigned long long h[2];
    double warm = 0, cold = 0, wev = 0, cev = 0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int R = 20;
    for (int i = 0; i < R; i++) {
        // cold: a stream over 18 MB first (same as a c3 scan)
        hipLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, 0, a, b, n);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_line<KB>, dim3(1), dim3(threads), 0, 0, d, 1);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); cev += ms * 1e3;
        CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
        cold += h[0] / 100.0;
        // warm: again, back to back
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_line<KB>, dim3(1), dim3(threads), 0, 0, d, 1);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1)); wev += ms * 1e3;
        CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
        warm += h[0] / 100.0;
    }
    printf("{\"code_kb\": %d, \"threads\": %d, \"cold_us\": %.2f, \"warm_us\": %.2f, \"cold_event_us\": %.2f, \"warm_event_us\": %.2f}\n",
           KB, threads, cold / R, warm / R, cev / R, wev / R);
    return 0;
}

int main() {
    const long n = 18l * 1024 * 1024 / 32;
    double4 *a, *b;
    unsigned long long* d;
    CK(hipMalloc(&a, n * 32)); CK(hipMalloc(&b, n * 32)); CK(hipMalloc(&d, 64));
    CK(hipMemset(a, 0, n * 32));
    for (int t : {64, 1024}) {
        if (probe<4>(t, a, b, n, d)) return 1;
        if (probe<16>(t, a, b, n, d)) return 1;
        if (probe<32>(t, a, b, n, d)) return 1;
        if (probe<64>(t, a, b, n, d)) return 1;
        if (probe<96>(t, a, b, n, d)) return 1;
    }
    return 0;
}
