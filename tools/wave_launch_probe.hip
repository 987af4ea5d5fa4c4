// wave_launch_probe.hip -- diagnostic (not part of the engine): how long do the 16
// waves of one 1024-thread workgroup take to all start?  k_step's first barrier is
// reached ~7 us after its first wave starts (stamps build, profiles/r02_b), so this
// times the wave-start spread of a workgroup for kernels with and without scratch,
// large LDS and many VGPRs, alone and right after a streaming kernel.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/wave_launch_probe tools/wave_launch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %s\n", hipGetErrorString(e_), #x); return 1; } } while (0)

// o[blockIdx][wave] = wall clock at the wave's first instruction; o2 = at the barrier exit
template <int MODE>
__global__ __launch_bounds__(1024) void k_probe(unsigned long long* o, int n, int sel) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    extern __shared__ unsigned char dl[];
    int x = threadIdx.x;
    if (MODE == 1) {                        // scratch: a dynamically indexed private array
        volatile int priv[64];
        for (int i = 0; i < 64; i++) priv[i] = i * x;
        x += priv[(sel + x) & 63];
    }
    if (MODE == 2) {                        // 128 live VGPRs
        asm volatile("v_mov_b32 v127, %0" :: "v"(x) : "v127");
    }
    if (MODE == 3) dl[threadIdx.x] = (unsigned char)x;     // large dynamic LDS (launch arg)
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        o[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 2] = t0;
        o[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 2 + 1] = t1;
    }
    if (x == 0x7FFFFFF && sel == 12345) o[0] = 1;
}

__global__ void k_stream(const double4* a, double4* b, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        double4 v = a[i];
        if (v.x == 12345.0) b[i] = v;
    }
}

template <int MODE>
static int run(const char* name, int grid, size_t lds, bool after_stream, const double4* a, double4* b, long n,
               unsigned long long* d) {
    static unsigned long long h[256 * 16 * 2];
    double spread = 0, tobar = 0;
    const int R = 20;
    for (int r = 0; r < R; r++) {
        if (after_stream) hipLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, 0, a, b, n);
        hipLaunchKernelGGL(k_probe<MODE>, dim3(grid), dim3(1024), lds, 0, d, grid, 0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, d, (size_t)grid * 16 * 2 * 8, hipMemcpyDeviceToHost));
        double sp = 0, tb = 0;
        for (int g = 0; g < grid; g++) {
            unsigned long long mn = ~0ull, mx = 0, bar = 0;
            for (int w = 0; w < 16; w++) {
                unsigned long long t0 = h[(g * 16 + w) * 2], t1 = h[(g * 16 + w) * 2 + 1];
                mn = t0 < mn ? t0 : mn; mx = t0 > mx ? t0 : mx; bar = t1 > bar ? t1 : bar;
            }
            sp += (mx - mn) * 0.01;          // 100 MHz -> us
            tb += (bar - mn) * 0.01;
        }
        spread += sp / grid;
        tobar += tb / grid;
    }
    printf("{\"mode\": \"%s\", \"grid\": %d, \"lds_kb\": %zu, \"after_stream\": %d, \"wave_start_spread_us\": %.2f, "
           "\"first_start_to_barrier_us\": %.2f}\n", name, grid, lds / 1024, (int)after_stream, spread / R, tobar / R);
    return 0;
}

int main() {
    const long n = 18l * 1024 * 1024 / 32;
    double4 *a, *b;
    unsigned long long* d;
    CK(hipMalloc(&a, n * 32)); CK(hipMalloc(&b, n * 32)); CK(hipMalloc(&d, 256 * 16 * 2 * 8));
    CK(hipMemset(a, 0, n * 32));
    CK(hipFuncSetAttribute((const void*)k_probe<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024));
    for (int st = 0; st < 2; st++) {
        if (run<0>("plain", 1, 0, st, a, b, n, d)) return 1;
        if (run<1>("scratch", 1, 0, st, a, b, n, d)) return 1;
        if (run<2>("vgpr128", 1, 0, st, a, b, n, d)) return 1;
        if (run<3>("lds120k", 1, 120 * 1024, st, a, b, n, d)) return 1;
        if (run<0>("plain", 256, 0, st, a, b, n, d)) return 1;
        if (run<1>("scratch", 256, 0, st, a, b, n, d)) return 1;
        if (run<2>("vgpr128", 256, 0, st, a, b, n, d)) return 1;
    }
    return 0;
}
