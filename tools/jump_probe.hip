// jump_probe.hip -- diagnostic (not part of the engine): the cost of a jump into code that
// is not in the instruction cache.  One wave runs a chain of NB blocks, each a few
// instructions followed by a jump over 2 KB of never-executed padding (so sequential
// instruction prefetch cannot bring in the next block), twice: pass 1 with cold code, pass 2
// with the same code now cached.  Run cold after an 18 MB stream (L2 churned, like a c3
// scan before k_step) and back to back.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/jump_probe tools/jump_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %s\n", hipGetErrorString(e_), #x); return 1; } } while (0)

#define CHAIN(NB) asm volatile(".rept %1\n v_add_u32 %0, 1, %0\n s_branch 1f\n .rept 512\n s_nop 0\n .endr\n1:\n .endr" : "+v"(x) : "i"(NB))

template <int NB>
__global__ __launch_bounds__(64) void k_jump(unsigned long long* o) {
    int x = threadIdx.x;
    unsigned long long t[3];
    t[0] = __builtin_amdgcn_s_memrealtime();
    CHAIN(NB);
    __builtin_amdgcn_s_waitcnt(0);
    t[1] = __builtin_amdgcn_s_memrealtime();
    CHAIN(NB);       // a second copy of the code: still cold
    __builtin_amdgcn_s_waitcnt(0);
    t[2] = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { o[0] = t[1] - t[0]; o[1] = t[2] - t[1]; o[2] = (unsigned long long)x; }
}

// the same chain run twice through a loop: pass 2 re-runs cached code
template <int NB>
__global__ __launch_bounds__(64) void k_jump2(unsigned long long* o) {
    int x = threadIdx.x;
    unsigned long long t[3];
    for (int p = 0; p < 2; p++) {
        t[p] = __builtin_amdgcn_s_memrealtime();
        CHAIN(NB);
        __builtin_amdgcn_s_waitcnt(0);
    }
    t[2] = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { o[0] = t[1] - t[0]; o[1] = t[2] - t[1]; o[2] = (unsigned long long)x; }
}

__global__ void k_stream(const double4* a, double4* b, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        double4 v = a[i];
        if (v.x == 12345.0) b[i] = v;
    }
}

template <int NB>
static int probe(const double4* a, double4* b, long n, unsigned long long* d, bool stream) {
    unsigned long long h[3];
    double p1 = 0, p2 = 0, q1 = 0, q2 = 0;
    const int R = 20;
    for (int i = 0; i < R; i++) {
        if (stream) hipLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, 0, a, b, n);
        hipLaunchKernelGGL(k_jump2<NB>, dim3(1), dim3(64), 0, 0, d);
        CK(hipMemcpy(h, d, 24, hipMemcpyDeviceToHost));
        p1 += h[0] / 100.0; p2 += h[1] / 100.0;
        if (stream) hipLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, 0, a, b, n);
        hipLaunchKernelGGL(k_jump<NB>, dim3(1), dim3(64), 0, 0, d);
        CK(hipMemcpy(h, d, 24, hipMemcpyDeviceToHost));
        q1 += h[0] / 100.0; q2 += h[1] / 100.0;
    }
    printf("{\"blocks\": %d, \"after_stream\": %d, \"loop_pass1_us\": %.3f, \"loop_pass2_us\": %.3f, "
           "\"copy1_us\": %.3f, \"copy2_us\": %.3f, \"us_per_cold_jump\": %.3f, \"us_per_warm_jump\": %.4f}\n",
           NB, stream ? 1 : 0, p1 / R, p2 / R, q1 / R, q2 / R, p1 / R / NB, p2 / R / NB);
    return 0;
}

int main() {
    const long n = 18l * 1024 * 1024 / 32;
    double4 *a, *b;
    unsigned long long* d;
    CK(hipMalloc(&a, n * 32)); CK(hipMalloc(&b, n * 32)); CK(hipMalloc(&d, 64));
    CK(hipMemset(a, 0, n * 32));
    for (int s = 0; s < 2; s++) {
        if (probe<8>(a, b, n, d, s)) return 1;
        if (probe<16>(a, b, n, d, s)) return 1;
        if (probe<24>(a, b, n, d, s)) return 1;
    }
    return 0;
}
