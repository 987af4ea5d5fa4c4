// microbench.hip -- latency probes for the serial k_step design (diagnostic tool,
// not part of the engine): dependent global-load latency (L2-warm, freshly
// written by another CU / XCD), __syncthreads cost at 1024 threads, in-kernel
// clock (s_memtime / s_memrealtime), empty-kernel duration, f64 add chain.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench tools/microbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %s\n", hipGetErrorString(e_), #x); return 1; } } while (0)

struct Out { unsigned long long t[16]; double d[4]; };

// pointer chase through `next` (dependent loads), one lane
__global__ void k_chase(const int* next, int steps, Out* o) {
    if (threadIdx.x != 0) return;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    int p = 0;
    for (int i = 0; i < steps; i++) p = next[p];
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    o->t[0] = t1 - t0; o->t[1] = r1 - r0; o->t[2] = (unsigned long long)p;
}

// producer: every block writes a slice of `next` (a random cycle), so the chase
// afterwards reads lines last written by other CUs / XCDs
__global__ void k_produce(int* next, const int* perm, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        next[perm[i]] = perm[(i + 1) % n];
}

__global__ __launch_bounds__(1024) void k_sync(int iters, Out* o) {
    __shared__ int s[1024];
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    int v = threadIdx.x;
    for (int i = 0; i < iters; i++) {
        s[threadIdx.x] = v;
        __syncthreads();
        v += s[(threadIdx.x + 1) & 1023];
        __syncthreads();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { o->t[3] = t1 - t0; o->t[4] = r1 - r0; o->t[5] = (unsigned long long)v; }
}

__global__ void k_fadd(const double* x, int n, Out* o) {
    if (threadIdx.x != 0) return;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    double acc = 0;
    for (int i = 0; i < n; i++) acc += x[i & 63] * 1.0000001;
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    o->t[6] = t1 - t0; o->t[7] = r1 - r0; o->d[0] = acc;
}

__global__ void k_empty(Out* o) { if (threadIdx.x == 0 && blockIdx.x == 1 << 30) o->t[15] = 1; }

int main() {
    const int n = 1 << 22;
    std::vector<int> perm(n);
    uint64_t s = 12345;
    for (int i = 0; i < n; i++) perm[i] = i;
    for (int i = n - 1; i > 0; i--) { s = s * 6364136223846793005ull + 1442695040888963407ull; int j = (int)((s >> 33) % (uint64_t)(i + 1)); std::swap(perm[i], perm[j]); }
    int *dn, *dp; Out* dout; double* dx;
    CK(hipMalloc(&dn, n * 4)); CK(hipMalloc(&dp, n * 4)); CK(hipMalloc(&dout, sizeof(Out))); CK(hipMalloc(&dx, 64 * 8));
    CK(hipMemcpy(dp, perm.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(dx, 0, 64 * 8));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    Out o;
    const int steps = 2000;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k_produce, dim3(1024), dim3(256), 0, 0, dn, dp, n);
        hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, dn, steps, dout);   // fresh lines, other CUs wrote them
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(&o, dout, sizeof o, hipMemcpyDeviceToHost));
        double clk = (double)o.t[0] / (double)o.t[1] * 100.0;
        printf("chase(fresh) : %.1f ns/load  %.0f cyc/load  clock %.0f MHz\n", o.t[1] * 10.0 / steps, (double)o.t[0] / steps, clk);
        hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, dn, steps, dout);   // same lines again (L2 warm)
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(&o, dout, sizeof o, hipMemcpyDeviceToHost));
        printf("chase(warm)  : %.1f ns/load  %.0f cyc/load\n", o.t[1] * 10.0 / steps, (double)o.t[0] / steps);
    }
    hipLaunchKernelGGL(k_sync, dim3(1), dim3(1024), 0, 0, 1000, dout);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(&o, dout, sizeof o, hipMemcpyDeviceToHost));
    printf("syncthreads  : %.1f ns per barrier (1024 thr)  %.0f cyc\n", o.t[4] * 10.0 / 2000, (double)o.t[3] / 2000);
    hipLaunchKernelGGL(k_fadd, dim3(1), dim3(64), 0, 0, dx, 100000, dout);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(&o, dout, sizeof o, hipMemcpyDeviceToHost));
    printf("f64 mul+add chain: %.2f ns/iter  %.1f cyc  clock %.0f MHz\n", o.t[7] * 10.0 / 100000, (double)o.t[6] / 100000, (double)o.t[6] / o.t[7] * 100.0);
    for (int g : {1, 256, 1024}) {
        for (int w = 0; w < 50; w++) hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, 0, dout);
        hipEventRecord(e0);
        for (int w = 0; w < 200; w++) hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, 0, dout);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("empty kernel grid %4d: %.2f us per launch (back to back)\n", g, ms * 1000 / 200);
    }
    return 0;
}
