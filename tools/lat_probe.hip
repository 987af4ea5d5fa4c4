// lat_probe.hip -- diagnostic (not part of the engine): latency of the primitives k_step is
// built from, inside one 1024-thread workgroup (16 waves) on gfx950, in shader clocks:
// a workgroup barrier, a dependent LDS read (all 16 waves / wave 0 alone), a wave
// reduction of a double (DPP), an f64 division, a dependent global load (L2-warm).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/lat_probe tools/lat_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../kafkabalancer_amd/csrc/wave_ops.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %s\n", hipGetErrorString(e_), #x); return 1; } } while (0)

constexpr int N = 64;

__global__ __launch_bounds__(1024) void k_lat(unsigned long long* o, const int* gchain, double* dout) {
    __shared__ int s_chain[4096];
    __shared__ double s_d[1024];
    const int tid = threadIdx.x, wid = tid >> 6;
    for (int i = tid; i < 4096; i += 1024) s_chain[i] = (i * 97 + 13) & 4095;
    s_d[tid] = 1.0 + tid;
    __syncthreads();
    unsigned long long t[8];
    int k = tid;
    t[0] = clock64();
    for (int i = 0; i < N; i++) __syncthreads();
    t[1] = clock64();
    for (int i = 0; i < N; i++) k = s_chain[k];                    // every wave
    __syncthreads();
    t[2] = clock64();
    if (wid == 0) for (int i = 0; i < N; i++) k = s_chain[k];      // wave 0 alone
    __syncthreads();
    t[3] = clock64();
    double v = s_d[tid];
    for (int i = 0; i < N; i++) v = kbe::wave_red_sum(v) * 1e-3 + v;   // every wave
    __syncthreads();
    t[4] = clock64();
    double q = v;
    if (wid == 0) for (int i = 0; i < N; i++) q = 1.0 / (q + 1.0);  // f64 division chain
    __syncthreads();
    t[5] = clock64();
    int g = tid & 63;
    if (wid == 0) for (int i = 0; i < N; i++) g = __builtin_nontemporal_load(gchain + g);   // dependent global loads
    __syncthreads();
    t[6] = clock64();
    if (tid == 0) for (int i = 0; i < 6; i++) o[i] = t[i + 1] - t[i];
    if (k == -1 || g == -1) dout[0] = v + q;
    dout[1 + tid] = q;
}

int main() {
    unsigned long long* d; int* gc; double* dd;
    CK(hipMalloc(&d, 64)); CK(hipMalloc(&gc, 4096 * 4)); CK(hipMalloc(&dd, 8 * 2048));
    int h[4096];
    for (int i = 0; i < 4096; i++) h[i] = (i * 131 + 7) & 63;
    CK(hipMemcpy(gc, h, sizeof(h), hipMemcpyHostToDevice));
    const char* names[6] = {"barrier", "lds_dep_read_16w", "lds_dep_read_1w", "wave_sum_f64_16w", "f64_div_1w", "global_dep_load_1w"};
    double acc[6] = {0};
    const int R = 20;
    for (int r = 0; r < R + 2; r++) {
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(1024), 0, 0, d, gc, dd);
        unsigned long long o[6];
        CK(hipMemcpy(o, d, 48, hipMemcpyDeviceToHost));
        if (r >= 2) for (int i = 0; i < 6; i++) acc[i] += (double)o[i] / N / R;
    }
    printf("{");
    for (int i = 0; i < 6; i++) printf("%s\"%s_clk\": %.1f", i ? ", " : "", names[i], acc[i]);
    printf("}\n");
    return 0;
}
