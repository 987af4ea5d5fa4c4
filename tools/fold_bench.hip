// fold_bench: cycles of one in-order f64 fold of n LDS-resident values by one wave
// (the exact getUnbalanceBL folds of k_step).  Diagnostic only.
//   A: element j of each 64-chunk read from lane j with readlane (the k_step code)
//   B: every lane runs the chain itself over broadcast LDS reads (b128, unrolled)
//   C: B with 32-element register batches (16 b128 reads issued, then 32 adds)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ double lane_val(double v, int j) {
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), j);
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), j);
    return __hiloint2double(hi, lo);
}

__global__ void k_fold(const double* in, int n, int variant, double* out, long long* cyc) {
    __shared__ double s[4096];
    const int lane = threadIdx.x;
    for (int i = lane; i < n; i += 64) s[i] = in[i];
    __syncthreads();
    double acc = 0.0;
    const long long t0 = wall_clock64();
    const long long c0 = clock64();
    if (variant == 0) {
        for (int k = 0; k < n; k += 64) {
            const double v = k + lane < n ? s[k + lane] : 0.0;
#pragma unroll
            for (int j = 0; j < 64; j++) acc += lane_val(v, j);
        }
    } else if (variant == 1) {
        const double2* s2 = reinterpret_cast<const double2*>(s);
        for (int k = 0; k < n / 2; k += 8) {
#pragma unroll
            for (int j = 0; j < 8; j++) { const double2 v = s2[k + j]; acc += v.x; acc += v.y; }
        }
    } else {
        const double2* s2 = reinterpret_cast<const double2*>(s);
        for (int k = 0; k < n / 2; k += 16) {
            double2 v[16];
#pragma unroll
            for (int j = 0; j < 16; j++) v[j] = s2[k + j];
#pragma unroll
            for (int j = 0; j < 16; j++) { acc += v[j].x; acc += v[j].y; }
        }
    }
    const long long c1 = clock64();
    const long long t1 = wall_clock64();
    if (lane == 0) { out[variant] = acc; cyc[2 * variant] = c1 - c0; cyc[2 * variant + 1] = t1 - t0; }
}

int main() {
    const int n = 4096;
    std::vector<double> h(n);
    srand(7);
    for (int i = 0; i < n; i++) h[i] = (double)rand() / RAND_MAX * 1e-3 + 1e-7 * i;
    double ref = 0.0;
    for (int i = 0; i < n; i++) ref += h[i];
    double *d_in, *d_out; long long* d_cyc;
    hipMalloc(&d_in, n * 8); hipMalloc(&d_out, 3 * 8); hipMalloc(&d_cyc, 6 * 8);
    hipMemcpy(d_in, h.data(), n * 8, hipMemcpyHostToDevice);
    int rate = 0; hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
    for (int rep = 0; rep < 3; rep++)
        for (int v = 0; v < 3; v++) {
            hipLaunchKernelGGL(k_fold, dim3(1), dim3(64), 0, 0, d_in, n, v, d_out, d_cyc);
            hipDeviceSynchronize();
            double o[3]; long long c[6];
            hipMemcpy(o, d_out, 24, hipMemcpyDeviceToHost);
            hipMemcpy(c, d_cyc, 48, hipMemcpyDeviceToHost);
            if (rep == 2)
                printf("variant %d: %lld cycles, %.2f us (wall), exact=%d\n", v, c[2 * v],
                       c[2 * v + 1] * 1000.0 / rate, o[v] == ref);
        }
    return 0;
}
