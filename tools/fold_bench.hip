// fold_bench: cycles of one in-order f64 fold of n LDS-resident values by one wave
// (the exact getUnbalanceBL folds of k_step).  Diagnostic only.
//   A: element j of each 64-chunk read from lane j with readlane (the k_step code)
//   B: every lane runs the chain itself over broadcast LDS reads (b128, unrolled)
//   C: B with 32-element register batches (16 b128 reads issued, then 32 adds)
//   D: B's loop with LDS address-space pointers over 1024-element chunks (chain_lds)
//   E: D software-pipelined (the next batch's reads issued before this batch's adds)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ double lane_val(double v, int j) {
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), j);
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), j);
    return __hiloint2double(hi, lo);
}

typedef __attribute__((address_space(3))) double lds_f64;
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) f64x2 lds_f64x2;
template <int D>
__device__ __forceinline__ double chain_d(double acc, const lds_f64* x, int m) {
    const lds_f64x2* x2 = (const lds_f64x2*)x;
    const int h = m >> 1;
    int k = 0;
    for (; k + D <= h; k += D) {
#pragma unroll
        for (int j = 0; j < D; j++) { const f64x2 v = x2[k + j]; acc += v.x; acc += v.y; }
    }
    for (; k < h; k++) { const f64x2 v = x2[k]; acc += v.x; acc += v.y; }
    if (m & 1) acc += x[m - 1];
    return acc;
}
template <int D>
__device__ __forceinline__ double chain_e(double acc, const lds_f64* x, int m) {
    const lds_f64x2* x2 = (const lds_f64x2*)x;
    const int nb = m / (2 * D);
    if (nb > 0) {
        f64x2 cur[D];
#pragma unroll
        for (int j = 0; j < D; j++) cur[j] = x2[j];
        for (int b = 0; b < nb; b++) {
            f64x2 nxt[D];
            const int o = (b + 1 < nb ? b + 1 : b) * D;
#pragma unroll
            for (int j = 0; j < D; j++) nxt[j] = x2[o + j];
#pragma unroll
            for (int j = 0; j < D; j++) { acc += cur[j].x; acc += cur[j].y; }
#pragma unroll
            for (int j = 0; j < D; j++) cur[j] = nxt[j];
        }
    }
    for (int k = nb * 2 * D; k < m; k++) acc += x[k];
    return acc;
}

__global__ void k_fold(const double* in, int n, int variant, double* out, long long* cyc) {
    __shared__ __align__(16) double s[4096];
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
    } else if (variant == 3) {
        for (int k = 0; k < n; k += 1024) acc = chain_d<8>(acc, (const lds_f64*)(s + k), n - k < 1024 ? n - k : 1024);
    } else if (variant == 4) {
        for (int k = 0; k < n; k += 1024) acc = chain_e<8>(acc, (const lds_f64*)(s + k), n - k < 1024 ? n - k : 1024);
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
    hipMalloc(&d_in, n * 8); hipMalloc(&d_out, 5 * 8); hipMalloc(&d_cyc, 10 * 8);
    hipMemcpy(d_in, h.data(), n * 8, hipMemcpyHostToDevice);
    int rate = 0; hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
    for (int rep = 0; rep < 3; rep++)
        for (int v = 0; v < 5; v++) {
            hipLaunchKernelGGL(k_fold, dim3(1), dim3(64), 0, 0, d_in, n, v, d_out, d_cyc);
            hipDeviceSynchronize();
            double o[5]; long long c[10];
            hipMemcpy(o, d_out, 40, hipMemcpyDeviceToHost);
            hipMemcpy(c, d_cyc, 80, hipMemcpyDeviceToHost);
            if (rep == 2)
                printf("variant %d: %lld cycles, %.2f us (wall), exact=%d\n", v, c[2 * v],
                       c[2 * v + 1] * 1000.0 / rate, o[v] == ref);
        }
    return 0;
}
