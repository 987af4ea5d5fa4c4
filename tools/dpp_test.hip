// dpp_test.hip -- checks the DPP wave reductions of kernels.hip against plain loops
// (diagnostic tool).  hipcc --offload-arch=gfx950 -O3 -o tools/dpp_test tools/dpp_test.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cfloat>
#include "../kafkabalancer_amd/csrc/wave_ops.h"

__global__ void k(const double* x, const unsigned long long* y, const uint32_t* z, double* o1, double* o2,
                  unsigned long long* o3, uint32_t* o4, uint32_t* o5, long long* o6, int* o7) {
    o7[blockIdx.x * 64 + threadIdx.x] = kbe::wave_incl_scan((int)(z[blockIdx.x * 64 + threadIdx.x] & 1023));
    const int i = blockIdx.x * 64 + threadIdx.x;
    double s = kbe::wave_red_sum(x[i]);
    double m = kbe::wave_red_min(x[i]);
    unsigned long long u = kbe::wave_red_sum(y[i]);
    uint32_t mm = kbe::wave_red_min(z[i]);
    uint32_t oo = kbe::wave_red_or(z[i]);
    long long sc = kbe::wave_red_max((long long)z[i] - 1000);
    if (threadIdx.x == 17) { o1[blockIdx.x] = s; o2[blockIdx.x] = m; o3[blockIdx.x] = u; o4[blockIdx.x] = mm; o5[blockIdx.x] = oo; o6[blockIdx.x] = sc; }
}

int main() {
    const int nb = 64, n = nb * 64;
    double* hx = new double[n]; unsigned long long* hy = new unsigned long long[n]; uint32_t* hz = new uint32_t[n];
    uint64_t s = 1;
    for (int i = 0; i < n; i++) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        hx[i] = (double)(s >> 11) * 0x1p-53 - 0.3; hy[i] = s >> 20; hz[i] = (uint32_t)(s >> 40);
        if ((i & 63) == 5 && (i / 64) % 3 == 0) hx[i] = -HUGE_VAL;
    }
    double *dx, *o1, *o2; unsigned long long *dy, *o3; uint32_t *dz, *o4, *o5; long long* o6; int* o7;
    hipMalloc(&o7, n * 4);
    hipMalloc(&dx, n * 8); hipMalloc(&dy, n * 8); hipMalloc(&dz, n * 4);
    hipMalloc(&o1, nb * 8); hipMalloc(&o2, nb * 8); hipMalloc(&o3, nb * 8); hipMalloc(&o4, nb * 4); hipMalloc(&o5, nb * 4); hipMalloc(&o6, nb * 8);
    hipMemcpy(dx, hx, n * 8, hipMemcpyHostToDevice); hipMemcpy(dy, hy, n * 8, hipMemcpyHostToDevice); hipMemcpy(dz, hz, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(nb), dim3(64), 0, 0, dx, dy, dz, o1, o2, o3, o4, o5, o6, o7);
    int* r7 = new int[n];
    hipMemcpy(r7, o7, n * 4, hipMemcpyDeviceToHost);
    int bad_scan = 0;
    for (int b = 0; b < nb; b++) { int acc = 0; for (int l = 0; l < 64; l++) { acc += (int)(hz[b * 64 + l] & 1023); if (r7[b * 64 + l] != acc) bad_scan++; } }
    printf("dpp inclusive scan: %s (%d bad lanes)\n", bad_scan ? "FAIL" : "ok", bad_scan);
    double r1[nb], r2[nb]; unsigned long long r3[nb]; uint32_t r4[nb], r5[nb]; long long r6[nb];
    hipMemcpy(r1, o1, nb * 8, hipMemcpyDeviceToHost); hipMemcpy(r2, o2, nb * 8, hipMemcpyDeviceToHost);
    hipMemcpy(r3, o3, nb * 8, hipMemcpyDeviceToHost); hipMemcpy(r4, o4, nb * 4, hipMemcpyDeviceToHost);
    hipMemcpy(r5, o5, nb * 4, hipMemcpyDeviceToHost); hipMemcpy(r6, o6, nb * 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int b = 0; b < nb; b++) {
        double m = HUGE_VAL; unsigned long long u = 0; uint32_t mm = 0xFFFFFFFFu, oo = 0; long long mx = -(1ll << 62);
        double lo = 0, hi = 0;
        for (int l = 0; l < 64; l++) { double v = hx[b * 64 + l]; if (v > -HUGE_VAL) { lo += v; } m = v < m ? v : m; u += hy[b * 64 + l];
            mm = hz[b * 64 + l] < mm ? hz[b * 64 + l] : mm; oo |= hz[b * 64 + l]; long long q = (long long)hz[b * 64 + l] - 1000; mx = q > mx ? q : mx; }
        (void)hi;
        const bool has_inf = (b % 3) == 0;
        bool ok = (has_inf ? r1[b] == -HUGE_VAL : fabs(r1[b] - lo) <= 1e-12 * (1 + fabs(lo))) && r2[b] == m && r3[b] == u && r4[b] == mm && r5[b] == oo && r6[b] == mx;
        if (!ok) { bad++; printf("block %d: sum %g/%g min %g/%g u %llu/%llu mm %u/%u or %u/%u max %lld/%lld\n", b, r1[b], lo, r2[b], m, r3[b], u, r4[b], mm, r5[b], oo, r6[b], mx); }
    }
    printf("dpp reductions: %s (%d bad of %d)\n", bad ? "FAIL" : "ok", bad, nb);
    return (bad || bad_scan) ? 1 : 0;
}
