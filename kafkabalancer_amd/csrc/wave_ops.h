// wave_ops.h -- wave-wide reductions on CDNA (wave64) with DPP row operations:
// quad_perm / row_ror within 16-lane rows, then row_bcast:15 / row_bcast:31 across
// rows; the total lands in lane 63 and is broadcast with v_readlane.  Pure VALU:
// unlike __shfl_xor (ds_bpermute) it does not queue on the CU's LDS pipeline.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace kbe {

template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}

template <int CTRL, typename T>
__device__ __forceinline__ T dpp_mov(T v) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit values");
    if constexpr (sizeof(T) == 4) {
        int x;
        __builtin_memcpy(&x, &v, 4);
        x = dpp_i32<CTRL>(x);
        T r;
        __builtin_memcpy(&r, &x, 4);
        return r;
    } else {
        int x[2];
        __builtin_memcpy(x, &v, 8);
        x[0] = dpp_i32<CTRL>(x[0]);
        x[1] = dpp_i32<CTRL>(x[1]);
        T r;
        __builtin_memcpy(&r, x, 8);
        return r;
    }
}

template <typename T>
__device__ __forceinline__ T lane63(T v) {
    if constexpr (sizeof(T) == 4) {
        int x;
        __builtin_memcpy(&x, &v, 4);
        x = __builtin_amdgcn_readlane(x, 63);
        T r;
        __builtin_memcpy(&r, &x, 4);
        return r;
    } else {
        int x[2];
        __builtin_memcpy(x, &v, 8);
        x[0] = __builtin_amdgcn_readlane(x[0], 63);
        x[1] = __builtin_amdgcn_readlane(x[1], 63);
        T r;
        __builtin_memcpy(&r, x, 8);
        return r;
    }
}

// all lanes of the wave must be active (full-wave code paths only)
template <typename T, typename Op>
__device__ __forceinline__ T wave_reduce(T v, Op op) {
    v = op(v, dpp_mov<0xb1>(v));    // quad_perm [1,0,3,2]
    v = op(v, dpp_mov<0x4e>(v));    // quad_perm [2,3,0,1]
    v = op(v, dpp_mov<0x124>(v));   // row_ror:4
    v = op(v, dpp_mov<0x128>(v));   // row_ror:8
    v = op(v, dpp_mov<0x142>(v));   // row_bcast:15
    v = op(v, dpp_mov<0x143>(v));   // row_bcast:31
    return lane63(v);
}

template <typename T>
__device__ __forceinline__ T wave_red_sum(T v) { return wave_reduce(v, [](T a, T b) { return a + b; }); }
template <typename T>
__device__ __forceinline__ T wave_red_min(T v) { return wave_reduce(v, [](T a, T b) { return b < a ? b : a; }); }
template <typename T>
__device__ __forceinline__ T wave_red_max(T v) { return wave_reduce(v, [](T a, T b) { return b > a ? b : a; }); }
template <typename T>
__device__ __forceinline__ T wave_red_or(T v) { return wave_reduce(v, [](T a, T b) { return a | b; }); }

// inclusive prefix sum over the 64 lanes (lane i: lanes 0..i): Hillis-Steele
// row_shr steps within the 16-lane rows, then the row totals via row_bcast
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

}  // namespace kbe
