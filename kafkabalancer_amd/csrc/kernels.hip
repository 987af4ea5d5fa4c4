// kernels.hip -- CDNA4 (gfx950) kernels of the kafkabalancer move-search engine.
//
// One Balance() step (balancer.go:49-65) is two launches on one stream:
//
//   k_scan   grid   the HBM stream over the SoA partition arrays.  Every workgroup
//                   stages the relative-load table r[B] and the per-set target
//                   records in LDS, then for each of its tiles of 2048 partitions
//                   evaluates the Remove / Add / Disallowed / distributeLeaders
//                   first-index predicates (from the packed meta word) and the
//                   O(1)-delta score of every leader / non-leader slot against its
//                   first eligible target (steps.go:167-222); the tile minimum is
//                   found with wave shuffles + LDS, and the near-tie census (all
//                   (partition, slot, target) within 4*eps of it) is taken right
//                   away, de-duplicated by key in LDS.  One record per workgroup.
//   k_step   1 WG   the serial half: combine the records; the reference's step
//                   order (RemoveExtra / AddMissing / MoveDisallowed /
//                   ReassignLeaders / MoveLeaders / MoveNonLeaders, balancer.go:34-44);
//                   certified decision or exact sequential folds for near ties
//                   (strict-< first minimum in (partition, slot, target) order,
//                   steps.go:211); the on-device apply (replacepl/addpl,
//                   utils.go:166-202); then the prep of the next step: incremental
//                   re-sort of the touched brokers (getBL, utils.go:107-117), bl_move
//                   compaction, relative loads, error bound eps, set records.
//
// Loads are exact in integral mode.  Otherwise a step updates the touched loads
// incrementally and tracks a rigorous error bound; whenever a decision or the
// broker order cannot be certified from the bounds, the step halts with
// H_NEED_EXACT, the host runs k_refresh (exact partition-ordered refolds,
// utils.go:92-105) and the step is re-run.  Values the reference's decision
// depends on are then computed in the reference's own operation order (IEEE
// binary64, no FMA: the file is built with -ffp-contract=off; true division).
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstddef>
#include <cstdint>
#include "engine_dev.h"
#include "kernels_api.h"
#include "wave_ops.h"

// The file builds as several translation units compiled in parallel (Makefile: -DKB_TU=0..10,
// each instantiating one group of kernels and their launch helpers); without KB_TU it is
// one unit holding everything.
#ifndef KB_TU
#define KB_TU (-1)
#endif
#define KB_IN_TU(n) (KB_TU < 0 || KB_TU == (n))

namespace kbe {

// --------------------------------------------------------------- helpers

#ifndef KB_EAGER_CODE
#define KB_EAGER_CODE 1   // (diagnostic A/B: 0 compiles the eager-refold code out)
#endif

__device__ __forceinline__ unsigned long long d2u(double d) { return (unsigned long long)__double_as_longlong(d); }
__device__ __forceinline__ double u2d(unsigned long long u) { return __longlong_as_double((long long)u); }

// plain loads / stores of objects of 8-byte multiples (record headers, keys,
// 16-B set-record units): the data crosses kernel boundaries only
__device__ __forceinline__ uint32_t ld32(const void* p) { return *(const uint32_t*)p; }
__device__ __forceinline__ void st32(void* p, uint32_t v) { *(uint32_t*)p = v; }
__device__ __forceinline__ double ldd(const double* p) { return *p; }
__device__ __forceinline__ void stdbl(double* p, double v) { *p = v; }
template <typename T>
__device__ __forceinline__ T ldobj(const T* p) { return *p; }
template <typename T>
__device__ __forceinline__ void stobj(T* p, const T& v) { *p = v; }
// write-through (sc1) stores of what a scan workgroup hands to k_step (records, spilled
// keys): the line leaves the XCD's L2 at once, so k_pair's step workgroup, acquiring after
// the workgroup's drained arrival, reads it with no L2 write-back on the producer's side
// (MI355X_MICROARCH.md, inter-workgroup visibility; the same cost as plain stores here)
template <typename T>
__device__ __forceinline__ void stobj_wt(T* p, const T& v) {
    static_assert(sizeof(T) % 8 == 0, "8-byte granules");
    const unsigned long long* src = (const unsigned long long*)&v;
    unsigned long long* dst = (unsigned long long*)p;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 8); i++)
        __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st32_wt(uint32_t* p, uint32_t v) {
    // (global address space: a global_store sc1 even where the pointer is generic)
    __hip_atomic_store((__attribute__((address_space(1))) uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// reference term (utils.go:136-143): r = L/avg - 1; r>0 ? r*r : r*r/2 (exact ops)
__device__ __forceinline__ double term_x(double L, double avg) {
    double r = L / avg - 1.0;
    if (r > 0) return r * r;
    return r * r / 2;
}

// scoring (approximate; error covered by eps): f(r) and the O(1) move delta
__device__ __forceinline__ double fsq(double r) {
    const double q = r * r;
    return __builtin_amdgcn_ldexp(q, r > 0 ? 0 : -1);   // q or q/2, exactly (power-of-two scaling)
}
// U(after) - U(before) for moving weight w (delta = w/avg) from source s to target t
__device__ __forceinline__ double dsrc(double rs, double delta) { return fsq(rs - delta) - fsq(rs); }
__device__ __forceinline__ double dtgt(double rt, double delta) { return fsq(rt + delta) - fsq(rt); }
// the same with f(r) from a (r, f(r)) table entry (bit-identical results)
__device__ __forceinline__ double dsrc_f(double2 rf, double delta) { return fsq(rf.x - delta) - rf.y; }
__device__ __forceinline__ double dtgt_f(double2 rf, double delta) { return fsq(rf.x + delta) - rf.y; }

__device__ __forceinline__ bool setbit(const uint64_t* sb, int b) {
    return (sb[b >> 6] >> (b & 63)) & 1ull;
}

// wave-wide reductions (full waves only): DPP row operations, no LDS traffic
template <typename T>
__device__ __forceinline__ T wave_min(T v) { return wave_red_min(v); }
template <typename T>
__device__ __forceinline__ T wave_max(T v) { return wave_red_max(v); }
template <typename T>
__device__ __forceinline__ T wave_sum(T v) { return wave_red_sum(v); }

// u16 field idx of a set record held in registers as U 16-B units (the unit picked by selects:
// a runtime index into the register array would put it in scratch)
template <int U>
__device__ __forceinline__ uint32_t rec_u16(const uint4 (&v)[U], int idx) {
    uint4 q = v[0];
#pragma unroll
    for (int u = 1; u < U; u++)
        if ((idx >> 3) == u) q = v[u];
    const int c = (idx >> 1) & 3;
    const uint32_t word = c == 0 ? q.x : (c == 1 ? q.y : (c == 2 ? q.z : q.w));
    return (idx & 1) ? (word >> 16) : (word & 0xFFFFu);
}

// gamma_n bound of a sequential n-term fold of non-negative terms (|fold - sum| <= gamma_n * sum)
__device__ __forceinline__ double gamma_n(int n) { return 1.01 * (double)(n > 1 ? n : 1) * (DBL_EPSILON / 2); }

// Sequential fold of n doubles held in LDS, in order (the reference's fold).
// Loads are batched FOLD_BATCH at a time so the dependent add chain, not LDS latency,
// sets the pace.
constexpr int FOLD_BATCH = 8;
__device__ __forceinline__ double fold_lds(const double* x, int n, double acc = 0.0) {
    int k = 0;
    for (; k + FOLD_BATCH <= n; k += FOLD_BATCH) {
        double v[FOLD_BATCH];
#pragma unroll
        for (int i = 0; i < FOLD_BATCH; i++) v[i] = x[k + i];
#pragma unroll
        for (int i = 0; i < FOLD_BATCH; i++) acc += v[i];
    }
    for (; k < n; k++) acc += x[k];
    return acc;
}

// Sequential fold of term_x(x[k], avg) in order.  The terms of a batch are
// independent (their IEEE divisions overlap); only the adds form the chain.
constexpr int TERM_BATCH = 16;
__device__ __forceinline__ double fold_terms_lds(const double* x, int n, double avg) {
    double U = 0.0;
    int k = 0;
    for (; k + TERM_BATCH <= n; k += TERM_BATCH) {
        double t[TERM_BATCH];
#pragma unroll
        for (int i = 0; i < TERM_BATCH; i++) t[i] = term_x(x[k + i], avg);
#pragma unroll
        for (int i = 0; i < TERM_BATCH; i++) U += t[i];
    }
    for (; k < n; k++) U += term_x(x[k], avg);
    return U;
}

// getUnbalanceBL (utils.go:119-147) of the bl order with bl[ps] = Ls and
// bl[pt] = Lt (steps.go:185,207): two sequential folds, the reference's order.
__device__ double exact_unbalance_lds(const double* Lm, int n, int ps, int pt, double Ls, double Lt) {
    double S = 0.0;
    int k = 0;
    for (; k + FOLD_BATCH <= n; k += FOLD_BATCH) {
        double v[FOLD_BATCH];
#pragma unroll
        for (int i = 0; i < FOLD_BATCH; i++) v[i] = Lm[k + i];
#pragma unroll
        for (int i = 0; i < FOLD_BATCH; i++) S += (k + i == ps) ? Ls : ((k + i == pt) ? Lt : v[i]);
    }
    for (; k < n; k++) S += (k == ps) ? Ls : ((k == pt) ? Lt : Lm[k]);
    const double avg = S / (double)n;
    double U = 0.0;
    k = 0;
    for (; k + FOLD_BATCH <= n; k += FOLD_BATCH) {
        double t[FOLD_BATCH];
#pragma unroll
        for (int i = 0; i < FOLD_BATCH; i++) {
            const double L = (k + i == ps) ? Ls : ((k + i == pt) ? Lt : Lm[k + i]);
            t[i] = term_x(L, avg);
        }
#pragma unroll
        for (int i = 0; i < FOLD_BATCH; i++) U += t[i];
    }
    for (; k < n; k++) U += term_x((k == ps) ? Ls : ((k == pt) ? Lt : Lm[k]), avg);
    return U;
}

// The same folds run by one whole wave (every lane gets the result).  The lanes load
// and compute 64 elements at a time in parallel (the 4096-broker case divides per term:
// one lane doing all of them was issue-bound on the division sequences) into a
// per-wave LDS row; then every lane runs the in-order additions itself over broadcast
// 16-byte LDS reads, one dependent add per element as in the reference.  The chain is
// bound by the f64 add latency: 11.3 cycles per element on gfx950 against 22 for
// reading element j from lane j with readlane (tools/fold_bench.hip, 4096 elements:
// 19.3 vs 37.4 us).  x must be 16-byte aligned.
typedef __attribute__((address_space(3))) double lds_f64;
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) f64x2 lds_f64x2;
template <int D = 8>
__device__ __forceinline__ double chain_lds(double acc, const lds_f64* x, int m) {
    const lds_f64x2* x2 = (const lds_f64x2*)x;
    int k = 0;
    for (; k + 2 * D <= m; k += 2 * D) {
        f64x2 v[D];
#pragma unroll
        for (int j = 0; j < D; j++) v[j] = x2[(k >> 1) + j];
#pragma unroll
        for (int j = 0; j < D; j++) { acc += v[j].x; acc += v[j].y; }
    }
    for (; k < m; k++) acc += x[k];
    return acc;
}
// The same in-order chain over m elements with the next 16 elements' LDS reads issued
// before the current 16 are added (two register sets, alternating; the reads are
// unconditional -- x must have 32 readable elements past m -- so the compiler waits for the
// older eight reads only), and the running sum stored after every 64th element (the list
// folds' checkpoints: ck[i] for the element i closing a 64-block, i relative to x; lane 0).
__device__ __forceinline__ double chain_lds_ck(double acc, const lds_f64* x, int m, double* ck, int lane) {
    const lds_f64x2* x2 = (const lds_f64x2*)x;
    f64x2 a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; j++) a[j] = x2[j];
    int k = 0;
    for (; k + 32 <= m; k += 32) {
#pragma unroll
        for (int j = 0; j < 8; j++) b[j] = x2[((k + 16) >> 1) + j];
#pragma unroll
        for (int j = 0; j < 8; j++) { acc += a[j].x; acc += a[j].y; }
        if (((k + 16) & 63) == 0 && lane == 0) ck[k + 15] = acc;
#pragma unroll
        for (int j = 0; j < 8; j++) a[j] = x2[((k + 32) >> 1) + j];
#pragma unroll
        for (int j = 0; j < 8; j++) { acc += b[j].x; acc += b[j].y; }
        if (((k + 32) & 63) == 0 && lane == 0) ck[k + 31] = acc;
    }
    if (k + 16 <= m) {
#pragma unroll
        for (int j = 0; j < 8; j++) { acc += a[j].x; acc += a[j].y; }
        if (((k + 16) & 63) == 0 && lane == 0) ck[k + 15] = acc;
        k += 16;
    }
    for (; k < m; k++) acc += x[k];
    return acc;
}
// a wave's own LDS writes are seen by its later reads (LDS executes a wave's
// operations in order); this keeps the compiler from moving them across
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// getUnbalanceBL of bl[] with bl[ps] = Ls, bl[pt] = Lt (ps / pt = -1: none); Lm is
// 16-byte aligned LDS, scr the calling wave's 64-double LDS row (wave-uniform call)
// (not inlined: k_step's 128-VGPR budget spills with the unrolled chains inside it;
// the pointers are cast to LDS so the call does not fall back to flat loads)
__device__ __attribute__((noinline)) double exact_unbalance_wave(const double* Lm_, int n, int ps, int pt, double Ls, double Lt, double* scr_) {
    const lds_f64* Lm = (const lds_f64*)Lm_;
    lds_f64* scr = (lds_f64*)scr_;
    const int lane = threadIdx.x & 63;
    double S = 0.0;
    for (int k = 0; k < n; k += 64) {
        const int m = n - k < 64 ? n - k : 64;
        if ((unsigned)(ps - k) < 64u || (unsigned)(pt - k) < 64u) {
            const int i = k + lane;
            if (lane < m) scr[lane] = i == ps ? Ls : (i == pt ? Lt : Lm[i]);
            wave_lds_sync();
            S = chain_lds(S, scr, m);
            wave_lds_sync();
        } else {
            S = chain_lds(S, Lm + k, m);
        }
    }
    const double avg = S / (double)n;
    double U = 0.0;
    for (int k = 0; k < n; k += 64) {
        const int m = n - k < 64 ? n - k : 64;
        const int i = k + lane;
        if (lane < m) scr[lane] = term_x(i == ps ? Ls : (i == pt ? Lt : Lm[i]), avg);
        wave_lds_sync();
        U = chain_lds(U, scr, m);
        wave_lds_sync();
    }
    return U;
}

// The same fold over bl-ordered loads in memory (k_step with its broker tables in memory,
// B > MAXB): the lanes load each 64-element chunk (the next one in flight while the
// current one is chained) into the wave's LDS row, and the chain runs from there.
__device__ __attribute__((noinline)) double exact_unbalance_wave_g(const double* Lm, int n, int ps, int pt, double Ls, double Lt, double* scr_) {
    lds_f64* scr = (lds_f64*)scr_;
    const int lane = threadIdx.x & 63;
    auto ld = [&](int k) -> double {
        const int i = k + lane;
        return i < n ? (i == ps ? Ls : (i == pt ? Lt : Lm[i])) : 0.0;
    };
    double S = 0.0, nx = ld(0);
    for (int k = 0; k < n; k += 64) {
        const int m = n - k < 64 ? n - k : 64;
        const double cur = nx;
        nx = ld(k + 64);
        scr[lane] = cur;
        wave_lds_sync();
        S = chain_lds(S, scr, m);
        wave_lds_sync();
    }
    const double avg = S / (double)n;
    double U = 0.0;
    nx = ld(0);
    for (int k = 0; k < n; k += 64) {
        const int m = n - k < 64 ? n - k : 64;
        const double cur = nx;
        nx = ld(k + 64);
        scr[lane] = term_x(cur, avg);
        wave_lds_sync();
        U = chain_lds(U, scr, m);
        wave_lds_sync();
    }
    return U;
}
template <bool GB>
__device__ __forceinline__ double exact_unb_w(const double* Lm, int n, int ps, int pt, double Ls, double Lt, double* scr) {
    if constexpr (GB) return exact_unbalance_wave_g(Lm, n, ps, pt, Ls, Lt, scr);
    else return exact_unbalance_wave(Lm, n, ps, pt, Ls, Lt, scr);
}

// ---------------------------------------------- near-tie de-duplication
// LDS open-addressing table keyed by (kind, source, target); the weight bits are
// claimed by the first insert; a different weight under the same key is a
// "conflict" handled by the caller.  Contenders with one key have one exact U,
// so only the earliest iteration index per key matters (steps.go:211).

struct Dedup {
    uint32_t* key;
    unsigned long long* wb;
    unsigned long long* it;
    int cap;
    int* n = nullptr;               // optional: count of distinct keys, per kind
    int* last = nullptr;            // optional: slot of a claimed key per kind (the one when n == 1)
};

__device__ __forceinline__ uint32_t ckey(int kind, int s, int t) {
    return ((uint32_t)kind << 30) | ((uint32_t)s << 15) | (uint32_t)t;
}

__device__ void dedup_clear(const Dedup& T) {
    for (int i = threadIdx.x; i < T.cap; i += blockDim.x) { T.key[i] = NONE32; T.wb[i] = NONE64; T.it[i] = NONE64; }
}

// >= 0 slot, -1 table full, -2 weight conflict
__device__ int dedup_insert(const Dedup& T, int kind, int s, int t, double w, unsigned long long iter) {
    const uint32_t k = ckey(kind, s, t);
    uint32_t h = (k * 2654435761u) & (uint32_t)(T.cap - 1);
    int probe = 0;
    for (; probe < T.cap; probe++) {
        uint32_t old = atomicCAS(&T.key[h], NONE32, k);
        if (old == NONE32 && T.n) { atomicAdd(&T.n[kind], 1); T.last[kind] = (int)h; }
        if (old == NONE32 || old == k) break;
        h = (h + 1) & (uint32_t)(T.cap - 1);
    }
    if (probe == T.cap) return -1;
    const unsigned long long wb = d2u(w);
    unsigned long long oldw = atomicCAS(&T.wb[h], NONE64, wb);
    if (oldw != NONE64 && oldw != wb) return -2;
    atomicMin(&T.it[h], iter);
    return (int)h;
}

__device__ __forceinline__ Contender dedup_entry(const Dedup& T, int h) {
    Contender c;
    const uint32_t k = T.key[h];
    c.kind = (int)(k >> 30);
    c.s = (int)((k >> 15) & 0x7FFF);
    c.t = (int)(k & 0x7FFF);
    c.w = u2d(T.wb[h]);
    c.iter = T.it[h];
    c.pad = 0;
    return c;
}

__device__ __forceinline__ double cont_delta(const double* r, const Contender& c, double inv_avg) {
    const double delta = c.w * inv_avg;
    return dsrc(r[c.s], delta) + dtgt(r[c.t], delta);
}

// ------------------------------------------------ per-broker list upkeep
// (partition lists sorted by index, for the exact refold of k_refresh)

// The list edits move up to LIST_K * blockDim entries per pass: every load of the pass is
// issued before one barrier, then every store.  A list of at most LIST_K * blockDim
// entries (c5: ~7300) is edited in one round trip -- the entries the search loaded are the
// ones stored shifted; one barrier pair per blockDim entries made an edit ~15 us of
// dependent round trips on the eager refolds' critical path.  Each edit lowers the
// broker's first changed position (Lists.dpos, the fold checkpoints).
constexpr int LIST_K = 8;

struct ListExt { uint32_t st, n, dp; };      // a list's start, length, first changed position

__device__ __forceinline__ ListExt list_ext(const Lists& L, int b) {
    ListExt x;
    x.st = L.lstart[b]; x.n = L.llen[b]; x.dp = L.dpos[b];
    return x;
}

// remove partition q from broker b's list (block-wide, all threads call); x follows
__device__ void list_remove_x(Lists L, int b, uint32_t q, ListExt& x, int* s_i) {
    const uint32_t st = x.st, n = x.n;
    const uint32_t nt = blockDim.x;
    if (threadIdx.x == 0) *s_i = -1;
    __syncthreads();
    if (n <= LIST_K * nt) {
        uint32_t v[LIST_K];
#pragma unroll
        for (int k = 0; k < LIST_K; k++) {
            const uint32_t i = k * nt + threadIdx.x;
            v[k] = i < n ? L.lent[st + i] : NONE32;
        }
#pragma unroll
        for (int k = 0; k < LIST_K; k++)
            if (v[k] == q) *s_i = (int)(k * nt + threadIdx.x);
        __syncthreads();
        const int at = *s_i;
        if (at < 0) return;
#pragma unroll
        for (int k = 0; k < LIST_K; k++) {
            const uint32_t i = k * nt + threadIdx.x;
            if (i > (uint32_t)at && i < n) L.lent[st + i - 1] = v[k];
        }
        if (threadIdx.x == 0) {
            L.llen[b] = n - 1;
            if ((uint32_t)at < x.dp) L.dpos[b] = (uint32_t)at;
        }
        __syncthreads();
        x.n = n - 1;
        x.dp = (uint32_t)at < x.dp ? (uint32_t)at : x.dp;
        return;
    }
    for (uint32_t i0 = 0; i0 < n; i0 += LIST_K * nt) {
        uint32_t v[LIST_K];
#pragma unroll
        for (int k = 0; k < LIST_K; k++) {
            const uint32_t i = i0 + k * nt + threadIdx.x;
            v[k] = i < n ? L.lent[st + i] : NONE32;
        }
#pragma unroll
        for (int k = 0; k < LIST_K; k++)
            if (v[k] == q) *s_i = (int)(i0 + k * nt + threadIdx.x);
    }
    __syncthreads();
    const int at = *s_i;
    if (at < 0) return;
    for (uint32_t c = (uint32_t)at; c + 1 < n; c += LIST_K * nt) {
        uint32_t v[LIST_K];
#pragma unroll
        for (int k = 0; k < LIST_K; k++) {
            const uint32_t j = c + k * nt + threadIdx.x;
            v[k] = j + 1 < n ? L.lent[st + j + 1] : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < LIST_K; k++) {
            const uint32_t j = c + k * nt + threadIdx.x;
            if (j + 1 < n) L.lent[st + j] = v[k];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        L.llen[b] = n - 1;
        if ((uint32_t)at < x.dp) L.dpos[b] = (uint32_t)at;
    }
    __syncthreads();
    x.n = n - 1;
    x.dp = (uint32_t)at < x.dp ? (uint32_t)at : x.dp;
}

// insert partition q into broker b's sorted list; false: no room (the list keeps q out)
__device__ bool list_insert_x(Lists L, int b, uint32_t q, ListExt& x, int* s_i) {
    const uint32_t st = x.st, n = x.n;
    const uint32_t nt = blockDim.x;
    if (n >= L.lcap[b]) return false;
    if (threadIdx.x == 0) *s_i = 0;
    __syncthreads();
    if (n <= LIST_K * nt) {
        uint32_t v[LIST_K];
#pragma unroll
        for (int k = 0; k < LIST_K; k++) {
            const uint32_t i = k * nt + threadIdx.x;
            v[k] = i < n ? L.lent[st + i] : NONE32;
        }
        int c = 0;
#pragma unroll
        for (int k = 0; k < LIST_K; k++) c += v[k] < q ? 1 : 0;
        c = wave_sum(c);
        if ((threadIdx.x & 63) == 0 && c) atomicAdd(s_i, c);
        __syncthreads();
        const uint32_t at = (uint32_t)*s_i;
#pragma unroll
        for (int k = 0; k < LIST_K; k++) {
            const uint32_t i = k * nt + threadIdx.x;
            if (i >= at && i < n) L.lent[st + i + 1] = v[k];
        }
        if (threadIdx.x == 0) {
            L.lent[st + at] = q; L.llen[b] = n + 1;
            if (at < x.dp) L.dpos[b] = at;
        }
        __syncthreads();
        x.n = n + 1;
        x.dp = at < x.dp ? at : x.dp;
        return true;
    }
    int c = 0;
    for (uint32_t i0 = 0; i0 < n; i0 += LIST_K * nt) {
        uint32_t v[LIST_K];
#pragma unroll
        for (int k = 0; k < LIST_K; k++) {
            const uint32_t i = i0 + k * nt + threadIdx.x;
            v[k] = i < n ? L.lent[st + i] : NONE32;
        }
#pragma unroll
        for (int k = 0; k < LIST_K; k++) c += v[k] < q ? 1 : 0;
    }
    c = wave_sum(c);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(s_i, c);
    __syncthreads();
    const uint32_t at = (uint32_t)*s_i;
    long long hi = (long long)n;
    while (hi > (long long)at) {
        long long lo = hi - (long long)LIST_K * nt;
        if (lo < (long long)at) lo = at;
        uint32_t v[LIST_K];
#pragma unroll
        for (int k = 0; k < LIST_K; k++) {
            const long long j = lo + k * (long long)nt + threadIdx.x;
            v[k] = j < hi ? L.lent[st + j] : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < LIST_K; k++) {
            const long long j = lo + k * (long long)nt + threadIdx.x;
            if (j < hi) L.lent[st + j + 1] = v[k];
        }
        __syncthreads();
        hi = lo;
    }
    if (threadIdx.x == 0) {
        L.lent[st + at] = q; L.llen[b] = n + 1;
        if (at < x.dp) L.dpos[b] = at;
    }
    __syncthreads();
    x.n = n + 1;
    x.dp = at < x.dp ? at : x.dp;
    return true;
}

__device__ void list_remove(Lists L, int b, uint32_t q, int* s_i) {
    ListExt x = list_ext(L, b);
    list_remove_x(L, b, q, x, s_i);
}
__device__ bool list_insert(Lists L, int b, uint32_t q, int* s_i) {
    ListExt x = list_ext(L, b);
    return list_insert_x(L, b, q, x, s_i);
}

// the list change of the last applied move (kind 1 replace, 2 remove, 3 add)
// (the lists by value: a reference into k_step's kernel-argument struct would make the
// struct's address escape -- copied to scratch, every field then a scratch load)
__device__ void do_list_op(DevCtl* ctl, Lists L, int* s_i) {
    if (!ctl->pending_list) return;
    const int kind = ctl->pl_kind, from = ctl->pl_from, to = ctl->pl_to;
    const uint32_t p = (uint32_t)ctl->pl_part;
    bool ok = true;
    if (kind == 1) { list_remove(L, from, p, s_i); ok = list_insert(L, to, p, s_i); }
    else if (kind == 2) list_remove(L, from, p, s_i);
    else if (kind == 3) ok = list_insert(L, to, p, s_i);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!ok) ctl->list_overflow = 1;
        ctl->pending_list = 0;
    }
    __syncthreads();
}

// --------------------------------------------------------------- k_scan
// census event counters (stamps build with -DKB_WALK_COUNTS only: their global atomics
// distort the census timing)
#ifdef KB_WALK_COUNTS
#define KB_COUNT_WALK(ctl, i, v) KB_COUNT(ctl, i, v)
#else
#define KB_COUNT_WALK(ctl, i, v) (void)0
#endif

static_assert(PER_LANE == 2, "the scan's register layout assumes two partitions per lane");

// one tile's data of one lane, as loaded (packed: unpacked where used, so the
// loads of a prefetched tile stay in flight until its scoring starts)
template <int RC>
struct PartRaw {
    double2 w;                      // weights of the lane's two partitions
    uint2 m;                        // their meta words
    uint32_t r[RC];                 // slot k: two u16 dense broker ids
    uint2 ps;                       // their allowed-set indices (set records in memory only:
                                    // ScanArgs.pset; else the meta word's set field)
    __device__ __forceinline__ double wt(int j) const { return j ? w.y : w.x; }
    __device__ __forceinline__ uint32_t mt(int j) const { return j ? m.y : m.x; }
    __device__ __forceinline__ uint32_t rp(int k, int j) const { return j ? (r[k] >> 16) : (r[k] & 0xFFFFu); }
};

// two consecutive partitions per lane: one 16-B weight load, one 8-B meta load
// and one 4-B load per replica slot (coalesced across the wave)
template <int RC, bool LSETS>
__device__ __forceinline__ void load_parts(const ScanArgs& a, long long base, PartRaw<RC>& P) {
    P.w = *(const double2*)(a.w + base);
    P.m = *(const uint2*)(a.meta + base);
#pragma unroll
    for (int k = 0; k < RC; k++) P.r[k] = *(const uint32_t*)(a.rep + (long long)k * a.Ppad + base);
    if (!LSETS) P.ps = *(const uint2*)(a.pset + base);
}
// a partition's allowed-set index: the meta word's 15-bit field when the set records
// live in LDS (at most 4096 sets), else the per-partition index array (any count)
template <int RC, bool LSETS>
__device__ __forceinline__ uint32_t set_of(const PartRaw<RC>& P, int j) {
    return LSETS ? meta_set(P.mt(j)) : (j ? P.ps.y : P.ps.x);
}

__device__ __forceinline__ void emit_global(const ScanArgs& a, const Contender& c) {
    uint32_t i = atomicAdd(a.ncont, 1u);
    if (i < a.cont_cap) stobj_wt(&a.cont[i], c);
    else st32_wt(a.cont_ovf, 1u);
}

__device__ __forceinline__ void emit(const ScanArgs& a, const Dedup& T, int kind, int s, int t, double w,
                                     unsigned long long iter) {
    KB_COUNT_WALK(a.ctl, 31, 1);
    if (dedup_insert(T, kind, s, t, w, iter) < 0) {   // table full or weight conflict: spill it raw
        KB_COUNT_WALK(a.ctl, 30, 1);
        Contender c;
        c.s = s; c.t = t; c.w = w; c.iter = iter; c.kind = kind; c.pad = 0;
        emit_global(a, c);
    }
}

// the 16-B units of a set record: from LDS (LSETS) or from memory
template <int RC, bool LSETS>
__device__ __forceinline__ void set_record(const ScanArgs& a, const uint4* s_set, uint32_t set,
                                           uint4 (&R)[sr_units(RC)]) {
    constexpr int U = sr_units(RC);
#pragma unroll
    for (int u = 0; u < U; u++) R[u] = LSETS ? s_set[set * U + u] : ldobj(a.setrec + (size_t)set * U + u);
}

// walk every allowed, non-replica target in bl order for one (partition, slot)
// and emit the ones within 4*eps of the tile minimum g; stop once 8*eps is
// exceeded (the approximate delta is monotone in the target load up to 2*eps).
// (ENT: the record's u16 field by index -- from LDS where the set records are staged, else
// from registers)
template <int RC, typename RF, typename PS, typename BL, typename ENT>
__device__ void walk_targets(const ScanArgs& a, const Dedup& T, RF s_rf, PS s_pos,
                             BL s_blm, ENT ent, int kind, long long p,
                             int slot, int src, const uint32_t (&reps)[RC], int nrep, int set, double w, double ds,
                             double g, double eps, double inv_avg, int nblm) {
    const unsigned long long ib = ((unsigned long long)p << 21) | ((unsigned long long)slot << 16);
    const double delta = w * inv_avg;
    const int nl = (int)ent(1);
    int last = -1;
    KB_COUNT_WALK(a.ctl, 29, 1);
    for (int i = 0; i < nl; i++) {                // the set's first KR eligible brokers
        const int b = (int)ent(2 + i);
        KB_COUNT_WALK(a.ctl, 28, 1);
        last = b;
        bool isrep = false;
#pragma unroll
        for (int q = 0; q < RC; q++) isrep |= (q < nrep) && ((int)reps[q] == b);
        if (isrep) continue;
        const double d = ds + dtgt_f(s_rf[b], delta);
        if (d <= g + 4.0 * eps) emit(a, T, kind, src, b, w, ib | (unsigned long long)s_pos[b]);
        if (d > g + 8.0 * eps) return;
    }
    // (the record lists the whole set, or the walk continues past its last member: a record
    // the fast prep merged may list fewer than KR members of a larger set)
    if (nl >= (int)ent(0) || last < 0) return;
    // rare: more than KR near-tied targets -- the walk goes on in bl order through the set's
    // membership words in memory, LA positions per round trip (their broker ids, then their
    // words, all in flight together): a set of 64 in 1000 brokers has a member every ~16
    // positions, and one position per dependent load made the few census workgroups that get
    // here the scan's last by ~2.5 us at c3
    // (32-bit halves of the words: the walk is inlined in the scoring loop, whose registers
    // it shares -- four positions of 64-bit words made every scan workgroup slower)
    const uint32_t* sb = (const uint32_t*)(a.setbits + (size_t)set * a.W64);
    constexpr int LA = 4;
    for (int k0 = s_pos[last] + 1; k0 < nblm; k0 += LA) {
        int bq[LA];
        uint32_t wq[LA];
#pragma unroll
        for (int q = 0; q < LA; q++) bq[q] = s_blm[k0 + q < nblm ? k0 + q : k0];
#pragma unroll
        for (int q = 0; q < LA; q++) wq[q] = sb[bq[q] >> 5];
#pragma unroll
        for (int q = 0; q < LA; q++) {
            const int k = k0 + q;
            if (k >= nblm) return;
            KB_COUNT_WALK(a.ctl, 27, 1);
            const int b = bq[q];
            if (!((wq[q] >> (b & 31)) & 1u)) continue;
            bool isrep = false;
#pragma unroll
            for (int x = 0; x < RC; x++) isrep |= (x < nrep) && ((int)reps[x] == b);
            if (isrep) continue;
            const double d = ds + dtgt_f(s_rf[b], delta);
            if (d <= g + 4.0 * eps) emit(a, T, kind, src, b, w, ib | (unsigned long long)k);
            if (d > g + 8.0 * eps) return;
        }
    }
}

// first allowed target in bl order that is not a replica (steps.go:192-201):
// among the first RC+1 entries of the partition's set record
template <int RC, bool LSETS>
__device__ __forceinline__ int first_target(const ScanArgs& a, const uint4* s_set, uint32_t set,
                                            const uint32_t (&reps)[RC], int nrep, int* nelig) {
    constexpr int U = sr_units(RC), UF = sr_units_first(RC);
    constexpr int KT = RC + 1;
    uint4 R[UF];
#pragma unroll
    for (int u = 0; u < UF; u++) R[u] = LSETS ? s_set[set * U + u] : ldobj(a.setrec + (size_t)set * U + u);
    *nelig = (int)rec_u16(R, 0);
    // slots past nrep compare against an id no record holds (ids < MAXB_G, NONE16 = padding);
    // padding is never a replica, so it is picked only when no valid target precedes it
    uint32_t rq[RC];
#pragma unroll
    for (int k = 0; k < RC; k++) rq[k] = k < nrep ? reps[k] : 0xFFFEu;
    uint32_t tb = NONE16;
#pragma unroll
    for (int i = KT - 1; i >= 0; i--) {
        const uint32_t b = rec_u16(R, 2 + i);
        bool isrep = false;
#pragma unroll
        for (int k = 0; k < RC; k++) isrep |= rq[k] == b;
        tb = isrep ? tb : b;
    }
    return tb == NONE16 ? -1 : (int)tb;
}

// order-preserving encoding of a double into u64 (LDS atomicMin of a minimum)
__device__ __forceinline__ unsigned long long enc(double d) {
    unsigned long long u = d2u(d);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double dec(unsigned long long e) {
    unsigned long long u = (e >> 63) ? (e & 0x7FFFFFFFFFFFFFFFull) : ~e;
    return u2d(u);
}


// the control values one scan round runs on (from DevCtl)
struct ScanParams {
    int run;
    double inv_avg, eps, ubL, ubN;
    int heavy, nblm;
    int tk_on;
    int ubpass;                     // census-free round whose minima close an open bound
    int incr;                       // incremental round: only the blocks with wmax >= wskip
    double wskip;
    double rlo, rhi;                // range of r[] (prune bound)
    // deferred prep pending (DevCtl.fp): posm holds the bl positions before the last move;
    // its touched brokers t move to n, every other bl_move broker follows (fixpos)
    int fp, fp_t0, fp_t1, fp_o0, fp_o1, fp_u0, fp_u1, fp_n0, fp_n1;
    // the bl position after the last move of broker b at position p before it (p < 0: not in
    // bl_move): drop the touched brokers, then count those now before the untouched rank
    __device__ __forceinline__ int fixpos(int b, int p) const {
        if (!fp || p < 0) return p;
        if (b == fp_t0) return fp_n0;
        if (b == fp_t1) return fp_n1;
        const int pc = p - (fp_o0 < p ? 1 : 0) - (fp_o1 < p ? 1 : 0);
        return pc + (fp_u0 <= pc ? 1 : 0) + (fp_u1 <= pc ? 1 : 0);
    }
};

// the lookup tables as loaded by one thread (issued with the control block, before the
// first tile: one round trip; written to LDS by scan_round)
// (pre: up to SCAN_THREADS brokers and set-record units, one of each per thread; larger
// tables are loaded by scan_round itself)
struct TabRaw {
    bool pre;
    double r;
    int32_t pos;
    uint4 set;
};

// Broker tables read from memory (GT: more brokers than the LDS tables hold, B > MAXB):
// the same indexing as the LDS tables, (r, f(r)) computed from r[] on each read; the
// tables stay L2-resident (B * 16 bytes)
struct RfMem {
    const double* r;
    __device__ __forceinline__ double2 operator[](int b) const { const double x = r[b]; return make_double2(x, fsq(x)); }
};
struct I32Mem {
    const int32_t* p;
    __device__ __forceinline__ int operator[](int i) const { return p[i]; }
};
template <bool GT> struct ScanTabs { double2* rf; int16_t* pos; uint16_t* blm; };
template <> struct ScanTabs<true> { RfMem rf; I32Mem pos; I32Mem blm; };

// One scan round of a workgroup over its tiles (its first tile and the tables already
// loaded into A / T): stage the tables, score, write the workgroup record.
template <int RC, bool LSETS, bool INCR, bool GT, bool BK>
__device__ __forceinline__ void scan_round(const ScanArgs& a, const ScanParams& q, unsigned char* smem,
                                           PartRaw<RC>& A, const TabRaw& TR,
                                           unsigned long long t_in,
                                           int wg, long long c0_in) {
    DevCtl* ctl = a.ctl;
    constexpr int U = sr_units(RC);
    constexpr int NW = SCAN_THREADS / 64;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

    const size_t rbytes = GT ? 0 : (size_t)a.B * 16;
    const size_t pbytes = GT ? 0 : ((size_t)a.B * 2 + 15) & ~(size_t)15;
    ScanTabs<GT> TB;
    if constexpr (GT) {
        TB.rf = RfMem{a.r}; TB.pos = I32Mem{a.posm}; TB.blm = I32Mem{a.blm};
    } else {
        TB.rf = (double2*)smem;                     // (r, f(r)) per broker
        TB.pos = (int16_t*)(smem + rbytes);
        TB.blm = (uint16_t*)(smem + rbytes + pbytes);
    }
    const auto s_rf = TB.rf;
    const auto s_pos = TB.pos;
    const auto s_blm = TB.blm;
    uint4* s_set = (uint4*)(smem + rbytes + 2 * pbytes);
    const size_t setbytes = LSETS ? (size_t)a.nsets * U * 16 : 0;
    uint32_t* s_key = (uint32_t*)(smem + rbytes + 2 * pbytes + setbytes);
    unsigned long long* s_wb = (unsigned long long*)(s_key + DEDUP_SCAN);
    unsigned long long* s_it = s_wb + DEDUP_SCAN;
    Dedup T{s_key, s_wb, s_it, DEDUP_SCAN};
    __shared__ uint32_t s_f[NF][NW];
    __shared__ unsigned long long s_c[2][NW];
    __shared__ uint32_t s_nk;
    __shared__ unsigned long long s_benc[2];
    __shared__ uint32_t s_bslot[2], s_nkk[2];
    __shared__ uint32_t s_fw[NW][NF];                // per wave: its first-index predicate minima
    __shared__ unsigned long long s_bke[2][NW];      // per wave and kind: its best non-census key
    __shared__ Contender s_bkc[2][NW];

    int tile = wg;
    // the lookup tables (loaded by the caller with the control block when they are small)
    if constexpr (GT) {
    } else if (TR.pre) {
        if (tid < a.B) {
            TB.rf[tid] = make_double2(TR.r, fsq(TR.r));
            // (bl order as the inverse of the positions: one table load fewer, and the
            // deferred prep's patch applies to both)
            const int p = q.fixpos(tid, TR.pos);
            TB.pos[tid] = (int16_t)p;
            if (p >= 0) TB.blm[p] = (uint16_t)tid;
        }
    } else {
        // (more brokers: every load first -- at most MAXB / SCAN_THREADS per thread --
        // then the LDS writes: one round trip, not one per loop iteration)
        constexpr int TQ = (MAXB + SCAN_THREADS - 1) / SCAN_THREADS;
        double rr[TQ];
        int32_t pp[TQ];
#pragma unroll
        for (int k = 0; k < TQ; k++) {
            const int i = min(k * SCAN_THREADS + tid, a.B - 1);
            rr[k] = ldd(a.r + i);
            pp[k] = (int32_t)ld32(a.posm + i);
        }
#pragma unroll
        for (int k = 0; k < TQ; k++) {
            const int i = k * SCAN_THREADS + tid;
            if (i < a.B) {
                TB.rf[i] = make_double2(rr[k], fsq(rr[k]));
                const int p = q.fixpos(i, pp[k]);
                TB.pos[i] = (int16_t)p;
                if (p >= 0) TB.blm[p] = (uint16_t)i;
            }
        }
    }
    if (LSETS) {
        if (TR.pre) { if (tid < a.nsets * U) s_set[tid] = TR.set; }
        else for (int i = tid; i < a.nsets * U; i += SCAN_THREADS) s_set[i] = ldobj(a.setrec + i);
    }
    for (int i = tid; i < DEDUP_SCAN; i += SCAN_THREADS) { s_key[i] = NONE32; s_wb[i] = NONE64; s_it[i] = NONE64; }
    if (tid == 0) s_nk = 0;
    if (tid < 2) { s_benc[tid] = NONE64; s_bslot[tid] = NONE32; s_nkk[tid] = 0; }
    if (tid < 2 * NW) (&s_bke[0][0])[tid] = NONE64;
    if (tid < NW * NF) (&s_fw[0][0])[tid] = NONE32;
    __shared__ unsigned long long s_cz[3];           // diagnostic (a.wgt): census clocks, waves, walk clocks
    if (tid < 3) s_cz[tid] = 0;
    const bool run = q.run != 0;
    const double inv_avg = q.inv_avg, eps = q.eps;
    const double ubL = q.ubL, ubN = q.ubN;
    const int heavy = q.heavy, nblm = q.nblm;
    const bool tk_on = q.tk_on != 0;
    __syncthreads();
    const bool ub_open = ubN == HUGE_VAL || (a.allow_leader && ubL == HUGE_VAL);
    if (!run || (a.dbg & 4) || (a.ubpass == 1 && !ub_open)) return;
    const bool census_off = (a.dbg & 1) || q.ubpass;
    // (bound keys are for the next step's census bound: none when this step's bound is
    // -inf -- the step after a first-index stage, whose successor is almost always one too
    // and which re-scans with the bound opened if it reaches move() after all)
    const bool bk_on = BK && !census_off && ubN != -HUGE_VAL;
    // Lower-bound prune.  The source delta f(r_s - delta) - f(r_s) decreases and the
    // target delta f(r_t + delta) - f(r_t) increases with the relative load (f is
    // convex), so every candidate of a partition with weight w scores
    //     d >= LB(delta) = [f(rmax - delta) - f(rmax)] + [f(rmin + delta) - f(rmin)],
    // delta = w / avg, over the range [rmin, rmax] of r[] (all brokers; absent ones
    // hold 0, which only widens it).  ub bounds the step's minimum per kind, and the
    // census never looks past ub + 12 eps (the wave gate below), so a wave whose
    // partitions all have LB > ub + 16 eps (rounding of d and LB: < 2 eps, see the
    // (1+R)^2 term of eps) holds neither the minimum nor a near tie: it only counts
    // its candidates.  With skewed weights that is almost every wave.
    // (the range [rmin, rmax] of r[] over every broker comes with the control block:
    // k_step's prep reduced it; a 16-wave reduction here costs ~0.3 us per scan)
    const double rmin = q.rlo, rmax = q.rhi;
    const double fmn = fsq(rmin), fmx = fsq(rmax);
    const double ubP = a.allow_leader ? (ubL > ubN ? ubL : ubN) : ubN;
    const double prune_t = (a.dbg & 16) ? HUGE_VAL : ubP + 16.0 * eps;    // dbg 16: no pruning

    double wgL = HUGE_VAL, wgN = HUGE_VAL;
    // the first-index predicates (rare once the plan is in shape): a wave's minima in LDS,
    // not eight registers held through the scoring loop (they pushed its loop-invariant
    // census thresholds to scratch, reloaded inside the loop behind a vmcnt(0) that also
    // waited for the prefetched tile)
    uint32_t fst[NF];
    auto fmin_ = [&](int f, uint32_t v) { if (v != NONE32) atomicMin(&s_fw[wid][f], v); };
    unsigned long long cL = 0, cN = 0;

    // score one tile held in P (partitions base, base + 1 of this lane)
    auto score = [&](const PartRaw<RC>& P, long long base) {
        if (a.dbg & 2) {                          // diagnostic: stream only
            uint32_t x = P.m.x ^ P.m.y ^ (uint32_t)__double2hiint(P.w.x) ^ (uint32_t)__double2hiint(P.w.y);
#pragma unroll
            for (int k = 0; k < RC; k++) x ^= P.r[k];
            fmin_(F_DUP, x | 0x80000000u);
            return;
        }
        double lL = HUGE_VAL, lN = HUGE_VAL;
        uint32_t cl = 0, cn = 0;                  // candidate counts of this tile (flushed to u64 below)
        // the first-index predicates are rare once the plan is in shape: one cheap
        // test per partition, the detailed path only for waves where one holds
        bool spec = false;
#pragma unroll
        for (int j = 0; j < PER_LANE; j++) {
            const uint32_t m = P.mt(j);
            uint32_t x = ((m ^ (m >> 5)) & 31u) | (m & 0x800u);      // want != nrep, Disallowed
            bool sp = x != 0 || (m & 31u) == 0;                         // ..., empty
            if (a.rebalance) sp |= P.rp(0, j) == (uint32_t)heavy;
            if (a.sem_go) {
                const int nrep = (int)meta_nrep(m);
#pragma unroll
                for (int q2 = 0; q2 < RC; q2++)
#pragma unroll
                    for (int y = q2 + 1; y < RC; y++) sp |= (y < nrep) && P.rp(q2, j) == P.rp(y, j);
            }
            spec |= sp && base + j < a.shard_end;
        }
        const bool anyspec = __ballot(spec) != 0;
        // the lower-bound prune (waves without a rare predicate only)
        bool need = anyspec;
        if (!need) {
            bool nd = false;
#pragma unroll
            for (int j = 0; j < PER_LANE; j++) {
                const double dl = P.wt(j) * inv_avg;
                const double lb = (fsq(rmax - dl) - fmx) + (fsq(rmin + dl) - fmn);
                nd |= !(lb > prune_t);
            }
            need = __ballot(nd) != 0;
        }
        if (!need) {
            // counts only: the eligible non-replica targets are |set ∩ bl_move| minus the
            // replicas inside the set (every replica broker is in bl_move), the same
            // number the scoring path derives from its first-target pick
            uint32_t cl = 0, cn = 0;
#pragma unroll
            for (int j = 0; j < PER_LANE; j++) {
                const uint32_t m = P.mt(j);
                const uint32_t nrep = meta_nrep(m), nin = meta_nin(m), set = set_of<RC, LSETS>(P, j);
                const uint32_t nelig = LSETS ? (uint32_t)((const uint16_t*)(s_set + (size_t)set * U))[0]
                                             : (ld32(a.setrec + (size_t)set * U) & 0xFFFFu);
                const bool ok = base + j < a.shard_end && meta_elig(m) && nrep > 0 && nelig > nin;
                const uint32_t ne = ok ? nelig - nin : 0u;
                if (a.allow_leader) cl += ne;
                cn += ne * (nrep > 0 ? nrep - 1 : 0u);
            }
            cL += cl;
            cN += cn;
            return;
        }
        if (anyspec) {
#pragma unroll
            for (int j = 0; j < PER_LANE; j++) {
                const long long p = base + j;
                const bool valid = p < a.shard_end;
                const uint32_t m = P.mt(j);
                const int nrep = (int)meta_nrep(m), want = (int)meta_want(m);
                const bool elig = valid && meta_elig(m);
                const uint32_t pi = valid ? (uint32_t)p : NONE32;
                if (a.sem_go) {
                    bool dup = false;
#pragma unroll
                    for (int x = 0; x < RC; x++)
#pragma unroll
                        for (int y = x + 1; y < RC; y++) dup |= (y < nrep) && P.rp(x, j) == P.rp(y, j);
                    if (dup) fmin_(F_DUP, pi);
                }
                if (want < nrep) fmin_(F_REMOVE, pi);
                if (want > nrep) fmin_(F_ADD, pi);
                if (nrep == 0) {
                    fmin_(F_EMPTY, pi);
                    if (elig) fmin_(F_EMPTY_ELIG, pi);
                }
                if (meta_dis(m)) fmin_(F_DIS, pi);
                if (a.rebalance && elig && nrep > 0 && (int)P.rp(0, j) == heavy) fmin_(F_LEAD, pi);
            }
        }
        // branch-free: every lane scores both partitions; invalid ones are masked
        const uint32_t bmax = (uint32_t)(a.B - 1);
        // (BK plans: the lane's argmin per kind, (target << 8) | (j << 4) | slot, for the wave's
        // bound key below -- two registers, in the BK instantiation only)
        uint32_t amL = 0, amN = 0;
#pragma unroll
        for (int j = 0; j < PER_LANE; j++) {
            const uint32_t m = P.mt(j);
            const int nrep = (int)meta_nrep(m);
            uint32_t reps[RC];
#pragma unroll
            for (int k = 0; k < RC; k++) reps[k] = P.rp(k, j);
            int nelig;
            const int tb0 = first_target<RC, LSETS>(a, s_set, set_of<RC, LSETS>(P, j), reps, nrep, &nelig);
            const bool ok = base + j < a.shard_end && meta_elig(m) && nrep > 0 && tb0 >= 0;
            const double delta = P.wt(j) * inv_avg;
            const double dt = dtgt_f(s_rf[tb0 >= 0 ? tb0 : 0], delta);
            const uint32_t ne = ok ? (uint32_t)(nelig - (int)meta_nin(m)) : 0u;
            const uint32_t r0 = min(reps[0], bmax);   // table index even where the slot is unused
            if (a.allow_leader) {
                const double d = dsrc_f(s_rf[r0], delta) + dt;
                const bool bt = ok && d < lL;
                lL = bt ? d : lL;
                if constexpr (BK) amL = bt ? (((uint32_t)tb0 << 8) | ((uint32_t)j << 4)) : amL;
                cl += ne;
            }
#pragma unroll
            for (int k = 1; k < RC; k++) {
                const double d = dsrc_f(s_rf[k < nrep ? reps[k] : r0], delta) + dt;
                const bool bt = ok && k < nrep && d < lN;
                lN = bt ? d : lN;
                if constexpr (BK) amN = bt ? (((uint32_t)tb0 << 8) | ((uint32_t)j << 4) | (uint32_t)k) : amN;
            }
            cn += ne * (uint32_t)(nrep - 1);
        }
        cL += cl;
        cN += cn;
        // wave minima; the census runs only where a wave minimum can be within 8*eps
        // of the step's global minimum, which is at most ub (k_step's upper bound)
        // (g <= ub + 2*eps: the first-target score is monotone in the target up to 2*eps)
        // (the wave minimum is within 12 eps of ub iff some lane's is: a ballot, and the
        // wave reduction only where it passes -- rare: the wave holding the step's minimum
        // always does, since ub bounds it from above.  The record carries the minimum over
        // the waves that passed, which is the step's minimum; a wave that did not pass
        // holds no candidate within 12 eps of ub)
        const bool hasL = __ballot(lL < HUGE_VAL && lL <= ubL + 12.0 * eps) != 0;
        const bool hasN = __ballot(lN < HUGE_VAL && lN <= ubN + 12.0 * eps) != 0;
        const double tL = hasL ? wave_min(lL) : HUGE_VAL, tN = hasN ? wave_min(lN) : HUGE_VAL;
        // A scored wave the census gate kept out still keeps its best candidate per kind (in
        // its slot of s_bk*, the minimum over its tiles): a workgroup whose waves all stayed
        // out of the census carries that as its record's best key, so every workgroup that
        // scored carries one.  The next step's census bound ub is the minimum of the records'
        // best keys re-scored; with keys only from the census waves -- the few around the
        // step's minimum, most often just the winning move -- no key survived the move and
        // the bound went open on every step (c3nl: 4000 of 5400 waves walked their targets,
        // 0.47 ms/step).  The record's minimum and key list stay the census waves' (k_step's
        // windows); this key only bounds.  (The scoring loop carries each lane's argmin in two
        // registers, in this instantiation only; re-scoring the lane's two partitions to find
        // it again cost every scored wave of a c3nl scan ~1 us per unit.)
        if (bk_on) {
            const bool needL = !hasL && a.allow_leader && __ballot(lL < HUGE_VAL);
            const bool needN = !hasN && __ballot(lN < HUGE_VAL);
            const double wL = needL ? wave_min(lL) : HUGE_VAL, wN = needN ? wave_min(lN) : HUGE_VAL;
            const unsigned long long bl = needL ? __ballot(lL == wL) : 0ull, bn = needN ? __ballot(lN == wN) : 0ull;
            const bool myL = bl && lane == __ffsll((long long)bl) - 1, myN = bn && lane == __ffsll((long long)bn) - 1;
            if ((myL && enc(wL) < s_bke[0][wid]) || (myN && enc(wN) < s_bke[1][wid])) {
                // (the lane's argmin from the scoring loop: the first (partition, slot) in
                // scoring order with the wave minimum, as a re-scoring would find it)
#pragma unroll
                for (int kind = 0; kind < 2; kind++) {
                    if (!(kind ? myN : myL)) continue;
                    const unsigned long long e = enc(kind ? wN : wL);
                    if (!(e < s_bke[kind][wid])) continue;
                    const uint32_t am = kind ? amN : amL;
                    const int tb = (int)(am >> 8), jm = (int)((am >> 4) & 15u), km = (int)(am & 15u);
                    uint32_t src = 0;
                    double wj = 0.0;
#pragma unroll
                    for (int jj = 0; jj < PER_LANE; jj++) {
                        if (jj == jm) wj = P.wt(jj);
#pragma unroll
                        for (int kk = 0; kk < RC; kk++) if (jj == jm && kk == km) src = P.rp(kk, jj);
                    }
                    Contender c;
                    c.s = (int)src; c.t = tb; c.w = wj; c.kind = kind; c.pad = 0;
                    c.iter = ((unsigned long long)(base + jm) << 21) | ((unsigned long long)km << 16) |
                             (unsigned long long)s_pos[tb];
                    s_bke[kind][wid] = e; s_bkc[kind][wid] = c;
                }
            }
        }
#ifdef KB_WALK_COUNTS
        if (lane == 0) {
            KB_COUNT(a.ctl, 7, 1);                                  // waves scored
            if (hasL || hasN) KB_COUNT(a.ctl, 15, 1);               // waves past the ub gate
        }
#endif
        if (!census_off && ((hasL && lL <= tL + 8.0 * eps) || (hasN && lN <= tN + 8.0 * eps))) {
            const unsigned long long cz0 = a.wgt ? clock64() : 0ull;
            // the (partition, slot) pairs within 8*eps of the wave minimum, as bits j*16 + slot
            uint32_t todo = 0;
#pragma unroll
            for (int j = 0; j < PER_LANE; j++) {
                const uint32_t m = P.mt(j);
                const int nrep = (int)meta_nrep(m);
                if (base + j >= a.shard_end || !meta_elig(m) || nrep == 0) continue;
                uint32_t reps[RC];
#pragma unroll
                for (int k = 0; k < RC; k++) reps[k] = P.rp(k, j);
                int nelig;
                const int tb = first_target<RC, LSETS>(a, s_set, set_of<RC, LSETS>(P, j), reps, nrep, &nelig);
                if (tb < 0) continue;
                const double delta = P.wt(j) * inv_avg;
                const double dt = dtgt_f(s_rf[tb], delta);
                if (hasL && a.allow_leader && dsrc_f(s_rf[reps[0]], delta) + dt <= tL + 8.0 * eps)
                    todo |= 1u << (j * 16);
#pragma unroll
                for (int k = 1; k < RC; k++)
                    if (hasN && k < nrep && dsrc_f(s_rf[reps[k]], delta) + dt <= tN + 8.0 * eps)
                        todo |= 1u << (j * 16 + k);
            }
            const unsigned long long cz1 = a.wgt ? clock64() : 0ull;
            // one walk call site (a compact, rarely executed code path)
            while (todo) {
                const int bit = __ffs(todo) - 1;
                todo &= todo - 1;
                const int j = bit >> 4, k = bit & 15;
                const uint32_t m = P.mt(j);
                const double w = P.wt(j);
                uint32_t reps[RC];
#pragma unroll
                for (int q2 = 0; q2 < RC; q2++) reps[q2] = P.rp(q2, j);
                uint32_t src = reps[0];
#pragma unroll
                for (int q2 = 1; q2 < RC; q2++) src = k == q2 ? reps[q2] : src;
                const int nrep = (int)meta_nrep(m), set = (int)set_of<RC, LSETS>(P, j);
                // (the record's fields: LDS reads where it is staged -- a runtime index into
                // a register copy of its units went through scratch)
                uint4 R[LSETS ? 1 : U];
                if (!LSETS) set_record<RC, LSETS>(a, s_set, (uint32_t)set, *(uint4(*)[U])R);
                const uint16_t* rs = (const uint16_t*)(s_set + (size_t)set * U);
                auto ent = [&](int idx) -> uint32_t {
                    if constexpr (LSETS) return rs[idx];
                    else return rec_u16(*(const uint4(*)[U])R, idx);
                };
                const double ds = dsrc_f(s_rf[src], w * inv_avg);
                walk_targets<RC>(a, T, s_rf, s_pos, s_blm, ent, k ? 1 : 0, base + j, k, (int)src, reps, nrep,
                                      set, w, ds, k ? tN : tL, eps, inv_avg, nblm);
            }
            if (a.wgt && lane == __ffsll((long long)__ballot(1)) - 1) {   // (the census lanes' first)
                const unsigned long long cz2 = clock64();
                atomicAdd(&s_cz[0], cz2 - cz0); atomicAdd(&s_cz[1], 1ull); atomicAdd(&s_cz[2], cz2 - cz1);
            }
        }
        wgL = tL < wgL ? tL : wgL;
        wgN = tN < wgN ? tN : wgN;
    };

    // ping-pong between two register sets: A and Bq; while one unit is scored, the next
    // one's loads are in flight.  A unit is one wave's 128 partitions: of this
    // workgroup's tiles (full round: A was issued by the caller before the tables;
    // issuing the second tile early as well was measured slower, 10.6 vs 10.2 us per c3
    // scan), or of the blocks an incremental round reads: the blocks in
    // descending wmax order, dealt wave-major across the workgroups (the few heavy
    // blocks land in different workgroups, whose near-tie tables they would otherwise
    // crowd); a block lighter than wskip holds no candidate within the census window
    // (k_step's certificate), and every later block is lighter still.
    // (the unit bases are wave-uniform: scalar registers; the lane adds its offset)
    const int widu = __builtin_amdgcn_readfirstlane(wid);
    const long long lofs = (long long)lane * PER_LANE;
    const long long i0 = (long long)widu * a.nscan + wg, istep = (long long)a.nscan * NW;
    auto unit = [&](long long k) -> long long {     // base of this wave's k-th unit, or -1
        if (!INCR || !q.incr) {
            const long long t = (long long)tile + k * a.nscan;
            return t < a.ntiles && widu < a.twaves ? a.shard_begin + t * ((long long)a.twaves * BLK) + (long long)widu * BLK : -1;
        }
        const long long i = i0 + k * istep;
        if (i >= a.nblk) return -1;
        const BlockDesc d = ldobj(a.bdesc + i);
        return d.wmax >= q.wskip ? d.blk * BLK : -1;
    };
    PartRaw<RC> Bq;
    // (an incremental round's first unit and its loads were issued by the caller)
    long long c0 = INCR && q.incr ? c0_in : unit(0), nu = 0;
    // (the prefetch is unconditional -- a last unit re-loads itself -- so that the
    // compiler waits for exactly the older unit's loads: vmcnt(N), not vmcnt(0))
    for (long long k = 0; c0 >= 0; k += 2) {
        const long long c1 = unit(k + 1);
        load_parts<RC, LSETS>(a, (c1 >= 0 ? c1 : c0) + lofs, Bq);
        score(A, c0 + lofs);
        nu++;
        if (c1 < 0) break;
        const long long c2 = unit(k + 2);
        load_parts<RC, LSETS>(a, (c2 >= 0 ? c2 : c1) + lofs, A);
        score(Bq, c1 + lofs);
        nu++;
        c0 = c2;
    }
    if (INCR && q.incr && !a.ubpass && lane == 0 && nu) atomicAdd(&ctl->total_blocks, (unsigned long long)nu);
    // workgroup record: counts, first-index predicates, minima, near-tie keys
    // (a wave's counts fit 32 bits unless the workgroup has tens of thousands of units:
    // a 32-bit reduction is one DPP add per step against two moves and a carry chain)
    const long long upw = (long long)(a.ntiles + a.nscan - 1) / a.nscan + (INCR ? (long long)a.nblk / ((long long)a.nscan * NW) + 1 : 0);
    if (upw * (PER_LANE * 64) * a.B * RC < (1ll << 32)) {
        cL = wave_sum((uint32_t)cL);
        cN = wave_sum((uint32_t)cN);
    } else {
        cL = wave_sum(cL);
        cN = wave_sum(cN);
    }
    bool anyf = false;
#pragma unroll
    for (int f = 0; f < NF; f++) { fst[f] = s_fw[wid][f]; anyf |= fst[f] != NONE32; }
    if (__ballot(anyf)) {                          // first-index predicates are rare
#pragma unroll
        for (int f = 0; f < NF; f++) fst[f] = wave_min(fst[f]);
    }
    __shared__ double s_wm[2][NW];
    if (lane == 0) {
        s_c[0][wid] = cL; s_c[1][wid] = cN;
        s_wm[0][wid] = wgL; s_wm[1][wid] = wgN;
#pragma unroll
        for (int f = 0; f < NF; f++) s_f[f][wid] = fst[f];
    }
    __syncthreads();   // also orders every census insert before the flush
    const unsigned long long t_sc = a.wgt ? wall_clock64() : 0ull;
    // the wave partials, combined lane-parallel by the waves that use them (the key
    // flush below: waves 0..3, one per SIMD)
    if (wid < DEDUP_SCAN / 64) {
        wgL = wave_min(lane < NW ? s_wm[0][lane] : HUGE_VAL);
        wgN = wave_min(lane < NW ? s_wm[1][lane] : HUGE_VAL);
    }
    RecHdr* hdr = a.R.h(wg);
    Contender* keys = a.R.k(wg);
    // the near-tie keys within 4*eps of the workgroup minima; the minimum-score key
    // per kind (smallest table slot among equal scores) goes into the header
    static_assert(DEDUP_SCAN <= SCAN_THREADS, "one table slot per thread");
    int myh = -1, mykind = 0;
    unsigned long long myenc = NONE64;
    if (tid < DEDUP_SCAN && s_key[tid] != NONE32 && s_wb[tid] != NONE64) {
        const Contender c = dedup_entry(T, tid);
        const double g = c.kind == 0 ? wgL : wgN;
        const double dl = c.w * inv_avg;
        const double d = dsrc_f(s_rf[c.s], dl) + dtgt_f(s_rf[c.t], dl);
        if (d <= g + 4.0 * eps) {
            myh = tid; mykind = c.kind; myenc = enc(d);
            atomicMin(&s_benc[c.kind], myenc);
            atomicAdd(&s_nkk[c.kind], 1u);
            const uint32_t k = atomicAdd(&s_nk, 1u);
            if (k < (uint32_t)TILE_KEYS) stobj_wt(&keys[k], c);
            else emit_global(a, c);
        }
    }
    __syncthreads();
    if (myh >= 0 && myenc == s_benc[mykind]) atomicMin(&s_bslot[mykind], (uint32_t)myh);
    __syncthreads();
    static_assert((NF * NW) % 64 == 0 && 64 % NW == 0, "(predicate, wave) partials in whole waves");
    if (wid == 0) {
        cL = wave_sum(lane < NW ? s_c[0][lane] : 0ull);
        cN = wave_sum(lane < NW ? s_c[1][lane] : 0ull);
        uint32_t fm = 0;
#pragma unroll
        for (int c0 = 0; c0 < NF * NW; c0 += 64) {
            const uint32_t fv = (&s_f[0][0])[c0 + lane];     // s_f[f][w] at f * NW + w
            if (__ballot(fv != NONE32)) {
#pragma unroll
                for (int f = c0 / NW; f < (c0 + 64) / NW; f++) {
                    fst[f] = wave_min((c0 + lane) / NW == f ? fv : NONE32);
                    fm |= fst[f] != NONE32 ? 1u << f : 0u;
                }
            }
        }
        // each kind's best key outside the census (BK plans): the first wave holding the
        // smallest, found lane-parallel (one lane per wave) rather than by lane 0 alone
        int bkw[2] = {-1, -1};
        if constexpr (BK) {
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const unsigned long long e = lane < NW ? s_bke[k][lane] : NONE64;
                const unsigned long long m = wave_min(e);
                const unsigned long long bb = __ballot(lane < NW && e == m && m != NONE64);
                bkw[k] = bb ? __ffsll((long long)bb) - 1 : -1;
            }
        }
      if (lane == 0) {
        RecHdr r;
        r.dmin[0] = wgL; r.dmin[1] = wgN;
        r.cand[0] = cL; r.cand[1] = cN;
        r.nkeys = s_nk < (uint32_t)TILE_KEYS ? s_nk : (uint32_t)TILE_KEYS;
        r.flags = 0;
        r.fmask = fm;
        r.nkk[0] = (uint16_t)min(s_nkk[0], 0xFFFFu);
        r.nkk[1] = (uint16_t)min(s_nkk[1], 0xFFFFu);
#pragma unroll
        for (int k = 0; k < 2; k++) {
            if (s_bslot[k] != NONE32) { r.best[k] = dedup_entry(T, (int)s_bslot[k]); continue; }
            // no census key: the best key of the waves outside the census (or none; plans
            // with -allow-leader keep no such keys)
            const int bw = bkw[k];
            if (bw >= 0) r.best[k] = s_bkc[k][bw];
            else { r.best[k].s = r.best[k].t = -1; r.best[k].w = 0.0; r.best[k].iter = NONE64; r.best[k].kind = k; r.best[k].pad = 0; }
        }
        stobj_wt(hdr, r);
        if (a.wgt) {
            unsigned long long* o = a.wgt + 6 * wg;
            o[0] = t_in; o[1] = t_sc; o[2] = wall_clock64(); o[3] = s_cz[0]; o[4] = s_cz[1]; o[5] = s_cz[2];
        }
        if (a.pred) {
            // k_pair: the record's minima, counts and predicate mask folded into this
            // workgroup's arrival line (performed at L2 before the arrival add: the step
            // workgroup reads the grid's reduction there after its wait)
            uint32_t* sh = a.done + (wg % PAIR_SHARDS) * PAIR_STRIDE;
            __hip_atomic_fetch_max((unsigned long long*)(sh + PRED_M0), ~enc(wgL), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_max((unsigned long long*)(sh + PRED_M1), ~enc(wgN), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cL) __hip_atomic_fetch_add((unsigned long long*)(sh + PRED_C0), cL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cN) __hip_atomic_fetch_add((unsigned long long*)(sh + PRED_C1), cN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (fm) __hip_atomic_fetch_or(sh + PRED_FM, fm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (fm) {
            uint32_t* fo = a.R.f(wg);
#pragma unroll
            for (int f = 0; f < NF; f++) st32_wt(fo + f, fst[f]);
        }
        if (tk_on && !a.ubpass) {              // the scan's interval (kernel timing; a bound
                                               // pass before it is timed by events, mode 2)
            atomicMin(&ctl->ts_beg, t_in);
            atomicMax(&ctl->ts_end, wall_clock64());
        }
      }
    }
}

__device__ __attribute__((noinline)) void refresh_in_scan(const RefreshArgs* rfp, int pend, int kind, int from, int to,
                                                          uint32_t part, double* buf, int ng);   // (k_refresh below)
__device__ __attribute__((noinline)) void eager_refold(const RefreshArgs* rfp, int k, double* buf, int cap);

template <int RC, bool LSETS, bool INCR, bool GT, bool BK = false>
__device__ __forceinline__ void scan_kernel_body(const ScanArgs& a) {
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int s_li;
    DevCtl* ctl = a.ctl;
    // eager refolds: the last workgroups of the grid refold the brokers the last step touched
    // (their lists already edited by k_step), concurrently with the scan
    if (KB_EAGER_CODE && a.eager && (int)blockIdx.x >= a.nscan + (a.listwg ? 1 : 0)) {
        eager_refold(a.rf, (int)blockIdx.x - a.nscan - (a.listwg ? 1 : 0), (double*)smem, a.dyn_lds / 8);
        return;
    }
    // (rfpass: if the last k_step halted for exact loads, this launch is the refresh,
    // refresh_in_scan; the scanning workgroups decide with their control words below)
    auto rf_run = [&]() {
        // (the workgroups that share the refolds: the scan's and the list workgroup -- not the
        // eager workgroups, which return at once on a halted step, nor k_pair's step workgroup)
        refresh_in_scan(a.rf, ctl->pending_list, ctl->pl_kind, ctl->pl_from, ctl->pl_to, (uint32_t)ctl->pl_part,
                        (double*)smem, a.nscan + (a.listwg ? 1 : 0));
    };
    if (a.listwg && (int)blockIdx.x == a.nscan) {
        // (the pending list edit of a step halted for exact loads waits for its refresh)
        const int h = ctl->halted;
        if (a.rfpass && h == H_NEED_EXACT) rf_run();
        else if (!(a.dbg & 8) && h != H_NEED_EXACT && !(KB_EAGER_CODE && a.eager && ctl->eg_n > 0)) do_list_op(ctl, a.L, &s_li);
        return;
    }
    const unsigned long long t_in = wall_clock64();
    // the control words the round reads do not change while a scan runs (it writes only
    // the spill counters, the timing interval and the list flags): read through the
    // constant address space, they are scalar loads on lgkmcnt, outside the in-order
    // vmcnt queue of the table and tile loads (the launch's acquire makes the last
    // k_step's writes visible to the scalar cache)
    typedef const __attribute__((address_space(4))) DevCtl* CtlK;
    const CtlK cc = (CtlK)ctl;
    // a conditional bound pass returns at once unless a bound is open: decided before
    // any partition word is loaded (it runs before every scan once a plan retried)
    if (a.ubpass == 1) {                 // (2: the sharded engines' tightening pass, every scan)
        const double ubL = cc->ub[0], ubN = cc->ub[1];
        const int h = cc->halted;
        if (!(ubN == HUGE_VAL || (a.allow_leader && ubL == HUGE_VAL))) {
            if (a.rfpass && h == H_NEED_EXACT) rf_run();
            return;
        }
    }
    // One round trip: the control words, the lookup tables and the first tile, issued in
    // that order in one straight-line block (no short-circuit between the control words,
    // clamped indices): vmcnt drains in issue order, so a load behind a branch on an
    // earlier load's value would wait for everything issued before it -- the first tile
    // included -- and each such split costs a round trip per workgroup.
    // (incremental kernel: the control block decides first whether the tiles are read)
    ScanParams q;
    const int c_halted = cc->halted, c_prepped = cc->prepped, c_steps = cc->steps, c_budget = cc->budget;
    q.inv_avg = cc->inv_avg; q.eps = cc->eps;
    q.ubL = cc->ub[0]; q.ubN = cc->ub[1];
    q.heavy = cc->heavy; q.nblm = cc->nblm;
    q.tk_on = cc->tk_on;
    q.rlo = cc->rlo; q.rhi = cc->rhi;
    const int c_incr_ok = cc->incr_ok, c_ub_sub = cc->ub_sub;
    q.fp = cc->fp;
    q.fp_t0 = cc->fp_t[0]; q.fp_t1 = cc->fp_t[1];
    q.fp_o0 = cc->fp_o[0]; q.fp_o1 = cc->fp_o[1];
    q.fp_u0 = cc->fp_u[0]; q.fp_u1 = cc->fp_u[1];
    q.fp_n0 = cc->fp_n[0]; q.fp_n1 = cc->fp_n[1];
    const double c_wskip = cc->wskip;
    TabRaw TR;
    const int nu = LSETS ? a.nsets * sr_units(RC) : 0;
    TR.pre = !GT && a.B <= SCAN_THREADS && nu <= SCAN_THREADS;
    if (TR.pre) {
        const int i = min((int)threadIdx.x, a.B - 1);
        TR.r = ldd(a.r + i);
        TR.pos = (int32_t)ld32(a.posm + i);
        if (LSETS) TR.set = ldobj(a.setrec + ((int)threadIdx.x < nu ? (int)threadIdx.x : 0));
    }
    PartRaw<RC> A;
    const bool own0 = (int)blockIdx.x < a.ntiles && (int)(threadIdx.x >> 6) < a.twaves;
    const long long a0 = own0 ? a.shard_begin + (long long)blockIdx.x * a.twaves * BLK + (long long)threadIdx.x * PER_LANE
                              : a.shard_begin + (long long)threadIdx.x * PER_LANE;
    // (unconditional: a branch here would make the table loads wait for the tile's;
    // every scanning wave has a first unit, an idle wave loads the shard's first tile,
    // and the arrays are padded by two tiles)
    if (!INCR) load_parts<RC, LSETS>(a, a0, A);
    __builtin_amdgcn_sched_barrier(0);                 // (no use of a control word moves above the loads)
    // incremental kernel: this wave's first block descriptor goes out with the control
    // block; the block's partition words follow as soon as both are in (two round trips
    // before the first score, none of them behind the table staging)
    BlockDesc d0;
    d0.wmax = -1.0; d0.blk = 0;
    const long long i0 = (long long)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) * a.nscan + blockIdx.x;
    if (INCR && i0 < a.nblk) d0 = ldobj(a.bdesc + i0);
    q.run = c_halted == H_RUN && c_prepped && c_steps < c_budget;
    if (a.rfpass && c_halted == H_NEED_EXACT) { rf_run(); return; }   // (the tile loads are dropped)
    q.ubpass = 0;
    // (a conditional bound pass launched on the block list of the last records' best
    // keys: those blocks only, when k_step left one, else every tile)
    q.incr = INCR && (a.ubpass ? c_ub_sub > 0 : c_incr_ok);
    q.wskip = INCR && !a.ubpass ? c_wskip : 0.0;
    long long c0 = -1;
    if (INCR && !q.incr && own0) load_parts<RC, LSETS>(a, a0, A);
    if (INCR && q.incr && d0.wmax >= q.wskip) {
        c0 = d0.blk * BLK;
        load_parts<RC, LSETS>(a, c0 + (long long)(threadIdx.x & 63) * PER_LANE, A);
    }
    scan_round<RC, LSETS, INCR, GT, BK>(a, q, smem, A, TR, t_in, (int)blockIdx.x, c0);
}

template <int RC, bool LSETS, bool INCR, bool GT = false>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan(ScanArgs a) {
    scan_kernel_body<RC, LSETS, INCR, GT>(a);
}

// --------------------------------------------------------------- k_step

struct Decision {
    int32_t status, step, kind, slot;
    long long part;
    int32_t from, to;
    double su, cu;
    double w;                       // move(): the partition weight of the winning key
    int32_t exact, err, err_broker, pad;
};

// broker flags (bfl / s_fl)
constexpr uint8_t BF_PRESENT = 1, BF_INCFG = 2, BF_DIRTY = 4, BF_TOUCHED = 8;

// the relative load the prep wrote to r[] for a bl_move broker, recomputed
// bit-identically from the load (same operands, same fused operation)
__device__ __forceinline__ double rel_ld(const double* s_ld, int b, double inv_avg) {
    return __fma_rn(s_ld[b], inv_avg, -1.0);
}
__device__ __forceinline__ double cont_delta_ld(const double* s_ld, const Contender& c, double inv_avg) {
    const double delta = c.w * inv_avg;
    return dsrc(rel_ld(s_ld, c.s, inv_avg), delta) + dtgt(rel_ld(s_ld, c.t, inv_avg), delta);
}

// every near-tie contender of `kind` within 4*eps of g: the keys of the
// records whose minimum is within 8*eps, then the raw spill buffer
template <typename F>
__device__ __forceinline__ void for_each_contender(const StepArgs& a, const double* s_ld, uint32_t ncont, int kind, double g,
                                   double eps, double inv_avg, F f) {
    const int nt = blockDim.x;
    for (int i = threadIdx.x; i < a.R.n; i += nt) {
        const RecHdr* h = a.R.h(i);
        if (!(ldd(&h->dmin[kind]) <= g + 8.0 * eps)) continue;
        const Contender* keys = a.R.k(i);
        const int nk = (int)min(ld32(&h->nkeys), (uint32_t)a.R.cap);
        for (int k = 0; k < nk; k++) {
            const Contender c = ldobj(keys + k);
            if (c.kind != kind) continue;
            if (cont_delta_ld(s_ld, c, inv_avg) <= g + 4.0 * eps) f(c);
        }
    }
    if (a.use_spill) {
        const uint32_t n = min(ncont, a.cont_cap);
        for (uint32_t i = threadIdx.x; i < n; i += nt) {
            const Contender c = ldobj(a.cont + i);
            if (c.kind != kind) continue;
            if (cont_delta_ld(s_ld, c, inv_avg) <= g + 4.0 * eps) f(c);
        }
    }
}

// Incremental mode: the certificate that lets the next scan skip whole
// partition blocks.  Every candidate of a partition with weight w scores at least
// LB(w / avg) (scan_round's lower-bound prune, over the range [rlo, rhi] of r[]), and LB
// is convex with LB(0) = 0.  Find dl > 0 with LB(dl) > thr (thr = the census window
// ub + 16 eps, the same bound the per-partition prune uses) and LB'(dl) < 0 (with a
// margin for the rounding of the slope): LB then decreases on [0, dl], so every weight
// w <= dl * avg scores above the window.  Wave 0 tries a 64 x 64 grid of
// [0, (rhi - rlo) / 2] (the minimum of LB lies below its midpoint) and keeps the
// largest certified point.  Returns the weight bound (blocks with wmax below it need no
// scan), 0 when nothing can be skipped; fl(wskip / avg) <= dl, as the scan computes it.
__device__ double incr_wskip(double rlo, double rhi, double thr, double avg, double iav, int lane) {
    if (!(thr < 0.0) || !(rhi > rlo) || !(avg > 0.0) || !(iav > 0.0)) return 0.0;
    const double fmn = fsq(rlo), fmx = fsq(rhi);
    auto ok = [&](double dl) {
        const double lb = (fsq(rhi - dl) - fmx) + (fsq(rlo + dl) - fmn);
        const double x1 = rhi - dl, x2 = rlo + dl;
        const double slope = (x2 > 0.0 ? 2.0 * x2 : x2) - (x1 > 0.0 ? 2.0 * x1 : x1);
        return lb > thr && slope < -1e-14 * (fabs(x1) + fabs(x2));
    };
    const double h = 0.5 * (rhi - rlo) / 64.0;
    const double d1 = h * (double)(lane + 1);
    unsigned long long bal = __ballot(ok(d1));
    double best = 0.0;
    if (bal) best = __shfl(d1, 63 - __clzll(bal));
    const double d2 = best + (h / 64.0) * (double)(lane + 1);
    bal = __ballot(ok(d2));
    if (bal) best = fmax(best, __shfl(d2, 63 - __clzll(bal)));
    if (!(best > 0.0)) return 0.0;
    double ws = best * avg;
    for (int it = 0; it < 16 && ws * iav > best; it++) ws *= 1.0 - 0x1p-50;
    return ws * iav <= best ? ws : 0.0;
}

#ifndef KB_FPABL
#define KB_FPABL 0   // diagnostic timing builds of the fast prep (1: no merge, 2: no counts / marks)
#endif
// the frozen average is folded again from scratch every FRZ_MAX steps (k_step's prep)
constexpr int FRZ_MAX = 1024;

#ifndef KB_SET_G
#define KB_SET_G 2   // records a wave rebuilds at once in the fused prep (A/B: 2 beat 4 and 1 at c3)
#endif

#ifndef KB_CLIST
#define KB_CLIST 1   // exact folds over a compact contender list (0: the table walk only; A/B)
#endif

// the control block lives in LDS for the whole k_step (one load round trip at the
// start, stores only at the end): the serial code never waits on a global RMW
constexpr int CTL_WORDS = (int)(offsetof(DevCtl, stamps) / 4);

// The serial half of one Balance() step (k_step): stage the control block, the
// broker tables and the allowed-set words in LDS, resolve the scan records (when
// prepped), apply the change and prep the next step.
template <bool BIG, bool GB, bool FUSED = false>
__device__ __forceinline__ void step_body(const StepArgs& a, DevCtl& C) {
    DevCtl* ctl = a.ctl;
    constexpr int MB = GB ? MAXB_G : MAXB;          // (GB: the per-broker tables in memory, a.gscr)
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    constexpr int NW = STEP_THREADS / 64;
    unsigned long long t_in = wall_clock64();       // (FUSED: reset when the scan is in)
    KB_STAMP_BEGIN();
    __shared__ unsigned long long s_span_from;      // (kernel timing: the scan's end, or 0)
    __shared__ unsigned long long s_pair_from;      // (k_pair: its first workgroup's start, or 0)
    // diagnostic phase stops: a -DKB_STOP_AT=k build returns after phase k (the code
    // after it is dead there); kb_engine_bench_step times such builds on a fixed input
#ifdef KB_STOP_AT
#define KB_STOP(k) do { if ((k) == KB_STOP_AT) { write_back(); return; } } while (0)
#else
#define KB_STOP(k) (void)0
#endif
    __shared__ Decision D;
    __shared__ int s_done, s_i, s_exact_need, s_retry, s_nT, s_unc, s_nblm;
    __shared__ unsigned long long s_u[NW];
    __shared__ double s_dv[NW];
    __shared__ int s_bs[NW], s_bt[NW];
    __shared__ double s_bw[NW];
    __shared__ double s_g[2];
    __shared__ unsigned long long s_cand[2];
    __shared__ uint32_t s_first[NF];
    __shared__ uint32_t s_flags, s_fm;
    __shared__ int s_kc[2], s_sok[2];
    __shared__ Contender s_single[2];
    __shared__ double s_sux;
    __shared__ __align__(16) double s_fold[NW * 64];   // per-wave rows of the exact folds
    __shared__ uint32_t s_key[DEDUP_STEP];
    __shared__ unsigned long long s_wb[DEDUP_STEP], s_it[DEDUP_STEP];
    extern __shared__ __align__(16) unsigned char dsm_lds[];
    unsigned char* dsm;
    if constexpr (GB) dsm = a.gscr; else dsm = dsm_lds;
    const StepLds LY = step_lds(a.B, a.NP2, a.sb_lds ? a.nsets * a.W64 : 0);
    double* s_ld = (double*)dsm;                     // loads by broker id
    double* s_e = (double*)(dsm + LY.e);             // load error bounds; zero whenever every load is
                                                     // exact, so then also sort keys / exact bl loads
    int32_t* s_ord = (int32_t*)(dsm + LY.ord);       // universe order by (load, id)
    uint64_t* s_sb = (uint64_t*)(dsm + LY.sb);       // allowed-set words (sb_lds)
    uint8_t* s_fl = dsm + LY.fl;                     // BF_* flags
    __shared__ int s_T[TMAX], s_posT[TMAX];
    __shared__ double s_Lold[TMAX], s_ebold[TMAX];  // touched brokers' load / bound before the apply
    __shared__ int s_memb;                          // the apply changed bl_move's membership
    __shared__ int s_cntT[TMAX];
    __shared__ uint64_t s_blmb[MB / 64], s_presb[MB / 64];
    __shared__ uint32_t s_smark[MAX_SETS / 32];
    __shared__ int s_nd[2], s_li[2], s_kfail[2];
    __shared__ int s_fpfail, s_fpnsub;
    __shared__ unsigned long long s_fpub[2];
    __shared__ double s_fpz[9];
    __shared__ __align__(16) uint16_t s_mrow[NW][8 * FP_MAXU];   // the fast prep's merged records, one row per wave
    Dedup T{s_key, s_wb, s_it, DEDUP_STEP, s_nd, s_li};
    const int B = a.B;

    // ---- one memory round trip: the control block, the broker state and the allowed-set
    // words (plain loads then LDS writes: at B <= 1024 one load of each array per thread,
    // all issued before the first LDS write; measured faster than LDS-DMA of the same
    // bytes, 16.5 vs 19.9 us per k_step at c3).  The record headers come to registers.
    auto stage_tables = [&]() {
        for (int b = tid; b < B; b += STEP_THREADS) {
            s_ld[b] = a.load[b];
            s_e[b] = a.eb[b];
            s_fl[b] = a.bfl[b];
            s_ord[b] = a.order[b];
        }
    };
    // ---- deferred prep (DevCtl.fp, round 6).  The last step applied a plain move() replace
    // and left the order work of its prep to this launch: the universe order after the move
    // (its touched brokers re-sorted, getBL's (load, id) order, utils.go:107-117), the bl_move
    // positions, the order certification, and the full records of the sets holding a touched
    // broker (the last step wrote their certain prefix).  In k_pair it runs before the wait,
    // beside the scan (whose workgroups patch the positions from the descriptor); the results
    // stay in LDS (s_pm, s_rec, s_ord) and go to memory after the wait (flush_deferred: the
    // scan reads posm / setrec while it runs).  The same phases as the prep below (P1-P5).
    int32_t* s_pm = (int32_t*)(dsm + (a.fp_lds ? a.fp_lds : 0));          // bl position per broker
    uint4* s_rec = (uint4*)(dsm + (a.fp_lds ? a.fp_lds + ((B * 4 + 15) & ~15) : 0));   // set records
    Contender* s_bk = (Contender*)(s_rec + (a.fp_lds ? a.nsets * a.units : 0));   // the records' best keys (fp_bk)
    int* s_dlist = (int*)s_smark;                    // sets rebuilt (free until the resolve's exact folds)
    __shared__ int s_dp, s_dn, s_dpunc, s_dlight, s_dheavy, s_dwc[NW];
    auto stage_fp = [&]() {                          // (fp_lds: the positions and the set records)
        for (int b = tid; b < B; b += STEP_THREADS) s_pm[b] = (int32_t)ld32(a.posm + b);
        for (int i = tid; i < a.nsets * a.units; i += STEP_THREADS) s_rec[i] = ldobj(a.setrec + i);
    };
    auto deferred_prep = [&](int t0, int t1) {
        const int dnT = t1 >= 0 ? 2 : 1;
        if (tid == 0) { s_T[0] = t0; s_T[1] = t1; s_dn = 0; s_dpunc = 0; s_cntT[0] = 0; s_cntT[1] = 0; }
        __syncthreads();
        // DP1: the touched brokers' old universe positions, the sets holding one (their records
        // are rebuilt below), the bl_move bits by broker id
        if (tid < dnT) s_fl[s_T[tid]] |= BF_TOUCHED;
        for (int i = tid; i < B; i += STEP_THREADS) {
            const int b = s_ord[i];
            if (b == t0) s_posT[0] = i;
            if (b == t1) s_posT[1] = i;
        }
        for (int set = tid; set < a.nsets; set += STEP_THREADS) {
            const uint64_t* sb = s_sb + (size_t)set * a.W64;
            bool hit = (sb[t0 >> 6] >> (t0 & 63)) & 1ull;
            if (t1 >= 0) hit |= (sb[t1 >> 6] >> (t1 & 63)) & 1ull;
            if (hit) s_dlist[atomicAdd(&s_dn, 1)] = set;     // (fp_lds: nsets <= 1024 words)
        }
        for (int b0 = wid * 64; b0 < B; b0 += STEP_THREADS) {
            const int b = b0 + lane;
            const bool in = b < B && (s_fl[b] & (BF_PRESENT | BF_INCFG));
            const unsigned long long m = __ballot(in);
            if (lane == 0) s_blmb[b0 >> 6] = m;
        }
        __syncthreads();
        // DP2: per untouched element, new position = old - (touched before it) + (touched
        // below it); for each touched broker the untouched ones below it
        constexpr int NQD = (MB + STEP_THREADS - 1) / STEP_THREADS;
        int nb[NQD], np[NQD];
#pragma unroll
        for (int q = 0; q < NQD; q++) {
            nb[q] = -1; np[q] = 0;
            if (q * STEP_THREADS >= B) continue;         // uniform
            const int i = q * STEP_THREADS + tid;
            const bool in = i < B;
            const int b = in ? s_ord[i] : 0;
            const bool untouched = in && !(s_fl[b] & BF_TOUCHED);
            const double Lb = s_ld[b];
            int below = 0, before = 0;
            for (int x = 0; x < dnT; x++) {
                const int t = s_T[x];
                const double Lt = s_ld[t];
                below += ((Lt < Lb) || (Lt == Lb && t < b)) ? 1 : 0;
                before += s_posT[x] < i ? 1 : 0;
                const bool b_lt_t = untouched && ((Lb < Lt) || (Lb == Lt && b < t));
                const unsigned long long bal = __ballot(b_lt_t);
                if (lane == 0 && bal) atomicAdd(&s_cntT[x], (int)__popcll(bal));
            }
            nb[q] = untouched ? b : -1;
            np[q] = i - before + below;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NQD; q++)
            if (q * STEP_THREADS < B && nb[q] >= 0) s_ord[np[q]] = nb[q];
        if (tid < dnT) {
            const int t = s_T[tid];
            const double Lt = s_ld[t];
            int rank = 0;
            for (int x = 0; x < dnT; x++) {
                const int t2 = s_T[x];
                const double L2 = s_ld[t2];
                rank += ((L2 < Lt) || (L2 == Lt && t2 < t)) ? 1 : 0;
            }
            s_ord[s_cntT[tid] + rank] = t;
        }
        __syncthreads();
        // DP3: bl_move positions along the new order (contiguous universe positions per
        // thread, a workgroup prefix of the bl_move counts), the order certification (with
        // approximate loads neighbours must be separated by more than their bounds), the
        // lightest / heaviest bl_move brokers
        {
            constexpr int FQ = MB / STEP_THREADS;
            int c = 0;
            const int base = tid * FQ;
            bool unc = false;
#pragma unroll
            for (int q = 0; q < FQ; q++) {
                const int i = base + q;
                if (i < B) {
                    const int b = s_ord[i];
                    c += (s_fl[b] & (BF_PRESENT | BF_INCFG)) ? 1 : 0;
                    if (i + 1 < B) {
                        const int b2 = s_ord[i + 1];
                        const double e = s_e[b] + s_e[b2];
                        unc |= e > 0.0 && !(s_ld[b2] - s_ld[b] > e);
                    }
                }
            }
            if (unc) s_dpunc = 1;
            const int incl = wave_incl_scan(c);
            if (lane == 63) s_dwc[wid] = incl;
            __syncthreads();
            const int wc = lane < NW ? s_dwc[lane] : 0;
            const int woff = wave_sum(lane < wid ? wc : 0), total = wave_sum(wc);
            int pos = woff + incl - c;
#pragma unroll
            for (int q = 0; q < FQ; q++) {
                const int i = base + q;
                if (i < B) {
                    const int b = s_ord[i];
                    if (s_fl[b] & (BF_PRESENT | BF_INCFG)) {
                        if (pos == 0) s_dlight = b;
                        if (pos == total - 1) s_dheavy = b;
                        s_pm[b] = pos++;
                    } else s_pm[b] = -1;
                }
            }
        }
        // DP4: the marked sets' records (the first KR brokers of set ∩ bl_move in the new bl
        // order, steps.go:192-201 targets), two per wave so their LDS chains overlap
        {
            constexpr int G = KB_SET_G;
            const int W64 = a.W64, KR = a.KR, U = a.units;
            const unsigned long long lt = (1ull << lane) - 1ull;
            const int mn = s_dn;
            for (int g = wid * G; g < mn; g += NW * G) {
                const int ng = mn - g < G ? mn - g : G;
                const uint64_t* sb[G];
                uint16_t* rec16[G];
                int found[G];
#pragma unroll
                for (int j = 0; j < G; j++) {
                    const int set = s_dlist[g + (j < ng ? j : 0)];
                    sb[j] = s_sb + (size_t)set * W64;
                    rec16[j] = (uint16_t*)(s_rec + (size_t)set * U);
                    found[j] = j < ng ? 0 : KR;
                }
                for (int base = 0; base < B; base += 64) {
                    bool need = false;
#pragma unroll
                    for (int j = 0; j < G; j++) need |= found[j] < KR;
                    if (!need) break;
                    const int k = base + lane;
                    const int b = s_ord[k < B ? k : 0];
                    const bool inb = k < B && ((s_blmb[b >> 6] >> (b & 63)) & 1ull);
                    uint64_t wj[G];
#pragma unroll
                    for (int j = 0; j < G; j++) wj[j] = sb[j][b >> 6];
#pragma unroll
                    for (int j = 0; j < G; j++) {
                        const bool mem = inb && ((wj[j] >> (b & 63)) & 1ull);
                        const unsigned long long m = __ballot(mem);
                        if (mem && found[j] < KR && j < ng) {
                            const int rk = found[j] + (int)__popcll(m & lt);
                            if (rk < KR) rec16[j][2 + rk] = (uint16_t)b;
                        }
                        found[j] += (int)__popcll(m);
                    }
                }
#pragma unroll
                for (int j = 0; j < G; j++) {
                    if (j >= ng) break;
                    for (int rk = found[j] + lane; rk < KR; rk += 64) rec16[j][2 + rk] = NONE16;
                    // (|set ∩ bl_move|, rec16[0], is unchanged: a plain replace keeps bl_move)
                    if (lane == 0) rec16[j][1] = (uint16_t)(found[j] < KR ? found[j] : KR);
                }
            }
        }
        if (tid < dnT) s_fl[s_T[tid]] &= ~BF_TOUCHED;
        __syncthreads();
    };
    // the deferred prep's tables to memory (after the wait: the scan read the old ones), by
    // threads t0, t0 + nt, ... -- on the fast path by the waves the apply leaves idle, else
    // before the first phase that reads them from memory (the general resolve) or at the end
    __shared__ int s_flushed;
    auto flush_deferred = [&](int t0, int nt) {
        for (int i = t0; i < B; i += nt) {
            const int b = s_ord[i];
            a.order[i] = b;
            a.posu[b] = i;
            const int p = s_pm[i];
            st32(a.posm + i, (uint32_t)p);
            if (p >= 0) st32(a.blm + p, (uint32_t)i);
        }
        const int U = a.units, n = s_dn * U;
        for (int q = t0; q < n; q += nt) {
            const int j = q / U, u = q - j * U;
            const int set = s_dlist[j];
            stobj(a.setrec + (size_t)set * U + u, s_rec[(size_t)set * U + u]);
        }
    };
    auto write_back = [&]() {
        KB_STAMP_FLUSH(ctl);
        __syncthreads();
        // (a deferred prep whose tables no earlier phase of this launch flushed)
        if (s_dp && !s_flushed) flush_deferred(tid, STEP_THREADS);
        unsigned long long t_out = 0;
        if (tid == 0 && C.tk_on) {
            // kernel timing: this launch (the scan's interval was folded in at the start:
            // a load here would wait for every store this thread issued)
            t_out = wall_clock64();
            C.tk_sum[1] += t_out - t_in;
            C.tk_n[1]++;
            if (s_span_from) { C.tk_span[1] += t_out - s_span_from; C.tk_span_n[1]++; }
            if (s_pair_from && t_out > s_pair_from) { C.tk_pair += t_out - s_pair_from; C.tk_pair_n++; }
        }
        __syncthreads();
        if (tid < CTL_WORDS) ((uint32_t*)ctl)[tid] = ((const uint32_t*)&C)[tid];
        if (tid == 0 && t_out) ctl->ts_prev_end = t_out;
    };
    if (tid == 0) { s_dp = 0; s_flushed = 0; }
    unsigned long long ts_b, ts_e, ts_pe;
    if constexpr (FUSED) {
        // k_pair's step workgroup (a resident workgroup of the scan's grid): the broker tables
        // and the allowed-set words are staged while the scan runs -- nothing changes them
        // then but the eager refolds of the last step's touched brokers (re-read below) and an
        // in-stream refresh (a step halted for exact loads: everything is staged again) --
        // then it waits for every other workgroup of the grid (scan, list, eager) to finish
        if (a.fuse_pre) stage_tables();
        if (a.sb_lds) {
            const int nq = a.nsets * a.W64;
            for (int q = 2 * tid; q < nq; q += 2 * STEP_THREADS) {
                if (q + 1 < nq) *(uint4*)(s_sb + q) = *(const uint4*)(a.setbits + q);
                else s_sb[q] = a.setbits[q];
            }
        }
        if (a.fp_lds) {
            // this state's bl positions and set records (the fast prep's inputs); a deferred
            // prep of the last move runs now, beside the scan (its control words do not change
            // while the scan runs; with eager refolds the touched brokers' loads do: after the
            // wait then)
            stage_fp();
            KB_STAMP(ctl, 7);
            if (a.fuse_pre && !a.eager && ctl->fp && ctl->halted == H_RUN && !ctl->full_prep) {
                deferred_prep(ctl->fp_t[0], ctl->fp_t[1]);
                if (tid == 0) s_dp = 1;
            }
            KB_STAMP(ctl, 15);
        }
        __shared__ int s_prehalt;
        int egb = -1;
        if (tid < EGW) {
            const int n = ctl->eg_n;
            egb = tid < n ? ctl->eg_b[tid] : -1;
        }
        __shared__ int s_wait_to;
        if (wid == 0) {
            if (lane == 0) s_prehalt = ctl->halted;
            // the arrival count is sharded over PAIR_SHARDS words (a workgroup adds to the
            // shard of blockIdx % 8, the blocks that share an XCD: 32 arrivals per word instead
            // of 255 serialised on one); lanes 0..7 poll one shard each.  (A bounded wait: 2 s
            // of the 100 MHz clock, orders of magnitude past any scan -- on expiry the plan
            // stops with an error instead of spinning on)
            const unsigned long long t0 = wall_clock64();
            int to = 0;
            for (;;) {
                // (the bound is tested first: a zero bound -- the tests' forced timeout --
                // gives up before the first poll)
                if (wall_clock64() - t0 >= a.wait_ticks) { to = 1; break; }
                const uint32_t v = lane < PAIR_SHARDS
                    ? __hip_atomic_load(a.wait_cnt + lane * PAIR_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
                if (wave_sum(v) >= (uint32_t)a.wait_n) break;
                __builtin_amdgcn_s_sleep(1);
            }
            // (tried: every handed-off byte read with sc1 loads instead of this acquire, the
            // producers' stores being write-through already -- c3 2 us per step slower, the
            // record and key loads as 8-byte atomic loads)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // (the other XCDs' writes)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // the grid's record reduction (ScanArgs.pred: every scanning workgroup folded its
            // record's minima, counts and predicate mask into its arrival line before counting
            // in), read once the count is complete, then every word of the line reset
            unsigned long long m0 = 0, m1 = 0, c0 = 0, c1 = 0;
            uint32_t fm = 0;
            if (!to && lane < PAIR_SHARDS) {
                uint32_t* sh = a.wait_cnt + lane * PAIR_STRIDE;
                m0 = __hip_atomic_load((unsigned long long*)(sh + PRED_M0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                m1 = __hip_atomic_load((unsigned long long*)(sh + PRED_M1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                c0 = __hip_atomic_load((unsigned long long*)(sh + PRED_C0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                c1 = __hip_atomic_load((unsigned long long*)(sh + PRED_C1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                fm = __hip_atomic_load(sh + PRED_FM, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            m0 = wave_red_max(m0); m1 = wave_red_max(m1);
            c0 = wave_sum(c0); c1 = wave_sum(c1);
            fm = wave_red_or(fm);
            if (!to && lane < PAIR_SHARDS) {
                // (after the loads: the reductions above consumed them)
                uint32_t* sh = a.wait_cnt + lane * PAIR_STRIDE;
                __hip_atomic_store(sh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((unsigned long long*)(sh + PRED_M0), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((unsigned long long*)(sh + PRED_M1), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((unsigned long long*)(sh + PRED_C0), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((unsigned long long*)(sh + PRED_C1), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(sh + PRED_FM, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (lane == 0) {
                s_wait_to = to;
                s_g[0] = m0 ? dec(~m0) : HUGE_VAL; s_g[1] = m1 ? dec(~m1) : HUGE_VAL;
                s_cand[0] = c0; s_cand[1] = c1;
                s_fm = fm;
            }
        }
        __syncthreads();
        if (s_wait_to) {
            if (tid == 0) {
                ChangeDev ch;
                ch.status = -1; ch.step = -1; ch.kind = 0; ch.slot = -1; ch.part = -1; ch.from = ch.to = -1;
                ch.su = ch.cu = 0.0; ch.exact = 0; ch.err_code = E_PAIR_TIMEOUT; ch.err_broker = -1; ch.pad = 0;
                const int lp = ctl->logpos;
                if (lp < ctl->logcap) a.log[lp] = ch;
                ctl->logpos = lp + 1;
                ctl->halted = H_DONE;
            }
            return;
        }
        t_in = wall_clock64();
        ts_b = ctl->ts_beg; ts_e = ctl->ts_end; ts_pe = ctl->ts_prev_end;
        if (tid < CTL_WORDS) ((uint32_t*)&C)[tid] = ((const uint32_t*)ctl)[tid];
        if (s_prehalt == H_NEED_EXACT || !a.fuse_pre) stage_tables();
        else if (egb >= 0 && egb < B) { s_ld[egb] = a.load[egb]; s_e[egb] = a.eb[egb]; s_fl[egb] = a.bfl[egb]; }

    } else {
    ts_b = ctl->ts_beg; ts_e = ctl->ts_end;         // (kernel timing, tk_on)
    ts_pe = ctl->ts_prev_end;
    if (tid < CTL_WORDS) ((uint32_t*)&C)[tid] = ((const uint32_t*)ctl)[tid];
    stage_tables();
    if (a.sb_lds) {
        const int nq = a.nsets * a.W64;                   // 16-B loads (the rows are contiguous)
        for (int q = 2 * tid; q < nq; q += 2 * STEP_THREADS) {
            if (q + 1 < nq) *(uint4*)(s_sb + q) = *(const uint4*)(a.setbits + q);
            else s_sb[q] = a.setbits[q];
        }
    }
    }
    KB_STAMP(ctl, 23);
    KB_STAMP(ctl, 27);
    double hd0 = HUGE_VAL, hd1 = HUGE_VAL;
    unsigned long long hc0 = 0, hc1 = 0;
    uint32_t hflg = 0, hfm = 0, hnk0 = 0, hnk1 = 0, hnks = 0;
    bool hpoison = false;
    if (tid < a.R.n) {
        const RecHdr* h = a.R.h(tid);
        hd0 = ldd(&h->dmin[0]); hd1 = ldd(&h->dmin[1]);
        hc0 = ldobj(&h->cand[0]); hc1 = ldobj(&h->cand[1]);
        hnks = ld32(&h->nkeys);
        hflg = ld32(&h->flags);
        hfm = ld32(&h->fmask);
        hpoison = !a.use_spill && (hflg & SUM_POISON);   // (a rank summary that timed out)
        hflg &= 1u;
        const uint32_t nkk = ld32(&h->nkk[0]);
        hnk0 = nkk & 0xFFFFu; hnk1 = nkk >> 16;
        // the best keys in the same round trip, straight to their LDS stash (the key count below
        // and the fast prep's upper bound read them there), not in a second round trip
        if (a.fp_lds && a.fp_bk) { s_bk[2 * tid] = ldobj(&h->best[0]); s_bk[2 * tid + 1] = ldobj(&h->best[1]); }
    }
    KB_STAMP(ctl, 28);
    dedup_clear(T);
    if (!a.use_spill && __syncthreads_or(hpoison)) {
        // some rank's summary workgroup timed out in its wait (k_scansum): its summary is not
        // this round's; every rank reads the same gathered summaries and stops here alike
        // (the rank that timed out logged the error in k_scansum and halted already)
        if (tid == 0 && ctl->halted == H_RUN) {
            ChangeDev ch;
            ch.status = -1; ch.step = -1; ch.kind = 0; ch.slot = -1; ch.part = -1; ch.from = ch.to = -1;
            ch.su = ch.cu = 0.0; ch.exact = 0; ch.err_code = E_PAIR_TIMEOUT; ch.err_broker = -1; ch.pad = 0;
            const int lp = ctl->logpos;
            if (lp < ctl->logcap) a.log[lp] = ch;
            ctl->logpos = lp + 1;
            ctl->halted = H_DONE;
        }
        return;
    }
    if (tid < 2) { s_nd[tid] = 0; s_li[tid] = -1; s_kfail[tid] = 0; }
    __syncthreads();                               // the control block copy
    if (a.fp_lds && !s_dp && C.fp && C.halted == H_RUN && !C.full_prep) {
        // (a deferred prep still pending: k_step's two-launch path, or eager refolds that changed
        // the touched brokers' loads while the scan ran)
        if (!FUSED) stage_fp();
        deferred_prep(C.fp_t[0], C.fp_t[1]);
        flush_deferred(tid, STEP_THREADS);
        if (tid == 0) { s_dp = 1; s_flushed = 1; }
        __syncthreads();
    }
    if (tid == 0 && (s_dp || C.fp)) {
        // (a pending deferred prep skipped here was for a state a full prep rebuilds)
        C.fp = 0;
        if (s_dp) { C.light = s_dlight; C.heavy = s_dheavy; }
    }
    if (s_dp && s_dpunc) {
        // the order after the last move is not certified by the load bounds: refold first
        // (as the prep's own certification does)
        __syncthreads();
        if (tid == 0) { C.halted = H_NEED_EXACT; C.prepped = 0; C.total_exact_halts++; }
        write_back();
        return;
    }
    {
        // this pair's first scan refolded the loads of a step halted for exact loads
        // (refresh_in_scan): resume as the host's refresh would, with a full prep
        const bool rfin = a.rf_final && C.halted == H_NEED_EXACT && !C.list_overflow;
        if (rfin) {
            __syncthreads();
            if (tid == 0) {
                C.halted = H_RUN; C.prepped = 0; C.full_prep = 1; C.ndirty = 0; C.want_refresh = 0;
                C.pending_list = 0;
                C.total_rf_stream++;
            }
            __syncthreads();
        }
    }
    if (tid == 0) { s_span_from = 0; s_pair_from = 0; }
    if (tid == 0 && C.tk_on) {
        // kernel timing: the interval of the scan that ran before this launch (if any), and
        // the spans: the scan's when it followed the last k_step back to back, this launch's
        // when it followed the scan (no host gap: within 10 us of the previous end); each
        // counted on its own (c5's bound passes sit between a step and the next scan)
        const unsigned long long b = ts_b, e = ts_e;
        if (FUSED && b != NONE64) s_pair_from = b;
        if (b != NONE64 && e > b) {
            C.tk_sum[0] += e - b; C.tk_n[0]++;
            if (ts_pe && b > ts_pe && b - ts_pe < 1000) { C.tk_span[0] += e - ts_pe; C.tk_span_n[0]++; }
            if (t_in > e && t_in - e < 1000) s_span_from = e;
        }
        ctl->ts_beg = NONE64;
        ctl->ts_end = 0;
    }
    const int halted = C.halted;
    const bool do_res = C.prepped && C.steps < C.budget;
    // (eager refolds: the launch that just ran refolded the last step's touched brokers and
    // did its pending list edit -- unless the step halted, then the in-stream refresh did it;
    // every thread reads the control words before thread 0 rewrites them)
    bool eg_done = false;
    if (KB_EAGER_CODE && a.eager) {
        eg_done = C.eg_n > 0 && halted == H_RUN && !C.list_overflow;
        __syncthreads();
        if (tid == 0) { if (eg_done) C.pending_list = 0; C.eg_n = 0; }
    }
    // the steps this Balance() may take (kb_engine_step's mask; SM_ALL = the whole table)
    const uint32_t sm = C.step_mask;
    const bool lead_on = a.allow_leader && (sm & SM_MOVE_LEADERS), non_on = (sm & SM_MOVE_NON_LEADERS) != 0;
    const double eps = C.eps, inv_avg = C.inv_avg, U0h = C.U0;
    const int nblm0 = C.nblm, ndirty0 = C.ndirty;
    const bool pend = !eg_done && C.pending_list != 0;   // (eg_done: thread 0 clears it)
    __shared__ long long s_moved;
    __shared__ int s_lkind, s_lpick;
    __shared__ uint32_t s_lpart;
    __shared__ int s_lrep[MAXR + 1];
    __shared__ unsigned long long s_lsb[MB / 64];
    if (tid == 0) { s_nT = 0; s_done = 0; s_exact_need = 0; s_retry = 0; s_moved = -1; s_lkind = 0; s_memb = 0; }
    // (the fast prep's counters: the deferred prep and its flush are done with them)
    if (tid == 0) { s_cntT[0] = 0; s_cntT[1] = 0; s_dn = 0; s_fpfail = 0; s_fpnsub = 0; s_fpub[0] = NONE64; s_fpub[1] = NONE64; }
    if (tid < NF) s_first[tid] = NONE32;
    if (tid < 2) { s_kc[tid] = 0; s_sok[tid] = -1; }   // (s_sok: -1 = no record offered its best key)
    if (halted != H_RUN) return;
    // the records' best keys (the single-key shortcut below): issued after the staging
    // round trip so they are not held in registers through it
    Contender hb0, hb1;
    hb0.s = hb1.s = -1;
    if (do_res && tid < a.R.n && !(a.fp_lds && a.fp_bk)) { hb0 = ldobj(&a.R.h(tid)->best[0]); hb1 = ldobj(&a.R.h(tid)->best[1]); }
    KB_STAMP(ctl, 12);
    KB_STOP(1);
    // ---- the scan records (or the gathered rank summaries): one per thread, reduced
    // per wave with DPP and across the waves by wave 0; then every thread collects
    // its record's near-tie keys of both kinds within 4*eps of the minima (distinct
    // keys, earliest iteration index per key)
    if (do_res) {
        // the first-level reductions run only on the waves holding records (one per SIMD
        // at 256 records: a wave reduction costs ~3.4x more with four waves per SIMD),
        // the second level on wave 0, published through LDS
        const int nrw = a.R.n >= STEP_THREADS ? NW : (a.R.n + 63) >> 6;
        __shared__ double s_pd[2][NW];
        __shared__ unsigned long long s_pc[2][NW];
        __shared__ uint32_t s_pf[2][NW];
        if constexpr (FUSED) {
            // k_pair: the scanning workgroups reduced their records into the arrival lines
            // (s_g / s_cand / s_fm are set from them after the wait); scan records carry no
            // overflow flag (flags == 0), only the raw spill buffer can have overflowed
            if (tid == 0) {
                if (a.incr) {
                    if (C.incr_ok) { s_cand[0] = C.cand_cache[0]; s_cand[1] = C.cand_cache[1]; }
                    else { C.cand_cache[0] = s_cand[0]; C.cand_cache[1] = s_cand[1]; }
                }
                s_flags = a.use_spill && C.cont_overflow ? 1u : 0u;
                C.last_fm = s_fm;
            }
        } else {
        if (wid < nrw) {
            double d0 = hd0, d1 = hd1;
            unsigned long long c0 = hc0, c1 = hc1;
            uint32_t flg = hflg, fm = hfm;
            for (int i = tid + STEP_THREADS; i < a.R.n; i += STEP_THREADS) {
                const RecHdr h = ldobj(a.R.h(i));
                d0 = h.dmin[0] < d0 ? h.dmin[0] : d0;
                d1 = h.dmin[1] < d1 ? h.dmin[1] : d1;
                c0 += h.cand[0]; c1 += h.cand[1];
                flg |= h.flags & 1u;
                fm |= h.fmask;
            }
            d0 = wave_min(d0); d1 = wave_min(d1); c0 = wave_sum(c0); c1 = wave_sum(c1);
            flg = wave_red_or(flg);
            fm = wave_red_or(fm);
            if (lane == 0) {
                s_pd[0][wid] = d0; s_pd[1][wid] = d1; s_pc[0][wid] = c0; s_pc[1][wid] = c1;
                s_pf[0][wid] = flg; s_pf[1][wid] = fm;
            }
        }
        __syncthreads();
        if (wid == 0) {
            const bool pin = lane < nrw;
            const double g0 = wave_min(pin ? s_pd[0][lane] : HUGE_VAL), g1 = wave_min(pin ? s_pd[1][lane] : HUGE_VAL);
            unsigned long long c0 = wave_sum(pin ? s_pc[0][lane] : 0ull), c1 = wave_sum(pin ? s_pc[1][lane] : 0ull);
            const uint32_t flg = wave_red_or(pin ? s_pf[0][lane] : 0u), fm = wave_red_or(pin ? s_pf[1][lane] : 0u);
            if (lane == 0) {
                if (a.incr) {
                    // an incremental scan read only some blocks: the counts are the last
                    // full scan's (move() steps keep nrep, the in-set replicas and bl_move)
                    if (C.incr_ok) { c0 = C.cand_cache[0]; c1 = C.cand_cache[1]; }
                    else { C.cand_cache[0] = c0; C.cand_cache[1] = c1; }
                }
                s_g[0] = g0; s_g[1] = g1; s_cand[0] = c0; s_cand[1] = c1;
                s_flags = flg | (a.use_spill && C.cont_overflow ? 1u : 0u);
                s_fm = fm;
                C.last_fm = fm;
            }
        }
        }
        __syncthreads();
        const double g0 = s_g[0], g1 = s_g[1];
    KB_STOP(2);
        if (s_fm) {
            // some record holds a first-index predicate (the plan is not in shape yet)
            uint32_t f[NF];
#pragma unroll
            for (int q = 0; q < NF; q++) f[q] = NONE32;
            for (int i = tid; i < a.R.n; i += STEP_THREADS) {
                if (!ld32(&a.R.h(i)->fmask)) continue;
                const uint32_t* fi = a.R.f(i);
#pragma unroll
                for (int q = 0; q < NF; q++) f[q] = min(f[q], ld32(fi + q));
            }
#pragma unroll
            for (int q = 0; q < NF; q++) {
                f[q] = wave_min(f[q]);
                if (lane == 0 && f[q] != NONE32) atomicMin(&s_first[q], f[q]);
            }
            __syncthreads();
        }
        KB_STAMP(ctl, 13);
        // keys within the window, per kind, over the records within 8*eps of the
        // minimum; a kind with exactly one such key needs no key round trip: it is
        // that record's best key (inserted here speculatively in any case)
        if (wid < nrw) {
            int kc0 = 0, kc1 = 0;
            if (tid < a.R.n) {
                const bool q0 = hd0 <= g0 + 8.0 * eps, q1 = hd1 <= g1 + 8.0 * eps;
                kc0 = q0 ? (int)hnk0 : 0;
                kc1 = q1 ? (int)hnk1 : 0;
                if (a.fp_lds && a.fp_bk) { hb0 = s_bk[2 * tid]; hb1 = s_bk[2 * tid + 1]; }   // (stashed with the headers)
                // (a kind with one key overall: this record's best key is it; the write
                // is meaningful only then)
                if (kc0 && hb0.s >= 0) { s_single[0] = hb0; s_sok[0] = cont_delta_ld(s_ld, hb0, inv_avg) <= g0 + 4.0 * eps; }
                if (kc1 && hb1.s >= 0) { s_single[1] = hb1; s_sok[1] = cont_delta_ld(s_ld, hb1, inv_avg) <= g1 + 4.0 * eps; }
            }
            kc0 = wave_sum(kc0); kc1 = wave_sum(kc1);
            if (lane == 0) {
                if (kc0) atomicAdd(&s_kc[0], kc0);
                if (kc1) atomicAdd(&s_kc[1], kc1);
            }
        }
        __syncthreads();
        // single-key kinds need the raw spill buffer to be empty (its keys are not counted)
        // (rank summaries always take the key path: a summary's best key is its records'
        // best, which need not be its one key when the census spilled past a workgroup
        // table -- the summary's key list holds it; and a single key whose record
        // offered no best key is collected rather than guessed)
        const bool many = a.R.n > STEP_THREADS || (a.use_spill && C.ncont > 0) || !a.use_spill;
        // (s_kc counts every key of the scan records in the windows, stored or spilled: a kind
        // with none has nothing to collect -- the step after a first-index stage, census off)
        const bool counted = a.R.n <= STEP_THREADS && a.use_spill;
        const bool need0 = (many || s_kc[0] > 1 || s_sok[0] < 0) && !(counted && s_kc[0] == 0);
        const bool need1 = (many || s_kc[1] > 1 || s_sok[1] < 0) && !(counted && s_kc[1] == 0);
        if (tid < 2 && !(tid ? need1 : need0) && s_kc[tid] == 1) {
            s_nd[tid] = s_sok[tid] ? 1 : 0;          // resolve takes s_single (s_li == -2)
            s_li[tid] = -2;
        }

        if ((need0 || need1) && a.R.n <= NW * 128) {
            // one record per thread: its window tests and key count into LDS (the exact folds'
            // rows, free until the resolve); then every key slot of every record, one per
            // thread, so a record's keys are loaded in parallel instead of one dependent
            // round trip per key (c2's all-tie records: 7.1 -> ~1 us)
            uint32_t* s_rq = (uint32_t*)s_fold;
            const int cap = a.R.cap;
            for (int i = tid; i < a.R.n; i += STEP_THREADS) {
                double d0 = hd0, d1 = hd1;              // (this thread's record: its registers)
                uint32_t nks = hnks;
                if (i != tid) {
                    const RecHdr* h = a.R.h(i);
                    d0 = ldd(&h->dmin[0]); d1 = ldd(&h->dmin[1]); nks = ld32(&h->nkeys);
                }
                const bool q0 = need0 && d0 <= g0 + 8.0 * eps;
                const bool q1 = need1 && d1 <= g1 + 8.0 * eps;
                const uint32_t nk = (q0 || q1) ? min(nks, (uint32_t)cap) : 0u;
                s_rq[i] = (nk << 2) | (q1 ? 2u : 0u) | (q0 ? 1u : 0u);
            }
            __syncthreads();
            const int tot = a.R.n * cap;
            // (two slots per thread and pass, both loads issued before either is used: one round
            // trip for up to 2 * STEP_THREADS slots -- c2's 79 records of 16 slots took two)
            auto take = [&](const Contender& c, uint32_t rq) {
                if (!((rq >> (c.kind ? 1 : 0)) & 1u)) return;
                if (cont_delta_ld(s_ld, c, inv_avg) <= (c.kind ? g1 : g0) + 4.0 * eps &&
                    dedup_insert(T, c.kind, c.s, c.t, c.w, c.iter) < 0)
                    s_kfail[c.kind] = 1;
            };
            for (int x0 = tid; x0 < tot; x0 += 2 * STEP_THREADS) {
                const int x1 = x0 + STEP_THREADS;
                const int i0 = x0 / cap, k0 = x0 - i0 * cap;
                const int i1 = x1 < tot ? x1 / cap : i0, k1 = x1 - i1 * cap;
                const uint32_t rq0 = s_rq[i0], rq1 = x1 < tot ? s_rq[i1] : 0u;
                const bool v0 = k0 < (int)(rq0 >> 2), v1 = x1 < tot && k1 < (int)(rq1 >> 2);
                Contender c0, c1;
                if (v0) c0 = ldobj(a.R.k(i0) + k0);
                if (v1) c1 = ldobj(a.R.k(i1) + k1);
                if (v0) take(c0, rq0);
                if (v1) take(c1, rq1);
            }
        } else {
            for (int i = tid; (need0 || need1) && i < a.R.n; i += STEP_THREADS) {
                const RecHdr* h = a.R.h(i);
                const bool q0 = need0 && ldd(&h->dmin[0]) <= g0 + 8.0 * eps;
                const bool q1 = need1 && ldd(&h->dmin[1]) <= g1 + 8.0 * eps;
                if (!q0 && !q1) continue;
                const Contender* keys = a.R.k(i);
                const int nk = (int)min(ld32(&h->nkeys), (uint32_t)a.R.cap);
                for (int k = 0; k < nk; k++) {
                    const Contender c = ldobj(keys + k);
                    if (!(c.kind ? q1 : q0)) continue;
                    if (cont_delta_ld(s_ld, c, inv_avg) <= (c.kind ? g1 : g0) + 4.0 * eps &&
                        dedup_insert(T, c.kind, c.s, c.t, c.w, c.iter) < 0)
                        s_kfail[c.kind] = 1;
                }
            }
        }
    }
    __syncthreads();
    KB_STAMP(ctl, 14);
    KB_STOP(3);
    if (do_res && a.use_spill && C.ncont > 0) {
        // raw spills of the scan (rare): every thread
        const uint32_t n = min(C.ncont, a.cont_cap);
        for (uint32_t i = tid; i < n; i += STEP_THREADS) {
            const Contender c = ldobj(a.cont + i);
            if (cont_delta_ld(s_ld, c, inv_avg) <= s_g[c.kind] + 4.0 * eps &&
                dedup_insert(T, c.kind, c.s, c.t, c.w, c.iter) < 0)
                s_kfail[c.kind] = 1;
        }
        __syncthreads();
    }
    KB_STAMP(ctl, 1);

    // the apply's operands for the single-key kinds (the usual move() decision), issued
    // now so their round trip overlaps the resolve: replica counts and load error
    // bounds of the key's source / target (lanes 2k, 2k + 1), the leader key's meta word
    // and NumConsumers (a leader move carries W * (len(R) + NumConsumers))
    int pf_cnt = 0, pf_nc = 0;
    uint32_t pf_meta = 0;
    double pf_lerr = 0.0;
    if (do_res && wid == 0 && lane < 4) {
        const int k = lane >> 1;
        if (s_li[k] == -2) {
            const Contender c = s_single[k];
            const int b = (lane & 1) ? c.t : c.s;
            pf_cnt = a.cnt[b];
            if (!a.integral) pf_lerr = a.lerr[b];
            if (lane == 0) {
                const long long p = (long long)(c.iter >> 21);
                pf_meta = a.meta[p];
                pf_nc = a.nc[p];
            }
        }
    }

    // ================================================================ resolve
    if (do_res) {
        if (pend) {                      // not consumed by a scan: do it here
            do_list_op(ctl, a.L, &s_i);
            if (tid == 0) { C.pending_list = 0; C.list_overflow = ctl->list_overflow; }
            __syncthreads();
        }
        KB_STAMP(ctl, 2);

        // ---- fast path (one thread, one barrier): no first-index predicate, no
        // ReassignLeaders, and every move() kind decided by the bounds on at most one key;
        // anything else takes the general path below
        __shared__ int s_fast;
        if (tid == 0) {
            const bool census_off = C.ub[0] == -HUGE_VAL || C.ub[1] == -HUGE_VAL;
            int fast = !C.list_overflow && !s_fm && !(a.rebalance && (sm & SM_REASSIGN)) && !(s_flags & 1u) &&
                       !a.exact_unb && !census_off;
            Decision d;
            d.status = 0; d.step = -1; d.kind = 0; d.slot = -1; d.part = -1; d.from = -1; d.to = -1;
            d.su = U0h; d.cu = U0h; d.w = 0.0; d.exact = 0; d.err = E_NONE; d.err_broker = -1; d.pad = 0;
            for (int kind = 0; fast && kind < 2; kind++) {
                if (!(kind ? non_on : lead_on)) continue;
                const int step = kind == 0 ? 7 : 8;
                const int ndist = s_nd[kind];
                if (s_kfail[kind] || ndist > 1) { fast = 0; break; }
                if (ndist == 1) {
                    const Contender cw = s_li[kind] == -2 ? s_single[kind] : dedup_entry(T, s_li[kind]);
                    const double Ua = U0h + cont_delta_ld(s_ld, cw, inv_avg);
                    // the general path's certification (3*eps margins on both decisions)
                    const double thr = U0h - a.min_unbalance;
                    const double rel = 4.0 * DBL_EPSILON * fabs(thr);
                    const bool imp_t = Ua + 3.0 * eps < U0h, imp_f = Ua - 3.0 * eps >= U0h;
                    const bool take_t = Ua + 3.0 * eps + rel < thr, take_f = Ua - 3.0 * eps - rel >= thr;
                    if (!((imp_t || imp_f) && (take_t || take_f))) { fast = 0; break; }
                    if (take_t) {
                        if (!imp_t) { d.status = -1; d.step = step; d.err = E_PANIC; }
                        else {
                            d.status = 1; d.step = step; d.kind = 1;
                            d.part = (long long)(cw.iter >> 21); d.slot = (int)((cw.iter >> 16) & 31);
                            d.from = cw.s; d.to = cw.t; d.w = cw.w; d.su = U0h; d.cu = Ua; d.exact = 0;
                        }
                        break;
                    }
                    d.su = U0h; d.cu = U0h; d.exact = 0;
                } else {
                    // no candidate: cu = su; the decision is su < fl(su - MinUnbalance)
                    const bool t_t = -a.min_unbalance > 4.0 * DBL_EPSILON * (fabs(U0h) + eps);
                    const bool t_f = a.min_unbalance >= 0.0;
                    if (!(t_t || t_f)) { fast = 0; break; }
                    if (t_t) { d.status = -1; d.step = step; d.err = E_PANIC; break; }
                    d.su = U0h; d.cu = U0h; d.exact = 0;
                }
            }
            if (fast) { D = d; s_done = 1; }
            s_fast = fast;
        }
        __syncthreads();
        if (!s_fast) {
            // (the general path reads the bl positions / order from memory: a deferred prep's
            // tables go out first)
            if (s_dp && !s_flushed) {
                flush_deferred(tid, STEP_THREADS);
                __syncthreads();
                if (tid == 0) s_flushed = 1;
            }
            // ---- Validate(dup) / RemoveExtra / AddMissing / MoveDisallowed / ReassignLeaders
            if (tid == 0) {
                const double su = U0h;
                D.status = 0; D.step = -1; D.kind = 0; D.slot = -1; D.part = -1;
                D.from = -1; D.to = -1; D.su = su; D.cu = su; D.exact = 0; D.err = E_NONE; D.err_broker = -1;
                const uint32_t* F = s_first;
                auto rd = [&](uint32_t p, int k) -> int { return (int)a.rep[(long long)k * a.Ppad + p]; };
                if (C.list_overflow) {
                    // a per-broker partition list ran out of slack: the host lays the
                    // lists out again (refresh) and the step runs again
                    s_exact_need = 1;
                } else if (a.sem_go && F[F_DUP] != NONE32 && (sm & SM_VALIDATE_REPLICAS)) {
                    D.status = -1; D.step = 1; D.err = E_DUP; D.part = F[F_DUP]; s_done = 1;
                } else if (a.sem_go && F[F_DUP] != NONE32 && (sm & (SM_ALL & ~7u))) {
                    // a step mask without ValidateReplicas over duplicated replicas (a Go-aliased
                    // remove): the reference goes on over them, the engine's loads and
                    // lists hold distinct replicas only -- an explicit error, never a guess
                    D.status = -1; D.step = __ffs(sm & (SM_ALL & ~7u)) - 1; D.err = E_DUP_UNSUP;
                    D.part = F[F_DUP]; s_done = 1;
                } else if (F[F_REMOVE] != NONE32 && (sm & SM_REMOVE)) {  // steps.go:70-89
                    const uint32_t p = F[F_REMOVE];
                    const uint32_t m = a.meta[p];
                    const int nrep = (int)meta_nrep(m), set = (int)(BIG && a.pset ? a.pset[p] : meta_set(m));
                    const uint64_t* sb = a.setbits + (size_t)set * a.W64;
                    // lightest allowed replica in (load, id) order = smallest universe position
                    int best = -1, bslot = -1, bpos = 0x7FFFFFFF;
                    for (int k = 0; k < nrep; k++) {
                        const int b = rd(p, k);
                        if (!setbit(sb, b)) continue;
                        const int ps = a.posu[b];
                        if (ps < bpos) { bpos = ps; best = b; bslot = k; }
                    }
                    D.step = 3; D.part = p;
                    if (best < 0) { D.status = -1; D.err = E_REMOVE; }
                    else {
                        // replacepl removes the FIRST slot holding that broker (utils.go:167-178)
                        D.status = 1; D.kind = 2; D.slot = bslot; D.from = best; D.to = -1;
                    }
                    s_done = 1;
                } else if (F[F_ADD] != NONE32 && (sm & SM_ADD)) {       // steps.go:93-113
                    s_lkind = 2; s_lpart = F[F_ADD];                      // pick list below
                } else if (F[F_DIS] != NONE32 && (sm & SM_DISALLOWED)) { // steps.go:117-143
                    s_lkind = 1; s_lpart = F[F_DIS];
                } else if (a.rebalance && (sm & SM_REASSIGN)) {           // steps.go:234-282
                    // su < MinUnbalance decides; certify it against eps or use the exact su
                    const bool lo = su + 2.0 * eps < a.min_unbalance, hi = su - 2.0 * eps >= a.min_unbalance;
                    if (!lo && !hi) {
                        s_exact_need = (!a.integral && ndirty0 > 0) ? 1 : 2;
                    } else if (hi) {
                        s_exact_need = 3;                                 // leader pick below
                    }
                }
            }
            __syncthreads();
            if (s_lkind) {
                // AddMissingReplicas / MoveDisallowedReplicas pick from the allowed brokers in
                // (load, id) order from the heaviest down: getBrokerListByLoad over the load
                // map with absent brokers at 0 (Add, utils.go:66-79), getBrokerListByLoadBL
                // over the brokers holding replicas (Disallowed, utils.go:81-90)
                const uint32_t p = s_lpart;
                const uint32_t m = a.meta[p];
                const int nrep = (int)meta_nrep(m), set = (int)(BIG && a.pset ? a.pset[p] : meta_set(m));
                if (wid == 0) {
                    if (lane < nrep) s_lrep[lane] = (int)a.rep[(long long)lane * a.Ppad + p];
#pragma unroll
                    for (int q = 0; q < MB / 4096; q++) {
                        const int wi = q * 64 + lane;
                        const unsigned long long sbw = wi < a.W64 ? (unsigned long long)a.setbits[(size_t)set * a.W64 + wi] : 0ull;
                        s_lsb[wi] = sbw;
                    }
                    if (lane == 0) s_lpick = -1;
                    const unsigned long long lt = (1ull << lane) - 1ull;
                    bool done = false;
                    for (int base = 0; base < B && !done; base += 64) {
                        const int k = base + lane;
                        const int b = k < B ? s_ord[B - 1 - k] : 0;
                        bool mem = k < B && ((s_lsb[b >> 6] >> (b & 63)) & 1ull);
                        if (s_lkind == 1) mem = mem && (s_fl[b] & BF_PRESENT);
                        bool isrep = false;
                        for (int q = 0; q < nrep; q++) isrep |= s_lrep[q] == b;
                        const bool ok = mem && !isrep;
                        const unsigned long long bal = __ballot(ok);
                        if (bal) {
                            if (ok && (bal & lt) == 0) s_lpick = b;      // first eligible from the heavy end
                            done = true;
                        }
                    }
                }
                __syncthreads();
                if (tid == 0) {
                    const int t = s_lpick;
                    if (s_lkind == 2) {
                        D.step = 4; D.part = p;
                        if (t < 0) { D.status = -1; D.err = E_ADD; }
                        else { D.status = 1; D.kind = 3; D.slot = nrep; D.from = -1; D.to = t; }
                    } else {
                        int vslot = -1;
                        for (int k = 0; k < nrep && vslot < 0; k++)
                            if (!((s_lsb[s_lrep[k] >> 6] >> (s_lrep[k] & 63)) & 1ull)) vslot = k;
                        D.step = 5; D.part = p; D.slot = vslot; D.from = s_lrep[vslot];
                        if (t < 0) { D.status = -1; D.err = E_DIS; D.err_broker = D.from; }
                        else { D.status = 1; D.kind = 1; D.to = t; }
                    }
                    s_done = 1;
                }
                __syncthreads();
            }
            // exact su (sequential folds in bl order); s_e doubles as the bl-ordered loads
            // (every load is exact here, so every error bound is zero).  k_pair with the deferred
            // prep's region holds this state's bl positions in LDS (s_pm: staged before the wait,
            // moved by a deferred prep): the bl-ordered loads are scattered from them and the
            // contenders' positions read there, no round trip to memory
            double* s_Lm = s_e;
            const bool pm_lds = FUSED && a.fp_lds;
            auto bpos = [&](int b) -> int { return pm_lds ? (int)s_pm[b] : (int)ld32(a.posm + b); };
            auto stage_exact = [&]() {
                if (pm_lds) {
                    // (every error bound is zero: the positions' loads are read before any is
                    // overwritten -- s_Lm aliases s_e, not s_ld)
                    for (int b = tid; b < B; b += STEP_THREADS) {
                        const int p = s_pm[b];
                        if (p >= 0) s_Lm[p] = s_ld[b];
                    }
                } else {
                    for (int k = tid; k < nblm0; k += STEP_THREADS) s_Lm[k] = s_ld[(int)ld32(a.blm + k)];
                }
                __syncthreads();
            };
            auto su_wave = [&]() {               // (wave 0, after stage_exact)
                const double su = exact_unb_w<GB>(s_Lm, nblm0, -1, -1, 0.0, 0.0, s_fold);
                if (lane == 0) { s_sux = su; atomicAdd(&C.total_folds, 1ull); }
            };
            auto exact_su = [&]() {
                stage_exact();
                if (wid == 0) su_wave();
                __syncthreads();
            };
            auto unstage = [&]() {
                for (int b = tid; b < B; b += STEP_THREADS) s_e[b] = 0.0;
                __syncthreads();
            };
            // (read into a register: thread 0 clears the word below, and a wave that read it
            // only after that would skip the block and its barriers)
            const int xneed = s_exact_need;
            if (xneed >= 2) {
                bool take = xneed == 3;
                if (xneed == 2) {
                    exact_su();
                    unstage();
                    take = !(s_sux < a.min_unbalance);
                }
                __syncthreads();                 // every thread has read s_exact_need
                if (tid == 0) {
                    s_exact_need = 0;
                    const uint32_t* F = s_first;
                    if (take) {
                        auto rd = [&](uint32_t p, int k) -> int { return (int)a.rep[(long long)k * a.Ppad + p]; };
                        if (F[F_EMPTY] != NONE32 || nblm0 == 0) {
                            D.status = -1; D.step = 6; D.err = E_PANIC; D.part = F[F_EMPTY]; s_done = 1;
                        } else if (F[F_LEAD] != NONE32) {
                            const uint32_t p = F[F_LEAD];
                            const int nrep = (int)meta_nrep(a.meta[p]);
                            const int light = C.light;
                            int ex = -1;
                            for (int k = 0; k < nrep && ex < 0; k++) if (rd(p, k) == light) ex = k;
                            D.status = 1; D.step = 6; D.part = p; D.slot = 0; D.from = rd(p, 0); D.to = light;
                            D.kind = ex >= 0 ? 4 : 1;       // swap when bl[0] is already a replica
                            s_done = 1;
                        }
                    }
                }
                __syncthreads();
            }
            KB_STAMP(ctl, 3);

            // ---- move(): leader step (if allowed), then non-leader step (steps.go:284-298)
            for (int kind = 0; kind < 2 && !s_done && !s_exact_need; kind++) {
                if (!(kind ? non_on : lead_on)) continue;        // (uniform: the step mask)
                const int step = kind == 0 ? 7 : 8;
                const double g = s_g[kind];
                if (tid == 0) {
                    if (s_first[F_EMPTY_ELIG] != NONE32) {
                        D.status = -1; D.step = step; D.err = E_PANIC; D.part = s_first[F_EMPTY_ELIG]; s_done = 1;
                    } else if (a.use_spill && (C.ub[0] == -HUGE_VAL || C.ub[1] == -HUGE_VAL)) {
                        s_retry = 1;                 // census was off (after a first-index stage)
                    } else if (s_flags & 1u) {
                        // near-tie spill overflow.  If the scan's census gate ran on a loose
                        // upper bound (ub > g: no surviving best keys, e.g. 4096 brokers with
                        // tiny weights), tighten it to the minima g just found and re-run
                        // this step's scan (the state is untouched; the next enqueued pair
                        // scans again); with ub already at g the host grows the spill buffer
                        // and the step runs again (rank summaries: a capacity error)
                        const bool loose = a.use_spill && (C.ub[1] > s_g[1] || (a.allow_leader && C.ub[0] > s_g[0]));
                        if (loose) s_retry = 1;
                        else s_retry = 2;            // (rank summaries: the host grows them)
                    }
                }
                __syncthreads();
                if (s_done || s_retry) break;
                // (1) the distinct keys of this kind were collected with the records
                const int ndist = s_nd[kind];
                const bool fail = s_kfail[kind] != 0;
                const bool have = ndist > 0 || fail;
                // (2) certified decision for one key; exact folds otherwise
                double Ua = 0.0;
                Contender cw;
                cw.s = cw.t = -1; cw.w = 0; cw.iter = NONE64; cw.kind = kind; cw.pad = 0;
                bool certain = false, c_improved = false, c_take = false;
                if (!fail && ndist == 1) {
                    cw = s_li[kind] == -2 ? s_single[kind] : dedup_entry(T, s_li[kind]);   // the one key
                    Ua = U0h + cont_delta_ld(s_ld, cw, inv_avg);
                    // |Ua - U'| <= eps and |U0h - su| <= eps; margins of 3*eps on both decisions
                    const double thr = U0h - a.min_unbalance;
                    const double rel = 4.0 * DBL_EPSILON * fabs(thr);
                    const bool imp_t = Ua + 3.0 * eps < U0h, imp_f = Ua - 3.0 * eps >= U0h;
                    const bool take_t = Ua + 3.0 * eps + rel < thr, take_f = Ua - 3.0 * eps - rel >= thr;
                    certain = (imp_t || imp_f) && (take_t || take_f) && !a.exact_unb;
                    c_improved = imp_t;
                    c_take = take_t;
                } else if (!have) {
                    // no candidate: cu = su; the decision is su < fl(su - MinUnbalance)
                    const bool t_t = -a.min_unbalance > 4.0 * DBL_EPSILON * (fabs(U0h) + eps);
                    const bool t_f = a.min_unbalance >= 0.0;
                    certain = (t_t || t_f) && !a.exact_unb;
                    c_improved = false;
                    c_take = t_t;
                }
                if (!certain && !a.integral && ndirty0 > 0) {
                    if (tid == 0) s_exact_need = 1;
                    __syncthreads();
                    break;
                }
                double Ustar = U0h, sux = U0h;
                unsigned long long witer = NONE64;
                int exact = 0;
                bool improved = false, take = false;
                if (certain) {
                    improved = c_improved;
                    take = c_take;
                    Ustar = Ua;
                    witer = cw.iter;
                } else {
                    exact = 1;
                    // exact su on wave 0 while the other waves fold the contenders
                    stage_exact();
                    // the contenders of this kind as a compact list with their bl positions
                    // (one pass over the key table by every thread and one round trip for the
                    // positions, instead of each fold wave walking the 2048 table slots and
                    // loading its contender's positions itself); kept in the set-mark words,
                    // which only the prep uses.  More than CLMAX keys: the table walk below.
                    constexpr int CLMAX = 640;
                    uint16_t* s_cl = (uint16_t*)s_smark;
                    int16_t* s_cps = (int16_t*)(s_cl + CLMAX);
                    int16_t* s_cpt = s_cps + CLMAX;
                    static_assert(3 * CLMAX * 2 <= (int)sizeof(s_smark), "contender list fits the mark words");
                    static_assert(DEDUP_STEP == 2 * STEP_THREADS, "two table slots per thread");
                    __shared__ int s_cwc[NW], s_ncl;
                    if (KB_CLIST && !fail && ndist != 1 && have) {
                        const int h0 = tid, h1 = tid + STEP_THREADS;
                        const bool v0 = s_key[h0] != NONE32 && (int)(s_key[h0] >> 30) == kind;
                        const bool v1 = s_key[h1] != NONE32 && (int)(s_key[h1] >> 30) == kind;
                        const unsigned long long m0 = __ballot(v0), m1 = __ballot(v1);
                        const unsigned long long lt = (1ull << lane) - 1ull;
                        if (lane == 0) s_cwc[wid] = (int)(__popcll(m0) + __popcll(m1));
                        __syncthreads();
                        const int wc = lane < NW ? s_cwc[lane] : 0;
                        const int woff = wave_sum(lane < wid ? wc : 0), tot = wave_sum(wc);
                        if (tot <= CLMAX) {
                            auto put = [&](int pos, int h) {
                                s_cl[pos] = (uint16_t)h;
                                const uint32_t k = s_key[h];
                                s_cps[pos] = (int16_t)bpos((int)((k >> 15) & 0x7FFF));
                                s_cpt[pos] = (int16_t)bpos((int)(k & 0x7FFF));
                            };
                            if (v0) put(woff + (int)__popcll(m0 & lt), h0);
                            if (v1) put(woff + (int)__popcll(m0) + (int)__popcll(m1 & lt), h1);
                        }
                        if (tid == 0) s_ncl = tot;
                        __syncthreads();
                    }
                    if (wid == 0) su_wave();
                    if (!fail && ndist == 1) {
                        if (wid == 1) {
                            const double u = exact_unb_w<GB>(s_Lm, nblm0, bpos(cw.s), bpos(cw.t),
                                                                  s_ld[cw.s] - cw.w, s_ld[cw.t] + cw.w, s_fold + 64);
                            if (lane == 0) { s_dv[0] = u; atomicAdd(&C.total_folds, 1ull); }
                        }
                        __syncthreads();
                        sux = s_sux;
                        Ustar = s_dv[0];
                        witer = cw.iter;
                    } else if (have) {
                        // several keys (or an overfull table): exact sequential folds, lexicographic min
                        double bu = HUGE_VAL;
                        unsigned long long bi = NONE64;
                        int bs = -1, bt = -1;
                        double bw = 0.0;
                        unsigned long long nf = 0;
                        auto better = [&](double u, const Contender& c) {
                            if (u < bu || (u == bu && c.iter < bi)) { bu = u; bi = c.iter; bs = c.s; bt = c.t; bw = c.w; }
                        };
                        if (KB_CLIST && !fail && s_ncl <= CLMAX) {
                            // one contender per wave (waves 1..NW-1) from the compact list
                            const int ncl = s_ncl;
                            if (wid > 0)
                                for (int i = wid - 1; i < ncl; i += NW - 1) {
                                    const Contender c = dedup_entry(T, (int)s_cl[i]);
                                    const double u = exact_unb_w<GB>(s_Lm, nblm0, (int)s_cps[i], (int)s_cpt[i],
                                                                          s_ld[c.s] - c.w, s_ld[c.t] + c.w, s_fold + 64 * wid);
                                    if (lane == 0) nf++;
                                    better(u, c);
                                }
                        } else if (!fail) {
                            // one contender per wave (waves 1..NW-1; the table slot is wave-uniform)
                            if (wid > 0)
                                for (int h = wid - 1; h < DEDUP_STEP; h += NW - 1) {
                                    if (!(s_key[h] != NONE32 && (int)(s_key[h] >> 30) == kind)) continue;
                                    const Contender c = dedup_entry(T, h);
                                    const double u = exact_unb_w<GB>(s_Lm, nblm0, bpos(c.s), bpos(c.t),
                                                                          s_ld[c.s] - c.w, s_ld[c.t] + c.w, s_fold + 64 * wid);
                                    if (lane == 0) nf++;
                                    better(u, c);
                                }
                        } else {
                            // (the spill path: per-thread folds over the records and the buffer)
                            __syncthreads();
                            for_each_contender(a, s_ld, C.ncont, kind, g, eps, inv_avg, [&](const Contender& c) {
                                const double u = exact_unbalance_lds(s_Lm, nblm0, bpos(c.s), bpos(c.t),
                                                                     s_ld[c.s] - c.w, s_ld[c.t] + c.w);
                                nf++;
                                better(u, c);
                            });
                        }
                        nf = wave_sum(nf);
                        if (lane == 0 && nf) atomicAdd(&C.total_folds, nf);
                        for (int o = 32; o > 0; o >>= 1) {
                            const double ou = __shfl_xor(bu, o);
                            const unsigned long long oi = __shfl_xor(bi, o);
                            const int os = __shfl_xor(bs, o), ot = __shfl_xor(bt, o);
                            const double ow = __shfl_xor(bw, o);
                            if (ou < bu || (ou == bu && oi < bi)) { bu = ou; bi = oi; bs = os; bt = ot; bw = ow; }
                        }
                        __syncthreads();
                        if (lane == 0) { s_dv[wid] = bu; s_u[wid] = bi; s_bs[wid] = bs; s_bt[wid] = bt; s_bw[wid] = bw; }
                        __syncthreads();
                        if (tid == 0) {
                            for (int q = 1; q < NW; q++)
                                if (s_dv[q] < s_dv[0] || (s_dv[q] == s_dv[0] && s_u[q] < s_u[0])) {
                                    s_dv[0] = s_dv[q]; s_u[0] = s_u[q]; s_bs[0] = s_bs[q]; s_bt[0] = s_bt[q]; s_bw[0] = s_bw[q];
                                }
                        }
                        __syncthreads();
                        sux = s_sux;
                        Ustar = s_dv[0]; witer = s_u[0];
                        cw.s = s_bs[0]; cw.t = s_bt[0]; cw.w = s_bw[0]; cw.iter = witer;
                    } else {
                        __syncthreads();
                        sux = s_sux;
                    }
                    unstage();
                    // cu starts at su and only a strictly smaller u replaces it (steps.go:163,211)
                    improved = have && Ustar < sux;
                    const double cu = improved ? Ustar : sux;
                    take = cu < sux - a.min_unbalance;
                }
                __syncthreads();
                if (tid == 0) {
                    if (take) {
                        if (!improved) {
                            // replacepl on the zero Partition: the reference panics
                            D.status = -1; D.step = step; D.err = E_PANIC; s_done = 1;
                        } else {
                            D.status = 1; D.step = step; D.kind = 1;
                            D.part = (long long)(witer >> 21); D.slot = (int)((witer >> 16) & 31);
                            D.from = cw.s; D.to = cw.t; D.w = cw.w; D.su = sux; D.cu = Ustar; D.exact = exact;
                            s_done = 1;
                        }
                    } else {
                        D.su = sux; D.cu = sux; D.exact = exact;
                    }
                }
                __syncthreads();
            }
        }
        KB_STAMP(ctl, 4);

        if (s_retry) {
            if (tid == 0 && s_retry == 2) {
                C.halted = H_NEED_SPILL;                // the host grows the spill buffer (and
                C.ncont = 0;                            // the rank summaries); it clears the flag
            } else if (tid == 0) {
                if (C.ub[0] == -HUGE_VAL || C.ub[1] == -HUGE_VAL) {
                    // the scan pruned every wave: its minima are not the step's; open the
                    // bound (the host's bound pass, or a full census, closes it)
                    C.ub[0] = HUGE_VAL;
                    C.ub[1] = HUGE_VAL;
                } else {
                    C.ub[0] = C.ub[0] < s_g[0] ? C.ub[0] : s_g[0];
                    C.ub[1] = C.ub[1] < s_g[1] ? C.ub[1] : s_g[1];
                }
                C.ncont = 0;
                C.cont_overflow = 0;
                C.total_retries++;
            }
            write_back();
            return;
        }
        if (s_exact_need) {
            // the bounds cannot decide and some loads are approximate: refold first
            if (tid == 0) {
                C.halted = H_NEED_EXACT;
                C.prepped = 0;
                C.total_exact_halts++;
            }
            write_back();
            return;
        }

        // ---------------------------------------------------------- apply
        // wave 0, one lane per replica slot (lanes 0..15 the old replicas, 16..31 the
        // new ones); cross-lane work by ballot / readlane.  A move() replacement takes
        // a one-round-trip path: no partition holds a disallowed replica when move()
        // runs (MoveDisallowedReplicas comes first, balancer.go:34-44) and the target is
        // inside the set, so the meta word is unchanged and only the source and the
        // target change (contribution W, or W * (len(R) + NumConsumers) at slot 0)
        KB_STAMP(ctl, 11);
    KB_STOP(4);
        if (wid == 0) {
            int nT = 0;
            const bool chg = D.status == 1;
            const long long p = D.part;
            const int kind = D.kind, slot = D.slot, to = D.to;
            // (a step mask without MoveDisallowedReplicas may run move() while some partition
            // holds a disallowed replica: then the meta word can change, the general path)
            const bool fast = chg && kind == 1 && (D.step == 7 || D.step == 8) && !(s_fm & (1u << F_DIS));
            bool upd = false, act = false;
            int b = -1, dcnt = 0, cv = 0;
            double oldc = 0.0, newc = 0.0, av = 0.0;
            if (fast) {
                b = lane == 0 ? D.from : to;
                // (the operands prefetched before the resolve when the decision is the
                // kind's single key; else one round trip)
                const int k = D.step == 7 ? 0 : 1;
                bool pf = s_li[k] == -2;
                if (pf) {
                    const Contender& c = s_single[k];
                    pf = c.s == D.from && c.t == to && (long long)(c.iter >> 21) == p;
                }
                if (lane < 2) {                              // every load in one round trip
                    if (pf) {
                        cv = lane == 0 ? __builtin_amdgcn_readlane(pf_cnt, 2 * k) : __builtin_amdgcn_readlane(pf_cnt, 2 * k + 1);
                        if (!a.integral) {
                            const long long lo = __double_as_longlong(pf_lerr);
                            const int l0 = __builtin_amdgcn_readlane((int)lo, 2 * k), h0 = __builtin_amdgcn_readlane((int)(lo >> 32), 2 * k);
                            const int l1 = __builtin_amdgcn_readlane((int)lo, 2 * k + 1), h1 = __builtin_amdgcn_readlane((int)(lo >> 32), 2 * k + 1);
                            av = lane == 0 ? __longlong_as_double(((long long)h0 << 32) | (uint32_t)l0)
                                           : __longlong_as_double(((long long)h1 << 32) | (uint32_t)l1);
                        }
                    } else {
                        cv = a.cnt[b];
                        if (!a.integral) av = a.lerr[b];
                    }
                }
                double c = D.w;
                if (slot == 0) {
                    uint32_t m;
                    int ncp;
                    if (pf && k == 0) { m = (uint32_t)__builtin_amdgcn_readlane((int)pf_meta, 0); ncp = __builtin_amdgcn_readlane(pf_nc, 0); }
                    else { m = a.meta[p]; ncp = a.nc[p]; }
                    c = D.w * (double)((int)meta_nrep(m) + ncp);
                }
                if (lane == 0) a.rep[(long long)slot * a.Ppad + p] = (uint16_t)to;
                act = lane < 2;
                oldc = lane == 0 ? c : 0.0;
                newc = lane == 0 ? 0.0 : c;
                dcnt = lane == 0 ? -1 : 1;
                upd = true;
            } else {
                int ro = -1;                                 // old replica at slot `lane`
                uint32_t m = 0, setx = 0;
                double wv = 0.0;
                int ncp = 0;
                if (chg) {
                    if (lane < a.RC) ro = (int)a.rep[(long long)lane * a.Ppad + p];
                    m = a.meta[p];
                    wv = a.w[p];
                    ncp = a.nc[p];
                    setx = BIG && a.pset ? a.pset[p] : meta_set(m);
                }
                const int nrep = (int)meta_nrep(m);
                if (lane >= nrep) ro = -1;
                // the new replica list (replacepl / addpl, utils.go:166-202)
                int rn = ro, nn = nrep;
                bool state_changed = chg;
                const unsigned long long ball_to = __ballot(ro == to && lane < 16);
                if (kind == 1) {                             // replace at slot (utils.go:186-190)
                    if (lane == slot) rn = to;
                } else if (kind == 4) {                      // swap with the existing replica (utils.go:179-185)
                    const int ex = ball_to ? (int)__ffsll((long long)ball_to) - 1 : 0;
                    const int ro_slot = __builtin_amdgcn_readlane(ro, __builtin_amdgcn_readfirstlane(slot));
                    if (lane == slot) rn = to;
                    else if (lane == ex) rn = ro_slot;
                } else if (kind == 2) {                      // remove (utils.go:176-178)
                    const int nxt = __shfl(ro, (lane + 1) & 63);
                    if (lane >= slot && lane + 1 < nrep) rn = nxt;
                    if (a.sem_go) state_changed = false;     // pl keeps its length: duplicates
                    else { nn = nrep - 1; if (lane == nn) rn = -1; }
                } else if (kind == 3) {                      // add (utils.go:199-202)
                    if (a.sem_go) state_changed = false;     // the append is not visible through pl
                    else { nn = nrep + 1; if (lane == nrep) rn = to; }
                }
                const bool go_remove = chg && a.sem_go && kind == 2;
                const int nw = go_remove ? nrep : nn;        // the replica slots written
                if (state_changed || go_remove) {
                    // the allowed-set words of the new replicas (Disallowed trigger, in-set count)
                    bool in = false;
                    if (lane < nw) {
                        // (typed LDS pointer: the two loads must not merge into one flat load)
                        const size_t wi = (size_t)setx * a.W64 + (rn >> 6);
                        const uint64_t wd = a.sb_lds ? ((const __attribute__((address_space(3))) uint64_t*)s_sb)[wi]
                                                     : a.setbits[wi];
                        in = (wd >> (rn & 63)) & 1ull;
                    }
                    const unsigned long long bin = __ballot(in && lane < nw), bout = __ballot(!in && lane < nw);
                    if (lane < nw) a.rep[(long long)lane * a.Ppad + p] = (uint16_t)rn;
                    const uint32_t nmeta = make_meta((uint32_t)nw, meta_want(m), meta_elig(m), bout ? 1u : 0u,
                                                     (uint32_t)__popcll(bin), meta_set(m));
                    if (lane == 0) a.meta[p] = nmeta;
                }
                if (state_changed) {
                    // contributions of getBrokerLoad (utils.go:92-105): the leader slot carries
                    // W * (len(R) + NumConsumers); lanes 0..15 hold the old replicas, 16..31 the new
                    const int j = lane & 15;
                    const bool old_lane = lane < 16 && j < nrep, new_lane = lane >= 16 && lane < 32 && j < nn;
                    const int rnew_j = __shfl(rn, j);
                    b = old_lane ? ro : (new_lane ? rnew_j : -1);
                    const double oc = old_lane ? (j == 0 ? wv * (double)(nrep + ncp) : wv) : 0.0;
                    const double nc_here = new_lane ? (j == 0 ? wv * (double)(nn + ncp) : wv) : 0.0;
                    // pair an old replica with the same broker among the new ones
                    double cn_other = 0.0;
                    bool matched = false;
                    for (int q = 0; q < 16; q++) {
                        const int bq = __builtin_amdgcn_readlane(rn, q);   // new replica q
                        const int bo = __builtin_amdgcn_readlane(ro, q);   // old replica q
                        const double ncq = q < nn ? (q == 0 ? wv * (double)(nn + ncp) : wv) : 0.0;
                        if (old_lane && q < nn && bq == b) { cn_other = ncq; matched = true; }
                        if (new_lane && q < nrep && bo == b) matched = true;
                    }
                    // per broker: (old, new) contribution; new-only brokers from the new lanes
                    act = old_lane || (new_lane && !matched);
                    oldc = old_lane ? oc : 0.0;
                    newc = old_lane ? cn_other : nc_here;
                    dcnt = old_lane ? (matched ? 0 : -1) : 1;
                    if (act && (oldc != newc || dcnt != 0)) {    // their counts and error terms
                        cv = a.cnt[b];
                        if (!a.integral) av = a.lerr[b];
                    }
                    upd = true;
                }
            }
            KB_STAMP(ctl, 21);
            if (upd) {
                const bool touched = act && oldc != newc;
                const bool cnt_changes = act && dcnt != 0;
                int dd = 0;
                double Lold = 0.0, ebold = 0.0;
                bool mchg = false;
                if (touched || cnt_changes) {
                    const int cnew = cv + dcnt;
                    if (dcnt) a.cnt[b] = cnew;
                    if (touched) {
                        const double L = s_ld[b];
                        Lold = L;
                        ebold = s_e[b];
                        const uint8_t fl0 = s_fl[b];
                        uint8_t fl = s_fl[b] & ~BF_PRESENT;
                        if (cnew > 0) fl |= BF_PRESENT;
                        double Ln, eb = 0.0;
                        if (a.integral) {
                            Ln = (L - oldc) + newc;
                        } else {
                            // bounded incremental update; the exact fold comes with k_refresh
                            const double u = DBL_EPSILON / 2;
                            const double x1 = L - oldc;
                            Ln = x1 + newc;
                            double ae = av + 1.01 * u * (fabs(x1) + fabs(Ln));
                            if (!(Ln > 0.0)) Ln = 0.0;               // loads are sums of non-negative terms
                            if (cnew == 0) { Ln = 0.0; ae = 0.0; }  // empty fold: exactly 0
                            a.lerr[b] = ae;
                            const bool dirty = cnew > 0;
                            if (dirty != ((fl & BF_DIRTY) != 0)) dd = dirty ? 1 : -1;
                            fl = dirty ? (uint8_t)(fl | BF_DIRTY) : (uint8_t)(fl & ~BF_DIRTY);
                            eb = dirty ? ae + gamma_n(cnew) * (Ln + ae) : 0.0;
                        }
                        a.load[b] = Ln; s_ld[b] = Ln;
                        a.eb[b] = eb; s_e[b] = eb;
                        a.bfl[b] = fl; s_fl[b] = fl;
                        if (!a.integral) {
                            // fold checkpoints: a broker whose list is edited gets its first
                            // changed position from the edit (list_remove / list_insert); one
                            // whose contribution changed in place (the leader's weight after a
                            // remove / add, a swap's two brokers) is refolded from the start
                            const bool ledit = (kind == 1 && (b == D.from || b == to)) ||
                                               (kind == 2 && b == D.from) || (kind == 3 && b == to);
                            if (!ledit) a.L.dpos[b] = 0u;
                        }
                        mchg = ((fl0 ^ fl) & BF_PRESENT) && !(fl & BF_INCFG);
                    }
                }
                KB_STAMP(ctl, 22);
                dd = wave_sum(dd);
                const unsigned long long bt = __ballot(touched);
                if (touched) {
                    const int k = (int)__popcll(bt & ((1ull << lane) - 1ull));
                    if (k < TMAX) { s_T[k] = b; s_Lold[k] = Lold; s_ebold[k] = ebold; }
                }
                if (__ballot(mchg) && lane == 0) s_memb = 1;
                nT = (int)__popcll(bt);
                if (nT > TMAX) nT = TMAX;
                if (lane == 0) {
                    if (dd) C.ndirty += dd;
                    // the per-broker partition lists follow in the next scan (k_scan's list workgroup)
                    if (!a.integral && (kind == 1 || kind == 2 || kind == 3)) {
                        C.pl_kind = kind; C.pl_from = D.from; C.pl_to = to; C.pl_part = p;
                        C.pending_list = 1;
                    }
                }
            }
            if (lane == 0) {
            s_nT = nT;
            if (D.status == 1) s_moved = D.part;
            // log the step
            ChangeDev ch;
            ch.status = D.status; ch.step = D.step; ch.kind = D.kind; ch.slot = D.slot;
            ch.part = D.part; ch.from = D.from; ch.to = D.to; ch.su = D.su; ch.cu = D.cu;
            ch.exact = D.exact; ch.err_code = D.err; ch.err_broker = D.err_broker; ch.pad = 0;
            if (C.logpos < C.logcap) a.log[C.logpos] = ch;
            C.logpos++;
            C.steps++;
            // (kb_engine_plan_until: a change on another partition ends the plan after it; the
            // budget goes too, so no later launch of the batch -- a refresh's resumed prep
            // included -- takes another step)
            if (D.status == 1 && C.stop_part >= 0 && D.part != C.stop_part) { C.budget = C.steps; C.halted = H_DONE; }
            // reference candidate count of the steps that actually ran this iteration
            unsigned long long add = 0;
            if (D.step < 0 || D.step >= 7) {
                if (lead_on) add += s_cand[0];
                if (D.step != 7 && non_on) add += s_cand[1];
            }
            C.total_cand += add;
            C.total_cont += (unsigned long long)(s_nd[0] + s_nd[1]);
            // (a step mask's no-change leaves the state and its prep as they were: the
            // next masked step resolves the same scan records, kb_engine_step)
            if (D.status != 1) { C.halted = H_DONE; if (!(D.status == 0 && sm != SM_ALL)) C.prepped = 0; }
            }
        } else if (s_dp && !s_flushed) {
            // (the fast path's flush: the waves the apply leaves idle; before the prep below,
            // whose merged set records must land after the rebuilt ones)
            flush_deferred(tid - 64, STEP_THREADS - 64);
            if (tid == 64) s_flushed = 1;
        }
        __syncthreads();
        if (D.status != 1) { write_back(); return; }
        // eager refolds: the next scan's extra workgroups edit the touched brokers' lists
        // (the pending edit, each its own broker's half) and refold them; more touched brokers
        // than EGW: the old way (the edit in the scan's list workgroup, the brokers stay dirty
        // until a refresh)
        if (KB_EAGER_CODE && tid == 0 && a.eager && !a.integral) {
            C.eg_n = s_nT <= EGW ? s_nT : 0;
            for (int k = 0; k < C.eg_n; k++) C.eg_b[k] = s_T[k];
        }
        KB_STAMP(ctl, 5);
    KB_STOP(5);
    }

    // ================================================================== prep
    // (next step): getBL's (load, id) order, bl_move, relative loads, eps, sets
    const bool full = C.full_prep != 0;
    // The next step's census bound ub is the minimum of last step's best keys (one per
    // record and kind) re-scored on the new loads: any legal move bounds the new minimum
    // from above.  A key whose brokers the applied move touched is still a legal move after
    // a replace that left bl_move's membership alone (its partition kept its replicas, its
    // target is still in the set and in bl_move): only the moved partition's keys are
    // dropped.  (Dropping every touched key as well left no key at all on most steps of a
    // non-leader plan -- the records' keys come from the census waves, which mostly share
    // the step's source or target -- so the bound went open and every wave walked its
    // targets: 4000 of 5400 waves per step, c3nl 0.47 ms/step.)  After a remove / add /
    // swap or a membership change the touched brokers' keys are dropped as before.
    auto keep_touched_keys = [&]() -> bool {
        return do_res && D.status == 1 && D.kind == 1 && !s_memb;
    };
#if KB_ABL & 2
    // diagnostic timing build (tools/ablate.sh): no incremental prep at all
    if (!full) { if (tid == 0) C.prepped = 1; write_back(); return; }
#endif
    const int nT = s_nT;
    bool marked = false;                              // (unused: the fused path returns itself)
    // ---- fast prep (round 6; DevCtl.fp): a plain move() replace -- frozen average, bl_move's
    // membership unchanged, two touched brokers -- writes only what the next scan cannot derive
    // and leaves the broker order, the positions and the full set records to the next launch's
    // step workgroup (deferred_prep, before its wait, beside the scan):
    //   FP1  the touched brokers' new bl positions (the bl_move brokers below each), the sets
    //        holding one, r[] of the touched and the frozen totals (as the frozen prep below),
    //        the upper bound from the records' best keys;
    //   FP2  each marked set's record merged from its current one (LDS, s_rec): its untouched
    //        members keep their order, the touched ones go in at their new positions; entries
    //        up to the last untouched member are certain (a member past the record's end
    //        could precede a touched broker inserted after it).  With <= 2 touched among KR = 6
    //        listed, >= 4 = RC + 1 remain, so the scan's first target is right; walk_targets
    //        continues in memory past a short record.  A set left with fewer certain members
    //        sends the step to the full prep below instead.
    if (FUSED && a.fp_ok && a.fp_lds && a.fp_bk && !full && do_res && D.status == 1 && D.kind == 1 &&
        (D.step == 7 || D.step == 8) && !s_memb && nT >= 1 && nT <= 2 && C.frz_n > 0 && C.frz_n < FRZ_MAX &&
        !a.eager && a.use_spill && !a.rebalance && !a.incr && !(KB_ABL & 32)) {
        const int t0 = s_T[0], t1 = nT > 1 ? s_T[1] : -1;
        const double iav = C.inv_avg;
        // FP1, one job per group of waves so that no wave runs two of them in series (the barrier
        // waits for the slowest): waves 0-3 the upper bound (records 0..255, then every 256th),
        // wave 4 the frozen totals and eps (lane 0), waves 8-15 the counts and the marks
        const double L0 = s_ld[t0], L1 = t1 >= 0 ? s_ld[t1] : 0.0;
        if (wid >= 8) {
            const int t8 = tid - 8 * 64;
            int c0 = 0, c1 = 0;
            for (int b = t8; b < ((KB_FPABL & 2) ? 0 : B); b += STEP_THREADS - 8 * 64) {   // (KB_FPABL: timing only)
                const bool in = (s_fl[b] & (BF_PRESENT | BF_INCFG)) && b != t0 && b != t1;
                const double Lb = s_ld[b];
                c0 += in && (Lb < L0 || (Lb == L0 && b < t0)) ? 1 : 0;
                c1 += in && t1 >= 0 && (Lb < L1 || (Lb == L1 && b < t1)) ? 1 : 0;
            }
            for (int set = t8; set < ((KB_FPABL & 2) ? 0 : a.nsets); set += STEP_THREADS - 8 * 64) {
                const uint64_t* sb = s_sb + (size_t)set * a.W64;
                bool hit = (sb[t0 >> 6] >> (t0 & 63)) & 1ull;
                if (t1 >= 0) hit |= (sb[t1 >> 6] >> (t1 & 63)) & 1ull;
                if (hit) s_dlist[atomicAdd(&s_dn, 1)] = set;
            }
            c0 = wave_sum(c0); c1 = wave_sum(c1);
            if (lane == 0) { if (c0) atomicAdd(&s_cntT[0], c0); if (c1) atomicAdd(&s_cntT[1], c1); }
        } else if (wid == 4) {
            if (lane < nT) stdbl(a.r + s_T[lane], rel_ld(s_ld, s_T[lane], iav));
            if (lane == 0) {
                // the frozen totals after the move (as the frozen prep below: the base's sum and
                // average, the touched brokers' increments, each bound grown by a few ulps) and eps
                double dU = 0.0, aU = 0.0, dV = 0.0, dE = 0.0, rl = HUGE_VAL, rh = -HUGE_VAL;
                for (int k = 0; k < nT; k++) {
                    const int b = s_T[k];
                    const double rn = rel_ld(s_ld, b, iav);
                    const double ro = __fma_rn(s_Lold[k], iav, -1.0);   // the r[] the base wrote
                    const double fn = fsq(rn), fo = fsq(ro);
                    dU += fn - fo;
                    aU += fn + fo;
                    dV += fabs(rn) * (1.0 + fabs(rn)) - fabs(ro) * (1.0 + fabs(ro));
                    dE += s_e[b] - s_ebold[k];
                    rl = rn < rl ? rn : rl;
                    rh = rn > rh ? rn : rh;
                }
                const double uu = DBL_EPSILON / 2;
                const double U0 = C.U0 + dU;
                const double uerr = C.uerr + 8.0 * uu * (fabs(C.U0) + fabs(U0) + aU);
                const double V = (C.V + dV) * (1.0 + 8.0 * uu);
                const double E = (C.E + dE) * (1.0 + 8.0 * uu);
                const double Rm = fmax(C.rm_bound, fmax(fabs(rl), fabs(rh)));
                const double n = (double)C.nblm;
                const double R = Rm + a.wmax * iav;
                const double Ea = E * iav;
                const double epsf = 64.0 * uu * ((n + 8.0) * (U0 + 2.0 * V) + 4.0 * (1.0 + R) * (1.0 + R));
                const double epsl = 16.0 * Ea * (V / (n > 0 ? n : 1.0) + R + 1.0) + 4.0 * Ea * Ea;
                double ep = 2.0 * (epsf + epsl) + uerr;
                if (!(ep > 1e-300)) ep = 1e-300;
                s_fpz[0] = U0; s_fpz[1] = uerr; s_fpz[2] = V; s_fpz[3] = E; s_fpz[4] = rl; s_fpz[5] = rh;
                s_fpz[6] = Rm; s_fpz[7] = ep; s_fpz[8] = epsl > epsf ? 1.0 : 0.0;
            }
        } else if (wid < 4) {
            // the best keys of every record but the moved partition's stay legal moves after a
            // plain replace (keep_touched_keys), re-scored on the new loads
            double ub0 = HUGE_VAL, ub1 = HUGE_VAL;
            int nkeep = 0;
            const long long pm = s_moved;
            for (int i = tid; i < a.R.n; i += 4 * 64) {
                const Contender bk[2] = {s_bk[2 * i], s_bk[2 * i + 1]};   // (stashed with the headers)
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    const Contender& c = bk[k];
                    const bool keep = c.s >= 0 && (long long)(c.iter >> 21) != pm;
                    if (a.ubdesc) {
                        BlockDesc d;
                        d.wmax = keep ? HUGE_VAL : -1.0;
                        d.blk = keep ? (long long)(c.iter >> 21) / BLK : 0;
                        stobj(a.ubdesc + 2 * i + k, d);
                    }
                    nkeep += keep ? 1 : 0;
                    if (!keep) continue;
                    const double d2 = cont_delta_ld(s_ld, c, iav);
                    if (k == 0) ub0 = d2 < ub0 ? d2 : ub0;
                    else ub1 = d2 < ub1 ? d2 : ub1;
                }
            }
            // (one LDS atomic per wave: same-address atomics of a whole wave serialise)
            ub0 = wave_min(ub0); ub1 = wave_min(ub1);
            nkeep = wave_sum(nkeep);
            if (lane == 0) {
                atomicMin(&s_fpub[0], enc(ub0)); atomicMin(&s_fpub[1], enc(ub1));
                if (a.ubdesc && nkeep) atomicAdd(&s_fpnsub, nkeep);
            }
        }
        KB_STAMP(ctl, 20);
        __syncthreads();                                // FP #1
        KB_STAMP(ctl, 6);
        // FP2: the touched brokers' bl positions before (s_pm: this state's) and after the move;
        // u = the untouched bl_move brokers before each (the scan's patch, below)
        const int o0 = s_pm[t0], o1 = t1 >= 0 ? s_pm[t1] : 0x7FFFFFFF;
        const bool t1lt = t1 >= 0 && (L1 < L0 || (L1 == L0 && t1 < t0));
        const int u0 = s_cntT[0], u1 = t1 >= 0 ? s_cntT[1] : 0x7FFFFFFF;
        const int n0 = u0 + (t1lt ? 1 : 0), n1 = t1 >= 0 ? u1 + (t1lt ? 0 : 1) : 0x7FFFFFFF;
        // (one wave per marked set, one lane per listed member: its position and its output index
        // by ballots -- no serial merge in one lane)
        const int nmk = (KB_FPABL & 1) ? 0 : s_dn, KR = a.KR;
        const unsigned long long ltm = (1ull << lane) - 1ull;
        for (int g = wid; g < nmk; g += NW) {
            const int set = s_dlist[g];
            const uint16_t* r16 = (const uint16_t*)(s_rec + (size_t)set * a.units);   // (fp_lds: a.units 16-B units)
            const int nelig = (int)r16[0], nl = (int)r16[1];
            const uint64_t* sb = s_sb + (size_t)set * a.W64;
            const bool in0 = (sb[t0 >> 6] >> (t0 & 63)) & 1ull;
            const bool in1 = t1 >= 0 && ((sb[t1 >> 6] >> (t1 & 63)) & 1ull);
            const int e = (int)r16[2 + (lane < KR ? lane : KR - 1)];
            const bool v = lane < KR && lane < nl && e != t0 && e != t1;
            const int p = s_pm[v ? e : 0];
            const int pc = p - (o0 < p ? 1 : 0) - (o1 < p ? 1 : 0);
            const int pe = pc + (u0 <= pc ? 1 : 0) + (u1 <= pc ? 1 : 0);
            const unsigned long long vm = __ballot(v);
            const int nv = (int)__popcll(vm);
            const int lastpe = vm ? __shfl(pe, 63 - __clzll(vm)) : -1;
            // a touched member is certain when a listed untouched member follows it, or when the
            // record listed the whole set
            const bool all = nl >= nelig;
            const bool c0 = in0 && (all || n0 < lastpe), c1 = in1 && (all || n1 < lastpe);
            const int no = nv + (c0 ? 1 : 0) + (c1 ? 1 : 0);
            const int nn = no < KR ? no : KR;
            const int kt = a.RC + 1 < nelig ? a.RC + 1 : nelig;
            if (nn < kt) { if (lane == 0) s_fpfail = 1; continue; }
            uint16_t* row = &s_mrow[wid][0];
            if (lane < 8 * a.units) row[lane] = NONE16;
            __builtin_amdgcn_wave_barrier();
            const int idx = (int)__popcll(vm & ltm) + (c0 && n0 < pe ? 1 : 0) + (c1 && n1 < pe ? 1 : 0);
            if (v && idx < KR) row[2 + idx] = (uint16_t)e;
            const int i0 = (int)__popcll(__ballot(v && pe < n0)) + (c1 && n1 < n0 ? 1 : 0);
            const int i1 = (int)__popcll(__ballot(v && pe < n1)) + (c0 && n0 < n1 ? 1 : 0);
            if (lane == 0) {
                if (c0 && i0 < KR) row[2 + i0] = (uint16_t)t0;
                if (c1 && i1 < KR) row[2 + i1] = (uint16_t)t1;
                row[0] = (uint16_t)nelig;
                row[1] = (uint16_t)nn;
            }
            __builtin_amdgcn_wave_barrier();
            if (lane < a.units) {
                // (entries past nn: NONE16 -- the row held NONE16 before the writes, and nn <= KR)
                stobj(a.setrec + (size_t)set * a.units + lane, *(const uint4*)(row + 8 * lane));
            }
            __builtin_amdgcn_wave_barrier();
        }
        KB_STAMP(ctl, 0);
        __syncthreads();                                // FP #2
        KB_STAMP(ctl, 8);
        if (!s_fpfail) {
            if (tid == 0) {
                C.U0 = s_fpz[0]; C.uerr = s_fpz[1]; C.V = s_fpz[2]; C.E = s_fpz[3];
                C.rm_bound = s_fpz[6]; C.eps = s_fpz[7];
                C.rlo = fmin(C.rlo, s_fpz[4]); C.rhi = fmax(C.rhi, s_fpz[5]);
                C.incr_ok = 0; C.wskip = 0.0;
                C.ub_sub = a.ubdesc && a.R.n <= STEP_THREADS && (s_fpnsub > 0 || a.ub_heavy) ? 1 : 0;
                C.frz_n = C.frz_n + 1;
                C.ub[0] = s_fpub[0] == NONE64 ? HUGE_VAL : dec(s_fpub[0]);
                C.ub[1] = s_fpub[1] == NONE64 ? HUGE_VAL : dec(s_fpub[1]);
                C.want_refresh = (s_fpz[8] != 0.0 || C.ndirty >= 256) ? 1 : 0;
                C.ncont = 0;
                C.cont_overflow = 0;
                C.fp = 1;
                C.fp_t[0] = t0; C.fp_t[1] = t1;
                C.fp_o[0] = o0; C.fp_o[1] = o1;
                C.fp_n[0] = n0; C.fp_n[1] = n1;
                C.fp_u[0] = u0; C.fp_u[1] = u1;
                C.prepped = 1; C.full_prep = 0;
                C.total_fp++;
            }
            KB_STAMP(ctl, 10);
            write_back();
            return;
        }
        // (a set left with too short a certain prefix: the full prep below; the records FP2
        // wrote are rewritten there, the r[] it wrote are the same values)
        if (tid == 0) { s_cntT[0] = 0; s_cntT[1] = 0; }
        __syncthreads();
    }
    if (!GB && !full && a.sb_lds) {
        // ---- fused incremental prep, wave-specialised.  A wave reduction of a double
        // costs ~340 clocks when all 16 waves run one (four per SIMD, issue-bound) and
        // ~100 when one wave per SIMD does (tools/lat_probe.hip), while a workgroup
        // barrier costs ~25: so the reductions run on the four "sum waves" (one per
        // SIMD: S -> avg -> r -> U0 / V / Rm, the upper bound), the other twelve
        // "order waves" re-sort the touched brokers and mark the sets meanwhile, and
        // the phases are joined by barriers.  Four barriers, then the bl_move
        // positions and the set records.
        constexpr int NRW = 4;                          // sum waves (waves 0..3)
        constexpr int OT = STEP_THREADS - NRW * 64;     // order-wave threads
        constexpr int NQ = (MAXB + OT - 1) / OT;
        const int ot = tid - NRW * 64;                  // order-wave thread index (< 0: sum wave)
        // frozen average: after a plain move (bl_move unchanged) the real load sum is what the
        // last full recompute folded, so avg / inv_avg stay; only the touched brokers' r
        // change, and U0 / V / E / R / the r range follow incrementally (the sums over every
        // broker and their reductions are skipped).  eps doubles (the frozen fold's rounding
        // next to a fresh fold's) plus uerr, the rounding of the incremental U0 updates.  A
        // full recompute every FRZ_MAX steps, after a membership change and after a full prep.
        // (replace / swap keep the real load sum: the weight changes brokers; a remove or an
        // add changes it, and then the sums are folded again)
        const bool frz = do_res && D.status == 1 && (D.kind == 1 || D.kind == 4) && !s_memb && C.frz_n > 0 &&
                         C.frz_n < FRZ_MAX && !a.eager && !(KB_ABL & 32);
        __shared__ double s_fz[6];                      // frozen step: dU, |updates|, dV, dE, r lo / hi
        __shared__ double s_fq[2][NRW], s_fq2[7][NW];
        __shared__ int s_fcnt[NRW];
        __shared__ int s_rt[MAXB / 64];                 // bl_move brokers per 64 universe positions
        __shared__ int s_nsub, s_mn, s_mw;
        // the marked sets in set order from word w0 on, at most MCAP of them (wave 1):
        // the compact list of the record rebuild
        constexpr int MCAP = 2 * DEDUP_STEP;
        int* s_mlist = (int*)s_it;                      // (the key table is free after the resolve)
        const int nwords = (a.nsets + 31) / 32;
        auto compact = [&](int w0) {
            int n = 0, w = w0;
            while (w < nwords) {
                const int ww = w + lane;
                const uint32_t bits = ww < nwords ? s_smark[ww] : 0u;
                const int c = __popc(bits);
                const int incl = wave_incl_scan(c);
                const bool fits = ww < nwords && n + incl <= MCAP;
                const int nfit = (int)__popcll(__ballot(fits));   // a prefix of the lanes
                if (fits) {
                    int k = n + incl - c;
                    for (uint32_t m = bits; m; m &= m - 1) s_mlist[k++] = ww * 32 + __ffs(m) - 1;
                }
                if (nfit > 0) n += __shfl(incl, nfit - 1);
                w += nfit;
                if (nfit < 64) break;
            }
            if (lane == 0) { s_mn = n; s_mw = w; }
        };
        // ---- P1.  sum waves: S, E, |bl_move| partials and the bl_move bits by broker id;
        // order waves: old positions of the touched brokers, the sets holding one
        // the records' best keys for the upper bound (P2): issued now, in flight during P1
        // (held in registers from the header load, they would stay live through the
        // resolve, the apply and the exact folds)
        const bool bkeys = do_res && tid < a.R.n;
        Contender bk0, bk1, bx0, bx1;
        bk0.s = bk1.s = bx0.s = bx1.s = -1;
        if (bkeys) { bk0 = ldobj(&a.R.h(tid)->best[0]); bk1 = ldobj(&a.R.h(tid)->best[1]); }
        if (bkeys && !a.use_spill) {                  // rank summaries: the second-best keys too
            bx0 = ldobj(a.R.k(tid) + (a.R.cap - 2)); bx1 = ldobj(a.R.k(tid) + (a.R.cap - 1));
        }
        if (tid < nT) { s_fl[s_T[tid]] |= BF_TOUCHED; s_cntT[tid] = 0; }
        if (tid == 0) { s_unc = 0; s_nsub = 0; }
        if (wid < NRW) {
            double sS = 0.0, sE = 0.0;
            int cn = 0;
            for (int b0 = wid * 64; b0 < ((KB_ABL & 4) ? 0 : B); b0 += NRW * 64) {
                const int b = b0 + lane;
                const bool in = b < B && (s_fl[b] & (BF_PRESENT | BF_INCFG));
                if (in) { sS += s_ld[b]; sE += s_e[b]; cn++; }
                const unsigned long long m = __ballot(in);
                if (lane == 0) s_blmb[b0 >> 6] = m;
            }
            if (!frz) {
                sS = wave_sum(sS); sE = wave_sum(sE); cn = wave_sum(cn);
                if (KB_ABL & 4) { sS = wid ? 0.0 : C.S; sE = wid ? 0.0 : C.E; cn = wid ? 0 : C.nblm; }   // (timing only)
                if (lane == 0) { s_fq[0][wid] = sS; s_fq[1][wid] = sE; s_fcnt[wid] = cn; }
            }
        } else {
            if (nT > 0)
                for (int i = ot; i < B; i += OT) {
                    const int b = s_ord[i];
                    for (int x = 0; x < nT; x++) if (s_T[x] == b) s_posT[x] = i;
                }
            // a set is marked when it holds a touched broker: one lane per set, one
            // ballot per 64 sets (no clear, no atomics)
            for (int s0 = ot - lane; s0 < a.nsets; s0 += OT) {
                const int set = s0 + lane;
                bool hit = false;
                if (set < a.nsets) {
                    const uint64_t* sb = s_sb + (size_t)set * a.W64;
                    for (int x = 0; x < nT; x++) {
                        const int t = s_T[x];
                        hit |= (sb[t >> 6] >> (t & 63)) & 1ull;
                    }
                }
                const unsigned long long m = __ballot(hit);
                if (lane == 0) { s_smark[s0 >> 5] = (uint32_t)m; s_smark[(s0 >> 5) + 1] = (uint32_t)(m >> 32); }
            }
        }
        __syncthreads();                                // #1
        KB_STAMP(ctl, 6);
    KB_STOP(6);
        // ---- P2.  sum waves (and any wave holding a record's best keys): avg, r, U0 /
        // V / Rm partials, the upper bound; order waves: the new positions
        int nb[NQ], np[NQ];
        if (wid < NRW || wid * 64 < (do_res ? a.R.n : 0)) {
            // (the same fixed-order combination on every such wave: identical bits)
            const double S = ((s_fq[0][0] + s_fq[0][1]) + s_fq[0][2]) + s_fq[0][3];
            const int nblm = (s_fcnt[0] + s_fcnt[1]) + (s_fcnt[2] + s_fcnt[3]);
            const double avg = frz ? C.avg : S / (double)nblm;
            const double iav = frz ? C.inv_avg : 1.0 / avg;
            double su = 0.0, v = 0.0, rm = 0.0, rlo = HUGE_VAL, rhi = -HUGE_VAL;
            if (frz && wid == 0) {
                // the touched brokers' new r (lane k: s_T[k]); lane 0 folds the updates
                // (all of them in bl_move: membership is unchanged)
                if (lane < nT) {
                    const int b = s_T[lane];
                    stdbl(a.r + b, rel_ld(s_ld, b, iav));
                }
                if (lane == 0) {
                    double dU = 0.0, aU = 0.0, dV = 0.0, dE = 0.0, rl = HUGE_VAL, rh = -HUGE_VAL;
                    for (int k = 0; k < nT; k++) {
                        const int b = s_T[k];
                        const double rn = rel_ld(s_ld, b, iav);
                        const double ro = __fma_rn(s_Lold[k], iav, -1.0);   // the r[] the base wrote
                        const double fn = fsq(rn), fo = fsq(ro);
                        dU += fn - fo;
                        aU += fn + fo;
                        dV += fabs(rn) * (1.0 + fabs(rn)) - fabs(ro) * (1.0 + fabs(ro));
                        dE += s_e[b] - s_ebold[k];
                        rl = rn < rl ? rn : rl;
                        rh = rn > rh ? rn : rh;
                    }
                    s_fz[0] = dU; s_fz[1] = aU; s_fz[2] = dV; s_fz[3] = dE; s_fz[4] = rl; s_fz[5] = rh;
                }
            } else if (!frz && wid < NRW) {
#pragma unroll 4
                for (int b = wid * 64 + lane; b < ((KB_ABL & 4) ? 0 : B); b += NRW * 64) {
                    double r = 0.0;
                    if (s_fl[b] & (BF_PRESENT | BF_INCFG)) {
                        r = rel_ld(s_ld, b, iav);
                        su += fsq(r);
                        const double ar = fabs(r);
                        v += ar * (1.0 + ar);
                        rm = ar > rm ? ar : rm;
                    }
                    stdbl(a.r + b, r);
                    rlo = r < rlo ? r : rlo;            // the scan's range of r[] (prune bound)
                    rhi = r > rhi ? r : rhi;
                }
            }
            // upper bound of the next step's minimum per kind: the best keys of the scan
            // just resolved whose partition and brokers the applied move did not touch
            // are still candidates; re-scored on the new loads they bound the new minimum
            double ub0 = HUGE_VAL, ub1 = HUGE_VAL;
            int nkeep = 0;
            if (bkeys) {
                const long long pm = s_moved;
                const bool keep_t = keep_touched_keys();
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    const Contender& c = k ? bk1 : bk0;
                    // the block of every best key other than the moved partition's: if no
                    // key survives below, the conditional bound pass scans only these blocks
                    // and the heaviest blocks by weight (engine.cpp fills that part once):
                    // census-free, their minima bound the step's minimum from above, and
                    // they hold last step's best candidates, so the bound stays tight
                    const bool keep = c.s >= 0 && (long long)(c.iter >> 21) != pm;
                    BlockDesc d;
                    d.wmax = keep ? HUGE_VAL : -1.0;
                    d.blk = keep ? (long long)(c.iter >> 21) / BLK : 0;
                    if (a.ubdesc) stobj(a.ubdesc + 2 * tid + k, d);
                    nkeep += keep ? 1 : 0;
                    if (!keep) continue;
                    if (!keep_t && ((s_fl[c.s] | s_fl[c.t]) & BF_TOUCHED)) continue;
                    const double d2 = cont_delta_ld(s_ld, c, iav);
                    if (k == 0) ub0 = d2 < ub0 ? d2 : ub0;
                    else ub1 = d2 < ub1 ? d2 : ub1;
                }
#pragma unroll
                for (int k = 0; k < 2; k++) {                 // (rank summaries' second-best keys)
                    const Contender& c = k ? bx1 : bx0;
                    if (c.s < 0 || (long long)(c.iter >> 21) == pm) continue;
                    if (!keep_t && ((s_fl[c.s] | s_fl[c.t]) & BF_TOUCHED)) continue;
                    const double d2 = cont_delta_ld(s_ld, c, iav);
                    if (k == 0) ub0 = d2 < ub0 ? d2 : ub0;
                    else ub1 = d2 < ub1 ? d2 : ub1;
                }
            }
            ub0 = wave_min(ub0); ub1 = wave_min(ub1);
            // (the kept keys counted per wave: same-address LDS atomics of a whole wave serialise)
            if (a.ubdesc) {
                nkeep = wave_sum(nkeep);
                if (lane == 0 && nkeep) atomicAdd(&s_nsub, nkeep);
            }
            if (!frz && wid < NRW) {
                su = wave_sum(su); v = wave_sum(v); rm = wave_max(rm);
                rlo = wave_min(rlo); rhi = wave_max(rhi);
                if (KB_ABL & 4) { su = wid ? 0.0 : C.U0; v = wid ? 0.0 : C.V; rm = 1.0; rlo = C.rlo; rhi = C.rhi; }   // (timing only)
            }
            if (lane == 0) {
                s_fq2[3][wid] = ub0; s_fq2[4][wid] = ub1;
                if (wid < NRW) {
                    s_fq2[0][wid] = su; s_fq2[1][wid] = v; s_fq2[2][wid] = rm;
                    s_fq2[5][wid] = rlo; s_fq2[6][wid] = rhi;
                }
            }
        } else if (lane == 0) {
            s_fq2[3][wid] = HUGE_VAL; s_fq2[4][wid] = HUGE_VAL;
        }
        if (ot >= 0 && nT > 0) {
            // per untouched element: new position = old - (touched before it) + (touched
            // keys below it); for every touched broker the untouched brokers below it
#pragma unroll
            for (int q = 0; q < NQ; q++) {
                nb[q] = -1;
                np[q] = 0;
                if (q * OT >= B) continue;                  // uniform
                const int i = q * OT + ot;
                const bool in = i < B;
                const int b = in ? s_ord[i] : 0;
                const bool untouched = in && !(s_fl[b] & BF_TOUCHED);
                const double Lb = s_ld[b];
                int below = 0, before = 0;
                for (int x = 0; x < nT; x++) {
                    const int t = s_T[x];
                    const double Lt = s_ld[t];
                    below += ((Lt < Lb) || (Lt == Lb && t < b)) ? 1 : 0;
                    before += s_posT[x] < i ? 1 : 0;
                    const bool b_lt_t = untouched && ((Lb < Lt) || (Lb == Lt && b < t));
                    const unsigned long long bal = __ballot(b_lt_t);
                    if (lane == 0 && bal) atomicAdd(&s_cntT[x], (int)__popcll(bal));
                }
                nb[q] = untouched ? b : -1;
                np[q] = i - before + below;
            }
        }
        __syncthreads();                                // #2
        KB_STAMP(ctl, 8);
    KB_STOP(7);
        // ---- P3.  order waves: scatter into the new order; wave 0: the step totals,
        // eps and the control block; wave 1: the list of marked sets
        if (ot >= 0 && nT > 0) {
#pragma unroll
            for (int q = 0; q < NQ; q++)
                if (q * OT < B && nb[q] >= 0) s_ord[np[q]] = nb[q];
            if (ot < nT) {
                const int t = s_T[ot];
                const double Lt = s_ld[t];
                int rank = 0;
                for (int x = 0; x < nT; x++) {
                    const int t2 = s_T[x];
                    const double L2 = s_ld[t2];
                    rank += ((L2 < Lt) || (L2 == Lt && t2 < t)) ? 1 : 0;
                }
                s_ord[s_cntT[ot] + rank] = t;
            }
        }
        if (wid == 0) {
            const double uu = DBL_EPSILON / 2;
            double S, E, avg, iav, U0, V, Rm, uerr;
            int nblm;
            if (frz) {
                // (the base's sum and average; the increments of this step's touched brokers,
                // each bound grown by a few ulps so it stays a bound)
                S = C.S; nblm = C.nblm; avg = C.avg; iav = C.inv_avg;
                U0 = C.U0 + s_fz[0];
                uerr = C.uerr + 8.0 * uu * (fabs(C.U0) + fabs(U0) + s_fz[1]);
                V = (C.V + s_fz[2]) * (1.0 + 8.0 * uu);
                E = (C.E + s_fz[3]) * (1.0 + 8.0 * uu);
                Rm = fmax(C.rm_bound, fmax(fabs(s_fz[4]), fabs(s_fz[5])));
            } else {
                S = ((s_fq[0][0] + s_fq[0][1]) + s_fq[0][2]) + s_fq[0][3];
                E = ((s_fq[1][0] + s_fq[1][1]) + s_fq[1][2]) + s_fq[1][3];
                nblm = (s_fcnt[0] + s_fcnt[1]) + (s_fcnt[2] + s_fcnt[3]);
                avg = S / (double)nblm;
                iav = 1.0 / avg;
                U0 = ((s_fq2[0][0] + s_fq2[0][1]) + s_fq2[0][2]) + s_fq2[0][3];
                V = ((s_fq2[1][0] + s_fq2[1][1]) + s_fq2[1][2]) + s_fq2[1][3];
                Rm = fmax(fmax(s_fq2[2][0], s_fq2[2][1]), fmax(s_fq2[2][2], s_fq2[2][3]));
                uerr = 0.0;
            }
            const double ub0 = wave_min(lane < NW ? s_fq2[3][lane] : HUGE_VAL);
            const double ub1 = wave_min(lane < NW ? s_fq2[4][lane] : HUGE_VAL);
            // (every lane: the incremental certificate below needs eps on the whole wave)
            const double u = DBL_EPSILON / 2;
            const double n = (double)nblm;
            const double R = Rm + a.wmax * iav;
            const double Ea = E * iav;
            double epsf = 64.0 * u * ((n + 8.0) * (U0 + 2.0 * V) + 4.0 * (1.0 + R) * (1.0 + R));
            double epsl = 16.0 * Ea * (V / (n > 0 ? n : 1.0) + R + 1.0) + 4.0 * Ea * Ea;
            double ep = frz ? 2.0 * (epsf + epsl) + uerr : epsf + epsl;
            if (!(ep > 1e-300)) ep = 1e-300;
            // incremental mode: after a move() with bl_move and the first-index predicates
            // unchanged, the next scan may skip the blocks lighter than wskip
            double ws = 0.0;
            const bool inc = a.incr && do_res && D.status == 1 && D.kind == 1 && (D.step == 7 || D.step == 8) &&
                             nblm == nblm0 && !s_fm && !a.rebalance && !a.sem_go && a.use_spill;
            // (the r range over every broker: frozen steps widen the base's range by the new r)
            const double rlo = frz ? fmin(C.rlo, s_fz[4])
                                   : fmin(fmin(s_fq2[5][0], s_fq2[5][1]), fmin(s_fq2[5][2], s_fq2[5][3]));
            const double rhi = frz ? fmax(C.rhi, s_fz[5])
                                   : fmax(fmax(s_fq2[6][0], s_fq2[6][1]), fmax(s_fq2[6][2], s_fq2[6][3]));
            if (inc) {
                const double ubP = a.allow_leader ? (ub0 > ub1 ? ub0 : ub1) : ub1;
                ws = incr_wskip(rlo, rhi, ubP + 16.0 * ep, avg, iav, lane);
            }
            if (lane == 0) {
                C.rlo = rlo; C.rhi = rhi;
                C.incr_ok = ws > 0.0 ? 1 : 0;
                C.wskip = ws;
                C.ub_sub = a.ubdesc && a.R.n <= STEP_THREADS && (s_nsub > 0 || a.ub_heavy) ? 1 : 0;
                C.S = S; C.avg = avg; C.inv_avg = iav; C.U0 = U0;
                C.V = V; C.eps = ep; C.E = E; C.nblm = nblm;
                C.uerr = uerr; C.rm_bound = Rm;
                C.frz_n = frz ? C.frz_n + 1 : 1;
                // after a first-index stage (Remove/Add/Disallowed) the next step is most
                // likely one too: no census (ub = -inf; k_step re-scans if move() is reached)
                const bool sup = a.use_spill && do_res && D.status == 1 && D.step >= 3 && D.step <= 5;
                C.ub[0] = sup ? -HUGE_VAL : ub0; C.ub[1] = sup ? -HUGE_VAL : ub1;
                C.want_refresh = (epsl > epsf || C.ndirty >= 256) ? 1 : 0;
                C.ncont = 0;
                C.cont_overflow = 0;
            }
        } else if (wid == 1) {
            compact(0);
        }
        __syncthreads();                                // #3
        KB_STAMP(ctl, 9);
    KB_STOP(8);
        // ---- P4.  bl_move = brokers present in the load map or listed in -broker-ids
        // (steps.go:150-157), interleaved (position i = q * STEP_THREADS + tid): order
        // and position writes, order certification, bl_move counts per 64 positions
        constexpr int PQ = (MAXB + STEP_THREADS - 1) / STEP_THREADS;
        int pb[PQ];
        unsigned long long pm[PQ];
        const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
        for (int q = 0; q < PQ; q++) {
            pb[q] = -1; pm[q] = 0;
            if (q * STEP_THREADS >= B) continue;         // uniform
            const int i = q * STEP_THREADS + tid;
            bool f = false;
            if (i < B) {
                const int b = s_ord[i];
                pb[q] = b;
                f = (s_fl[b] & (BF_PRESENT | BF_INCFG)) != 0;
                a.order[i] = b;
                a.posu[b] = i;
                // with approximate loads, neighbours must be separated by more than
                // their error bounds (else the exact order is unknown)
                if (i + 1 < B) {
                    const int b2 = s_ord[i + 1];
                    const double e = s_e[b] + s_e[b2];
                    if (e > 0.0 && !(s_ld[b2] - s_ld[b] > e)) s_unc = 1;
                }
            }
            pm[q] = __ballot(f);
            if (lane == 0 && (i >> 6) < MAXB / 64) s_rt[i >> 6] = (int)__popcll(pm[q]);
        }
        __syncthreads();                                // #4
        KB_STAMP(ctl, 16);
    KB_STOP(9);
        if (s_unc) {
            if (tid == 0) { C.halted = H_NEED_EXACT; C.prepped = 0; C.total_exact_halts++; }
            write_back();
            return;
        }
        // positions: the bl_move brokers before each 64-position row (lane-parallel prefix)
        {
            const int nrows = (B + 63) >> 6;
            const int rc = lane < nrows ? s_rt[lane] : 0;
            const int rincl = wave_incl_scan(rc);
            const int nblm = __builtin_amdgcn_readlane(rincl, 63);
            const int widu = __builtin_amdgcn_readfirstlane(wid);
#pragma unroll
            for (int q = 0; q < PQ; q++) {
                if (q * STEP_THREADS >= B) continue;     // uniform
                // exclusive prefix of this wave's row (rows are wave-uniform)
                const int off = __builtin_amdgcn_readlane(rincl - rc, q * NW + widu);
                if (pb[q] < 0) continue;
                const int b = pb[q];
                if ((pm[q] >> lane) & 1ull) {
                    const int pos = off + (int)__popcll(pm[q] & lt);
                    if (pos == 0) C.light = b;
                    if (pos == nblm - 1) C.heavy = b;
                    st32(a.blm + pos, (uint32_t)b); st32(a.posm + b, (uint32_t)pos);
                } else st32(a.posm + b, NONE32);
            }
            if (tid == 0 && nblm == 0) { C.light = -1; C.heavy = -1; }
        }
        KB_STAMP(ctl, 19);
    KB_STOP(10);
        // ---- P5.  set records of the marked sets (steps.go:192-201 targets): each wave
        // rebuilds G records at a time so their LDS chains overlap
        for (;;) {
            constexpr int G = KB_SET_G;
            const int W64 = a.W64, KR = a.KR;
            const int mn = (KB_ABL & 8) ? 0 : s_mn;
            constexpr int MAXU = sr_units(MAXR);
            __shared__ __align__(16) uint16_t s_rs2[NW][G][8 * MAXU];
            for (int g = wid * G; g < mn; g += NW * G) {
                const int ng = mn - g < G ? mn - g : G;
                const uint64_t* sb[G];
                uint16_t* rec16[G];
                int found[G];
#pragma unroll
                for (int j = 0; j < G; j++) {
                    const int jj = j < ng ? j : 0;
                    sb[j] = s_sb + (size_t)s_mlist[g + jj] * W64;
                    rec16[j] = &s_rs2[wid][j][0];
                    found[j] = j < ng ? 0 : KR;
                }
                for (int base = 0; base < B; base += 64) {
                    bool need = false;
#pragma unroll
                    for (int j = 0; j < G; j++) need |= found[j] < KR;
                    if (!need) break;
                    const int k = base + lane;
                    const int b = s_ord[k < B ? k : 0];
                    const bool inb = k < B && ((s_blmb[b >> 6] >> (b & 63)) & 1ull);
                    uint64_t wj[G];
#pragma unroll
                    for (int j = 0; j < G; j++) wj[j] = sb[j][b >> 6];
#pragma unroll
                    for (int j = 0; j < G; j++) {
                        const bool mem = inb && ((wj[j] >> (b & 63)) & 1ull);
                        const unsigned long long m = __ballot(mem);
                        if (mem && found[j] < KR) {
                            const int rk = found[j] + (int)__popcll(m & lt);
                            if (rk < KR) rec16[j][2 + rk] = (uint16_t)b;
                        }
                        found[j] += (int)__popcll(m);
                    }
                }
                int nj[G];
#pragma unroll
                for (int j = 0; j < G; j++) nj[j] = lane < W64 ? (int)__popcll(sb[j][lane] & s_blmb[lane]) : 0;
#pragma unroll
                for (int j = 0; j < G; j++) nj[j] = wave_sum(nj[j]);   // (independent chains: they overlap)
#pragma unroll
                for (int j = 0; j < G; j++) {
                    if (j >= ng) break;
                    for (int rk = found[j] + lane; rk < KR; rk += 64) rec16[j][2 + rk] = NONE16;
                    if (lane == 0) {
                        rec16[j][1] = (uint16_t)(found[j] < KR ? found[j] : KR);
                        rec16[j][0] = (uint16_t)nj[j];
                    }
                }
                __builtin_amdgcn_wave_barrier();
                if (lane < ng * a.units) {
                    const int j = lane / a.units, u = lane - j * a.units;
                    stobj(a.setrec + (size_t)s_mlist[g + j] * a.units + u, *(const uint4*)&s_rs2[wid][j][8 * u]);
                }
                __builtin_amdgcn_wave_barrier();
            }
            // (more marked sets than one list holds: the next chunk)
            const int mw = s_mw;
            if (mw >= nwords) break;
            __syncthreads();
            if (wid == 1) compact(mw);
            __syncthreads();
        }
        KB_STAMP(ctl, 20);
    KB_STOP(11);
        if (tid == 0) { C.prepped = 1; C.full_prep = 0; }
        write_back();
        return;
    } else {
    if (full) {
        // every load is exact here (fresh state or after k_refresh): s_e holds the sort keys
        unsigned long long* s_k64 = (unsigned long long*)s_e;
        const int NP2 = a.NP2;
        for (int i = tid; i < NP2; i += STEP_THREADS) {
            s_k64[i] = i < B ? d2u(s_ld[i]) : NONE64;
            s_ord[i] = i < B ? i : 0x7FFFFFFF;
        }
        __syncthreads();
        // bitonic sort by (load bits, dense id); loads are finite and >= 0, so the
        // IEEE bit pattern orders like the value (byBrokerLoad.Less, utils.go:23-28)
        for (int k = 2; k <= NP2; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = tid; i < NP2; i += STEP_THREADS) {
                    int ixj = i ^ j;
                    if (ixj > i) {
                        unsigned long long ki = s_k64[i], kj = s_k64[ixj];
                        int32_t ii = s_ord[i], ij = s_ord[ixj];
                        bool less = (kj < ki) || (kj == ki && ij < ii);
                        bool up = (i & k) == 0;
                        if (up == less) { s_k64[i] = kj; s_k64[ixj] = ki; s_ord[i] = ij; s_ord[ixj] = ii; }
                    }
                }
                __syncthreads();
            }
        }
        for (int b = tid; b < B; b += STEP_THREADS) s_e[b] = 0.0;
    } else if (nT > 0) {
        // incremental: only the touched brokers moved (their loads changed)
        if (tid < nT) { s_fl[s_T[tid]] |= BF_TOUCHED; s_cntT[tid] = 0; }
        __syncthreads();
        for (int i = tid; i < B; i += STEP_THREADS) {
            const int b = s_ord[i];
            if (s_fl[b] & BF_TOUCHED)
                for (int x = 0; x < nT; x++) if (s_T[x] == b) s_posT[x] = i;
        }
        __syncthreads();
        // per untouched element: new position = old - (touched before it) + (touched keys below it)
        int nb[(MB + STEP_THREADS - 1) / STEP_THREADS], np[(MB + STEP_THREADS - 1) / STEP_THREADS];
#pragma unroll
        for (int q = 0; q < (MB + STEP_THREADS - 1) / STEP_THREADS; q++) {
            nb[q] = -1;
            if (q * STEP_THREADS >= B) continue;         // uniform
            const int i = q * STEP_THREADS + tid;
            const bool in = i < B;
            const int b = in ? s_ord[i] : 0;
            const bool untouched = in && !(s_fl[b] & BF_TOUCHED);
            const double Lb = s_ld[b];
            int below = 0, before = 0;
            for (int x = 0; x < nT; x++) {
                const int t = s_T[x];
                const double Lt = s_ld[t];
                below += ((Lt < Lb) || (Lt == Lb && t < b)) ? 1 : 0;
                before += s_posT[x] < i ? 1 : 0;
                // count, for touched t, the untouched brokers below it
                const bool b_lt_t = untouched && ((Lb < Lt) || (Lb == Lt && b < t));
                const unsigned long long bal = __ballot(b_lt_t);
                if (lane == 0 && bal) atomicAdd(&s_cntT[x], (int)__popcll(bal));
            }
            nb[q] = untouched ? b : -1;
            np[q] = i - before + below;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < (MB + STEP_THREADS - 1) / STEP_THREADS; q++)
            if (nb[q] >= 0) s_ord[np[q]] = nb[q];
        if (tid < nT) {
            const int t = s_T[tid];
            const double Lt = s_ld[t];
            int rank = 0;
            for (int x = 0; x < nT; x++) {
                const int t2 = s_T[x];
                const double L2 = s_ld[t2];
                rank += ((L2 < Lt) || (L2 == Lt && t2 < t)) ? 1 : 0;
            }
            s_ord[s_cntT[tid] + rank] = t;
        }
    }
    __syncthreads();
    KB_STAMP(ctl, 6);
    // bl_move = brokers present in the load map or listed in -broker-ids (steps.go:150-157)
    for (int w = tid; w < MB / 64; w += STEP_THREADS) { s_blmb[w] = 0; s_presb[w] = 0; }
    if (tid == 0) s_unc = 0;
    __syncthreads();
    {
        constexpr int FQ = MB / STEP_THREADS;           // universe positions per thread
        int flag[FQ], c = 0;
        const int base = tid * FQ;
#pragma unroll
        for (int q = 0; q < FQ; q++) {
            const int i = base + q;
            flag[q] = 0;
            if (i < B) {
                const int b = s_ord[i];
                const uint8_t fl = s_fl[b];
                const bool pres = (fl & BF_PRESENT) != 0;
                flag[q] = (fl & (BF_PRESENT | BF_INCFG)) ? 1 : 0;
                if (flag[q]) atomicOr((unsigned long long*)&s_blmb[b >> 6], 1ull << (b & 63));
                if (pres) atomicOr((unsigned long long*)&s_presb[b >> 6], 1ull << (b & 63));
                c += flag[q];
                a.order[i] = b;
                a.posu[b] = i;
                // order certification: with approximate loads, neighbours must be
                // separated by more than their error bounds (else the exact order is unknown)
                if (i + 1 < B) {
                    const int b2 = s_ord[i + 1];
                    const double e = s_e[b] + s_e[b2];
                    if (e > 0.0 && !(s_ld[b2] - s_ld[b] > e)) s_unc = 1;
                }
            }
        }
        int incl = c;
        incl = wave_incl_scan(incl);
        __shared__ int s_wcnt[NW];
        if (lane == 63) s_wcnt[wid] = incl;
        __syncthreads();
        const int wc = lane < NW ? s_wcnt[lane] : 0;
        const int woff = wave_sum(lane < wid ? wc : 0), total = wave_sum(wc);
        int pos = woff + incl - c;
#pragma unroll
        for (int q = 0; q < FQ; q++) {
            const int i = base + q;
            if (i < B) {
                const int b = s_ord[i];
                if (flag[q]) {
                    // the first / last bl_move broker: getBL's lightest / heaviest
                    if (pos == 0) C.light = b;
                    if (pos == total - 1) C.heavy = b;
                    st32(a.blm + pos, (uint32_t)b); st32(a.posm + b, (uint32_t)pos); pos++;
                } else st32(a.posm + b, NONE32);
            }
        }
        if (tid == 0) {
            s_nblm = total;
            if (total == 0) { C.light = -1; C.heavy = -1; }
        }
    }
    __syncthreads();
    const int nblm = s_nblm;
    if (s_unc) {
        if (tid == 0) { C.halted = H_NEED_EXACT; C.prepped = 0; C.total_exact_halts++; }
        write_back();
        return;
    }
    KB_STAMP(ctl, 8);
    // the records' best keys (re-scored below for the next step's upper bound; one
    // record per thread): loaded first, their latency overlaps the sums
    const bool bkeys = do_res && !full && tid < a.R.n;
    Contender bk0, bk1, bx0, bx1;
    bk0.s = bk1.s = bx0.s = bx1.s = -1;
    if (bkeys) { bk0 = ldobj(&a.R.h(tid)->best[0]); bk1 = ldobj(&a.R.h(tid)->best[1]); }
    if (bkeys && !a.use_spill) {                      // rank summaries: the second-best keys too
        bx0 = ldobj(a.R.k(tid) + (a.R.cap - 2)); bx1 = ldobj(a.R.k(tid) + (a.R.cap - 1));
    }
    // approximate S (exact in integral mode: integers below 2^52), total load error E
    double sS = 0.0, sE = 0.0;
    for (int b = tid; b < B; b += STEP_THREADS)
        if (s_fl[b] & (BF_PRESENT | BF_INCFG)) { sS += s_ld[b]; sE += s_e[b]; }
    __shared__ double s_q[3][NW];
    sS = wave_sum(sS); sE = wave_sum(sE);
    if (lane == 0) { s_q[0][wid] = sS; s_q[1][wid] = sE; }
    __syncthreads();
    // the wave partials, combined lane-parallel (no serial LDS chain)
    const double S = wave_sum(lane < NW ? s_q[0][lane] : 0.0), E = wave_sum(lane < NW ? s_q[1][lane] : 0.0);
    const double avg = S / (double)nblm;
    const double iav = 1.0 / avg;
    double su = 0.0, v = 0.0, rm = 0.0, rlo = HUGE_VAL, rhi = -HUGE_VAL;
    for (int b = tid; b < B; b += STEP_THREADS) {
        double r = 0.0;
        if (s_fl[b] & (BF_PRESENT | BF_INCFG)) {
            r = rel_ld(s_ld, b, iav);
            su += fsq(r);
            const double ar = fabs(r);
            v += ar * (1.0 + ar);
            rm = ar > rm ? ar : rm;
        }
        stdbl(a.r + b, r);
        rlo = r < rlo ? r : rlo;                    // the scan's range of r[] (prune bound)
        rhi = r > rhi ? r : rhi;
    }
    su = wave_sum(su); v = wave_sum(v); rm = wave_max(rm);
    rlo = wave_min(rlo); rhi = wave_max(rhi);
    __shared__ double s_rr2[2][NW];
    if (lane == 0) { s_rr2[0][wid] = rlo; s_rr2[1][wid] = rhi; }
    // upper bound of the next step's minimum per kind: the near-tie keys of the scan
    // just resolved whose partition and brokers the applied move did not touch are
    // still candidates; re-scored on the new loads they bound the new minimum
    double ub0 = HUGE_VAL, ub1 = HUGE_VAL;
    if (bkeys) {
        const long long pm = s_moved;
        const bool keep_t = keep_touched_keys();
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const Contender& c = k == 0 ? bk0 : k == 1 ? bk1 : k == 2 ? bx0 : bx1;
            if (c.s < 0 || (long long)(c.iter >> 21) == pm) continue;
            if (!keep_t && ((s_fl[c.s] | s_fl[c.t]) & BF_TOUCHED)) continue;
            const double d = cont_delta_ld(s_ld, c, iav);
            if ((k & 1) == 0) ub0 = d < ub0 ? d : ub0;          // (k = 0, 2: leader keys)
            else ub1 = d < ub1 ? d : ub1;
        }
    }
    KB_STAMP(ctl, 0);
    ub0 = wave_min(ub0); ub1 = wave_min(ub1);
    __shared__ double s_ubw[2][NW];
    __syncthreads();
    if (lane == 0) { s_q[0][wid] = su; s_q[1][wid] = v; s_q[2][wid] = rm; s_ubw[0][wid] = ub0; s_ubw[1][wid] = ub1; }
    __syncthreads();
    KB_STAMP(ctl, 17);
    if (wid == 0) {
        const bool in = lane < NW;
        const double U0 = wave_sum(in ? s_q[0][lane] : 0.0), V = wave_sum(in ? s_q[1][lane] : 0.0);
        const double Rm = wave_max(in ? s_q[2][lane] : 0.0);
        ub0 = wave_min(in ? s_ubw[0][lane] : HUGE_VAL);
        ub1 = wave_min(in ? s_ubw[1][lane] : HUGE_VAL);
        const double rlo2 = wave_min(in ? s_rr2[0][lane] : HUGE_VAL), rhi2 = wave_max(in ? s_rr2[1][lane] : -HUGE_VAL);
#ifdef KB_STAMPS
        if (lane == 0) KB_STAMP(ctl, 18);
#endif
      if (lane == 0) {
        const double u = DBL_EPSILON / 2;
        const double n = (double)nblm;
        const double R = Rm + a.wmax * iav;
        const double Ea = E * iav;
        double epsf = 64.0 * u * ((n + 8.0) * (U0 + 2.0 * V) + 4.0 * (1.0 + R) * (1.0 + R));
        double epsl = 16.0 * Ea * (V / (n > 0 ? n : 1.0) + R + 1.0) + 4.0 * Ea * Ea;
        double ep = epsf + epsl;
        if (!(ep > 1e-300)) ep = 1e-300;
        C.S = S; C.avg = avg; C.inv_avg = iav; C.U0 = U0;
        C.V = V; C.eps = ep; C.E = E; C.nblm = nblm;
        C.rlo = rlo2; C.rhi = rhi2;
        const bool sup = a.use_spill && do_res && !full && D.status == 1 && D.step >= 3 && D.step <= 5;
        C.ub[0] = sup ? -HUGE_VAL : ub0; C.ub[1] = sup ? -HUGE_VAL : ub1;
        C.incr_ok = 0;                      // (the next scan reads every block)
        C.wskip = 0.0;
        C.ub_sub = 0;                       // (a bound pass, if any, scans every tile)
        C.want_refresh = (epsl > epsf || C.ndirty >= 256) ? 1 : 0;
        C.ncont = 0;
        C.cont_overflow = 0;
      }
    }
    }
    KB_STAMP(ctl, 9);
    // ---- set records: full, or the sets containing a touched broker.  Past MAX_SETS sets
    // (the LDS bitmap's capacity) the sets come as a list instead: every set, or the
    // touched brokers' set lists (a set in two of them is rebuilt twice, identically)
    const bool bigm = BIG && a.nsets > (int)MAX_SETS;
    __shared__ int s_bo[TMAX + 1], s_bb[TMAX];
    for (int w = tid; !bigm && !marked && w < (a.nsets + 31) / 32; w += STEP_THREADS) {
        const int rem = a.nsets - w * 32;                 // only bits of existing sets
        s_smark[w] = full ? (rem >= 32 ? 0xFFFFFFFFu : (1u << rem) - 1u) : 0u;
    }
    if (marked) {
        // (marked by the fused prep)
    } else if (!full && a.sb_lds) {
        // resident words: a set is marked when it holds a touched broker
        __syncthreads();
        for (int set = tid; set < a.nsets; set += STEP_THREADS) {
            const uint64_t* sb = s_sb + (size_t)set * a.W64;
            bool hit = false;
            for (int x = 0; x < nT; x++) {
                const int t = s_T[x];
                hit |= (sb[t >> 6] >> (t & 63)) & 1ull;
            }
            if (hit) atomicOr(&s_smark[set >> 5], 1u << (set & 31));
        }
    } else if (!full) {
        // two memory round trips: the touched brokers' set-list extents, then the lists
        if (tid < nT) {
            const int t = s_T[tid];
            const int o0 = a.bset_off[t], o1 = a.bset_off[t + 1];
            s_bb[tid] = o0;
            s_bo[tid] = o1 - o0;
        }
        __syncthreads();
        if (wid == 0) {
            const int c = lane < nT ? s_bo[lane] : 0;
            int incl = c;
            incl = wave_incl_scan(incl);
            if (lane < nT) s_bo[lane] = incl - c;
            if (lane == nT - 1) s_bo[nT] = incl;
            if (nT == 0 && lane == 0) s_bo[0] = 0;
        }
        __syncthreads();
        const int tot = s_bo[nT];
        for (int q = tid; !bigm && q < tot; q += STEP_THREADS) {
            int x = 0;
            while (x + 1 < nT && s_bo[x + 1] <= q) x++;
            const int set = a.bset_ids[s_bb[x] + q - s_bo[x]];
            atomicOr(&s_smark[set >> 5], 1u << (set & 31));
        }
    }
    __syncthreads();
    KB_STAMP(ctl, 16);
    if (!(KB_ABL & 1) || full) {     // (KB_ABL & 1: diagnostic timing build without the rebuild)
        // marked sets in chunks of the compact list (allowed-set words resident in LDS,
        // or staged per chunk: one round trip); each wave rebuilds four records at a
        // time so their LDS chains overlap
        constexpr int G = 4;
        uint64_t* s_stage = (uint64_t*)s_wb;               // [CH * W64] (dedup table: free here)
        int* s_mlist = (int*)s_it;                         // [CH]
        __shared__ int s_mn, s_cursor;
        const int W64 = a.W64, KR = a.KR;
        // (past MAXB brokers the words are read from memory where they lie: a staged chunk
        // of DEDUP_STEP / W64 < 32 sets could not take a whole mark word, the compaction
        // below needs room for 32)
        const bool stage = !GB && !a.sb_lds;
        const int CH = stage ? DEDUP_STEP / W64 : 2 * DEDUP_STEP;   // >= 32
        const int nwords = (a.nsets + 31) / 32;
        const unsigned long long lt = (1ull << lane) - 1ull;
        // each wave builds its records in LDS, then writes them as whole 16-B units
        constexpr int MAXU = sr_units(MAXR);
        __shared__ __align__(16) uint16_t s_rs[NW][G][8 * MAXU];
        if (tid == 0) s_cursor = 0;
        __syncthreads();
        const int lim = bigm ? (full ? a.nsets : s_bo[nT]) : nwords;
        for (;;) {
            // (every thread reads the cursor before wave 0 may advance it: a wave reading
            // the advanced cursor would leave the loop, skip its records and the barriers)
            const int c0 = s_cursor;
            if (c0 >= lim) break;
            __syncthreads();
            int bn = 0;
            if (bigm) {
                // the next CH sets of the list
                bn = min(CH, lim - c0);
                for (int q = tid; q < bn; q += STEP_THREADS) {
                    int set = c0 + q;
                    if (!full) {
                        int x = 0;
                        while (x + 1 < nT && s_bo[x + 1] <= set) x++;
                        set = a.bset_ids[s_bb[x] + set - s_bo[x]];
                    }
                    s_mlist[q] = set;
                }
                if (tid == 0) s_mn = bn;
            } else if (wid == 0) {
                // the next marked sets, up to CH, in set order
                int n = 0, w = c0;
                while (w < nwords) {
                    const int ww = w + lane;
                    const uint32_t bits = ww < nwords ? s_smark[ww] : 0u;
                    const int c = __popc(bits);
                    int incl = c;
                    incl = wave_incl_scan(incl);
                    const bool fits = ww < nwords && n + incl <= CH;
                    const int nfit = (int)__popcll(__ballot(fits));       // a prefix of the lanes
                    if (fits) {
                        int k = n + incl - c;
                        for (uint32_t m = bits; m; m &= m - 1) s_mlist[k++] = ww * 32 + __ffs(m) - 1;
                    }
                    if (nfit > 0) n += __shfl(incl, nfit - 1);
                    w += nfit;
                    if (nfit < 64) break;                  // the words are exhausted or the chunk is full
                }
                if (lane == 0) { s_mn = n; s_cursor = w; }
            }
            __syncthreads();
            KB_STAMP(ctl, 19);
            if (bigm && tid == 0) s_cursor = c0 + bn;      // (every thread has read the old cursor)
            const int mn = s_mn;
            if (stage) {
                for (int q = tid; q < mn * W64; q += STEP_THREADS) {
                    const int i = q / W64, wd = q - i * W64;
                    s_stage[q] = a.setbits[(size_t)s_mlist[i] * W64 + wd];
                }
                __syncthreads();
            }
            for (int g = wid * G; g < mn; g += NW * G) {
                const int ng = mn - g < G ? mn - g : G;
                const uint64_t* sb[G];
                uint16_t* rec16[G];
                int found[G];
#pragma unroll
                for (int j = 0; j < G; j++) {
                    const int jj = j < ng ? j : 0;
                    const int set = s_mlist[g + jj];
                    sb[j] = a.sb_lds ? s_sb + (size_t)set * W64
                                     : (GB ? a.setbits + (size_t)set * W64 : s_stage + (size_t)(g + jj) * W64);
                    rec16[j] = &s_rs[wid][j][0];
                    found[j] = j < ng ? 0 : KR;
                }
                // the first KR brokers of set ∩ bl_move in bl order (move targets, steps.go:192-201);
                // PP positions per lane and iteration (one iteration almost always suffices)
#ifndef KB_SET_PP
#define KB_SET_PP 1
#endif
                constexpr int PP = KB_SET_PP;
                for (int base = 0; base < B; base += 64 * PP) {
                    bool need = false;
#pragma unroll
                    for (int j = 0; j < G; j++) need |= found[j] < KR;
                    if (!need) break;
                    // every word read unconditionally: one LDS round trip for all of them
                    int bq[PP];
                    bool inb[PP];
                    uint64_t wj[PP][G];
#pragma unroll
                    for (int q = 0; q < PP; q++) {
                        const int k = base + q * 64 + lane;
                        bq[q] = s_ord[k < B ? k : 0];
                    }
#pragma unroll
                    for (int q = 0; q < PP; q++) {
                        const int b = bq[q];
                        inb[q] = base + q * 64 + lane < B && ((s_blmb[b >> 6] >> (b & 63)) & 1ull);
#pragma unroll
                        for (int j = 0; j < G; j++) wj[q][j] = sb[j][b >> 6];
                    }
#pragma unroll
                    for (int j = 0; j < G; j++) {
#pragma unroll
                        for (int q = 0; q < PP; q++) {
                            const int b = bq[q];
                            const bool mem = inb[q] && ((wj[q][j] >> (b & 63)) & 1ull);
                            const unsigned long long m = __ballot(mem);
                            if (mem && found[j] < KR) {
                                const int rk = found[j] + (int)__popcll(m & lt);
                                if (rk < KR) rec16[j][2 + rk] = (uint16_t)b;
                            }
                            found[j] += (int)__popcll(m);
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < G; j++) {
                    if (j >= ng) break;
                    for (int rk = found[j] + lane; rk < KR; rk += 64) rec16[j][2 + rk] = NONE16;
                    if (lane == 0) rec16[j][1] = (uint16_t)(found[j] < KR ? found[j] : KR);
                    int n = 0;
#pragma unroll
                    for (int q = 0; q < MB / 4096; q++) {
                        const int wi = q * 64 + lane;
                        n += wi < W64 ? (int)__popcll(sb[j][wi] & s_blmb[wi]) : 0;
                    }
                    n = wave_sum(n);
                    if (lane == 0) rec16[j][0] = (uint16_t)n;
                }
                __builtin_amdgcn_wave_barrier();
                if (lane < ng * a.units) {
                    const int j = lane / a.units, u = lane - j * a.units;
                    const int set = s_mlist[g + j];
                    stobj(a.setrec + (size_t)set * a.units + u, *(const uint4*)&s_rs[wid][j][8 * u]);
                }
                __builtin_amdgcn_wave_barrier();
            }
            __syncthreads();
            KB_STAMP(ctl, 20);
        }
    }
    if (tid == 0) { C.prepped = 1; C.full_prep = 0; C.frz_n = 0; }   // (no frozen base)
    KB_STAMP(ctl, 10);
    write_back();
}

// (BIG: more broker lists than the meta word's set field / the LDS mark bitmap hold --
// a separate instantiation, so the common kernel's register allocation is untouched)
template <bool BIG, bool GB = false>
__global__ __launch_bounds__(STEP_THREADS) void k_step(StepArgs a) {
    __shared__ DevCtl C;
    step_body<BIG, GB>(a, C);
}

// One Balance() step in one launch: the scan's grid (scan, list and eager workgroups) plus
// one resident step workgroup, the last of the grid.  Every other workgroup publishes its
// writes (agent-scope release) and counts itself in; the step workgroup stages the broker
// tables while the scan runs, waits for the count, and resolves, applies and preps as
// k_step does.  Dispatch is in grid order within an XCD, so every workgroup the step
// workgroup waits for was dispatched before it or on another XCD: no wait can starve.
// (Replaces the k_step launch of a pair: its dispatch gap behind the scan and the staging
// round trip leave the step's critical path.)
// (BK: the scanning workgroups keep bound keys -- the best key of every scored wave outside
// the census, scan_round -- the instantiation launched for plans without -allow-leader)
template <int RC, bool LSETS, bool BK = false>
__global__ __launch_bounds__(SCAN_THREADS) void k_pair(ScanArgs a, StepArgs sa) {
    static_assert(SCAN_THREADS == STEP_THREADS, "one workgroup shape for both roles");
    if ((int)blockIdx.x == (int)gridDim.x - 1) {
        __shared__ DevCtl C;
        step_body<false, false, true>(sa, C);
        return;
    }
    // (a scanning workgroup's hand-off is write-through stores; the list and eager workgroups
    // and an in-stream refresh write plain and publish with an agent-scope release)
    const bool wt = (int)blockIdx.x < a.nscan && !(a.rfpass && a.ctl->halted == H_NEED_EXACT);
    scan_kernel_body<RC, LSETS, false, false, BK>(a);
    // publish (MI355X_MICROARCH.md, inter-workgroup visibility): every wave drains its stores,
    // then one lane (after an L2 write-back where the stores were plain) counts the
    // workgroup in
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!wt) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __hip_atomic_fetch_add(a.done + (blockIdx.x % PAIR_SHARDS) * PAIR_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ------------------------------------------------------------- k_listop

#if KB_IN_TU(0)
__global__ __launch_bounds__(1024) void k_listop(DevCtl* ctl, Lists L) {
    __shared__ int s_i;
    do_list_op(ctl, L, &s_i);
}
#endif

// ------------------------------------------------------------ k_refresh
// exact partition-ordered refold (getBrokerLoad, utils.go:92-105) of every
// dirty broker: one workgroup per broker; contributions staged in LDS chunks,
// folded sequentially by one lane.

[[maybe_unused]] constexpr int REFRESH_THREADS = 256;
[[maybe_unused]] constexpr int REFRESH_CHUNK = 1024;
// The exact getBrokerLoad fold (utils.go:92-105) of broker b's contributions in partition
// order by one workgroup of NT threads (every thread calls; the result is wave 0's).
// Double-buffered: while wave 0 folds chunk j (a broadcast-LDS add chain), waves 1..
// gather chunk j + 1 from the partition list -- every list load of a thread first, then
// the partition words they index, then the LDS writes (two round trips per chunk, not
// two per element).  buf: 2 * CH doubles of LDS.
// (x: the list's extent when the caller has it -- the eager refold, right after its edit)
template <int NT, int CH>
__device__ __forceinline__ double refold_broker(const RefreshArgs& a, int b, double* buf, const ListExt* xk = nullptr) {
    constexpr int GT = NT - 64, PER = (CH + GT - 1) / GT;
    static_assert(CH % 64 == 0, "whole checkpoint blocks per chunk");
    const ListExt x = xk ? *xk : list_ext(a.L, b);
    const uint32_t st = x.st, n = x.n;
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    // restart at the last checkpoint below the first changed position: the fold of the
    // unchanged prefix is that checkpoint's value, bit for bit (the same chain)
    const uint32_t dp = x.dp;
    const uint32_t base = (dp < n ? dp : n) & ~63u;
    const double acc0 = base ? a.L.ck[st + base - 1] : 0.0;
    auto gather = [&](uint32_t c0, double* dst) {
        const int t = tid - 64;
        uint32_t q[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const uint32_t i = (uint32_t)(t + k * GT);
            q[k] = i < (uint32_t)CH && c0 + i < n ? a.L.lent[st + c0 + i] : NONE32;
        }
        double w[PER];
        uint32_t mq[PER];
        int32_t ncq[PER];
        uint16_t r0[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const uint32_t qq = q[k] != NONE32 ? q[k] : 0u;
            w[k] = a.w[qq]; mq[k] = a.meta[qq]; ncq[k] = a.nc[qq]; r0[k] = a.rep[qq];
        }
#pragma unroll
        for (int k = 0; k < PER; k++)
            if (q[k] != NONE32)   // slot 0 carries the leader weight W * (len(R) + NumConsumers)
                dst[t + k * GT] = r0[k] == (uint16_t)b ? w[k] * (double)((int)meta_nrep(mq[k]) + ncq[k]) : w[k];
    };
    double acc = acc0;
    if (wid > 0 && base < n) gather(base, buf);
    __syncthreads();
    for (uint32_t c0 = base, j = 0; c0 < n; c0 += CH, j++) {
        const uint32_t m = n - c0 < (uint32_t)CH ? n - c0 : (uint32_t)CH;
        if (wid > 0 && c0 + CH < n) gather(c0 + CH, buf + ((j + 1) & 1) * CH);
        if (wid == 0) {
            // the chain in 64-element blocks, a checkpoint after each whole one
            const lds_f64* x = (const lds_f64*)(buf + (j & 1) * CH);
            for (uint32_t u = 0; u < m; u += 64) {
                const int mm = m - u < 64u ? (int)(m - u) : 64;
                acc = chain_lds(acc, x + u, mm);
                if (mm == 64 && lane == 0) a.L.ck[st + c0 + u + 63] = acc;
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        a.load[b] = acc;
        a.lerr[b] = gamma_n((int)n) * acc;
        a.eb[b] = 0.0;
        a.bfl[b] = a.bfl[b] & ~BF_DIRTY;
        a.L.dpos[b] = NONE32;
    }
    return acc;
}

// One workgroup per dirty broker (the host's refresh after a batch halted for exact loads)
#if KB_IN_TU(0)
__global__ __launch_bounds__(REFRESH_THREADS) void k_refresh(RefreshArgs a) {
    const int b = blockIdx.x;
    if (b >= a.B || !(a.bfl[b] & BF_DIRTY)) return;
    __shared__ __align__(16) double s_c[2 * REFRESH_CHUNK];
    refold_broker<REFRESH_THREADS, REFRESH_CHUNK>(a, b, s_c);
}
#endif

// The same refresh inside the stream: the first scan launch of the pair after a k_step
// that halted for exact loads (ScanArgs.rfpass) refolds the dirty brokers instead of
// scanning -- workgroup 0 first applies the pending per-broker list edit and then folds
// the edited lists' brokers itself; every workgroup folds the dirty brokers of its
// grid stride -- and the pair's k_step resumes with a full prep (StepArgs.rf_final).
// No host round trip, and the pairs enqueued behind the halt do real steps.  (The
// arguments come from device memory, not the kernel-argument struct: a by-value copy
// passed to this call would give every scan wave a stack frame.)
__device__ __attribute__((noinline)) void refresh_in_scan(const RefreshArgs* rfp, int pend, int kind, int from, int to,
                                                          uint32_t part, double* buf, int ng) {
    const RefreshArgs rf = *rfp;
    // (a list that overflowed earlier: the host relists and refreshes; k_step leaves the
    // halt to it, StepArgs.rf_final)
    if (rf.ctl->list_overflow) return;
    __shared__ int s_i;
    const int g = blockIdx.x;
    const bool ef = pend && kind != 3 && from >= 0, et = pend && kind != 2 && to >= 0;
    bool ok = true;                       // (workgroup-uniform: list_insert reads llen / lcap)
    if (g == 0 && pend) {
        if (kind == 1) { list_remove(rf.L, from, part, &s_i); ok = list_insert(rf.L, to, part, &s_i); }
        else if (kind == 2) list_remove(rf.L, from, part, &s_i);
        else if (kind == 3) ok = list_insert(rf.L, to, part, &s_i);
        if (!ok && threadIdx.x == 0) rf.ctl->list_overflow = 1;   // the host relists (refresh)
        __syncthreads();
    }
    // A failed insert left `to`'s list without the moved partition: neither edited broker
    // is folded here, both stay dirty, and the host's refresh refolds them after the relist
    // (the other workgroups' brokers have intact lists: their folds stand).
    for (int b = g; b < rf.B; b += ng) {
        if ((g != 0 || !ok) && ((ef && b == from) || (et && b == to))) continue;   // workgroup 0's
        if (!(rf.bfl[b] & BF_DIRTY)) continue;                                     // (uniform)
        refold_broker<SCAN_THREADS, RF_CHUNK>(rf, b, buf);
    }
    if (g == 0 && ok) {
        if (ef && from % ng != 0 && (rf.bfl[from] & BF_DIRTY)) refold_broker<SCAN_THREADS, RF_CHUNK>(rf, from, buf);
        if (et && to % ng != 0 && to != from && (rf.bfl[to] & BF_DIRTY)) refold_broker<SCAN_THREADS, RF_CHUNK>(rf, to, buf);
    }
}

// One touched broker of the last applied step (DevCtl.eg_b[k]) refolded exactly by an extra
// workgroup of the next scan launch (ScanArgs.eager), after its own half of the pending list
// edit (each list belongs to one workgroup; the list workgroup skips the edit), while the
// scan runs (it never reads the loads): the next k_step resolves on exact loads, with no halt
// for a refresh when its decision needs the exact folds.  A halted step's launch is the
// in-stream refresh's instead (it does the edit and refolds every dirty broker).
// The edit and the refold in one pass over the list (a list of at most LIST_K * blockDim
// entries whose suffix fits the workgroup's LDS): the entries the edit loads are the ones
// whose partition words the refold gathers, at their new positions, so the refold costs one
// memory round trip -- the partition words -- then the chain from the last checkpoint below
// the first changed position.  (Under the scan's full-rate stream a round trip costs ~10 us:
// the chunked refold's two per chunk made an eager workgroup ~50 us at c5, longer than the
// scan it runs beside.)  Returns false (nothing done) when the list does not qualify.
__device__ bool eager_edit_refold(const RefreshArgs& rf, int b, int op, uint32_t q, ListExt& x, double* buf, int cap) {
    const uint32_t st = x.st, n = x.n, nt = blockDim.x;
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    // LDS: two chunks of contributions (a ring, +32 for the chain's read-ahead), then the new
    // list's partition ids from position base on.  (Chunks of 512: the gather before the first
    // fold and the last chunk's fold after the last gather are what the overlap leaves
    // exposed -- c5 eager workgroup 42.4 us at 1024, 38.0-38.7 at 512, 39.1 at 384, 39.7 at
    // 256, 41.5 at 768, 45.0 at 2048)
    constexpr int ECH = 512;
    uint32_t* ids = (uint32_t*)(buf + 2 * ECH + 32);
    if (n + 1 > LIST_K * nt || 2 * ECH + 32 + ((int)n + 2) / 2 > cap) return false;
    if (op == 2 && n >= rf.L.lcap[b]) return false;          // (the general path reports it)
    __shared__ int s_at;
    __shared__ double s_acc0;
    if (tid == 0) s_at = op == 1 ? -1 : 0;
    __syncthreads();
    uint32_t v[LIST_K];
#pragma unroll
    for (int k = 0; k < LIST_K; k++) {
        const uint32_t i = k * nt + tid;
        v[k] = i < n ? rf.L.lent[st + i] : NONE32;
    }
    if (op == 1) {
#pragma unroll
        for (int k = 0; k < LIST_K; k++)
            if (v[k] == q) s_at = (int)(k * nt + tid);
    } else if (op == 2) {
        int c = 0;
#pragma unroll
        for (int k = 0; k < LIST_K; k++) c += v[k] < q ? 1 : 0;
        c = wave_sum(c);
        if (lane == 0 && c) atomicAdd(&s_at, c);
    }
    __syncthreads();
    int at = s_at;
    if (op == 1 && at < 0) op = 0;                           // (not listed: nothing to remove)
    if (op == 0) at = (int)n;
    const uint32_t nn = op == 1 ? n - 1 : (op == 2 ? n + 1 : n);
    const uint32_t dp = (uint32_t)at < x.dp ? (uint32_t)at : x.dp;
    const uint32_t base = (dp < nn ? dp : nn) & ~63u;
    // the edit's stores, and the new list's partition ids from position base on (LDS)
#pragma unroll
    for (int k = 0; k < LIST_K; k++) {
        const uint32_t i = k * nt + tid;
        if (i >= n) continue;
        uint32_t np = i;
        if (op == 1) { if (i == (uint32_t)at) continue; if (i > (uint32_t)at) { np = i - 1; rf.L.lent[st + np] = v[k]; } }
        if (op == 2 && i >= (uint32_t)at) { np = i + 1; rf.L.lent[st + np] = v[k]; }
        if (np >= base) ids[np - base] = v[k];
    }
    if (tid == 0) {
        if (op == 2) {
            rf.L.lent[st + at] = q;
            if ((uint32_t)at >= base) ids[at - base] = q;
        }
        rf.L.llen[b] = nn;
        s_acc0 = base ? rf.L.ck[st + base - 1] : 0.0;
    }
    // The contributions (getBrokerLoad's terms, utils.go:92-105: slot 0 carries the leader
    // weight W * (len(R) + NumConsumers)) are gathered a chunk ahead of the chain: waves 1..
    // gather chunk c + 1 from the partition words into the ring's other half while wave 0 folds
    // chunk c in order -- the random partition-word loads (~half the refold's time at c5,
    // 7300-entry lists) overlap the add-latency-bound chain instead of preceding it
    const int mtot = (int)(nn - base);
    auto gather = [&](int c1, int c2, int t, int ntt) {
        double* dst = buf + ((c1 / ECH) & 1) * ECH - c1;
        for (int i = c1 + t; i < c2; i += ntt) {
            const uint32_t pp = ids[i];
            const double w = rf.w[pp];
            const uint32_t m = rf.meta[pp];
            const int32_t ncp = rf.nc[pp];
            const uint16_t r0 = rf.rep[pp];
            dst[i] = r0 == (uint16_t)b ? w * (double)((int)meta_nrep(m) + ncp) : w;
        }
    };
    __syncthreads();
    gather(0, mtot < ECH ? mtot : ECH, tid, (int)nt);
    __syncthreads();
    double acc = s_acc0;
    for (int c0 = 0; c0 < mtot; c0 += ECH) {
        const int c1 = c0 + ECH < mtot ? c0 + ECH : mtot;
        if (wid > 0) {
            gather(c1, c1 + ECH < mtot ? c1 + ECH : mtot, tid - 64, (int)nt - 64);
        } else {
            // (in-order chain over the chunk's ring slot; checkpoints relative to its start, a
            // multiple of 64; the read-ahead past its end reads the other slot, unused)
            acc = chain_lds_ck(acc, (const lds_f64*)(buf + ((c0 / ECH) & 1) * ECH), c1 - c0,
                               rf.L.ck + st + base + c0, lane);
        }
        __syncthreads();
    }
    if (wid == 0) {
        if (lane == 0) {
            rf.load[b] = acc;
            rf.lerr[b] = gamma_n((int)nn) * acc;
            rf.eb[b] = 0.0;
            rf.bfl[b] = rf.bfl[b] & ~BF_DIRTY;
            rf.L.dpos[b] = NONE32;
        }
    }
    __syncthreads();
    x.n = nn;
    x.dp = NONE32;
    return true;
}

__device__ __attribute__((noinline)) void eager_refold(const RefreshArgs* rfp, int k, double* buf, int cap) {
    const RefreshArgs rf = *rfp;
    DevCtl* ctl = rf.ctl;
    if (ctl->halted != H_RUN || k >= ctl->eg_n || ctl->list_overflow) return;   // (uniform)
    const int b = ctl->eg_b[k];
    if (b < 0 || b >= rf.B) return;
    const bool tk = ctl->tk_on != 0;
    const unsigned long long t0 = tk ? wall_clock64() : 0ull;
    ListExt x = list_ext(rf.L, b);                // (one round trip with the flags below)
    const bool dirty = (rf.bfl[b] & BF_DIRTY) != 0;
    // this broker's half of the last step's list edit (replace = remove from `from`, insert
    // into `to`: different lists, different workgroups)
    int op = 0;
    uint32_t p = 0;
    if (ctl->pending_list) {
        const int kind = ctl->pl_kind;
        p = (uint32_t)ctl->pl_part;
        if (b == ctl->pl_from && (kind == 1 || kind == 2)) op = 1;
        else if (b == ctl->pl_to && (kind == 1 || kind == 3)) op = 2;
    }
    const bool one = dirty && eager_edit_refold(rf, b, op, p, x, buf, cap);
    const unsigned long long t1 = tk ? wall_clock64() : 0ull;
    if (!one) {
        __shared__ int s_i;
        bool ok = true;
        if (op == 1) list_remove_x(rf.L, b, p, x, &s_i);
        if (op == 2) ok = list_insert_x(rf.L, b, p, x, &s_i);
        if (!ok) {                                 // (the broker stays dirty: the host relists)
            if (threadIdx.x == 0) ctl->list_overflow = 1;
            return;
        }
        if (dirty) refold_broker<SCAN_THREADS, RF_CHUNK>(rf, b, buf, &x);
    }
    if (threadIdx.x == 0) {
        if (dirty) atomicSub(&ctl->ndirty, 1);
        if (tk) {                                  // (kernel timing: the eager workgroups' spans)
            atomicAdd(&ctl->tk_eg, wall_clock64() - t0);
            atomicAdd(&ctl->tk_eg_edit, t1 - t0);
            atomicAdd(&ctl->tk_eg_n, 1ull);
        }
    }
}

// --------------------------------------------------- multi-GPU summaries

// pack this rank's scan result + its distinct near-tie keys (within 4*eps of the
// rank's minimum, a superset of those within 4*eps of the global one)
// One rank's summary of its scan records (multi-GPU): minima, candidate counts and
// first-index words of the rank, its best key per kind (the records' best keys re-scored on
// r) and a second-best key of another partition, and its near-tie keys within 4 eps of its
// own minima.  One record per thread (R.n <= SUM_RECS; the host keeps a sharded engine's
// scan grid within it), so every record field is loaded once; the near-tie keys are then
// loaded one key slot per thread, all in flight at once.
// (s_r: LDS for the relative loads r, B doubles: every key is re-scored from LDS; staged:
// the caller already copied r there -- k_scansum does it while the scan runs)
__device__ __forceinline__ void summary_body(const SumArgs& a, double* s_r, bool staged) {
    DevCtl* ctl = a.ctl;
    RecHdr* out = a.out.h(0);
    Contender* okeys = a.out.k(0);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // a halted batch: the rounds after the halt are no-ops (k_step returns at once), and
    // the summary is left as the halted round wrote it, so the gathered flags every rank
    // reads when it grows its summaries (grow_summary: bit 2, a spill it can still grow)
    // are that round's, whichever round of the batch halted
    if (!(ctl->halted == H_RUN && ctl->prepped)) return;
    __shared__ uint32_t s_key[DEDUP_STEP];
    __shared__ unsigned long long s_wb[DEDUP_STEP], s_it[DEDUP_STEP];
    __shared__ uint32_t s_n, s_fail;
    __shared__ double s_d[2][16];
    __shared__ unsigned long long s_c[2][16];
    __shared__ uint32_t s_f[NF];
    __shared__ uint32_t s_fm[16];
    __shared__ double s_g[2];
    __shared__ unsigned long long s_benc[2], s_benc2[2];
    __shared__ uint32_t s_brec[2], s_brec2[2], s_nkk[2];
    __shared__ long long s_bp[2];
    __shared__ uint32_t s_rk[SUM_RECS];              // stored keys per record
    Dedup T{s_key, s_wb, s_it, DEDUP_STEP};
    dedup_clear(T);
    if (tid == 0) { s_n = 0; s_fail = a.R.n > SUM_RECS ? 1u : 0u; }   // (the host's clamp; never)
    if (tid < NF) s_f[tid] = NONE32;
    if (tid < 2) {
        s_benc[tid] = NONE64; s_brec[tid] = NONE32; s_benc2[tid] = NONE64; s_brec2[tid] = NONE32;
        s_nkk[tid] = 0; s_bp[tid] = -1;
    }
    // the near-tie keys take the first cap - 2 slots; the last two carry, per kind, the best
    // key of another partition than the summary's best (k_step's census bound: the best key
    // is most often the applied move itself, whose partition's keys are dropped)
    const uint32_t capk = (uint32_t)a.out.cap - 2u;
    const double eps = ctl->eps, inv_avg = ctl->inv_avg;
    const bool mine = tid < a.R.n;
    double d0 = HUGE_VAL, d1 = HUGE_VAL;
    unsigned long long c0 = 0, c1 = 0;
    uint32_t fm = 0, nks = 0;
    Contender bk[2];
    bk[0].s = bk[1].s = -1;
    if (mine) {
        const RecHdr* h = a.R.h(tid);
        d0 = ldd(&h->dmin[0]); d1 = ldd(&h->dmin[1]);
        c0 = ldobj(&h->cand[0]); c1 = ldobj(&h->cand[1]);
        nks = min(ld32(&h->nkeys), (uint32_t)a.R.cap);
        fm = ld32(&h->fmask);
        bk[0] = ldobj(&h->best[0]); bk[1] = ldobj(&h->best[1]);
    }
    if (!staged)                                     // (the header loads above are in flight)
        for (int b = tid; b < a.B; b += 1024) s_r[b] = a.r[b];
    if (tid < SUM_RECS) s_rk[tid] = nks;
    const uint32_t myfm = fm;
    d0 = wave_min(d0); d1 = wave_min(d1); c0 = wave_sum(c0); c1 = wave_sum(c1);
    fm = wave_red_or(fm);
    if (lane == 0) {
        s_d[0][wid] = d0; s_d[1][wid] = d1; s_c[0][wid] = c0; s_c[1][wid] = c1;
        s_fm[wid] = fm;
    }
    __syncthreads();
    if (myfm) {
        const uint32_t* fi = a.R.f(tid);
        for (int q = 0; q < NF; q++) {
            const uint32_t v = ld32(fi + q);
            if (v != NONE32) atomicMin(&s_f[q], v);
        }
    }
    if (tid == 0) {
        for (int x = 1; x < 16; x++) {
            d0 = s_d[0][x] < d0 ? s_d[0][x] : d0;
            d1 = s_d[1][x] < d1 ? s_d[1][x] : d1;
            c0 += s_c[0][x]; c1 += s_c[1][x];
        }
        s_g[0] = d0; s_g[1] = d1;
        out->dmin[0] = d0; out->dmin[1] = d1; out->cand[0] = c0; out->cand[1] = c1;
    }
    // the rank's best key per kind: the records' best keys re-scored on r
    unsigned long long me[2] = {NONE64, NONE64};
    for (int k = 0; k < 2; k++)
        if (bk[k].s >= 0) {
            me[k] = enc(cont_delta(s_r, bk[k], inv_avg));
            atomicMin(&s_benc[k], me[k]);
        }
    __syncthreads();
    auto ins = [&](const Contender& c) {
        const double g = s_g[c.kind];
        if (!(g < HUGE_VAL)) return;               // (no census wave on this rank for the kind)
        if (!(cont_delta(s_r, c, inv_avg) <= g + 4.0 * eps)) return;
        if (dedup_insert(T, c.kind, c.s, c.t, c.w, c.iter) < 0) s_fail = 1;
    };
    {
        // (tried: the first 4 key slots per thread loaded speculatively beside the headers --
        // 130 KB through one workgroup per step at c3, the summary 2.2 us slower)
        const int kc = a.R.cap, tot = a.R.n * kc;
        for (int x = tid; x < tot; x += 1024) {
            const int i = x / kc, k = x - i * kc;
            if (k < (int)s_rk[i]) ins(ldobj(a.R.k(i) + k));
        }
        const uint32_t nc = min(ctl->ncont, a.cont_cap);
        for (uint32_t i = tid; i < nc; i += 1024) ins(ldobj(a.cont + i));
    }
    for (int k = 0; k < 2; k++)
        if (me[k] != NONE64 && me[k] == s_benc[k]) atomicMin(&s_brec[k], (uint32_t)tid);
    __syncthreads();
    // second-best keys: the best key per kind among the records whose best key lies in
    // another partition than the summary's best
    for (int k = 0; k < 2; k++)
        if ((uint32_t)tid == s_brec[k]) s_bp[k] = (long long)(bk[k].iter >> 21);
    __syncthreads();
    unsigned long long e2[2] = {NONE64, NONE64};
    for (int k = 0; k < 2; k++)
        if (me[k] != NONE64 && (long long)(bk[k].iter >> 21) != s_bp[k]) {
            e2[k] = me[k];
            atomicMin(&s_benc2[k], e2[k]);
        }
    __syncthreads();
    for (int k = 0; k < 2; k++)
        if (e2[k] != NONE64 && e2[k] == s_benc2[k]) atomicMin(&s_brec2[k], (uint32_t)tid);
    for (int h = tid; h < DEDUP_STEP; h += 1024) {
        if (s_key[h] == NONE32) continue;
        const uint32_t k = atomicAdd(&s_n, 1u);
        atomicAdd(&s_nkk[s_key[h] >> 30], 1u);
        if (k < capk) okeys[k] = dedup_entry(T, h);
    }
    __syncthreads();
    for (int k = 0; k < 2; k++) {
        // (the record that holds the best / second-best key writes it from its registers)
        if ((uint32_t)tid == s_brec[k]) out->best[k] = bk[k];
        if ((uint32_t)tid == s_brec2[k]) okeys[capk + k] = bk[k];
    }
    if (tid < 2) {
        Contender x;
        x.s = x.t = -1; x.w = 0.0; x.iter = NONE64; x.kind = tid; x.pad = 0;
        if (s_brec[tid] == NONE32) out->best[tid] = x;
        if (s_brec2[tid] == NONE32) okeys[capk + tid] = x;
    }
    if (tid == 0) {
        const uint32_t ovf = ctl->cont_overflow;
        out->nkeys = s_n < capk ? s_n : capk;
        out->flags = (ovf || s_fail || s_n > capk) ? 1u : 0u;
        out->flags |= 2u;
        if (ovf && a.spill_growable) out->flags |= 4u;   // (grow_summary)
        out->nkk[0] = (uint16_t)min(s_nkk[0], 0xFFFFu);
        out->nkk[1] = (uint16_t)min(s_nkk[1], 0xFFFFu);
        uint32_t m = 0;
        for (int q = 0; q < NF; q++) m |= s_f[q] != NONE32 ? 1u << q : 0u;
        out->fmask = m;
        uint32_t* fo = a.out.f(0);
        for (int q = 0; q < NF; q++) fo[q] = s_f[q];
    }
}

#if KB_IN_TU(0)
__global__ __launch_bounds__(1024) void k_summary(SumArgs a) {
    // (r in LDS up to SUM_RLDS brokers; past that, the keys are re-scored from memory)
    extern __shared__ __align__(16) double sum_dyn[];
    if (a.B <= SUM_RLDS) summary_body(a, sum_dyn, false);
    else summary_body(a, const_cast<double*>(a.r), true);
}
#endif

// The scan and the rank summary in one launch (sharded engines): the scan's grid plus one
// resident summary workgroup, the last of the grid, which waits for the others' arrivals
// (k_pair's sharded count, bounded wait) and then runs summary_body.  The all-gather and
// the resolve follow as before; this removes the summary's launch and dispatch gap.
template <int RC, bool LSETS, bool BK>
__global__ __launch_bounds__(SCAN_THREADS) void k_scansum(ScanArgs a, SumArgs sa) {
    static_assert(SCAN_THREADS == 1024, "summary_body runs 1024 threads");
    if ((int)blockIdx.x == (int)gridDim.x - 1) {
        const int tid = threadIdx.x, lane = tid & 63;
        __shared__ int s_to;
        // r does not change while the scan runs: staged into this workgroup's dynamic LDS
        // (the scan's tables' space, at least 16 B per broker) before the wait
        extern __shared__ __align__(16) unsigned char smem_sum[];
        double* s_r = (double*)smem_sum;
        for (int b = tid; b < sa.B; b += 1024) s_r[b] = sa.r[b];
        if (tid < 64) {
            const unsigned long long t0 = wall_clock64();
            int to = 0;
            for (;;) {
                if (wall_clock64() - t0 >= sa.wait_ticks) { to = 1; break; }
                const uint32_t v = lane < PAIR_SHARDS
                    ? __hip_atomic_load(sa.wait_cnt + lane * PAIR_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
                if (wave_sum(v) >= (uint32_t)sa.wait_n) break;
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // (the other XCDs' writes)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (!to && lane < PAIR_SHARDS)
                __hip_atomic_store(sa.wait_cnt + lane * PAIR_STRIDE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (lane == 0) s_to = to;
        }
        __syncthreads();
        if (s_to) {
            // (as k_pair's step workgroup: an explicit error in the step log, the plan halts;
            // the host resets the count and refuses further work.)  This rank's summary slot
            // carries SUM_POISON, so every rank's resolve of this round reads it from the
            // gathered summaries and halts with the same error: no rank applies a change the
            // others do not, and no rank stays behind in a later collective.
            if (tid == 0) {
                RecHdr* out = sa.out.h(0);
                __hip_atomic_store(&out->flags, SUM_POISON, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&out->nkeys, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                DevCtl* ctl = sa.ctl;
                ChangeDev ch;
                ch.status = -1; ch.step = -1; ch.kind = 0; ch.slot = -1; ch.part = -1; ch.from = ch.to = -1;
                ch.su = ch.cu = 0.0; ch.exact = 0; ch.err_code = E_PAIR_TIMEOUT; ch.err_broker = -1; ch.pad = 0;
                const int lp = ctl->logpos;
                if (lp < ctl->logcap) sa.log[lp] = ch;
                ctl->logpos = lp + 1;
                ctl->halted = H_DONE;
            }
            return;
        }
        summary_body(sa, s_r, true);
        return;
    }
    const bool wt = (int)blockIdx.x < a.nscan && !(a.rfpass && a.ctl->halted == H_NEED_EXACT);
    scan_kernel_body<RC, LSETS, false, false, BK>(a);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!wt) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __hip_atomic_fetch_add(a.done + (blockIdx.x % PAIR_SHARDS) * PAIR_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ------------------------------------------------------- launch helpers
// (compiled as several translation units, KB_TU = 0..10, in parallel: Makefile)

// (the scan's instantiations per slot count spread over TUs 1, 8, 9, 10)
#define KB_SCAN_TU(RC)                                                                                    \
    void launch_scan_##RC(const ScanArgs& a, bool lds_sets, size_t lds, hipStream_t st) {                \
        const int grid = a.nscan + (a.listwg ? 1 : 0) + a.eager;                                         \
        /* (incremental mode: with the set records in LDS only; engine.cpp gates it.  Broker           \
           tables in memory (a.gt, B > MAXB): set records in memory too) */                              \
        if (a.gt) hipLaunchKernelGGL((k_scan<RC, false, false, true>), dim3(grid), dim3(SCAN_THREADS), lds, st, a); \
        else if (lds_sets && a.incr) hipLaunchKernelGGL((k_scan<RC, true, true>), dim3(grid), dim3(SCAN_THREADS), lds, st, a); \
        else if (lds_sets) hipLaunchKernelGGL((k_scan<RC, true, false>), dim3(grid), dim3(SCAN_THREADS), lds, st, a); \
        else hipLaunchKernelGGL((k_scan<RC, false, false>), dim3(grid), dim3(SCAN_THREADS), lds, st, a);  \
    }                                                                                                     \
    int scan_occ_##RC(bool lds_sets, bool gt, size_t lds) {                                              \
        int n = 0, m = 0;                                                                                 \
        if (gt) hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_scan<RC, false, false, true>, SCAN_THREADS, lds); \
        else if (lds_sets) {                                                                              \
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_scan<RC, true, false>, SCAN_THREADS, lds); \
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&m, k_scan<RC, true, true>, SCAN_THREADS, lds);  \
            n = n < m ? n : m;                                                                            \
        } else hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_scan<RC, false, false>, SCAN_THREADS, lds); \
        return n;                                                                                         \
    }
#if KB_IN_TU(1)
KB_SCAN_TU(1) KB_SCAN_TU(2) KB_SCAN_TU(3)
#endif
#if KB_IN_TU(8)
KB_SCAN_TU(4) KB_SCAN_TU(6)
#endif
#if KB_IN_TU(9)
KB_SCAN_TU(8) KB_SCAN_TU(12)
#endif
#if KB_IN_TU(10)
KB_SCAN_TU(16)
#endif
#undef KB_SCAN_TU

#if KB_IN_TU(0)
#define KB_SCAN_DECL(RC)                                                                                  \
    void launch_scan_##RC(const ScanArgs& a, bool lds_sets, size_t lds, hipStream_t st);                \
    int scan_occ_##RC(bool lds_sets, bool gt, size_t lds);
KB_SCAN_DECL(1) KB_SCAN_DECL(2) KB_SCAN_DECL(3) KB_SCAN_DECL(4) KB_SCAN_DECL(6) KB_SCAN_DECL(8)
KB_SCAN_DECL(12) KB_SCAN_DECL(16)
#undef KB_SCAN_DECL
void launch_scan(const ScanArgs& a, int rc, bool lds_sets, size_t lds, hipStream_t st) {
    switch (rc) {
        case 1: launch_scan_1(a, lds_sets, lds, st); break;
        case 2: launch_scan_2(a, lds_sets, lds, st); break;
        case 3: launch_scan_3(a, lds_sets, lds, st); break;
        case 4: launch_scan_4(a, lds_sets, lds, st); break;
        case 6: launch_scan_6(a, lds_sets, lds, st); break;
        case 8: launch_scan_8(a, lds_sets, lds, st); break;
        case 12: launch_scan_12(a, lds_sets, lds, st); break;
        default: launch_scan_16(a, lds_sets, lds, st); break;
    }
}
int scan_blocks_per_cu(int rc, bool lds_sets, bool gt, size_t lds) {
    switch (rc) {
        case 1: return scan_occ_1(lds_sets, gt, lds);
        case 2: return scan_occ_2(lds_sets, gt, lds);
        case 3: return scan_occ_3(lds_sets, gt, lds);
        case 4: return scan_occ_4(lds_sets, gt, lds);
        case 6: return scan_occ_6(lds_sets, gt, lds);
        case 8: return scan_occ_8(lds_sets, gt, lds);
        case 12: return scan_occ_12(lds_sets, gt, lds);
        default: return scan_occ_16(lds_sets, gt, lds);
    }
}
#endif

#if KB_IN_TU(0)

__global__ __launch_bounds__(1024) void k_touch(double* r, int B, int32_t* blm, int32_t* posm, uint4* setrec, int nrec) {
    for (int i = threadIdx.x; i < B; i += 1024) {
        const double x = r[i]; const int32_t y = blm[i], z = posm[i];
        __syncthreads();
        r[i] = x; blm[i] = y; posm[i] = z;
    }
    for (int i = threadIdx.x; i < nrec; i += 1024) { const uint4 v = setrec[i]; __syncthreads(); setrec[i] = v; }
}

// Upper bound of the first step's minimum.  Without a previous step's best keys
// ub = +inf, which sends every wave of the scan through the near-tie census (and
// defeats the lower-bound prune); with many near-tied targets per wave (4096
// brokers, tiny weights) that overflows the spill buffer.  The minima of a
// census-free scan of the same state are the step minimum g itself, so ub = g is
// valid for the census gate (tL <= ub + 12 eps) and the prune (LB > ub + 16 eps).
// Only a bound that is +inf is set (the records are this pass's only when a bound
// was open: otherwise the bound pass returned at once and they are stale).
// (tighten: the sharded engines' pass runs on every scan and lowers a finite bound too -- a
// rank's bound from its one gathered summary's few keys can sit far above its minimum)
__global__ __launch_bounds__(256) void k_ubinit(DevCtl* ctl, Recs R, int allow_leader, int tighten) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const bool run = ctl->halted == H_RUN && ctl->prepped && ctl->steps < ctl->budget;
    if (!run) return;                            // uniform over the workgroup
    double m0 = HUGE_VAL, m1 = HUGE_VAL;
    for (int i = tid; i < R.n; i += 256) {
        const RecHdr* h = R.h(i);
        m0 = h->dmin[0] < m0 ? h->dmin[0] : m0;
        m1 = h->dmin[1] < m1 ? h->dmin[1] : m1;
    }
    m0 = wave_min(m0);
    m1 = wave_min(m1);
    __shared__ double s_m[2][4];
    if (lane == 0) { s_m[0][wid] = m0; s_m[1][wid] = m1; }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 4; w++) {
            m0 = s_m[0][w] < m0 ? s_m[0][w] : m0;
            m1 = s_m[1][w] < m1 ? s_m[1][w] : m1;
        }
        m0 = s_m[0][0] < m0 ? s_m[0][0] : m0;
        m1 = s_m[1][0] < m1 ? s_m[1][0] : m1;
        const double u0 = ctl->ub[0], u1 = ctl->ub[1];
        if (tighten) {                           // (-inf: census off, left alone)
            if (u1 != -HUGE_VAL && m1 < u1) ctl->ub[1] = m1;
            if (allow_leader && u0 != -HUGE_VAL && m0 < u0) ctl->ub[0] = m0;
        } else {
            const bool open1 = u1 == HUGE_VAL, open0 = allow_leader && u0 == HUGE_VAL;
            if (open0 || open1) {                // the bound pass ran on this state
                if (open0) ctl->ub[0] = m0;
                if (open1) ctl->ub[1] = m1;
            }
        }
    }
}

void launch_ubinit(DevCtl* ctl, const Recs& R, int allow_leader, int tighten, hipStream_t st) {
    hipLaunchKernelGGL(k_ubinit, dim3(1), dim3(256), 0, st, ctl, R, allow_leader, tighten);
}

void launch_touch(double* r, int B, int32_t* blm, int32_t* posm, uint4* setrec, int nrec, hipStream_t st) {
    hipLaunchKernelGGL(k_touch, dim3(1), dim3(1024), 0, st, r, B, blm, posm, setrec, nrec);
}
#endif

#if KB_IN_TU(2)

int step_static_lds(bool gb) {
    hipFuncAttributes fa, fb;
    if (hipFuncGetAttributes(&fa, gb ? (const void*)k_step<false, true> : (const void*)k_step<false>) != hipSuccess) return -1;
    if (hipFuncGetAttributes(&fb, gb ? (const void*)k_step<true, true> : (const void*)k_step<true>) != hipSuccess) return -1;
    return (int)(fa.sharedSizeBytes > fb.sharedSizeBytes ? fa.sharedSizeBytes : fb.sharedSizeBytes);
}

void launch_step(const StepArgs& a, hipStream_t st) {
    if (a.gscr) {
        if (a.pset && a.nsets > (int)MAX_SETS)
            hipLaunchKernelGGL((k_step<true, true>), dim3(1), dim3(STEP_THREADS), a.lds_bytes, st, a);
        else
            hipLaunchKernelGGL((k_step<false, true>), dim3(1), dim3(STEP_THREADS), a.lds_bytes, st, a);
    } else if (a.pset && a.nsets > (int)MAX_SETS)
        hipLaunchKernelGGL(k_step<true>, dim3(1), dim3(STEP_THREADS), a.lds_bytes, st, a);
    else
        hipLaunchKernelGGL(k_step<false>, dim3(1), dim3(STEP_THREADS), a.lds_bytes, st, a);
}
#endif

// the fused pair (k_pair) for the device slot counts of the common replication factors
// (one translation unit per (slot count, bound keys): TUs 3 / 6 for RC = 3 without / with
// bound keys, 4 / 7 for RC = 4)
#define KB_PAIR_TU(R, BKV, NAME)                                                                      \
    int pair_attr_##NAME(bool lds_sets, size_t lds, int* static_lds) {                               \
        hipFuncAttributes fa;                                                                          \
        const void* f = lds_sets ? (const void*)k_pair<R, true, BKV> : (const void*)k_pair<R, false, BKV>; \
        if (hipFuncGetAttributes(&fa, f) != hipSuccess) return -1;                                   \
        *static_lds = (int)fa.sharedSizeBytes;                                                         \
        int n = 0;                                                                                     \
        if (lds_sets) hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_pair<R, true, BKV>, SCAN_THREADS, lds);  \
        else hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_pair<R, false, BKV>, SCAN_THREADS, lds);          \
        return n;                                                                                      \
    }                                                                                                  \
    void launch_pair_##NAME(const ScanArgs& a, const StepArgs& sa, bool lds_sets, size_t lds, hipStream_t st) { \
        const int grid = a.nscan + (a.listwg ? 1 : 0) + a.eager + 1;                                 \
        if (lds_sets) hipLaunchKernelGGL((k_pair<R, true, BKV>), dim3(grid), dim3(SCAN_THREADS), lds, st, a, sa); \
        else hipLaunchKernelGGL((k_pair<R, false, BKV>), dim3(grid), dim3(SCAN_THREADS), lds, st, a, sa);         \
    }
#if KB_IN_TU(3)
KB_PAIR_TU(3, false, 3n)
#endif
#if KB_IN_TU(6)
KB_PAIR_TU(3, true, 3b)
#endif
#if KB_IN_TU(4)
KB_PAIR_TU(4, false, 4n)
#endif
#if KB_IN_TU(7)
KB_PAIR_TU(4, true, 4b)
#endif
#undef KB_PAIR_TU

#if KB_IN_TU(0)
#define KB_PAIR_DECL(NAME)                                                                             \
    int pair_attr_##NAME(bool lds_sets, size_t lds, int* static_lds);                                \
    void launch_pair_##NAME(const ScanArgs& a, const StepArgs& sa, bool lds_sets, size_t lds, hipStream_t st);
KB_PAIR_DECL(3n) KB_PAIR_DECL(3b) KB_PAIR_DECL(4n) KB_PAIR_DECL(4b)
#undef KB_PAIR_DECL
bool pair_supported(int rc) { return rc == 3 || rc == 4; }
// (both instantiations: the grid is sized so every workgroup is resident in either)
int pair_blocks_per_cu(int rc, bool lds_sets, size_t lds, int* static_lds) {
    if (rc != 3 && rc != 4) return -1;
    int s0 = 0, s1 = 0;
    const int n0 = rc == 3 ? pair_attr_3n(lds_sets, lds, &s0) : pair_attr_4n(lds_sets, lds, &s0);
    const int n1 = rc == 3 ? pair_attr_3b(lds_sets, lds, &s1) : pair_attr_4b(lds_sets, lds, &s1);
    *static_lds = s0 > s1 ? s0 : s1;
    return n0 < n1 ? n0 : n1;
}
void launch_pair(const ScanArgs& a, const StepArgs& sa, int rc, bool lds_sets, size_t lds, hipStream_t st) {
    // bound keys for plans without -allow-leader: there every step moves another partition
    // and the census waves' keys rarely outlive it (the -allow-leader headline keeps the
    // instantiation without them: its kernel is unchanged)
    const bool bk = !a.allow_leader;
    if (rc == 3) { if (bk) launch_pair_3b(a, sa, lds_sets, lds, st); else launch_pair_3n(a, sa, lds_sets, lds, st); }
    else { if (bk) launch_pair_4b(a, sa, lds_sets, lds, st); else launch_pair_4n(a, sa, lds_sets, lds, st); }
}

void launch_listop(DevCtl* ctl, const Lists& L, hipStream_t st) {
    hipLaunchKernelGGL(k_listop, dim3(1), dim3(1024), 0, st, ctl, L);
}
void launch_refresh(const RefreshArgs& a, hipStream_t st) {
    if (a.B > 0) hipLaunchKernelGGL(k_refresh, dim3(a.B), dim3(REFRESH_THREADS), 0, st, a);
}
void launch_summary(const SumArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_summary, dim3(1), dim3(1024), a.B <= SUM_RLDS ? (size_t)a.B * 8 : 0, st, a);
}
#endif

#if KB_IN_TU(5)

template <int RC, bool LSETS, bool BK>
static int scansum_attr1(size_t lds, int* static_lds) {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, (const void*)k_scansum<RC, LSETS, BK>) != hipSuccess) return -1;
    *static_lds = (int)fa.sharedSizeBytes;
    int n = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_scansum<RC, LSETS, BK>, SCAN_THREADS, lds);
    return n;
}
template <int RC, bool LSETS>
static int scansum_attr(size_t lds, int* static_lds) {
    int s0 = 0, s1 = 0;
    const int n0 = scansum_attr1<RC, LSETS, false>(lds, &s0), n1 = scansum_attr1<RC, LSETS, true>(lds, &s1);
    *static_lds = s0 > s1 ? s0 : s1;
    return n0 < n1 ? n0 : n1;
}
int scansum_blocks_per_cu(int rc, bool lds_sets, size_t lds, int* static_lds) {
    if (rc == 3) return lds_sets ? scansum_attr<3, true>(lds, static_lds) : scansum_attr<3, false>(lds, static_lds);
    if (rc == 4) return lds_sets ? scansum_attr<4, true>(lds, static_lds) : scansum_attr<4, false>(lds, static_lds);
    return -1;
}
void launch_scansum(const ScanArgs& a, const SumArgs& sa, int rc, bool lds_sets, size_t lds, hipStream_t st) {
    const int grid = a.nscan + (a.listwg ? 1 : 0) + a.eager + 1;
    const bool bk = !a.allow_leader;
#define KB_SCANSUM_LAUNCH(R, L)                                                                          \
    do {                                                                                                 \
        if (bk) hipLaunchKernelGGL((k_scansum<R, L, true>), dim3(grid), dim3(SCAN_THREADS), lds, st, a, sa);  \
        else hipLaunchKernelGGL((k_scansum<R, L, false>), dim3(grid), dim3(SCAN_THREADS), lds, st, a, sa);    \
    } while (0)
    if (rc == 3) {
        if (lds_sets) KB_SCANSUM_LAUNCH(3, true); else KB_SCANSUM_LAUNCH(3, false);
    } else {
        if (lds_sets) KB_SCANSUM_LAUNCH(4, true); else KB_SCANSUM_LAUNCH(4, false);
    }
#undef KB_SCANSUM_LAUNCH
}
#endif

#if KB_IN_TU(0)

// Control-block / step-log transfers between the device and the host's pinned
// (fine-grained, mapped) mirror as one small kernel on the engine's stream instead of
// hipMemcpyAsync: a copy engine round trip costs more than a one-workgroup launch, and a
// kernel in the stream needs no cross-engine dependency.  Plain vector loads / stores;
// with a flag, the copies are released to system scope before the flag's store, so the
// host may read them as soon as it sees the sequence number.
__global__ void __launch_bounds__(256) k_xfer(XferArgs a) {
    const int tid = threadIdx.x;
    for (int k = 0; k < 2; k++)
        for (int i = tid; i < a.n[k]; i += 256) a.dst[k][i] = a.src[k][i];
    if (!a.flag) return;
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(a.flag, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

void launch_xfer(const XferArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_xfer, dim3(1), dim3(256), 0, st, a);
}
#endif

}  // namespace kbe
