// kernels.hip -- CDNA4 (gfx950) kernels of the kafkabalancer move-search engine.
//
// One Balance() step (balancer.go:49-65) is six launches on one stream:
//   k_prep      1 WG   sort brokers by (load, id) (getBL, utils.go:107-117), exact
//                      sequential folds of su (getUnbalanceBL, utils.go:119-147),
//                      relative loads r = L/avg - 1, error bound eps
//   k_setlists  nsets/4 WGs  per allowed-broker set: the first K brokers of the set
//                      in bl order with their r (move targets, steps.go:257-266), and
//                      the last K (Add / Disallowed picks, steps.go:102,130-134)
//   k_scan      P/1024 WGs  the HBM stream over the SoA partition arrays: the Remove /
//                      Add / Disallowed / distributeLeaders first-index predicates
//                      (from the packed meta word) and the O(1)-delta score of every
//                      leader / non-leader slot against its first eligible target
//                      (steps.go:232-288); one 64-B record per workgroup
//   k_reduce    1 WG   combines the per-workgroup records
//   k_census    P/1024 WGs  exits unless its minimum is within 8*eps of the global one;
//                      then enumerates the near-tie (partition, slot, target) moves and
//                      de-duplicates them by key (source, target, weight) in LDS
//   k_resolve   1 WG   the reference's step order; exact sequential folds for the
//                      distinct near-tie keys (strict-< first minimum in (partition,
//                      slot, target) order, steps.go:276); the certified decision; the
//                      on-device apply (replacepl/addpl, utils.go:166-202) with an exact
//                      partition-ordered refold of touched loads (utils.go:92-105).
//
// Exactness: values the reference's decision depends on are computed in the
// reference's own operation order (IEEE binary64, no FMA: the file is built with
// -ffp-contract=off; true division), or bounded by eps and resolved exactly when
// the bound does not decide (DESIGN.md "Exactness").
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>
#include "engine_dev.h"
#include "kernels_api.h"

namespace kbe {

// --------------------------------------------------------------- helpers

__device__ __forceinline__ unsigned long long d2u(double d) { return (unsigned long long)__double_as_longlong(d); }
__device__ __forceinline__ double u2d(unsigned long long u) { return __longlong_as_double((long long)u); }

// order-preserving encoding of a double into u64
__device__ __forceinline__ unsigned long long enc(double d) {
    unsigned long long u = d2u(d);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double dec(unsigned long long e) {
    unsigned long long u = (e >> 63) ? (e & 0x7FFFFFFFFFFFFFFFull) : ~e;
    return u2d(u);
}

// reference term (utils.go:136-143): r = L/avg - 1; r>0 ? r*r : r*r/2 (exact ops)
__device__ __forceinline__ double term_x(double L, double avg) {
    double r = L / avg - 1.0;
    if (r > 0) return r * r;
    return r * r / 2;
}

// scoring (approximate; error covered by eps): f(r) and the O(1) move delta
__device__ __forceinline__ double fsq(double r) {
    double q = r * r;
    return r > 0 ? q : 0.5 * q;
}
// U(after) - U(before) for moving weight w (delta = w/avg) from source s to target t
__device__ __forceinline__ double dsrc(double rs, double delta) { return fsq(rs - delta) - fsq(rs); }
__device__ __forceinline__ double dtgt(double rt, double delta) { return fsq(rt + delta) - fsq(rt); }

__device__ __forceinline__ bool setbit(const uint64_t* sb, int b) {
    return (sb[b >> 6] >> (b & 63)) & 1ull;
}

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { T x = __shfl_xor(v, o); v = x < v ? x : v; }
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Sequential fold of n doubles held in LDS, in order (the reference's fold).
// Loads are batched 16 at a time so the dependent add chain, not LDS latency,
// sets the pace.
__device__ __forceinline__ double fold_lds(const double* x, int n, double acc = 0.0) {
    int k = 0;
    for (; k + 16 <= n; k += 16) {
        double v[16];
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = x[k + i];
#pragma unroll
        for (int i = 0; i < 16; i++) acc += v[i];
    }
    for (; k < n; k++) acc += x[k];
    return acc;
}

// getUnbalanceBL (utils.go:119-147) of the bl_move order with bl[ps] = Ls and
// bl[pt] = Lt (steps.go:250,272): two sequential folds, the reference's order.
__device__ double exact_unbalance_lds(const double* Lm, int n, int ps, int pt, double Ls, double Lt) {
    double S = 0.0;
    int k = 0;
    for (; k + 16 <= n; k += 16) {
        double v[16];
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = Lm[k + i];
#pragma unroll
        for (int i = 0; i < 16; i++) S += (k + i == ps) ? Ls : ((k + i == pt) ? Lt : v[i]);
    }
    for (; k < n; k++) S += (k == ps) ? Ls : ((k == pt) ? Lt : Lm[k]);
    const double avg = S / (double)n;
    double U = 0.0;
    k = 0;
    for (; k + 16 <= n; k += 16) {
        double t[16];
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const double L = (k + i == ps) ? Ls : ((k + i == pt) ? Lt : Lm[k + i]);
            t[i] = term_x(L, avg);
        }
#pragma unroll
        for (int i = 0; i < 16; i++) U += t[i];
    }
    for (; k < n; k++) U += term_x((k == ps) ? Ls : ((k == pt) ? Lt : Lm[k]), avg);
    return U;
}

// ---------------------------------------------- near-tie de-duplication
// LDS open-addressing table keyed by (kind, source, target); the weight bits are
// claimed by the first insert; a different weight under the same key is a
// "conflict" handled by the caller.  Contenders with one key have one exact U,
// so only the earliest iteration index per key matters (steps.go:276).

struct Dedup {
    uint32_t* key;
    unsigned long long* wb;
    unsigned long long* it;
    int cap;
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

// --------------------------------------------------------------- k_prep

__global__ __launch_bounds__(PREP_THREADS) void k_prep(PrepArgs a) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int NP2 = a.NP2;
    unsigned long long* keys = (unsigned long long*)smem;        // NP2
    double* Tm = (double*)(keys + NP2);                           // NP2
    uint32_t* idx = (uint32_t*)(Tm + NP2);                        // NP2
    __shared__ double s_red[PREP_THREADS / 64];
    __shared__ int s_wcnt[PREP_THREADS / 64];
    __shared__ double s_avg, s_S, s_U0;
    __shared__ int s_nblm;
    DevCtl* ctl = a.ctl;
    const int tid = threadIdx.x;
    if (ctl->halted) return;
    KB_STAMP_BEGIN();
    if (tid == 0) {
        ctl->gmin[0] = ctl->gmin[1] = NONE64;
        for (int f = 0; f < NF; f++) ctl->first[f] = NONE32;
        ctl->ncand[0] = ctl->ncand[1] = 0;
        ctl->ncont = 0;
        ctl->cont_overflow = 0;
    }
    for (int i = tid; i < NP2; i += PREP_THREADS) {
        if (i < a.B) { keys[i] = d2u(a.load[i]); idx[i] = (uint32_t)i; }
        else { keys[i] = NONE64; idx[i] = NONE32; }
    }
    __syncthreads();
    KB_STAMP(ctl, 0);
    // bitonic sort by (load bits, dense id); loads are finite and >= 0, so the
    // IEEE bit pattern orders like the value (byBrokerLoad.Less, utils.go:23-28)
    for (int k = 2; k <= NP2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < NP2; i += PREP_THREADS) {
                int ixj = i ^ j;
                if (ixj > i) {
                    unsigned long long ki = keys[i], kj = keys[ixj];
                    uint32_t ii = idx[i], ij = idx[ixj];
                    bool less = (kj < ki) || (kj == ki && ij < ii);
                    bool up = (i & k) == 0;
                    if (up == less) { keys[i] = kj; keys[ixj] = ki; idx[i] = ij; idx[ixj] = ii; }
                }
            }
            __syncthreads();
        }
    }
    KB_STAMP(ctl, 1);
    // compaction of the bl_move subsequence (NP2 <= 4096 => 4 elements / thread)
    int base = tid * 4;
    int flag[4]; unsigned long long kv[4]; uint32_t iv[4];
    int c = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        int i = base + q;
        flag[q] = 0;
        kv[q] = 0; iv[q] = NONE32;
        if (i < a.B) {
            uint32_t b = idx[i];
            kv[q] = keys[i]; iv[q] = b;
            a.order[i] = (int32_t)b;
            flag[q] = (a.cnt[b] > 0 || a.incfg[b]) ? 1 : 0;
            c += flag[q];
        }
    }
    const int lane = tid & 63, wid = tid >> 6;
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) { int y = __shfl_up(incl, o); if (lane >= o) incl += y; }
    if (lane == 63) s_wcnt[wid] = incl;
    __syncthreads();
    int woff = 0, total = 0;
    for (int w = 0; w < PREP_THREADS / 64; w++) { if (w < wid) woff += s_wcnt[w]; total += s_wcnt[w]; }
    int pos = woff + incl - c;
    __syncthreads();   // all reads of keys[] done before the in-place compaction
#pragma unroll
    for (int q = 0; q < 4; q++) {
        int i = base + q;
        if (i < a.B) {
            uint32_t b = iv[q];
            if (flag[q]) { keys[pos] = kv[q]; a.blm[pos] = (int32_t)b; a.posm[b] = pos; pos++; }
            else a.posm[b] = -1;
        }
    }
    if (tid == 0) s_nblm = total;
    __syncthreads();
    const int nblm = s_nblm;
    const double* Lm = (const double*)keys;
    KB_STAMP(ctl, 2);
    // S: sequential fold in bl order (utils.go:123-128)
    if (tid == 0) {
        const double S = fold_lds(Lm, nblm);
        s_S = S;
        s_avg = S / (double)nblm;
    }
    __syncthreads();
    KB_STAMP(ctl, 3);
    const double avg = s_avg;
    for (int k = tid; k < nblm; k += PREP_THREADS) Tm[k] = term_x(Lm[k], avg);
    __syncthreads();
    KB_STAMP(ctl, 4);
    // su: sequential fold of the terms (utils.go:134-143)
    if (tid == 0) s_U0 = fold_lds(Tm, nblm);
    KB_STAMP(ctl, 5);
    // error-bound ingredients: V = sum |r|(1+|r|), Rmax = max |r|
    const double inv_avg = 1.0 / avg;
    double v = 0.0, rm = 0.0;
    for (int k = tid; k < nblm; k += PREP_THREADS) {
        double r = fabs(Lm[k] * inv_avg - 1.0);
        v += r * (1.0 + r);
        rm = r > rm ? r : rm;
    }
    v = wave_sum(v);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { double x = __shfl_xor(rm, o); rm = x > rm ? x : rm; }
    if (lane == 0) s_red[wid] = v;
    __syncthreads();
    double V = 0.0;
    for (int w = 0; w < PREP_THREADS / 64; w++) V += s_red[w];
    __syncthreads();
    if (lane == 0) s_red[wid] = rm;
    __syncthreads();
    double Rm = 0.0;
    for (int w = 0; w < PREP_THREADS / 64; w++) Rm = s_red[w] > Rm ? s_red[w] : Rm;
    KB_STAMP(ctl, 6);
    for (int b = tid; b < a.B; b += PREP_THREADS)
        a.r[b] = a.posm[b] >= 0 ? __fma_rn(a.load[b], inv_avg, -1.0) : 0.0;
    if (tid == 0) {
        const double u = DBL_EPSILON / 2;
        double R = Rm + a.rmax_w * inv_avg;
        double eps = 64.0 * u * ((double)(nblm + 8) * (s_U0 + 2.0 * V) + 4.0 * (1.0 + R) * (1.0 + R));
        if (!(eps > 1e-300)) eps = 1e-300;
        ctl->S = s_S; ctl->avg = avg; ctl->inv_avg = inv_avg; ctl->U0 = s_U0;
        ctl->V = V; ctl->eps = eps; ctl->nblm = nblm;
        ctl->heavy = nblm > 0 ? a.blm[nblm - 1] : -1;
        ctl->light = nblm > 0 ? a.blm[0] : -1;
    }
    KB_STAMP(ctl, 7);
}

// ------------------------------------------------------------ k_setlists

__global__ __launch_bounds__(256) void k_setlists(SetArgs a) {
    if (a.ctl->halted) return;
    __shared__ int32_t s_order[MAXB];
    __shared__ unsigned long long s_blm[MAXB / 64], s_pres[MAXB / 64];
    __shared__ unsigned long long s_sb[4][MAXB / 64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < a.W64; i += 256) { s_blm[i] = 0; s_pres[i] = 0; }
    const int set = blockIdx.x * 4 + wv;
    for (int i = lane; i < a.W64; i += 64) s_sb[wv][i] = set < a.nsets ? a.setbits[(size_t)set * a.W64 + i] : 0ull;
    __syncthreads();
    for (int i = tid; i < a.B; i += 256) {
        s_order[i] = a.order[i];
        if (a.posm[i] >= 0) atomicOr(&s_blm[i >> 6], 1ull << (i & 63));
        if (a.cnt[i] > 0) atomicOr(&s_pres[i >> 6], 1ull << (i & 63));
    }
    __syncthreads();
    if (set >= a.nsets) return;
    const unsigned long long* sb = s_sb[wv];
    const unsigned long long lt = (1ull << lane) - 1ull;
    unsigned char* rec = a.setrec + (size_t)set * a.stride;
    int32_t* ids = (int32_t*)(rec + sr_ids_off());
    double* rr = (double*)(rec + sr_r_off(a.K));
    // kind 0: first K of set ∩ bl_move ascending; 1: last K of set ∩ present; 2: last K of set
    for (int kind = 0; kind < 3; kind++) {
        int found = 0;
        for (int base = 0; base < a.B && found < a.K; base += 64) {
            const int k = base + lane;
            bool mem = false;
            int b = -1;
            if (k < a.B) {
                b = s_order[kind == 0 ? k : a.B - 1 - k];
                mem = (sb[b >> 6] >> (b & 63)) & 1ull;
                if (kind == 0) mem = mem && ((s_blm[b >> 6] >> (b & 63)) & 1ull);
                else if (kind == 1) mem = mem && ((s_pres[b >> 6] >> (b & 63)) & 1ull);
            }
            const unsigned long long m = __ballot(mem);
            if (mem) {
                const int rk = found + __popcll(m & lt);
                if (rk < a.K) {
                    if (kind == 0) { ids[rk] = b; rr[rk] = a.r[b]; }
                    else a.lists[((size_t)set * 2 + (kind - 1)) * a.K + rk] = b;
                }
            }
            found += __popcll(m);
        }
        for (int rk = found + lane; rk < a.K; rk += 64) {
            if (kind == 0) { ids[rk] = -1; rr[rk] = 0.0; }
            else a.lists[((size_t)set * 2 + (kind - 1)) * a.K + rk] = -1;
        }
        if (kind == 0 && lane == 0) ((int32_t*)rec)[1] = found < a.K ? found : a.K;
    }
    int n = 0;
    for (int i = lane; i < a.W64; i += 64) n += __popcll(sb[i] & s_blm[i]);
    n = wave_sum(n);
    if (lane == 0) ((int32_t*)rec)[0] = n;
}

// --------------------------------------------------------------- k_scan

template <int RC>
struct PartRegs {
    double w[PER_LANE];
    uint32_t m[PER_LANE];
    uint32_t r[RC][PER_LANE];
};

template <int RC>
__device__ __forceinline__ void load_parts(const ScanArgs& a, long long base, PartRegs<RC>& P) {
    const double2 w01 = *(const double2*)(a.w + base);
    const double2 w23 = *(const double2*)(a.w + base + 2);
    P.w[0] = w01.x; P.w[1] = w01.y; P.w[2] = w23.x; P.w[3] = w23.y;
    const uint4 m4 = *(const uint4*)(a.meta + base);
    P.m[0] = m4.x; P.m[1] = m4.y; P.m[2] = m4.z; P.m[3] = m4.w;
#pragma unroll
    for (int k = 0; k < RC; k++) {
        const uint2 r2 = *(const uint2*)(a.rep + (long long)k * a.Ppad + base);
        P.r[k][0] = r2.x & 0xFFFFu; P.r[k][1] = r2.x >> 16;
        P.r[k][2] = r2.y & 0xFFFFu; P.r[k][3] = r2.y >> 16;
    }
}

// the first KT entries of a set record always contain the first eligible target
// (at most nrep <= RC of them are replicas)
template <int RC>
struct TargetRegs {
    static constexpr int KT = RC + 1;
    int32_t id[PER_LANE][KT];
    double r[PER_LANE][KT];
    int32_t nelig[PER_LANE];
    double rs[PER_LANE][RC];
};

template <int RC>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan(ScanArgs a) {
    DevCtl* ctl = a.ctl;
    if (ctl->halted) return;
    const double inv_avg = ctl->inv_avg;
    const int heavy = ctl->heavy;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const long long base = a.shard_begin + (long long)blockIdx.x * TILE + (long long)tid * PER_LANE;
    constexpr int KT = TargetRegs<RC>::KT;
    const int roff = sr_r_off(a.K);

    PartRegs<RC> P;
    load_parts<RC>(a, base, P);
    // issue every per-broker lookup of the 4 partitions before using any
    // (one L1/L2 round trip): set records and source relative loads
    TargetRegs<RC> T;
#pragma unroll
    for (int j = 0; j < PER_LANE; j++) {
        const unsigned char* rec = a.setrec + (size_t)meta_set(P.m[j]) * a.stride;
        T.nelig[j] = ((const int32_t*)rec)[0];
#pragma unroll
        for (int i = 0; i < KT; i++) {
            T.id[j][i] = ((const int32_t*)(rec + sr_ids_off()))[i];
            T.r[j][i] = ((const double*)(rec + roff))[i];
        }
#pragma unroll
        for (int k = 0; k < RC; k++) T.rs[j][k] = a.r[P.r[k][j]];
    }

    double dminL = HUGE_VAL, dminN = HUGE_VAL;
    uint32_t fst[NF];
#pragma unroll
    for (int f = 0; f < NF; f++) fst[f] = NONE32;
    unsigned long long cL = 0, cN = 0;

#pragma unroll
    for (int j = 0; j < PER_LANE; j++) {
        const long long p = base + j;
        const bool valid = p < a.shard_end;
        const uint32_t m = P.m[j];
        const int nrep = (int)meta_nrep(m), want = (int)meta_want(m);
        const bool elig = valid && meta_elig(m);
        const uint32_t pi = valid ? (uint32_t)p : NONE32;
        if (a.sem_go) {
            bool dup = false;
#pragma unroll
            for (int x = 0; x < RC; x++)
#pragma unroll
                for (int y = x + 1; y < RC; y++) dup |= (y < nrep) && P.r[x][j] == P.r[y][j];
            if (dup) fst[F_DUP] = min(fst[F_DUP], pi);
        }
        if (want < nrep) fst[F_REMOVE] = min(fst[F_REMOVE], pi);
        if (want > nrep) fst[F_ADD] = min(fst[F_ADD], pi);
        if (nrep == 0) {
            fst[F_EMPTY] = min(fst[F_EMPTY], pi);
            if (elig) fst[F_EMPTY_ELIG] = min(fst[F_EMPTY_ELIG], pi);
        }
        if (meta_dis(m)) fst[F_DIS] = min(fst[F_DIS], pi);
        if (a.rebalance && elig && nrep > 0 && (int)P.r[0][j] == heavy) fst[F_LEAD] = min(fst[F_LEAD], pi);
        // first allowed target in bl order that is not a replica (steps.go:257-266)
        double rt = 0.0;
        bool have = false;
#pragma unroll
        for (int i = KT - 1; i >= 0; i--) {
            const int b = T.id[j][i];
            bool isrep = false;
#pragma unroll
            for (int k = 0; k < RC; k++) isrep |= (k < nrep) && ((int)P.r[k][j] == b);
            if (b >= 0 && !isrep) { rt = T.r[j][i]; have = true; }
        }
        if (elig && nrep > 0 && have) {
            const double delta = P.w[j] * inv_avg;
            const double dt = dtgt(rt, delta);
            const unsigned long long ne = (unsigned long long)(T.nelig[j] - (int)meta_nin(m));
            if (a.allow_leader) {
                const double d = dsrc(T.rs[j][0], delta) + dt;
                dminL = d < dminL ? d : dminL;
                cL += ne;
            }
#pragma unroll
            for (int k = 1; k < RC; k++) {
                if (k < nrep) {
                    const double d = dsrc(T.rs[j][k], delta) + dt;
                    dminN = d < dminN ? d : dminN;
                }
            }
            cN += ne * (unsigned long long)(nrep - 1);
        }
    }
    // workgroup reduction: wave shuffles, then LDS across the 4 waves
    __shared__ double s_d[2][SCAN_THREADS / 64];
    __shared__ uint32_t s_f[NF][SCAN_THREADS / 64];
    __shared__ unsigned long long s_c[2][SCAN_THREADS / 64];
    dminL = wave_min(dminL);
    dminN = wave_min(dminN);
    cL = wave_sum(cL);
    cN = wave_sum(cN);
#pragma unroll
    for (int f = 0; f < NF; f++) fst[f] = wave_min(fst[f]);
    if (lane == 0) {
        s_d[0][wid] = dminL; s_d[1][wid] = dminN;
        s_c[0][wid] = cL; s_c[1][wid] = cN;
#pragma unroll
        for (int f = 0; f < NF; f++) s_f[f][wid] = fst[f];
    }
    __syncthreads();
    if (tid == 0) {
        for (int x = 1; x < SCAN_THREADS / 64; x++) {
            dminL = s_d[0][x] < dminL ? s_d[0][x] : dminL;
            dminN = s_d[1][x] < dminN ? s_d[1][x] : dminN;
            cL += s_c[0][x]; cN += s_c[1][x];
#pragma unroll
            for (int f = 0; f < NF; f++) fst[f] = min(fst[f], s_f[f][x]);
        }
        BlockRec r;
        r.dmin[0] = dminL; r.dmin[1] = dminN;
        r.cand[0] = cL; r.cand[1] = cN;
#pragma unroll
        for (int f = 0; f < NF; f++) r.first[f] = fst[f];
        a.blockrec[blockIdx.x] = r;
    }
}

// ------------------------------------------------------------- k_reduce
// one workgroup combines the per-tile records (instead of same-address atomics,
// which serialise at ~90 ops/us per word)
__global__ __launch_bounds__(1024) void k_reduce(ReduceArgs a) {
    DevCtl* ctl = a.ctl;
    if (ctl->halted) return;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    double d0 = HUGE_VAL, d1 = HUGE_VAL;
    unsigned long long c0 = 0, c1 = 0;
    uint32_t f[NF];
#pragma unroll
    for (int q = 0; q < NF; q++) f[q] = NONE32;
    for (int i = tid; i < a.tiles; i += 1024) {
        const BlockRec r = a.blockrec[i];
        d0 = r.dmin[0] < d0 ? r.dmin[0] : d0;
        d1 = r.dmin[1] < d1 ? r.dmin[1] : d1;
        c0 += r.cand[0]; c1 += r.cand[1];
#pragma unroll
        for (int q = 0; q < NF; q++) f[q] = min(f[q], r.first[q]);
    }
    d0 = wave_min(d0); d1 = wave_min(d1); c0 = wave_sum(c0); c1 = wave_sum(c1);
#pragma unroll
    for (int q = 0; q < NF; q++) f[q] = wave_min(f[q]);
    __shared__ double s_d[2][16];
    __shared__ unsigned long long s_c[2][16];
    __shared__ uint32_t s_f[NF][16];
    if (lane == 0) {
        s_d[0][wid] = d0; s_d[1][wid] = d1; s_c[0][wid] = c0; s_c[1][wid] = c1;
#pragma unroll
        for (int q = 0; q < NF; q++) s_f[q][wid] = f[q];
    }
    __syncthreads();
    if (tid == 0) {
        for (int x = 1; x < 16; x++) {
            d0 = s_d[0][x] < d0 ? s_d[0][x] : d0;
            d1 = s_d[1][x] < d1 ? s_d[1][x] : d1;
            c0 += s_c[0][x]; c1 += s_c[1][x];
            for (int q = 0; q < NF; q++) f[q] = min(f[q], s_f[q][x]);
        }
        ctl->gmin[0] = d0 < HUGE_VAL ? enc(d0) : NONE64;
        ctl->gmin[1] = d1 < HUGE_VAL ? enc(d1) : NONE64;
        ctl->ncand[0] = c0; ctl->ncand[1] = c1;
        for (int q = 0; q < NF; q++) ctl->first[q] = f[q];
    }
}

// ------------------------------------------------------------- k_census

__device__ __forceinline__ void emit_global(const ScanArgs& a, const Contender& c) {
    uint32_t i = atomicAdd(&a.ctl->ncont, 1u);
    if (i < a.cont_cap) a.cont[i] = c;
    else a.ctl->cont_overflow = 1;
}

__device__ __forceinline__ void emit(const ScanArgs& a, const Dedup& T, int kind, int s, int t, double w,
                                     unsigned long long iter) {
    if (dedup_insert(T, kind, s, t, w, iter) < 0) {   // table full or weight conflict: keep it raw
        Contender c;
        c.s = s; c.t = t; c.w = w; c.iter = iter; c.kind = kind; c.pad = 0;
        emit_global(a, c);
    }
}

// walk every allowed, non-replica target in bl_move order for one (partition, slot)
// and emit the ones within 4*eps of the minimum; stop once 8*eps is exceeded
// (the approximate delta is monotone in the target load up to 2*eps).
template <int RC>
__device__ void walk_targets(const ScanArgs& a, const Dedup& T, int kind, long long p, int slot, int src,
                             const uint32_t (&reps)[RC], int nrep, int set, double w, double ds,
                             double g, double eps, int nblm, double inv_avg) {
    const unsigned long long ib = ((unsigned long long)p << 21) | ((unsigned long long)slot << 16);
    const double delta = w * inv_avg;
    const unsigned char* rec = a.setrec + (size_t)set * a.stride;
    const int32_t* ids = (const int32_t*)(rec + sr_ids_off());
    const double* rr = (const double*)(rec + sr_r_off(a.K));
    const int nl = ((const int32_t*)rec)[1];
    int start = 0;
    for (int i = 0; i < nl; i++) {                // the set's first K eligible brokers
        const int b = ids[i];
        start = a.posm[b] + 1;
        bool isrep = false;
#pragma unroll
        for (int q = 0; q < RC; q++) isrep |= (q < nrep) && ((int)reps[q] == b);
        if (isrep) continue;
        const double d = ds + dtgt(rr[i], delta);
        if (d <= g + 4.0 * eps) emit(a, T, kind, src, b, w, ib | (unsigned long long)(start - 1));
        if (d > g + 8.0 * eps) return;
    }
    if (nl < a.K) return;                          // the set is exhausted
    const uint64_t* sb = a.setbits + (size_t)set * a.W64;
    for (int k = start; k < nblm; k++) {           // rare: more than K near-tied targets
        const int b = a.blm[k];
        if (!setbit(sb, b)) continue;
        bool isrep = false;
#pragma unroll
        for (int q = 0; q < RC; q++) isrep |= (q < nrep) && ((int)reps[q] == b);
        if (isrep) continue;
        const double d = ds + dtgt(a.r[b], delta);
        if (d <= g + 4.0 * eps) emit(a, T, kind, src, b, w, ib | (unsigned long long)k);
        if (d > g + 8.0 * eps) return;
    }
}

template <int RC>
__global__ __launch_bounds__(SCAN_THREADS) void k_census(ScanArgs a) {
    DevCtl* ctl = a.ctl;
    if (ctl->halted) return;
    const double eps = ctl->eps;
    const unsigned long long eL = ctl->gmin[0], eN = ctl->gmin[1];
    const double gL = eL == NONE64 ? HUGE_VAL : dec(eL);
    const double gN = eN == NONE64 ? HUGE_VAL : dec(eN);
    const BlockRec& br = a.blockrec[blockIdx.x];
    const bool doL = a.allow_leader && eL != NONE64 && br.dmin[0] <= gL + 8.0 * eps;
    const bool doN = eN != NONE64 && br.dmin[1] <= gN + 8.0 * eps;
    if (!doL && !doN) return;
    __shared__ uint32_t s_key[DEDUP_CENSUS];
    __shared__ unsigned long long s_wb[DEDUP_CENSUS], s_it[DEDUP_CENSUS];
    Dedup T{s_key, s_wb, s_it, DEDUP_CENSUS};
    dedup_clear(T);
    __syncthreads();
    const double inv_avg = ctl->inv_avg;
    const int nblm = ctl->nblm;
    const int roff = sr_r_off(a.K);
    const long long base = a.shard_begin + (long long)blockIdx.x * TILE + (long long)threadIdx.x * PER_LANE;
    PartRegs<RC> P;
    load_parts<RC>(a, base, P);
    for (int j = 0; j < PER_LANE; j++) {
        const long long p = base + j;
        if (p >= a.shard_end) continue;
        const uint32_t m = P.m[j];
        const int nrep = (int)meta_nrep(m), set = (int)meta_set(m);
        if (!meta_elig(m) || nrep == 0) continue;
        uint32_t reps[RC];
#pragma unroll
        for (int k = 0; k < RC; k++) reps[k] = P.r[k][j];
        const unsigned char* rec = a.setrec + (size_t)set * a.stride;
        const int32_t* ids = (const int32_t*)(rec + sr_ids_off());
        const double* rr = (const double*)(rec + roff);
        double rt = 0.0;
        bool have = false;
        for (int i = 0; i < a.K && !have; i++) {
            const int b = ids[i];
            if (b < 0) break;
            bool isrep = false;
#pragma unroll
            for (int k = 0; k < RC; k++) isrep |= (k < nrep) && ((int)reps[k] == b);
            if (!isrep) { rt = rr[i]; have = true; }
        }
        if (!have) continue;
        const double w = P.w[j];
        const double delta = w * inv_avg;
        const double dt = dtgt(rt, delta);
        if (doL) {
            const double ds = dsrc(a.r[reps[0]], delta);
            if (ds + dt <= gL + 8.0 * eps)
                walk_targets<RC>(a, T, 0, p, 0, (int)reps[0], reps, nrep, set, w, ds, gL, eps, nblm, inv_avg);
        }
        if (doN) {
#pragma unroll
            for (int k = 1; k < RC; k++) {
                if (k < nrep) {
                    const double ds = dsrc(a.r[reps[k]], delta);
                    if (ds + dt <= gN + 8.0 * eps)
                        walk_targets<RC>(a, T, 1, p, k, (int)reps[k], reps, nrep, set, w, ds, gN, eps, nblm, inv_avg);
                }
            }
        }
    }
    __syncthreads();
    // flush the workgroup's distinct keys (earliest iteration index per key)
    for (int h = threadIdx.x; h < DEDUP_CENSUS; h += SCAN_THREADS)
        if (s_key[h] != NONE32 && s_wb[h] != NONE64) emit_global(a, dedup_entry(T, h));
}

// ------------------------------------------------------------ k_resolve

struct Decision {
    int32_t status, step, kind, slot;
    long long part;
    int32_t from, to;
    double su, cu;
    int32_t exact, err, err_broker, pad;
};

__device__ __forceinline__ double contribution(const ResolveArgs& a, uint32_t q, int b) {
    const uint32_t m = a.meta[q];
    const int lead = a.rep[q] == (uint16_t)b;   // slot 0 of partition q
    const double w = a.w[q];
    if (lead) return w * (double)((int)meta_nrep(m) + a.nc[q]);
    return w;
}

// remove partition q from broker b's list (block-wide, all threads call)
__device__ void list_remove(const ResolveArgs& a, int b, uint32_t q, int* s_i) {
    const uint32_t st = a.lstart[b], n = a.llen[b];
    if (threadIdx.x == 0) *s_i = -1;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += RESOLVE_THREADS)
        if (a.lent[st + i] == q) *s_i = (int)i;
    __syncthreads();
    const int at = *s_i;
    if (at < 0) return;
    for (uint32_t c = (uint32_t)at; c + 1 < n; c += RESOLVE_THREADS) {
        uint32_t j = c + threadIdx.x;
        uint32_t v = 0;
        bool act = j + 1 < n;
        if (act) v = a.lent[st + j + 1];
        __syncthreads();
        if (act) a.lent[st + j] = v;
        __syncthreads();
    }
    if (threadIdx.x == 0) a.llen[b] = n - 1;
    __syncthreads();
}

// insert partition q into broker b's sorted list
__device__ bool list_insert(const ResolveArgs& a, int b, uint32_t q, int* s_i) {
    const uint32_t st = a.lstart[b], n = a.llen[b];
    if (n >= a.lcap[b]) return false;
    if (threadIdx.x == 0) *s_i = 0;
    __syncthreads();
    int c = 0;
    for (uint32_t i = threadIdx.x; i < n; i += RESOLVE_THREADS) c += a.lent[st + i] < q ? 1 : 0;
    c = wave_sum(c);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(s_i, c);
    __syncthreads();
    const uint32_t at = (uint32_t)*s_i;
    long long hi = (long long)n;
    while (hi > (long long)at) {
        long long lo = hi - RESOLVE_THREADS;
        if (lo < (long long)at) lo = at;
        long long j = lo + threadIdx.x;
        bool act = j < hi;
        uint32_t v = 0;
        if (act) v = a.lent[st + j];
        __syncthreads();
        if (act) a.lent[st + j + 1] = v;
        __syncthreads();
        hi = lo;
    }
    if (threadIdx.x == 0) { a.lent[st + at] = q; a.llen[b] = n + 1; }
    __syncthreads();
    return true;
}

__global__ __launch_bounds__(RESOLVE_THREADS) void k_resolve(ResolveArgs a) {
    DevCtl* ctl = a.ctl;
    if (ctl->halted) return;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    constexpr int NW = RESOLVE_THREADS / 64;
    constexpr int FOLD_CHUNK = 512;
    __shared__ Decision D;
    __shared__ int s_done, s_i, s_fail, s_ndist;
    __shared__ unsigned long long s_u[NW];
    __shared__ double s_dv[NW];
    __shared__ int s_flag[NW];
    __shared__ double s_fold[8][FOLD_CHUNK];     // refold staging (non-integral mode)
    __shared__ double s_Lm[MAXB];                // exact loads in bl_move order
    __shared__ uint32_t s_key[DEDUP_RESOLVE];
    __shared__ unsigned long long s_wb[DEDUP_RESOLVE], s_it[DEDUP_RESOLVE];
    Dedup T{s_key, s_wb, s_it, DEDUP_RESOLVE};
    const double su = ctl->U0;
    const double eps = ctl->eps;
    const int nblm = ctl->nblm;
    KB_STAMP_BEGIN();
    for (int k = tid; k < nblm; k += RESOLVE_THREADS) s_Lm[k] = a.load[a.blm[k]];

    if (tid == 0) {
        D.status = 0; D.step = -1; D.kind = 0; D.slot = -1; D.part = -1;
        D.from = -1; D.to = -1; D.su = su; D.cu = su; D.exact = 1; D.err = E_NONE; D.err_broker = -1;
        s_done = 0;
        const uint32_t* F = ctl->first;
        auto rd = [&](uint32_t p, int k) -> int { return (int)a.rep[(long long)k * a.Ppad + p]; };
        if (a.sem_go && F[F_DUP] != NONE32) {
            D.status = -1; D.step = 1; D.err = E_DUP; D.part = F[F_DUP]; s_done = 1;
        } else if (F[F_REMOVE] != NONE32) {                      // steps.go:70-89
            const uint32_t p = F[F_REMOVE];
            const uint32_t m = a.meta[p];
            const int nrep = (int)meta_nrep(m), set = (int)meta_set(m);
            const uint64_t* sb = a.setbits + (size_t)set * a.W64;
            // lightest allowed replica in (load, id) order = smallest bl position
            int best = -1, bslot = -1, bpos = 0x7FFFFFFF;
            for (int k = 0; k < nrep; k++) {
                const int b = rd(p, k);
                if (!setbit(sb, b)) continue;
                const int ps = a.posm[b];
                if (ps < bpos) { bpos = ps; best = b; bslot = k; }
            }
            D.step = 3; D.part = p;
            if (best < 0) { D.status = -1; D.err = E_REMOVE; }
            else {
                // replacepl removes the FIRST slot holding that broker (utils.go:167-178)
                D.status = 1; D.kind = 2; D.slot = bslot; D.from = best; D.to = -1;
            }
            s_done = 1;
        } else if (F[F_ADD] != NONE32) {                         // steps.go:93-113
            const uint32_t p = F[F_ADD];
            const uint32_t m = a.meta[p];
            const int nrep = (int)meta_nrep(m), set = (int)meta_set(m);
            const int32_t* dl = a.lists + ((size_t)set * 2 + 1) * a.K;
            int t = -1;
            for (int i = 0; i < a.K && t < 0; i++) {
                const int b = dl[i];
                if (b < 0) break;
                bool isrep = false;
                for (int k = 0; k < nrep; k++) isrep |= rd(p, k) == b;
                if (!isrep) t = b;
            }
            D.step = 4; D.part = p;
            if (t < 0) { D.status = -1; D.err = E_ADD; }
            else { D.status = 1; D.kind = 3; D.slot = nrep; D.from = -1; D.to = t; }
            s_done = 1;
        } else if (F[F_DIS] != NONE32) {                         // steps.go:117-143
            const uint32_t p = F[F_DIS];
            const uint32_t m = a.meta[p];
            const int nrep = (int)meta_nrep(m), set = (int)meta_set(m);
            const uint64_t* sb = a.setbits + (size_t)set * a.W64;
            int vslot = -1;
            for (int k = 0; k < nrep && vslot < 0; k++) if (!setbit(sb, rd(p, k))) vslot = k;
            const int32_t* dl = a.lists + ((size_t)set * 2 + 0) * a.K;
            int t = -1;
            for (int i = 0; i < a.K && t < 0; i++) {
                const int b = dl[i];
                if (b < 0) break;
                bool isrep = false;
                for (int k = 0; k < nrep; k++) isrep |= rd(p, k) == b;
                if (!isrep) t = b;
            }
            D.step = 5; D.part = p; D.slot = vslot; D.from = rd(p, vslot);
            if (t < 0) { D.status = -1; D.err = E_DIS; D.err_broker = D.from; }
            else { D.status = 1; D.kind = 1; D.to = t; }
            s_done = 1;
        } else if (a.rebalance && !(su < a.min_unbalance)) {     // steps.go:299-347
            if (F[F_EMPTY] != NONE32 || nblm == 0) {
                D.status = -1; D.step = 6; D.err = E_PANIC; D.part = F[F_EMPTY]; s_done = 1;
            } else if (F[F_LEAD] != NONE32) {
                const uint32_t p = F[F_LEAD];
                const int nrep = (int)meta_nrep(a.meta[p]);
                const int light = ctl->light;
                int ex = -1;
                for (int k = 0; k < nrep && ex < 0; k++) if (rd(p, k) == light) ex = k;
                D.status = 1; D.step = 6; D.part = p; D.slot = 0; D.from = rd(p, 0); D.to = light;
                D.kind = ex >= 0 ? 4 : 1;       // swap when bl[0] is already a replica
                s_done = 1;
            }
        }
    }
    __syncthreads();
    KB_STAMP(ctl, 8);

    // move(): leader step (if allowed), then non-leader step (steps.go:284-298)
    for (int kind = a.allow_leader ? 0 : 1; kind < 2 && !s_done; kind++) {
        const int step = kind == 0 ? 7 : 8;
        if (tid == 0) {
            if (ctl->first[F_EMPTY_ELIG] != NONE32) {
                D.status = -1; D.step = step; D.err = E_PANIC; D.part = ctl->first[F_EMPTY_ELIG]; s_done = 1;
            } else if (ctl->cont_overflow) {
                D.status = -1; D.step = step; D.err = E_CONT_OVERFLOW; s_done = 1;
            }
            s_fail = 0;
            s_ndist = 0;
        }
        dedup_clear(T);
        __syncthreads();
        if (s_done) break;
        const uint32_t nc = min(ctl->ncont, a.cont_cap);
        // (1) distinct keys of this kind (earliest iteration index per key)
        for (uint32_t i = tid; i < nc; i += RESOLVE_THREADS) {
            const Contender c = a.cont[i];
            if (c.kind == kind && dedup_insert(T, c.kind, c.s, c.t, c.w, c.iter) < 0) s_fail = 1;
        }
        __syncthreads();
        int nd = 0;
        for (int h = tid; h < DEDUP_RESOLVE; h += RESOLVE_THREADS) nd += s_key[h] != NONE32 ? 1 : 0;
        nd = wave_sum(nd);
        if (lane == 0 && nd) atomicAdd(&s_ndist, nd);
        __syncthreads();
        const int ndist = s_ndist;
        const bool fail = s_fail != 0;
        double Ustar = su;
        unsigned long long witer = NONE64;
        Contender cw;
        cw.s = cw.t = -1; cw.w = 0; cw.iter = NONE64; cw.kind = kind; cw.pad = 0;
        int exact = 1;
        const double thr = su - a.min_unbalance;          // steps.go:292
        const bool have = ndist > 0 || fail;
        if (!fail && ndist == 1) {
            // one key: every contender scores the same exact U; the first in iteration order wins
            if (tid == 0) s_i = -1;
            __syncthreads();
            for (int h = tid; h < DEDUP_RESOLVE; h += RESOLVE_THREADS) if (s_key[h] != NONE32) s_i = h;
            __syncthreads();
            cw = dedup_entry(T, s_i);
            witer = cw.iter;
            const double delta = cw.w * ctl->inv_avg;
            const double Ua = su + (dsrc(a.r[cw.s], delta) + dtgt(a.r[cw.t], delta));
            const double lim = thr < su ? thr : su;
            const bool certain = (Ua + 2.0 * eps < lim) || (Ua - 2.0 * eps >= (thr > su ? thr : su));
            if (certain && !a.exact_unb) { Ustar = Ua; exact = 0; }
            else {
                if (tid == 0) {
                    s_dv[0] = exact_unbalance_lds(s_Lm, nblm, a.posm[cw.s], a.posm[cw.t],
                                                  a.load[cw.s] - cw.w, a.load[cw.t] + cw.w);
                    atomicAdd(&ctl->total_folds, 1ull);
                }
                __syncthreads();
                Ustar = s_dv[0];
            }
        } else if (have) {
            // several keys (or an overfull table): exact sequential folds, lexicographic min
            double bu = HUGE_VAL;
            unsigned long long bi = NONE64;
            int bs = -1, bt = -1;
            double bw = 0.0;
            unsigned long long nf = 0;
            if (!fail) {
                for (int h = tid; h < DEDUP_RESOLVE; h += RESOLVE_THREADS) {
                    if (s_key[h] == NONE32) continue;
                    const Contender c = dedup_entry(T, h);
                    const double u = exact_unbalance_lds(s_Lm, nblm, a.posm[c.s], a.posm[c.t],
                                                         a.load[c.s] - c.w, a.load[c.t] + c.w);
                    nf++;
                    if (u < bu || (u == bu && c.iter < bi)) { bu = u; bi = c.iter; bs = c.s; bt = c.t; bw = c.w; }
                }
            } else {
                for (uint32_t i = tid; i < nc; i += RESOLVE_THREADS) {
                    const Contender c = a.cont[i];
                    if (c.kind != kind) continue;
                    const double u = exact_unbalance_lds(s_Lm, nblm, a.posm[c.s], a.posm[c.t],
                                                         a.load[c.s] - c.w, a.load[c.t] + c.w);
                    nf++;
                    if (u < bu || (u == bu && c.iter < bi)) { bu = u; bi = c.iter; bs = c.s; bt = c.t; bw = c.w; }
                }
            }
            nf = wave_sum(nf);
            if (lane == 0 && nf) atomicAdd(&ctl->total_folds, nf);
            for (int o = 32; o > 0; o >>= 1) {
                const double ou = __shfl_xor(bu, o);
                const unsigned long long oi = __shfl_xor(bi, o);
                const int os = __shfl_xor(bs, o), ot = __shfl_xor(bt, o);
                const double ow = __shfl_xor(bw, o);
                if (ou < bu || (ou == bu && oi < bi)) { bu = ou; bi = oi; bs = os; bt = ot; bw = ow; }
            }
            if (lane == 0) { s_dv[wid] = bu; s_u[wid] = bi; s_flag[wid] = wid; }
            __shared__ int s_bs[NW], s_bt[NW];
            __shared__ double s_bw[NW];
            if (lane == 0) { s_bs[wid] = bs; s_bt[wid] = bt; s_bw[wid] = bw; }
            __syncthreads();
            if (tid == 0) {
                for (int q = 1; q < NW; q++)
                    if (s_dv[q] < s_dv[0] || (s_dv[q] == s_dv[0] && s_u[q] < s_u[0])) {
                        s_dv[0] = s_dv[q]; s_u[0] = s_u[q]; s_bs[0] = s_bs[q]; s_bt[0] = s_bt[q]; s_bw[0] = s_bw[q];
                    }
            }
            __syncthreads();
            Ustar = s_dv[0]; witer = s_u[0];
            cw.s = s_bs[0]; cw.t = s_bt[0]; cw.w = s_bw[0]; cw.iter = witer;
        }
        __syncthreads();
        if (tid == 0) {
            // cu starts at su and only a strictly smaller u replaces it (steps.go:227-229,276)
            const bool improved = have && Ustar < su;
            const double cu = improved ? Ustar : su;
            if (cu < thr) {
                if (!improved) {
                    // replacepl on the zero Partition: the reference panics
                    D.status = -1; D.step = step; D.err = E_PANIC; s_done = 1;
                } else {
                    D.status = 1; D.step = step; D.kind = 1;
                    D.part = (long long)(witer >> 21); D.slot = (int)((witer >> 16) & 31);
                    D.from = cw.s; D.to = cw.t; D.su = su; D.cu = cu; D.exact = exact;
                    s_done = 1;
                }
            }
        }
        __syncthreads();
    }
    KB_STAMP(ctl, 9);

    // ---------------------------------------------------------- apply
    __shared__ int s_aff[2 * MAXR + 2];
    __shared__ double s_oldc[2 * MAXR + 2];
    __shared__ int s_naff;
    if (tid == 0) {
        s_naff = 0;
        if (D.status == 1) {
            const long long p = D.part;
            const uint32_t m = a.meta[p];
            const int nrep = (int)meta_nrep(m);
            int r[MAXR + 1];
            for (int k = 0; k < nrep; k++) r[k] = (int)a.rep[(long long)k * a.Ppad + p];
            const double wv = a.w[p];
            const int ncp = a.nc[p];
            for (int k = 0; k < nrep; k++) {             // old contributions of p's brokers
                s_aff[s_naff] = r[k];
                s_oldc[s_naff] = k == 0 ? wv * (double)(nrep + ncp) : wv;
                s_naff++;
            }
            int nn = nrep;
            bool state_changed = true;
            if (D.kind == 1) {                           // replace at slot (utils.go:186-190)
                r[D.slot] = D.to;
            } else if (D.kind == 4) {                    // swap with the existing replica (utils.go:179-185)
                int ex = 0;
                for (int k = 0; k < nrep; k++) if (r[k] == D.to) { ex = k; break; }
                const int old = r[D.slot];
                r[D.slot] = D.to;
                r[ex] = old;
            } else if (D.kind == 2) {                    // remove (utils.go:176-178)
                for (int k = D.slot; k + 1 < nrep; k++) r[k] = r[k + 1];
                if (a.sem_go) state_changed = false;     // pl keeps its length: duplicates
                else nn = nrep - 1;
            } else if (D.kind == 3) {                    // add (utils.go:199-202)
                if (a.sem_go) state_changed = false;     // the append is not visible through pl
                else { r[nrep] = D.to; nn = nrep + 1; }
            }
            // the meta bits that depend on the replicas (Disallowed trigger, in-set count)
            const uint64_t* sb = a.setbits + (size_t)meta_set(m) * a.W64;
            auto remeta = [&](int n) {
                uint32_t dis = 0, nin = 0;
                for (int k = 0; k < n; k++) { const bool in = setbit(sb, r[k]); dis |= in ? 0u : 1u; nin += in ? 1u : 0u; }
                return make_meta((uint32_t)n, meta_want(m), meta_elig(m), dis, nin, meta_set(m));
            };
            if (a.sem_go && (D.kind == 2 || D.kind == 3)) {
                // Go aliasing: the remove shifted the shared backing array in place
                if (D.kind == 2) {
                    for (int k = 0; k < nrep; k++) a.rep[(long long)k * a.Ppad + p] = (uint16_t)r[k];
                    a.meta[p] = remeta(nrep);
                }
                s_naff = 0;
            } else if (state_changed) {
                for (int k = 0; k < nn; k++) a.rep[(long long)k * a.Ppad + p] = (uint16_t)r[k];
                a.meta[p] = remeta(nn);
                if (D.kind == 1) { a.cnt[D.from]--; a.cnt[D.to]++; }
                if (D.kind == 2) { a.cnt[D.from]--; }
                if (D.kind == 3) { a.cnt[D.to]++; }
                // new contributions; integral mode updates loads incrementally (exact)
                const int base_aff = s_naff;
                for (int k = 0; k < nn; k++) {
                    const int b = r[k];
                    const double cc = k == 0 ? wv * (double)(nn + ncp) : wv;
                    int f = -1;
                    for (int x = 0; x < base_aff; x++) if (s_aff[x] == b) f = x;
                    if (f >= 0) {
                        if (s_oldc[f] == cc) { s_aff[f] = -1 - s_aff[f]; }  // unchanged contribution
                        else if (a.integral) a.load[b] = (a.load[b] - s_oldc[f]) + cc;
                    } else {
                        if (a.integral) a.load[b] = a.load[b] + cc;
                        s_aff[s_naff] = b; s_oldc[s_naff] = 0.0; s_naff++;
                    }
                }
                for (int x = 0; x < base_aff; x++) {
                    const int b = s_aff[x];
                    if (b < 0) continue;
                    bool still = false;
                    for (int k = 0; k < nn; k++) still |= r[k] == b;
                    if (!still && a.integral) a.load[b] = a.load[b] - s_oldc[x];
                }
                int n2 = 0;                              // brokers whose contribution changed
                for (int x = 0; x < s_naff; x++) if (s_aff[x] >= 0) s_aff[n2++] = s_aff[x];
                s_naff = n2;
            } else {
                s_naff = 0;
            }
        }
    }
    __syncthreads();
    KB_STAMP(ctl, 10);
    // non-integral: maintain per-broker partition lists and refold touched loads exactly
    if (D.status == 1 && !a.integral && s_naff > 0) {
        const uint32_t p = (uint32_t)D.part;
        bool ok = true;
        if (D.kind == 1) {
            list_remove(a, D.from, p, &s_i);
            ok = list_insert(a, D.to, p, &s_i);
        } else if (D.kind == 2 && !a.sem_go) {
            list_remove(a, D.from, p, &s_i);
        } else if (D.kind == 3 && !a.sem_go) {
            ok = list_insert(a, D.to, p, &s_i);
        }
        KB_STAMP(ctl, 11);
        if (!ok) {
            if (tid == 0) { ctl->list_overflow = 1; D.status = -1; D.err = E_LIST_OVERFLOW; }
        } else {
            const int naff = s_naff;
            for (int x0 = 0; x0 < naff; x0 += 8) {
                // stage up to 8 brokers' contributions chunk by chunk; lane 0 of wave x folds
                const int nb = naff - x0 < 8 ? naff - x0 : 8;
                uint32_t maxn = 0;
                for (int x = 0; x < nb; x++) { const uint32_t n = a.llen[s_aff[x0 + x]]; maxn = n > maxn ? n : maxn; }
                double acc = 0.0;
                for (uint32_t c = 0; c < maxn; c += FOLD_CHUNK) {
                    for (int e = tid; e < nb * FOLD_CHUNK; e += RESOLVE_THREADS) {
                        const int x = e / FOLD_CHUNK, i = e % FOLD_CHUNK;
                        const int b = s_aff[x0 + x];
                        const uint32_t n = a.llen[b], st = a.lstart[b];
                        if (c + (uint32_t)i < n) s_fold[x][i] = contribution(a, a.lent[st + c + i], b);
                    }
                    __syncthreads();
                    if (lane == 0 && wid < nb) {
                        const int b = s_aff[x0 + wid];
                        const uint32_t n = a.llen[b];
                        if (c < n) acc = fold_lds(&s_fold[wid][0], (int)(n - c < FOLD_CHUNK ? n - c : FOLD_CHUNK), acc);
                    }
                    __syncthreads();
                }
                if (lane == 0 && wid < nb) a.load[s_aff[x0 + wid]] = acc;
                __syncthreads();
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        KB_STAMP(ctl, 12);
        ChangeDev ch;
        ch.status = D.status; ch.step = D.step; ch.kind = D.kind; ch.slot = D.slot;
        ch.part = D.part; ch.from = D.from; ch.to = D.to; ch.su = D.su; ch.cu = D.cu;
        ch.exact = D.exact; ch.err_code = D.err; ch.err_broker = D.err_broker; ch.pad = 0;
        if (ctl->logpos < ctl->logcap) a.log[ctl->logpos] = ch;
        ctl->logpos++;
        ctl->steps++;
        // reference candidate count of the steps that actually ran this iteration
        unsigned long long add = 0;
        if (D.step < 0 || D.step >= 7) {
            if (a.allow_leader) add += ctl->ncand[0];
            if (D.step != 7) add += ctl->ncand[1];
        }
        ctl->total_cand += add;
        ctl->total_cont += min(ctl->ncont, a.cont_cap);
        if (D.status != 1) ctl->halted = 1;
    }
}

// --------------------------------------------------- multi-GPU summaries

// pack this rank's scan result + its distinct local near-tie keys
__global__ __launch_bounds__(1024) void k_summary(SumArgs a) {
    DevCtl* ctl = a.ctl;
    Summary* s = a.out;
    __shared__ uint32_t s_key[DEDUP_RESOLVE];
    __shared__ unsigned long long s_wb[DEDUP_RESOLVE], s_it[DEDUP_RESOLVE];
    __shared__ uint32_t s_n;
    __shared__ int s_fail;
    Dedup T{s_key, s_wb, s_it, DEDUP_RESOLVE};
    dedup_clear(T);
    if (threadIdx.x == 0) { s_n = 0; s_fail = 0; }
    __syncthreads();
    const uint32_t nc = min(ctl->ncont, a.cont_cap);
    for (uint32_t i = threadIdx.x; i < nc; i += blockDim.x) {
        const Contender c = a.cont[i];
        if (dedup_insert(T, c.kind, c.s, c.t, c.w, c.iter) < 0) s_fail = 1;
    }
    __syncthreads();
    for (int h = threadIdx.x; h < DEDUP_RESOLVE; h += blockDim.x) {
        if (s_key[h] == NONE32) continue;
        const uint32_t k = atomicAdd(&s_n, 1u);
        if (k < (uint32_t)SUMMARY_CONT) s->cont[k] = dedup_entry(T, h);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        s->gmin[0] = ctl->gmin[0]; s->gmin[1] = ctl->gmin[1];
        for (int f = 0; f < NF; f++) s->first[f] = ctl->first[f];
        s->ncand[0] = ctl->ncand[0]; s->ncand[1] = ctl->ncand[1];
        s->ncont = s_n < (uint32_t)SUMMARY_CONT ? s_n : (uint32_t)SUMMARY_CONT;
        s->overflow = (ctl->cont_overflow || s_fail || s_n > (uint32_t)SUMMARY_CONT) ? 1u : 0u;
        if (ctl->halted) s->overflow |= 2u;
    }
}

// combine every rank's summary identically on every rank
__global__ __launch_bounds__(256) void k_merge(MergeArgs a) {
    DevCtl* ctl = a.ctl;
    if (ctl->halted) return;
    __shared__ unsigned long long g[2];
    __shared__ uint32_t total;
    if (threadIdx.x == 0) {
        g[0] = g[1] = NONE64;
        uint32_t f[NF];
        for (int q = 0; q < NF; q++) f[q] = NONE32;
        unsigned long long c0 = 0, c1 = 0;
        uint32_t ov = 0;
        for (int r = 0; r < a.nranks; r++) {
            const Summary* s = a.all + r;
            g[0] = s->gmin[0] < g[0] ? s->gmin[0] : g[0];
            g[1] = s->gmin[1] < g[1] ? s->gmin[1] : g[1];
            for (int q = 0; q < NF; q++) f[q] = min(f[q], s->first[q]);
            c0 += s->ncand[0]; c1 += s->ncand[1];
            ov |= s->overflow & 1u;
        }
        ctl->gmin[0] = g[0]; ctl->gmin[1] = g[1];
        for (int q = 0; q < NF; q++) ctl->first[q] = f[q];
        ctl->ncand[0] = c0; ctl->ncand[1] = c1;
        ctl->cont_overflow = ov;
        total = 0;
    }
    __syncthreads();
    const double eps = ctl->eps, inv_avg = ctl->inv_avg;
    for (int r = 0; r < a.nranks; r++) {
        const Summary* s = a.all + r;
        for (uint32_t i = threadIdx.x; i < s->ncont; i += blockDim.x) {
            const Contender c = s->cont[i];
            // each rank emitted relative to its own minimum; keep those within the
            // global bound (every rank holds the same loads, so d is identical)
            if (g[c.kind] == NONE64) continue;
            const double gm = dec(g[c.kind]);
            const double delta = c.w * inv_avg;
            const double d = dsrc(a.r[c.s], delta) + dtgt(a.r[c.t], delta);
            if (!(d <= gm + 4.0 * eps)) continue;
            const uint32_t k = atomicAdd(&total, 1u);
            if (k < a.cont_cap) a.cont[k] = c;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) ctl->ncont = total;
}

// ------------------------------------------------------- launch helpers

template <int RC>
static void launch_scan_rc(const ScanArgs& a, int tiles, hipStream_t st) {
    hipLaunchKernelGGL(k_scan<RC>, dim3(tiles), dim3(SCAN_THREADS), 0, st, a);
}
template <int RC>
static void launch_census_rc(const ScanArgs& a, int tiles, hipStream_t st) {
    hipLaunchKernelGGL(k_census<RC>, dim3(tiles), dim3(SCAN_THREADS), 0, st, a);
}

#define KB_RC_SWITCH(RCV, FN, ...)                  \
    switch (RCV) {                                   \
        case 1: FN<1>(__VA_ARGS__); break;           \
        case 2: FN<2>(__VA_ARGS__); break;           \
        case 3: FN<3>(__VA_ARGS__); break;           \
        case 4: FN<4>(__VA_ARGS__); break;           \
        case 6: FN<6>(__VA_ARGS__); break;           \
        case 8: FN<8>(__VA_ARGS__); break;           \
        case 12: FN<12>(__VA_ARGS__); break;         \
        default: FN<16>(__VA_ARGS__); break;         \
    }

void launch_prep(const PrepArgs& a, hipStream_t st) {
    const size_t lds = (size_t)a.NP2 * (8 + 8 + 4);
    hipLaunchKernelGGL(k_prep, dim3(1), dim3(PREP_THREADS), lds, st, a);
}
void launch_setlists(const SetArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_setlists, dim3((a.nsets + 3) / 4), dim3(256), 0, st, a);
}
void launch_scan(const ScanArgs& a, int rc, int tiles, hipStream_t st) {
    KB_RC_SWITCH(rc, launch_scan_rc, a, tiles, st);
}
void launch_census(const ScanArgs& a, int rc, int tiles, hipStream_t st) {
    KB_RC_SWITCH(rc, launch_census_rc, a, tiles, st);
}
void launch_reduce(const ReduceArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, st, a);
}
void launch_resolve(const ResolveArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_resolve, dim3(1), dim3(RESOLVE_THREADS), 0, st, a);
}
void launch_summary(const SumArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_summary, dim3(1), dim3(1024), 0, st, a);
}
void launch_merge(const MergeArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_merge, dim3(1), dim3(256), 0, st, a);
}

}  // namespace kbe
