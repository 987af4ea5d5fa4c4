// engine_dev.h -- device-side data layout shared by the HIP kernels and the
// host half of the engine (engine.cpp).  See DESIGN.md "Data layout in HBM".
#pragma once
#include <cstdint>

namespace kbe {

constexpr int MAXB = 4096;          // dense broker universe limit (prep sorts it in LDS)
constexpr int MAXR = 16;            // replica slots per partition
constexpr int TILE = 1024;          // partitions per scan/census workgroup
constexpr int SCAN_THREADS = 256;   // 4 consecutive partitions per lane
constexpr int PER_LANE = 4;
constexpr int RESOLVE_THREADS = 1024;
constexpr int PREP_THREADS = 1024;
constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr unsigned long long NONE64 = ~0ull;
constexpr int SUMMARY_CONT = 1024;  // distinct near-tie keys carried per rank in a summary
constexpr int DEDUP_RESOLVE = 2048; // LDS key table of k_resolve / k_summary
constexpr int DEDUP_CENSUS = 512;   // LDS key table of one k_census workgroup

// first-index predicates reduced by the scan (min over partition index)
enum {
    F_DUP = 0,         // ValidateReplicas (steps.go:27-36), only for Go-aliasing semantics
    F_REMOVE = 1,      // RemoveExtraReplicas trigger (steps.go:74)
    F_ADD = 2,         // AddMissingReplicas trigger (steps.go:97)
    F_DIS = 3,         // MoveDisallowedReplicas trigger (steps.go:124-126)
    F_LEAD = 4,        // distributeLeaders pick (steps.go:259-272)
    F_EMPTY = 5,       // partition with no replicas (distributeLeaders panics)
    F_EMPTY_ELIG = 6,  // ... and eligible for move() (slice bounds panic)
    NF = 8
};

// meta word of a partition:
//   [0..4] nrep  [5..9] want (NumReplicas, clamped to 31)  [10] eligible (want >= MinReplicas)
//   [11] a replica is outside the allowed set (MoveDisallowedReplicas trigger)
//   [12..16] replicas inside the allowed set  [17..31] allowed-set index
__host__ __device__ inline uint32_t meta_nrep(uint32_t m) { return m & 31u; }
__host__ __device__ inline uint32_t meta_want(uint32_t m) { return (m >> 5) & 31u; }
__host__ __device__ inline uint32_t meta_elig(uint32_t m) { return (m >> 10) & 1u; }
__host__ __device__ inline uint32_t meta_dis(uint32_t m) { return (m >> 11) & 1u; }
__host__ __device__ inline uint32_t meta_nin(uint32_t m) { return (m >> 12) & 31u; }
__host__ __device__ inline uint32_t meta_set(uint32_t m) { return m >> 17; }
__host__ __device__ inline uint32_t make_meta(uint32_t nrep, uint32_t want, uint32_t elig, uint32_t dis,
                                              uint32_t nin, uint32_t set) {
    return (nrep & 31u) | ((want > 31u ? 31u : want) << 5) | ((elig & 1u) << 10) | ((dis & 1u) << 11) |
           ((nin & 31u) << 12) | (set << 17);
}
constexpr uint32_t MAX_SETS = 1u << 15;

// per-set target record, rebuilt every step by k_setlists:
//   int32 nelig (|set ∩ bl_move|), int32 nlist, int32 ids[K] (first K eligible
//   brokers in bl_move order), double r[K] (their relative loads L/avg - 1)
__host__ __device__ inline int sr_ids_off() { return 8; }
__host__ __device__ inline int sr_r_off(int K) { return (8 + 4 * K + 15) & ~15; }
__host__ __device__ inline int sr_stride(int K) { return sr_r_off(K) + 8 * K; }

struct Contender {                  // a near-tie candidate move (32 B)
    int32_t s, t;                   // dense source / target broker
    double w;                       // partition weight (scored delta, steps.go:250,272)
    unsigned long long iter;        // (partition << 21) | (slot << 16) | target bl position
    int32_t kind;                   // 0 = leader move, 1 = non-leader move
    int32_t pad;
};

// per-tile scan record (64 B): no global atomics in the scan, k_reduce combines
struct BlockRec {
    double dmin[2];                 // min score delta {leader, non-leader}
    unsigned long long cand[2];     // reference candidate counts
    uint32_t first[NF];             // first-index predicates
};

struct ChangeDev {
    int32_t status, step, kind, slot;
    int64_t part;
    int32_t from, to;               // dense broker indices (-1 none)
    double su, cu;
    int32_t exact, err_code;
    int32_t err_broker, pad;
};

struct DevCtl {
    int32_t halted, steps, logpos, logcap;
    int32_t nblm, heavy, light, npresent;
    double S, avg, inv_avg, U0, eps, V;
    unsigned long long gmin[2];     // order-preserving encoded min score delta per kind
    uint32_t first[NF];
    unsigned long long ncand[2];    // reference candidate count of this step per kind
    uint32_t ncont, cont_overflow;
    int32_t list_overflow, pad0;
    unsigned long long total_cand, total_cont, total_folds;
    // diagnostic phase stamps (builds with -DKB_STAMPS): accumulated
    // wall_clock64 ticks (100 MHz) per phase of k_prep [0..7] and k_resolve [8..15]
    unsigned long long stamps[16];
};

#ifdef KB_STAMPS
#define KB_STAMP_BEGIN() unsigned long long _kb_t0 = wall_clock64()
#define KB_STAMP(ctl, i)                                                        \
    do {                                                                        \
        if (threadIdx.x == 0) {                                                 \
            unsigned long long _t = wall_clock64();                             \
            (ctl)->stamps[i] += _t - _kb_t0;                                    \
            _kb_t0 = _t;                                                        \
        }                                                                       \
    } while (0)
#else
#define KB_STAMP_BEGIN() (void)0
#define KB_STAMP(ctl, i) (void)0
#endif

// summary exchanged between ranks each step (multi-GPU)
struct Summary {
    unsigned long long gmin[2];
    uint32_t first[NF];
    unsigned long long ncand[2];
    uint32_t ncont, overflow;
    Contender cont[SUMMARY_CONT];
};

// errors recorded in ChangeDev.err_code
enum {
    E_NONE = 0, E_DUP = 1, E_REMOVE = 2, E_ADD = 3, E_DIS = 4, E_PANIC = 5,
    E_CONT_OVERFLOW = 6, E_LIST_OVERFLOW = 7
};

}  // namespace kbe
