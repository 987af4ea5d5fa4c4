// engine_dev.h -- device-side data layout shared by the HIP kernels and the
// host half of the engine (engine.hip).  See DESIGN.md "Data layout in HBM".
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
constexpr int SUMMARY_CONT = 1024;  // contenders carried per rank in a multi-GPU summary

// first-index predicates reduced by the scan (atomicMin over partition index)
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

// meta word of a partition: nrep | want | eligible | set
__host__ __device__ inline uint32_t meta_nrep(uint32_t m) { return m & 31u; }
__host__ __device__ inline uint32_t meta_want(uint32_t m) { return (m >> 5) & 31u; }
__host__ __device__ inline uint32_t meta_elig(uint32_t m) { return (m >> 10) & 1u; }
__host__ __device__ inline uint32_t meta_set(uint32_t m) { return m >> 11; }
__host__ __device__ inline uint32_t make_meta(uint32_t nrep, uint32_t want, uint32_t elig, uint32_t set) {
    return (nrep & 31u) | ((want > 31u ? 31u : want) << 5) | ((elig & 1u) << 10) | (set << 11);
}
constexpr uint32_t MAX_SETS = 1u << 21;

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
};

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
