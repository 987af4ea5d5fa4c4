// kernels_api.h -- argument blocks and launchers of the kernels in kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "engine_dev.h"

namespace kbe {

struct PrepArgs {
    DevCtl* ctl;
    const double* load;
    const int32_t* cnt;
    const uint8_t* incfg;
    int B, NP2;
    int32_t* order;        // [B] universe sorted by (load, id)
    int32_t* blm;          // [B] bl_move order (present or in cfg.Brokers)
    int32_t* posm;         // [B] position in bl_move or -1
    double* r;             // [B] relative load L/avg - 1 (approximate, scoring only)
    double rmax_w;         // max weight (for the eps bound)
};

struct SetArgs {
    const DevCtl* ctl;
    int nsets, B, W64, K, stride;
    const uint64_t* setbits;
    const int32_t* order;
    const int32_t* posm;
    const int32_t* cnt;
    const double* r;
    unsigned char* setrec;  // [nsets][stride] first K eligible targets + their r + nelig
    int32_t* lists;         // [nsets][2][K]: desc present (Disallowed), desc universe (Add)
};

struct ScanArgs {
    DevCtl* ctl;
    const double* w;
    const uint16_t* rep;      // [RC][Ppad] slot-major dense broker ids
    const uint32_t* meta;     // [Ppad]
    long long Ppad, shard_begin, shard_end;
    int K, W64, stride;
    const uint64_t* setbits;
    const unsigned char* setrec;
    const double* r;
    const int32_t* blm;
    const int32_t* posm;
    int allow_leader, rebalance, sem_go;
    BlockRec* blockrec;       // [tiles] per-tile record (k_reduce combines)
    Contender* cont;
    uint32_t cont_cap;
};

struct ReduceArgs {
    DevCtl* ctl;
    const BlockRec* blockrec;
    int tiles;
};

struct ResolveArgs {
    DevCtl* ctl;
    double* w;
    uint16_t* rep;
    uint32_t* meta;
    const int32_t* nc;        // NumConsumers
    long long Ppad;
    int RC, K, W64, B;
    const uint64_t* setbits;
    const int32_t* lists;
    const int32_t* blm;
    const int32_t* posm;
    const double* r;
    double* load;
    int32_t* cnt;
    const Contender* cont;
    uint32_t cont_cap;
    int allow_leader, rebalance, sem_go, integral, exact_unb;
    long long minrep;
    double min_unbalance;
    // per-broker partition lists (non-integral mode): CSR with slack
    uint32_t* lstart;
    uint32_t* llen;
    uint32_t* lcap;
    uint32_t* lent;
    ChangeDev* log;
};

struct SumArgs {
    DevCtl* ctl;
    const Contender* cont;
    uint32_t cont_cap;
    Summary* out;
};

struct MergeArgs {
    DevCtl* ctl;
    const Summary* all;
    int nranks;
    Contender* cont;
    uint32_t cont_cap;
    const double* r;
};

void launch_prep(const PrepArgs& a, hipStream_t st);
void launch_setlists(const SetArgs& a, hipStream_t st);
void launch_scan(const ScanArgs& a, int rc, int tiles, hipStream_t st);
void launch_census(const ScanArgs& a, int rc, int tiles, hipStream_t st);
void launch_reduce(const ReduceArgs& a, hipStream_t st);
void launch_resolve(const ResolveArgs& a, hipStream_t st);
void launch_summary(const SumArgs& a, hipStream_t st);
void launch_merge(const MergeArgs& a, hipStream_t st);

}  // namespace kbe
