// kernels_api.h -- argument blocks and launchers of the kernels in kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "engine_dev.h"

namespace kbe {

// per-broker partition lists (non-integral loads): CSR with slack, sorted by
// partition index, the fold order of getBrokerLoad (utils.go:92-105)
struct Lists {
    uint32_t* lstart;
    uint32_t* llen;
    uint32_t* lcap;
    uint32_t* lent;
    // fold checkpoints: ck[lstart + 64 i - 1] = the in-order fold of a list's first 64 i
    // contributions (i >= 1, the partial sums of getBrokerLoad's own chain), valid below
    // dpos[b], the first list position whose entry or contribution changed since the broker's
    // last refold (NONE32: all valid) -- a refold restarts at the checkpoint below dpos
    double* ck;
    uint32_t* dpos;
};

struct RefreshArgs {
    DevCtl* ctl;
    const double* w;
    const uint16_t* rep;
    const uint32_t* meta;
    const int32_t* nc;
    double* load;
    double* lerr;
    double* eb;
    uint8_t* bfl;
    int B;
    Lists L;
};

struct ScanArgs {
    DevCtl* ctl;
    const double* w;
    const uint16_t* rep;      // [RC][Ppad] slot-major dense broker ids
    const uint32_t* meta;     // [Ppad]
    long long Ppad, shard_begin, shard_end;
    int ntiles, nscan;        // tiles of twaves * BLK partitions; workgroups that scan
    int twaves;               // waves of a workgroup that score (a tile's blocks; the rest idle)
    int B, nsets, W64, units; // units: 16-B words per set record
    const uint64_t* setbits;
    const uint4* setrec;
    const double* r;
    const int32_t* blm;
    const int32_t* posm;
    int allow_leader, rebalance, sem_go;
    Recs R;                   // this scan's workgroup records (scan_recs layout)
    Contender* cont;          // spill buffer
    uint32_t cont_cap;
    uint32_t* ncont;          // its fill counter and overflow flag (DevCtl's)
    uint32_t* cont_ovf;
    int listwg;               // 1: the last workgroup applies the pending list op
    int ubpass;               // 1: census-free bound pass (k_ubinit follows); returns at once
                              //    unless a relevant upper bound is +inf
    int dbg;                  // diagnostic only (KB_DEBUG_SCAN): 1 = skip the census
    int rfpass;               // 1: if the last k_step halted for exact loads (H_NEED_EXACT),
                              //    this launch refolds the dirty brokers instead of scanning
    const RefreshArgs* rf;    //    (with the pending list edit) and the pair's k_step resumes
    Lists L;
    int incr;                 // incremental mode: block descriptors (DevCtl.incr_ok decides per step)
    int nblk;
    const BlockDesc* bdesc;
    const uint32_t* pset;     // [Ppad] allowed-set index per partition (set records in memory only)
    int eager;                // > 0: that many extra workgroups after the list workgroup refold the
                              //    last applied step's touched brokers (DevCtl.eg_*)
    int gt;                   // 1: the broker tables are read from memory (B > MAXB; k_scan<.., GT>)
    uint32_t* done;           // k_pair: every non-step workgroup counts itself in here when done
    unsigned long long* wgt;  // diagnostic (KB_WGT): per scan workgroup {start, scored, record written}
    int pred;                 // 1 (k_pair only): scanning workgroups fold their record's minima,
                              //    counts and predicate mask into their arrival line (PRED_*)
    int dyn_lds;              // the launch's dynamic LDS bytes (the eager refolds' buffer)
};

struct StepArgs {
    DevCtl* ctl;
    double* w;
    uint16_t* rep;
    uint32_t* meta;
    const int32_t* nc;        // NumConsumers
    long long Ppad;
    int RC, KR, K, units, W64, B, nsets, NP2;
    int sb_lds;               // 1: every set's allowed-set words are staged in LDS
    int lds_bytes;            // dynamic LDS (step_lds(B, NP2, sb_lds ? nsets * W64 : 0).total)
    const uint64_t* setbits;
    uint4* setrec;
    int32_t* order;           // [B] universe sorted by (load, id)
    int32_t* posu;            // [B] position in order
    int32_t* blm;             // [B] bl_move order
    int32_t* posm;            // [B] position in bl_move or -1
    double* r;                // [B] approximate relative loads
    double* load;             // [B] loads (exact in integral mode / when clean)
    double* lerr;             // [B] bound |load - real sum of contributions| (non-integral)
    double* eb;               // [B] bound |load - reference fold| (0 when exact)
    uint8_t* bfl;             // [B] BF_PRESENT | BF_INCFG | BF_DIRTY
    int32_t* cnt;             // [B] replicas held
    const int32_t* bset_off;  // [B+1] sets containing each broker
    const int32_t* bset_ids;
    Recs R;                   // scan records or gathered rank summaries
    const Contender* cont;    // spill buffer (single-GPU mode)
    uint32_t cont_cap;
    int use_spill;
    int allow_leader, rebalance, sem_go, integral, exact_unb;
    long long minrep;
    double min_unbalance, wmax;
    ChangeDev* log;
    Lists L;
    int incr;                 // incremental mode (single GPU): decide DevCtl.incr_ok / wskip
    BlockDesc* ubdesc;        // [2 * R.n] the blocks of the records' best keys (bound pass subset)
    int ub_heavy;             // 1: ubdesc also lists the heaviest blocks (the subset is never empty)
    const uint32_t* pset;     // [Ppad] allowed-set index per partition, or null (the meta word's field)
    int rf_final;             // 1: a halt for exact loads was refolded by this pair's first scan
                              //    (rfpass): resume with a full prep
    int eager;                // 1: leave the touched brokers (and their list edit) to the next
                              //    scan's eager refolds (ScanArgs.eager)
    unsigned char* gscr;      // non-null (B > MAXB): k_step's per-broker tables live in this
                              //    memory scratch (step_lds(B, NP2, 0) layout) instead of LDS
    uint32_t* wait_cnt;       // k_pair's step workgroup: waits until *wait_cnt == wait_n (the
    int wait_n;               //    grid's other workgroups), then resets it
    int fuse_pre;             // k_pair: stage the broker tables before the wait (diagnostic 0: after)
    unsigned long long wait_ticks;   // k_pair: the wait's bound (100 MHz ticks; 2 s, tests: 0)
    // deferred prep (DevCtl.fp): fp_lds > 0 = the byte offset of its LDS region in the dynamic
    // LDS (bl positions int32[B], then the set records uint4[nsets * units]); fp_ok = a step may
    // leave its prep deferred (engine.cpp decides; a pending one is finished whenever fp_lds > 0)
    int fp_lds, fp_ok;
    int fp_bk;                // 1: the fp region also holds the records' best keys (2 per record)
};


struct SumArgs {
    DevCtl* ctl;
    Recs R;                   // this rank's scan records
    const Contender* cont;
    uint32_t cont_cap;
    const double* r;
    int B;                    // brokers (r's length; k_summary stages r in LDS, B <= MAXB)
    Recs out;                 // one summary (summary_recs layout)
    int spill_growable;       // 1: this rank's spill buffer can still grow (summary flag bit 2)
    // k_scansum (the summary workgroup in the scan's grid): the arrival count it waits on
    // (wait_n workgroups, bounded by wait_ticks), and the step log for a timeout's error
    uint32_t* wait_cnt;
    int wait_n;
    unsigned long long wait_ticks;
    ChangeDev* log;
};

void launch_scan(const ScanArgs& a, int rc, bool lds_sets, size_t lds_bytes, hipStream_t st);
int scan_blocks_per_cu(int rc, bool lds_sets, bool gt, size_t lds_bytes);
void launch_step(const StepArgs& a, hipStream_t st);
bool pair_supported(int rc);
int pair_blocks_per_cu(int rc, bool lds_sets, size_t lds_bytes, int* static_lds);
void launch_pair(const ScanArgs& a, const StepArgs& sa, int rc, bool lds_sets, size_t lds_bytes, hipStream_t st);
int step_static_lds(bool gb);
// diagnostic: one workgroup rewrites the given tables in place (n = 0: nothing)
void launch_ubinit(DevCtl* ctl, const Recs& R, int allow_leader, int tighten, hipStream_t st);
void launch_touch(double* r, int B, int32_t* blm, int32_t* posm, uint4* setrec, int nrec, hipStream_t st);
void launch_listop(DevCtl* ctl, const Lists& L, hipStream_t st);
void launch_refresh(const RefreshArgs& a, hipStream_t st);
void launch_summary(const SumArgs& a, hipStream_t st);
int scansum_blocks_per_cu(int rc, bool lds_sets, size_t lds_bytes, int* static_lds);
void launch_scansum(const ScanArgs& a, const SumArgs& sa, int rc, bool lds_sets, size_t lds_bytes, hipStream_t st);

// k_xfer: up to two 32-bit word copies (device <-> the host's mapped pinned mirror), then,
// if flag is set, a system-scope release and *flag = seq (the host waits on it)
struct XferArgs {
    const uint32_t* src[2];
    uint32_t* dst[2];
    int n[2];
    uint32_t* flag;
    uint32_t seq;
};
void launch_xfer(const XferArgs& a, hipStream_t st);

}  // namespace kbe
