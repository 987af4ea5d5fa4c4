// engine_dev.h -- device-side data layout shared by the HIP kernels and the
// host half of the engine (engine.cpp).  See DESIGN.md "Data layout in HBM".
#pragma once
#include <cstddef>
#include <cstdint>

namespace kbe {

constexpr int MAXB = 4096;          // brokers whose tables k_scan / k_step keep in LDS
constexpr int MAXB_G = 16384;       // dense broker universe limit (past MAXB: tables in memory;
                                    // 15-bit ids in the near-tie keys, 16-bit bl positions)
constexpr int MAXR = 16;            // replica slots per partition
#ifndef KB_SCAN_THREADS
#define KB_SCAN_THREADS 1024
#endif
constexpr int SCAN_THREADS = KB_SCAN_THREADS;  // k_scan workgroup (one per CU at 1024)
constexpr int PER_LANE = 2;         // consecutive partitions per lane (vector loads)
constexpr int TILE = SCAN_THREADS * PER_LANE;   // 2048 partitions per scan tile
constexpr int SHARD_ALIGN = 1024;   // shard boundaries (multi-GPU) are multiples of this
#ifndef KB_STEP_THREADS
#define KB_STEP_THREADS 1024
#endif
constexpr int STEP_THREADS = KB_STEP_THREADS;  // k_step: one workgroup
#ifndef KB_ABL
#define KB_ABL 0                    // diagnostic ablation builds only (tools/ablate.sh)
#endif
constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr unsigned long long NONE64 = ~0ull;
constexpr uint16_t NONE16 = 0xFFFFu;
constexpr int TILE_KEYS = 16;       // near-tie keys carried in a scan workgroup record
constexpr int SUMMARY_KEYS = 56;    // key slots per rank summary to start with (1936-B summaries):
                                    // near-tie keys in the first 54, the last two the second-best
                                    // keys per kind (k_summary); grown 8x (up to DEDUP_STEP) when
                                    // the near-tie keys overflow
constexpr int SUMMARY_KEYS_MAX = 2048;
constexpr int SUM_RECS = 1024;      // scan records one rank summary reads (one per thread)
constexpr uint32_t SUM_POISON = 8u;  // rank summary flag: its summary workgroup timed out (every rank halts)
constexpr int SUM_RLDS = 8192;      // k_summary keeps r in LDS up to this many brokers
constexpr int DEDUP_STEP = 2048;    // LDS key table of k_step / k_summary
constexpr int DEDUP_SCAN = 256;     // LDS key table of one k_scan workgroup
constexpr int TMAX = 2 * MAXR + 4;  // brokers touched by one applied change (bound)
constexpr int EGW = 4;              // eager refold workgroups per scan launch (touched brokers)
constexpr int PAIR_SHARDS = 8;      // k_pair's arrival count: one word per XCD group of blocks,
constexpr int PAIR_STRIDE = 32;     // each on a 128-B line of its own
// k_pair's scan workgroups also fold their record's minima, candidate counts and predicate
// mask into their arrival line (u32 word offsets; the u64 words 8-byte aligned): the step
// workgroup reads the grid's reduction from the 8 lines instead of reducing every record
// after its wait.  Zero is every word's identity: the minima are stored as ~enc(d) and
// combined with max.
constexpr int PRED_M0 = 2, PRED_M1 = 4, PRED_C0 = 6, PRED_C1 = 8, PRED_FM = 10;
constexpr int RF_CHUNK = 2048;       // in-stream refresh: contributions per fold chunk (two buffers)
constexpr int RF_LDS_BYTES = 2 * RF_CHUNK * 8;
constexpr int BLK = 128;            // partitions of one wave in a scan tile = one block of
                                    // the incremental mode (64 lanes x PER_LANE)

// incremental mode: one descriptor per partition block, sorted by wmax descending
struct BlockDesc {
    double wmax;                    // largest weight in the block (after FillDefaults)
    long long blk;                  // block index: partitions [blk * BLK, blk * BLK + BLK)
};
constexpr int LDS_SETS_MAX = 65536; // set records staged in LDS when they fit in this

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

// Per-set target record, maintained by k_step (16-byte units, u16 fields):
//   [0] nelig = |set ∩ bl_move|, [1] nl = valid ids, [2 .. 2+KR) the first KR
//   brokers of set ∩ bl_move in bl order (dense ids, NONE16 past nl).
// KR >= RC + 1 so the first eligible non-replica target is always inside.  At least two
// units (KR = 14): a census walk that passes the record's last entry goes on through the set's
// membership words in memory, a round trip per four bl positions, and with KR = 6 the three c3
// census workgroups walked ~1000 positions per step there (~2.5 us behind every other scan
// workgroup); the scan's first-target pick reads only the first unit (RC + 1 <= 6).
__host__ __device__ constexpr int sr_units(int rc) { return (rc + 1 + 2 + 7) / 8 > 2 ? (rc + 1 + 2 + 7) / 8 : 2; }
// set-record units the fast prep's merge handles (engine.cpp: the deferred prep needs units <= this)
constexpr int FP_MAXU = 2;
// the units holding a record's first RC + 1 entries (the scan's first-target pick)
__host__ __device__ constexpr int sr_units_first(int rc) { return (rc + 1 + 2 + 7) / 8; }
__host__ __device__ constexpr int sr_kr(int rc) { return sr_units(rc) * 8 - 2; }

struct Contender {                  // a near-tie candidate move (32 B)
    int32_t s, t;                   // dense source / target broker
    double w;                       // partition weight (scored delta, steps.go:185,207)
    unsigned long long iter;        // (partition << 21) | (slot << 16) | target bl position
    int32_t kind;                   // 0 = leader move, 1 = non-leader move
    int32_t pad;
};

// header of a scan-workgroup record and of a rank summary (multi-GPU)
struct RecHdr {                     // 112 B
    double dmin[2];                 // min score delta {leader, non-leader}
    unsigned long long cand[2];     // reference candidate counts
    uint32_t nkeys;                 // near-tie keys stored for this record
    uint32_t flags;                 // bit0: keys overflowed (see k_step); bit1: summaries: the scan ran
    uint32_t fmask;                 // bit q: first[q] != NONE32 (first-index predicates)
    uint16_t nkk[2];                // keys per kind within the window (stored or spilled)
    Contender best[2];              // the record's minimum-score key per kind (s < 0: none);
                                    // k_step re-scores them for the next step's upper bound
};
static_assert(sizeof(RecHdr) == 112, "record header layout");

// a set of records: headers, first-index predicate words and near-tie keys, each
// with its own byte stride (scan records: three dense arrays; rank summaries: one
// self-contained block per rank)
struct Recs {
    unsigned char* hdr;
    unsigned char* first;           // uint32_t[NF] per record
    unsigned char* keys;            // Contender[cap] per record
    int hdr_stride, first_stride, key_stride;
    int n, cap;
    __host__ __device__ RecHdr* h(int i) const { return (RecHdr*)(hdr + (size_t)i * hdr_stride); }
    __host__ __device__ uint32_t* f(int i) const { return (uint32_t*)(first + (size_t)i * first_stride); }
    __host__ __device__ Contender* k(int i) const { return (Contender*)(keys + (size_t)i * key_stride); }
};
constexpr int FIRST_BYTES = NF * 4;
constexpr int WGREC_BYTES = (int)sizeof(RecHdr) + FIRST_BYTES + TILE_KEYS * (int)sizeof(Contender);
__host__ __device__ constexpr int summary_bytes(int keys) {
    return (int)sizeof(RecHdr) + FIRST_BYTES + keys * (int)sizeof(Contender);
}
inline Recs scan_recs(unsigned char* base, int nscan) {
    Recs r;
    r.hdr = base;
    r.first = base + (size_t)nscan * sizeof(RecHdr);
    r.keys = r.first + (size_t)nscan * FIRST_BYTES;
    r.hdr_stride = (int)sizeof(RecHdr); r.first_stride = FIRST_BYTES; r.key_stride = TILE_KEYS * (int)sizeof(Contender);
    r.n = nscan; r.cap = TILE_KEYS;
    return r;
}
inline Recs summary_recs(unsigned char* base, int n, int keys) {
    Recs r;
    r.hdr = base;
    r.first = base + sizeof(RecHdr);
    r.keys = r.first + FIRST_BYTES;
    r.hdr_stride = r.first_stride = r.key_stride = summary_bytes(keys);
    r.n = n; r.cap = keys;
    return r;
}

// dynamic LDS of k_step (byte offsets): loads [B], error bounds / sort keys [NP2],
// universe order [NP2], allowed-set words of every set when resident [sbw], flags [B]
struct StepLds { int e, ord, sb, fl, total; };
__host__ __device__ inline StepLds step_lds(int B, int NP2, int sbw) {
    auto al = [](int x) { return (x + 15) & ~15; };
    StepLds L;
    int o = al(B * 8);
    L.e = o;   o += al(NP2 * 8);
    L.ord = o; o += al(NP2 * 4);
    L.sb = o;  o += al(sbw * 8);
    L.fl = o;  o += al(B);
    L.total = o;
    return L;
}
constexpr int STEP_SB_MAX = 65536;  // allowed-set words kept in k_step's LDS up to this size

struct ChangeDev {
    int32_t status, step, kind, slot;
    int64_t part;
    int32_t from, to;               // dense broker indices (-1 none)
    double su, cu;
    int32_t exact, err_code;
    int32_t err_broker, pad;
};

// step-mask bits (1 << kb_step, include/kbengine.h): kb_engine_step runs a subset of the
// reference's steps table (balancer.go:34-44)
enum : uint32_t {
    SM_VALIDATE_WEIGHTS = 1u << 0, SM_VALIDATE_REPLICAS = 1u << 1, SM_FILL_DEFAULTS = 1u << 2,
    SM_REMOVE = 1u << 3, SM_ADD = 1u << 4, SM_DISALLOWED = 1u << 5, SM_REASSIGN = 1u << 6,
    SM_MOVE_LEADERS = 1u << 7, SM_MOVE_NON_LEADERS = 1u << 8, SM_ALL = 0x1FFu
};

// halted codes
// (H_NEED_SPILL: the near-tie spill buffer overflowed with the census bound already
// at the step minimum; the host grows the buffer and the step runs again)
enum { H_RUN = 0, H_DONE = 1, H_NEED_EXACT = 2, H_NEED_SPILL = 3 };

struct DevCtl {
    int32_t halted, steps, logpos, logcap;
    int32_t prepped, budget, full_prep, want_refresh;
    int32_t nblm, heavy, light, ndirty;
    double S, avg, inv_avg, U0, eps, V, E;
    double ub[2];                   // upper bound of the next step's minimum score delta per kind
    uint32_t ncont, cont_overflow;  // raw near-tie spill buffer (scan -> step)
    int32_t list_overflow, pending_list;
    int32_t pl_kind, pl_from, pl_to, pl_pad;  // pending per-broker list operation
    long long pl_part;
    unsigned long long total_cand, total_cont, total_folds, total_exact_halts;
    unsigned long long total_retries;   // steps re-scanned with a tightened census bound (k_step)
    // kernel timing (tk_on): summed device-clock durations (100 MHz ticks) and launch
    // counts, {k_scan, k_step}; k_step folds in the scan's interval below
    unsigned long long tk_sum[2], tk_n[2];
    // ... and the rocprofv3-comparable spans: a launch runs from the end of the kernel before
    // it (its dispatch included) to its own end -- {k_scan: previous k_step end .. last scan
    // workgroup end, k_step: scan end .. k_step end}; only launches queued back to back
    // (first workgroup within 10 us of the previous end) are counted
    unsigned long long tk_span[2], tk_span_n[2];
    // k_pair: its first workgroup's start .. the step workgroup's end (the fused launch less
    // its dispatch), summed with its count
    unsigned long long tk_pair, tk_pair_n;
    // eager refold workgroups (tk_on): summed start .. end and start .. list edit done, count
    unsigned long long tk_eg, tk_eg_edit, tk_eg_n;
    int32_t tk_on;
    uint32_t step_mask;             // steps the next Balance() may take (bit = kb_step; SM_ALL)
    // incremental mode (kb_engine_set_incremental): incr_ok = the next scan
    // may skip every partition block whose largest weight is below wskip (a lower-bound
    // certificate, see k_step); cand_cache = the candidate counts of the last full scan,
    // which move() steps leave unchanged
    int32_t incr_ok;
    int32_t ub_sub;                 // > 0: the conditional bound pass may scan only the blocks of
                                    // the last records' best keys (StepArgs.ubdesc), not all
    uint32_t last_fm;               // first-index predicates the last resolved scan found (bit q:
    int32_t last_fm_pad;            //   F_q somewhere; kb_engine_step answers a masked first-index
                                    //   step whose predicate is absent without a launch)

    double wskip;
    unsigned long long cand_cache[2];
    unsigned long long total_blocks;    // partition blocks the incremental scans read
    double rlo, rhi;                    // range of r[] (every broker; k_step's prep): the scan's
                                        // lower-bound prune reads it instead of reducing r[]
    unsigned long long total_rf_stream; // exact refolds run in the stream (the next pair's first
                                        // scan refolds, its k_step resumes: no host round trip)
    // frozen-average prep (k_step's fused incremental prep): between full recomputes of the
    // load sum, avg / inv_avg stay fixed (the real sum is invariant under moves), so only the
    // touched brokers' r[] change and U0 / V / E / R follow incrementally; uerr bounds the
    // rounding those updates added to U0, frz_n counts the steps since the base (0: none)
    double uerr, rm_bound;          // rm_bound: max |r| over bl_move (an upper bound when frozen)
    int32_t frz_n, frz_pad;
    // eager refolds (ScanArgs.eager): the brokers whose contribution the last applied step
    // changed, refolded exactly (after their half of the pending list edit) by extra
    // workgroups of the next scan launch, so the next resolve finds every load exact
    int32_t eg_n, eg_pad;
    int32_t eg_b[8];
    // deferred prep (round 6): after a plain move() replace (frozen average, bl_move unchanged,
    // at most two touched brokers) the step workgroup writes only what the next scan cannot
    // derive -- r[] of the touched brokers, eps / ub, the records of the sets holding them --
    // and leaves the broker order, the bl positions and the full set-record rebuild to the next
    // launch's step workgroup, which does them before its wait (beside the scan).  The scan's
    // workgroups patch the bl positions (posm / blm hold the state before the move) with this
    // descriptor: fp = 1 pending; fp_t the touched brokers (-1 none); fp_o their bl positions
    // before the move (INT_MAX none); fp_n after; fp_u = fp_n - (touched brokers before it)
    int32_t fp, fp_pad;
    int32_t fp_t[2], fp_o[2], fp_n[2], fp_u[2];
    unsigned long long total_fp;    // steps that took the fast prep
    // kb_engine_plan_until: the plan ends after the first applied change whose partition is
    // not stop_part (-1: no such stop) -- run()'s -complete-partition loop (kafkabalancer.go:
    // 193-221: the probe change that does not compare is applied, then the loop ends)
    long long stop_part;
    // diagnostic phase stamps (builds with -DKB_STAMPS): accumulated
    // shader-clock ticks (clock64) per phase of k_step; [24]/[25] the wall-clock
    // (100 MHz) and shader-clock length of k_step; [26] one stamp's own cost
    unsigned long long stamps[32];
    // the running scan's interval: earliest workgroup start, latest end (atomics;
    // outside the block k_step copies to LDS and back)
    unsigned long long ts_beg, ts_end;
    unsigned long long ts_prev_end;     // the last k_step's end (100 MHz), for the spans
};

#ifdef KB_STAMPS
// Wave 0's timeline: thread 0 writes the shader clock of each stamp point to LDS
// (one s_memtime + one ds_write: no barrier, no read-modify-write, nothing live in
// registers, so the measured code keeps its synchronisation and, as far as the
// compiler allows, its register allocation).  At the end thread 0 orders the points
// by time and charges each one the interval since the previous point (or the start);
// a point hit twice in one launch keeps its last time.  [24] / [25]: the launch's
// wall-clock (100 MHz) / shader-clock length; [29] / [30]: the start times.
#define KB_STAMP_BEGIN()                                                        \
    __shared__ unsigned long long _kb_st[32];                                   \
    if (threadIdx.x < 29) _kb_st[threadIdx.x] = 0;                              \
    if (threadIdx.x == 0) { _kb_st[29] = clock64(); _kb_st[30] = wall_clock64(); } \
    KB_STAMP(ctl, 26)
// (the shader clock by inline asm: clock64() made the compiler wait vmcnt(0) before the
// stamp's LDS write, charging outstanding stores to the phase that issued them)
#define KB_STAMP(ctl, i)                                                        \
    do {                                                                        \
        if (threadIdx.x == 0) {                                                 \
            unsigned long long _t;                                              \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t));    \
            _kb_st[i] = _t;                                                     \
        }                                                                       \
    } while (0)
#define KB_STAMP_FLUSH(ctl)                                                     \
    do {                                                                        \
        __syncthreads();                                                        \
        if (threadIdx.x == 0) {                                                 \
            const unsigned long long _c = clock64(), _w = wall_clock64();       \
            unsigned long long _d[24];                                          \
            for (int _i = 0; _i < 24; _i++) {                                   \
                const unsigned long long _ti = _kb_st[_i];                      \
                unsigned long long _p = _kb_st[29];                             \
                for (int _j = 0; _j < 29; _j++)                                 \
                    if (_j != 24 && _j != 25 && _kb_st[_j] < _ti && _kb_st[_j] > _p) _p = _kb_st[_j]; \
                _d[_i] = _ti ? _ti - _p : 0;                                    \
            }                                                                   \
            for (int _i = 0; _i < 24; _i++) if (_d[_i]) atomicAdd(&(ctl)->stamps[_i], _d[_i]); \
            atomicAdd(&(ctl)->stamps[24], _w - _kb_st[30]);                     \
            atomicAdd(&(ctl)->stamps[25], _c - _kb_st[29]);                     \
        }                                                                       \
        __syncthreads();                                                        \
    } while (0)
#define KB_COUNT(ctl, i, v) atomicAdd(&(ctl)->stamps[i], (unsigned long long)(v))
#else
#define KB_STAMP_BEGIN() (void)0
#define KB_STAMP(ctl, i) (void)0
#define KB_STAMP_FLUSH(ctl) (void)0
#define KB_COUNT(ctl, i, v) (void)0
#endif

// errors recorded in ChangeDev.err_code
enum {
    E_NONE = 0, E_DUP = 1, E_REMOVE = 2, E_ADD = 3, E_DIS = 4, E_PANIC = 5,
    E_CONT_OVERFLOW = 6, E_LIST_OVERFLOW = 7,
    E_DUP_UNSUP = 8,    // kb_engine_step without ValidateReplicas on a state holding duplicates (Go sem)
    E_PAIR_TIMEOUT = 9  // k_pair's step workgroup waited 2 s for the scan's workgroups (never expected)
};

}  // namespace kbe
