// engine.cpp -- host half of the MI355X kafkabalancer engine: the C ABI declared
// in include/kbengine.h.  Marshals the reference's PartitionList
// (kafkabalancer.go:40-58) into the device SoA layout, performs the one-time
// ValidateWeights / ValidateReplicas / FillDefaults (steps.go:7-66), and drives
// the per-step kernels of kernels.hip (k_scan -> k_step per Balance() call).
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (host folds must
// round exactly like Go on amd64: no FMA contraction).
#ifdef KB_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>   // host ranges per plan phase (rocprofv3 --marker-trace)
#else
// production build: no profiler dependency (make roctx builds the instrumented library)
#define roctxMark(msg) ((void)0)
#define roctxRangePush(msg) ((void)0)
#define roctxRangePop() ((void)0)
#endif
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>          // (types only: the symbols are resolved at run time, rccl_api)
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/kbengine.h"
#include "engine_dev.h"

#include "kernels_api.h"

using namespace kbe;

#define HIPCHK(x)                                                                  \
    do {                                                                           \
        hipError_t _e = (x);                                                       \
        if (_e != hipSuccess) {                                                    \
            e->last_err = std::string("HIP error: ") + hipGetErrorString(_e) +     \
                          " at " #x;                                               \
            return KB_ERR_HIP;                                                     \
        }                                                                          \
    } while (0)

static const char* kStepNames[9] = {
    "ValidateWeights", "ValidateReplicas", "FillDefaults", "RemoveExtraReplicas",
    "AddMissingReplicas", "MoveDisallowedReplicas", "ReassignLeaders",
    "MoveLeaders", "MoveNonLeaders"};

enum { TK_STEP = 0, TK_SCAN = 1, TK_REFRESH = 2, TK_BOUND = 3, TK_N = 4 };

// Diagnostic / A-B switches (KB_FUSE, KB_EAGER, KB_PAIR_WAIT_TICKS, ... -- INTEGRATION.md lists
// them) are read from the environment only after kb_set_diagnostics(1): a drop-in host never
// calls it, so an inherited environment cannot change the product library's kernel paths.
// The test suite and the bench scripts opt in (kafkabalancer_amd/engine.py, KB_DIAGNOSTICS=1).
static int g_diag = 0;
static const char* diag_getenv(const char* name) { return g_diag ? getenv(name) : nullptr; }
extern "C" void kb_set_diagnostics(int on) { g_diag = on ? 1 : 0; }
extern "C" int kb_diagnostics_enabled(void) { return g_diag; }

struct kb_engine {
    int dev = 0;
    hipStream_t st = nullptr;
    bool own_st = false;
    int64_t P = 0, Ppad = 0, B = 0, nsets = 0, ntiles = 0, nscan = 0;
    int twaves = SCAN_THREADS / 64;
    int rcap = 0, rc_dev = 1, K = 3, KR = 6, units = 1, W64 = 1, NP2 = 64;
    int sb_lds = 0, step_lds_bytes = 0;     // k_step: resident allowed-set words, dynamic LDS
    int sem = KB_SEM_APPLIED, allow_leader = 0, rebalance = 0;
    int64_t minrep = 2;
    double min_unb = 0.01;
    int64_t shard_begin = 0, shard_end = 0;
    bool integral = false;
    bool lds_sets = true;
    size_t scan_lds = 0;
    double wmax = 0;
    std::vector<int64_t> ids;
    std::vector<std::string> topics;
    std::vector<int64_t> pids;
    int pending = 0;                  // pending validation error (reported by every step)
    std::string pending_msg;
    int pending_step = 0;
    // device state
    double* w = nullptr;
    uint16_t* rep = nullptr;
    uint32_t* meta = nullptr;
    uint32_t* pset = nullptr;         // [Ppad] allowed-set index per partition (set records not in LDS)
    int32_t* nc = nullptr;
    double* load = nullptr;
    double* lerr = nullptr;
    double* eb = nullptr;
    uint8_t* bfl = nullptr;
    int32_t* cnt = nullptr;
    uint64_t* setbits = nullptr;
    uint4* setrec = nullptr;
    int32_t* order = nullptr;
    int32_t* posu = nullptr;
    int32_t* blm = nullptr;
    int32_t* posm = nullptr;
    double* r = nullptr;
    int32_t* bset_off = nullptr;
    int32_t* bset_ids = nullptr;
    unsigned char* gscr = nullptr;    // k_step's per-broker tables past MAXB brokers (StepArgs.gscr)
    uint32_t* pair_cnt = nullptr;     // k_pair's arrival count (ScanArgs.done / StepArgs.wait_cnt)
    bool fuse = false;                // pairs run as one k_pair launch (scan grid + step workgroup)
    bool fuse_sum = false;            // sharded scans: scan + rank summary as one k_scansum launch
    // resident workgroup slots of the scan / k_pair / k_scansum grids (blocks per CU x CUs),
    // kept for the switch to eager refolds, whose extra workgroups must fit beside them
    int64_t slots_scan = 0, slots_pair = 0, slots_sum = 0;
    bool eager_auto = false;          // lazy loads now; eager refolds once exact halts are frequent
    int64_t eager_switches = 0;
    int fp_lds = 0;                 // deferred prep: byte offset of its region in k_step's LDS (0: none)
    int64_t stop_part = -1;         // kb_engine_plan_until's partition for the plan running now
    int fp_bk = 0;                  // ... which also holds the records' best keys
    // the halt rate's window: the steps and exact halts at the checkpoint before last (w0)
    // and at the last one (w1), checkpoints at least 64 steps apart
    unsigned long long w0_steps = 0, w0_halts = 0, w1_steps = 0, w1_halts = 0;
    int fuse_pre = 1;                 // k_pair stages the tables before its wait (KB_FUSE_PRE=0: after)
    size_t pair_lds = 0;              // k_pair's dynamic LDS: max(scan, step)
    bool gb = false;                  // B > MAXB: broker tables in memory (k_scan GT, k_step GB)
    unsigned char* recs = nullptr;
    Contender* cont = nullptr;
    uint32_t cont_cap = 1u << 20;
    int64_t spill_grows = 0;           // spill buffer growths (grow_spill)
    Lists L{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    DevCtl* ctl = nullptr;
    ChangeDev* log = nullptr;
    int logcap = 0;
    DevCtl* h_ctl = nullptr;          // pinned
    bool ctl_mirror = false;          // h_ctl == the device block and the stream is idle
                                      // (set by run_steps; every other path clears it)
    ChangeDev* h_log = nullptr;       // pinned copy of the device step log (run_steps)
    int h_logcap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0;
    int64_t scan_bytes = 0;
    int exact_unb = 0;
    // per-kernel timing (cfg->time_kernels): one event per launch boundary
    int time_kernels = 0;
    std::vector<hipEvent_t> tev;
    std::vector<int> tkind;           // kernel kind between tev[i] and tev[i+1]
    int tev_used = 0;
    double kms[TK_N] = {0, 0, 0, 0};
    int64_t klaunch[TK_N] = {0, 0, 0, 0};
    int64_t refreshes = 0;
    bool rf_stream = false;        // in-stream refreshes (ScanArgs.rfpass / StepArgs.rf_final)
    bool eager = false;            // eager refolds of the touched brokers (ScanArgs.eager)
    RefreshArgs* rf_dev = nullptr; // the refresh's arguments in device memory (ScanArgs.rf)
    int dbg_scan = 0;
    unsigned long long* wgt = nullptr;     // diagnostic (KB_WGT=path): scan workgroup timeline
    std::string wgt_path;
    int incr = 0;                  // incremental mode (kb_engine_set_incremental)
    BlockDesc* bdesc = nullptr;    // partition blocks of the shard by wmax descending
    BlockDesc* ubdesc = nullptr;   // the bound pass's blocks (last best keys + heaviest)
    int64_t nubdesc = 0;
    int64_t nblk = 0;
    int batch = 64;                // (scan, step) pairs per enqueued batch (adaptive, run_steps)
    int sum_keys = SUMMARY_KEYS;   // near-tie keys per rank summary (grown on overflow)
    bool ub_mode = false;          // a step re-scanned: enqueue the conditional bound pass per scan
    bool ub_sticky = true;         // (diagnostic KB_UB_STICKY=0: a retry does not turn ub_mode on)
    uint32_t list_slack = 1024;        // free entries per broker list (doubled on every re-layout)
    int64_t relists = 0;
    const void* gath = nullptr;        // the last gathered rank summaries (device) and their count
    int gath_n = 0;                    //   (grow_summary reads their shared flags)
    uint32_t step_mask = SM_ALL;       // steps the running Balance() may take (kb_engine_step)
    bool recs_fresh = false;           // the scan records describe the current state (a masked
                                       //   step changed nothing): the next masked step reuses them
    bool reuse_now = false;            //   (the run about to start takes them)
    // control-block / step-log transfers (run_steps, reset_ctl): 0 = hipMemcpyAsync, 1 = k_xfer
    // (one-workgroup kernel to / from the pinned mirror, then a stream synchronisation),
    // 2 = k_xfer whose system-scope flag the host polls (KB_XFER, diagnostic A/B)
    int xfer = 2;
    DevCtl* h_ctl_d = nullptr;         // device addresses of the mapped pinned mirror
    ChangeDev* h_log_d = nullptr;
    uint32_t* h_flag = nullptr;        // k_xfer's sequence word (pinned, fine-grained)
    uint32_t* h_flag_d = nullptr;
    uint32_t xseq = 0;
    // host phases of the plan calls (us): reset_ctl, enqueue, wait for the batch, the rest of
    // kb_engine_plan (log conversion); [4] calls (kb_engine_host_timings, diagnostic)
    double host_us[5] = {0, 0, 0, 0, 0};
    // a k_pair step workgroup timed out waiting for its grid (never expected): the engine
    // refuses further work (its arrival count was reset, but a plan may have been cut short)
    bool dead = false;
    // the RCCL communicator of kb_engine_sharded_plan (kb_engine_comm_init) and its
    // exchange buffer: the gathered summaries of every rank, this rank's summary written in
    // place into its own slot (an in-place ncclAllGather)
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    unsigned char* sum_buf = nullptr;
    unsigned char* gath_buf = nullptr;
    int64_t xbuf_bytes = 0;            // summary bytes the buffers were sized for
    unsigned long long pair_wait_ticks = 200000000ull;   // k_pair's wait bound: 2 s of the 100 MHz clock
    std::string last_err;
};

// ------------------------------------------------------------ helpers

static double now_us() {
    return 1e-3 * (double)std::chrono::duration_cast<std::chrono::nanoseconds>(
                      std::chrono::steady_clock::now().time_since_epoch()).count();
}

// a fused launch's waiting workgroup (k_pair's step, k_scansum's summary) gave up on its grid:
// the stragglers still counted themselves in, so the arrival count is reset once the
// stream is idle, and the engine takes no more work
static int poison_after_timeout(kb_engine* e) {
    HIPCHK(hipStreamSynchronize(e->st));
    HIPCHK(hipMemsetAsync(e->pair_cnt, 0, PAIR_SHARDS * PAIR_STRIDE * 4, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    e->dead = true;
    return KB_OK;
}

// after a fused launch's timeout every step entry point refuses with this
static int dead_result(kb_engine* e) {
    e->last_err = "engine unusable: an earlier fused launch (scan + step or scan + summary) timed out waiting for its grid";
    return KB_ERR_HIP;
}

static std::string part_string(kb_engine* e, int64_t p, const std::vector<int64_t>& reps) {
    std::string t = p < (int64_t)e->topics.size() ? e->topics[p] : std::string();
    long long pid = p < (int64_t)e->pids.size() ? (long long)e->pids[p] : (long long)p;
    std::string s = "Partition(" + t + "," + std::to_string(pid) + ",[";
    for (size_t i = 0; i < reps.size(); i++) {
        if (i) s += " ";
        s += std::to_string((long long)reps[i]);
    }
    return s + "])";
}

static int64_t read_replicas(kb_engine* e, int64_t p, std::vector<int64_t>& out) {
    out.clear();
    uint32_t m = 0;
    if (hipMemcpy(&m, e->meta + p, 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    int n = (int)meta_nrep(m);
    for (int k = 0; k < n; k++) {
        uint16_t v = 0;
        if (hipMemcpy(&v, e->rep + (int64_t)k * e->Ppad + p, 2, hipMemcpyDeviceToHost) != hipSuccess) return -1;
        out.push_back(e->ids[v]);
    }
    return n;
}

template <typename T>
static hipError_t dalloc(T** p, size_t n) {
    return hipMalloc((void**)p, (n ? n : 1) * sizeof(T));
}

static int upload_rf(kb_engine* e);   // (step launch section)

static const int kRcChoices[] = {1, 2, 3, 4, 6, 8, 12, 16};

// ------------------------------------------------------------- RCCL (run-time bound)

// The sharded plan's all-gather goes through RCCL over xGMI.  The library is bound at run
// time (dlopen), not at link time: the engine (and the C++ CLI, which never shards) loads
// without it, and in a process that already holds an RCCL -- torch's -- the same copy is
// reused (RTLD_NOLOAD on its soname) rather than a second one loaded beside it.
struct RcclApi {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    std::string err;
};

static RcclApi& rccl_api() {
    static RcclApi api = [] {
        RcclApi a;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) { const char* d = dlerror(); a.err = std::string("RCCL not loadable: ") + (d ? d : "librccl.so.1"); return a; }
        a.get_unique_id = (decltype(a.get_unique_id))dlsym(h, "ncclGetUniqueId");
        a.comm_init_rank = (decltype(a.comm_init_rank))dlsym(h, "ncclCommInitRank");
        a.all_gather = (decltype(a.all_gather))dlsym(h, "ncclAllGather");
        a.comm_destroy = (decltype(a.comm_destroy))dlsym(h, "ncclCommDestroy");
        a.error_string = (decltype(a.error_string))dlsym(h, "ncclGetErrorString");
        if (!a.get_unique_id || !a.comm_init_rank || !a.all_gather || !a.comm_destroy || !a.error_string) {
            a.err = "RCCL: a required symbol is missing";
            a.get_unique_id = nullptr;
        }
        return a;
    }();
    return api;
}

// ------------------------------------------------------------- create

extern "C" int kb_abi_version(void) { return KB_ABI_VERSION; }

extern "C" int kb_engine_create(const kb_cluster* c, const kb_config* cfg, kb_engine** out) {
    if (!c || !cfg || !out) return KB_ERR_INVALID;
    *out = nullptr;
    kb_engine* e = new kb_engine();
    const int64_t n = c->n_partitions;
    if (n < 0 || (n > 0 && (!c->replica_off || !c->weight))) { delete e; return KB_ERR_INVALID; }
    e->P = n;
    e->sem = cfg->semantics == KB_SEM_GO ? KB_SEM_GO : KB_SEM_APPLIED;
    e->allow_leader = cfg->allow_leader ? 1 : 0;
    e->rebalance = cfg->rebalance_leaders ? 1 : 0;
    e->minrep = cfg->min_replicas;
    e->min_unb = cfg->min_unbalance;
    e->dev = cfg->device;
    e->exact_unb = cfg->exact_unbalance ? 1 : 0;
    e->time_kernels = cfg->time_kernels ? 1 : 0;
    if (c->topic_blob && c->topic_off) {
        e->topics.resize(n);
        for (int64_t i = 0; i < n; i++)
            e->topics[i].assign(c->topic_blob + c->topic_off[i], (size_t)(c->topic_off[i + 1] - c->topic_off[i]));
    }
    if (c->partition_id) e->pids.assign(c->partition_id, c->partition_id + n);

    // dense broker universe = sorted unique ids (so dense order == BrokerID order).
    // An open-addressing id table (at most MAXB_G distinct ids, else unsupported) instead of
    // sorting every replica id: one hash probe per replica (c3: 3M) and a sort of the
    // few distinct ids.
    int64_t nrep_total = n ? c->replica_off[n] - c->replica_off[0] : 0;
    constexpr uint32_t HCAP = 1u << 16;                  // > 2 * MAXB_G: short probe chains
    std::vector<int64_t> hkey(HCAP);
    std::vector<int32_t> hval(HCAP, -1);
    std::vector<int64_t> all;
    all.reserve(MAXB_G + 1);
    auto hslot = [&](int64_t id) -> uint32_t {
        uint64_t x = (uint64_t)id * 0x9E3779B97F4A7C15ull;
        uint32_t h = (uint32_t)(x >> 48);                // top 16 bits
        while (hval[h] >= 0 && hkey[h] != id) h = (h + 1) & (HCAP - 1);
        return h;
    };
    auto add_id = [&](int64_t id) {
        const uint32_t h = hslot(id);
        if (hval[h] < 0 && (int64_t)all.size() <= MAXB_G) { hkey[h] = id; hval[h] = 0; all.push_back(id); }
    };
    for (int64_t i = 0; i < nrep_total && (int64_t)all.size() <= MAXB_G; i++) add_id(c->replica_ids[c->replica_off[0] + i]);
    if (c->n_sets > 0 && c->set_off)
        for (int64_t i = c->set_off[0]; i < c->set_off[c->n_sets] && (int64_t)all.size() <= MAXB_G; i++) add_id(c->set_ids[i]);
    if (!cfg->brokers_nil)
        for (int64_t i = 0; i < cfg->n_brokers && (int64_t)all.size() <= MAXB_G; i++) add_id(cfg->brokers[i]);
    if ((int64_t)all.size() > MAXB_G) {
        e->last_err = "engine supports at most 16384 distinct brokers";
        *out = e;
        return KB_ERR_UNSUPPORTED;
    }
    std::sort(all.begin(), all.end());
    for (size_t i = 0; i < all.size(); i++) hval[hslot(all[i])] = (int)i;
    e->ids = all;
    e->B = (int64_t)all.size();
    auto dense_of = [&](int64_t id) -> int { return hval[hslot(id)]; };
    // replicas as dense ids, per partition (one lookup per replica, reused below)
    std::vector<uint16_t> dense((size_t)nrep_total);
    for (int64_t i = 0; i < nrep_total; i++) dense[i] = (uint16_t)dense_of(c->replica_ids[c->replica_off[0] + i]);
    auto dn = [&](int64_t i, int k) -> int { return dense[c->replica_off[i] - c->replica_off[0] + k]; };

    std::vector<int> len(n);
    std::vector<double> wt(c->weight, c->weight + n);
    std::vector<int64_t> want(n), ncon(n, 0);
    for (int64_t i = 0; i < n; i++) {
        len[i] = (int)(c->replica_off[i + 1] - c->replica_off[i]);
        want[i] = c->num_replicas ? c->num_replicas[i] : 0;
        if (c->num_consumers) ncon[i] = c->num_consumers[i];
    }
    auto rid = [&](int64_t i, int k) { return c->replica_ids[c->replica_off[i] + k]; };

    // ValidateWeights (steps.go:7-23) / ValidateReplicas (steps.go:27-36)
    auto reps_of = [&](int64_t i) {
        std::vector<int64_t> r;
        for (int k = 0; k < len[i]; k++) r.push_back(rid(i, k));
        return r;
    };
    if (n == 0) {
        e->pending = KB_ERR_PANIC; e->pending_step = 0;
        e->pending_msg = "ValidateWeights: panic: index out of range [0] with length 0";
    } else {
        bool has = wt[0] != 0;
        for (int64_t i = 0; i < n && !e->pending; i++) {
            if (has && wt[i] == 0) {
                e->pending = KB_ERR_STEP; e->pending_step = 0;
                e->pending_msg = std::string("ValidateWeights: partition ") + part_string(e, i, reps_of(i)) + " has no weight";
            } else if (!has && wt[i] != 0) {
                e->pending = KB_ERR_STEP; e->pending_step = 0;
                e->pending_msg = std::string("ValidateWeights: partition ") + part_string(e, 0, reps_of(0)) + " has no weight";
            } else if (wt[i] < 0) {
                e->pending = KB_ERR_STEP; e->pending_step = 0;
                e->pending_msg = std::string("ValidateWeights: partition ") + part_string(e, i, reps_of(i)) + " has negative weight";
            }
        }
        // (duplicates by dense id: the id map is a bijection; one epoch mark per broker, the
        // partition index, so a partition costs O(len) like toBrokerSet's map)
        std::vector<int64_t> seen_in(e->B ? e->B : 1, -1);
        for (int64_t i = 0; i < n && !e->pending; i++) {
            bool dup = false;
            for (int k = 0; k < len[i] && !dup; k++) {
                const int b = dn(i, k);
                dup = seen_in[b] == i;
                seen_in[b] = i;
            }
            if (dup) {
                e->pending = KB_ERR_STEP; e->pending_step = 1;
                e->pending_msg = std::string("ValidateReplicas: partition ") + part_string(e, i, reps_of(i)) + " has duplicated replicas";
            }
        }
    }
    // FillDefaults (steps.go:39-66)
    if (!e->pending) {
        if (wt[0] == 0) for (int64_t i = 0; i < n; i++) wt[i] = 1.0;
        for (int64_t i = 0; i < n; i++) if (want[i] == 0) want[i] = len[i];
    }
    // allowed-broker sets: the caller's lists + the default list for nil Brokers
    int64_t nsets_in = c->n_sets > 0 ? c->n_sets : 0;
    bool need_default = false;
    for (int64_t i = 0; i < n; i++) if (!c->set_idx || c->set_idx[i] < 0) need_default = true;
    std::vector<std::vector<int>> sets((size_t)nsets_in + (need_default ? 1 : 0));
    for (int64_t s = 0; s < nsets_in; s++)
        for (int64_t k = c->set_off[s]; k < c->set_off[s + 1]; k++) sets[s].push_back(dense_of(c->set_ids[k]));
    int64_t def_set = -1;
    if (need_default) {
        def_set = nsets_in;
        if (!cfg->brokers_nil) {
            for (int64_t k = 0; k < cfg->n_brokers; k++) sets[def_set].push_back(dense_of(cfg->brokers[k]));
        } else {
            // getBrokerList (utils.go:49-64): every broker holding a replica
            std::vector<char> seen(e->B, 0);
            for (int64_t i = 0; i < nrep_total; i++) seen[dense[i]] = 1;
            for (int64_t b = 0; b < e->B; b++) if (seen[b]) sets[def_set].push_back((int)b);
        }
    }
    e->nsets = (int64_t)sets.size();
    if (e->nsets == 0) { sets.emplace_back(); e->nsets = 1; }
    if (e->nsets > (1ll << 30)) {
        e->last_err = "engine supports at most 2^30 distinct broker lists";
        *out = e;
        return KB_ERR_UNSUPPORTED;
    }
    std::vector<int64_t> pset(n);
    for (int64_t i = 0; i < n; i++) pset[i] = (c->set_idx && c->set_idx[i] >= 0) ? c->set_idx[i] : def_set;

    // replica slots needed on the device
    int rcap = 1;
    for (int64_t i = 0; i < n; i++) {
        int64_t need = len[i];
        if (e->sem == KB_SEM_APPLIED && want[i] > len[i]) {
            int64_t grow = std::min<int64_t>(want[i], len[i] + (int64_t)sets[pset[i]].size());
            need = std::max<int64_t>(need, grow);
        }
        rcap = (int)std::max<int64_t>(rcap, need);
    }
    if (rcap > MAXR) {
        e->last_err = "engine supports at most 16 replicas per partition";
        *out = e;
        return KB_ERR_UNSUPPORTED;
    }
    e->rcap = rcap;
    for (int v : kRcChoices) if (v >= rcap) { e->rc_dev = v; break; }
    e->K = e->rc_dev + 2;
    e->units = sr_units(e->rc_dev);
    e->KR = sr_kr(e->rc_dev);
    e->W64 = (int)((e->B + 63) / 64);
    if (e->W64 < 1) e->W64 = 1;
    e->NP2 = 64;
    while (e->NP2 < e->B) e->NP2 <<= 1;

    // num_consumers must keep loads non-negative (sort on IEEE bits)
    for (int64_t i = 0; i < n; i++) {
        if (ncon[i] < 0 || ncon[i] > (1 << 30)) {
            e->last_err = "num_consumers outside [0, 2^30] is not supported";
            *out = e;
            return KB_ERR_UNSUPPORTED;
        }
        if (!(std::isfinite(wt[i]))) {
            e->last_err = "non-finite weight";
            *out = e;
            return KB_ERR_UNSUPPORTED;
        }
        e->wmax = std::max(e->wmax, wt[i]);
    }

    // exact initial loads: getBrokerLoad fold in partition order (utils.go:92-105)
    std::vector<double> ld(e->B, 0.0);
    std::vector<int32_t> cn(e->B, 0);
    for (int64_t i = 0; i < n; i++) {
        for (int k = 0; k < len[i]; k++) {
            const int b = dn(i, k);
            if (k == 0) ld[b] += wt[i] * (double)(len[i] + ncon[i]);
            else ld[b] += wt[i];
            cn[b]++;
        }
    }
    for (double v : ld) if (!std::isfinite(v)) {
        e->last_err = "non-finite broker load";
        *out = e;
        return KB_ERR_UNSUPPORTED;
    }
    // integral mode: all contributions are integers and every partial sum < 2^53,
    // so incremental +/- updates equal the reference's fold exactly
    {
        bool integ = true;
        long double tot = 0;
        for (int64_t i = 0; i < n && integ; i++) {
            if (wt[i] != std::floor(wt[i])) integ = false;
            tot += (long double)wt[i] * (long double)(2 * e->rc_dev + ncon[i] + 1);
        }
        e->integral = integ && tot < 4503599627370496.0L;  // 2^52
    }
    // error bounds of the exact folds against the real sums (non-integral mode)
    std::vector<double> le(e->B, 0.0);
    if (!e->integral)
        for (int64_t b = 0; b < e->B; b++)
            le[b] = 1.01 * (double)std::max(cn[b], 1) * (DBL_EPSILON / 2) * ld[b];

    // shard
    e->shard_begin = cfg->shard_begin;
    e->shard_end = (cfg->shard_begin == 0 && cfg->shard_end == 0) ? n : cfg->shard_end;
    if (e->shard_begin < 0 || e->shard_end > n || e->shard_begin > e->shard_end ||
        ((e->shard_begin % SHARD_ALIGN) != 0 && e->shard_begin != e->shard_end)) {
        e->last_err = "shard_begin must be a multiple of 1024 and 0 <= begin <= end <= n";
        delete e;
        return KB_ERR_INVALID;
    }
    // padding: the last tile of the shard may read up to TILE past shard_end
    e->Ppad = ((n + TILE - 1) / TILE) * TILE + 2 * TILE;

    // host SoA images
    std::vector<double> hw(e->Ppad, 0.0);
    std::vector<uint32_t> hm(e->Ppad, 0u);
    std::vector<uint16_t> hr((size_t)e->rc_dev * e->Ppad, 0);
    std::vector<int32_t> hnc(e->Ppad, 0);
    for (int64_t i = 0; i < n; i++) {
        hw[i] = wt[i];
        for (int k = 0; k < len[i]; k++) hr[(size_t)k * e->Ppad + i] = dense[c->replica_off[i] - c->replica_off[0] + k];
        hnc[i] = (int32_t)ncon[i];
    }
    // incremental mode: the shard's 128-partition blocks, heaviest largest weight first
    std::vector<BlockDesc> hbd;
    for (int64_t b0 = e->shard_begin; b0 < e->shard_end; b0 += BLK) {
        BlockDesc d;
        d.blk = b0 / BLK;
        d.wmax = 0.0;
        for (int64_t i = b0; i < std::min<int64_t>(b0 + BLK, e->shard_end); i++) d.wmax = std::max(d.wmax, wt[i]);
        hbd.push_back(d);
    }
    std::stable_sort(hbd.begin(), hbd.end(), [](const BlockDesc& x, const BlockDesc& y) { return x.wmax > y.wmax; });
    e->nblk = (int64_t)hbd.size();
    std::vector<uint64_t> hsb((size_t)e->nsets * e->W64, 0);
    for (int64_t s = 0; s < e->nsets; s++)
        for (int b : sets[s]) hsb[(size_t)s * e->W64 + (b >> 6)] |= 1ull << (b & 63);
    for (int64_t i = 0; i < n; i++) {
        // Disallowed trigger (a replica outside the allowed set) and the in-set count
        uint32_t dis = 0, nin = 0;
        const uint64_t* sb = &hsb[(size_t)pset[i] * e->W64];
        for (int k = 0; k < len[i]; k++) {
            const int b = dense[c->replica_off[i] - c->replica_off[0] + k];
            const bool in = (sb[b >> 6] >> (b & 63)) & 1ull;
            dis |= in ? 0u : 1u;
            nin += in ? 1u : 0u;
        }
        const uint32_t elig = want[i] >= e->minrep ? 1u : 0u;
        const uint32_t wnt = want[i] < 0 ? 0u : (uint32_t)std::min<int64_t>(want[i], 31);
        // (the meta word's 15-bit set field serves the LDS-resident set records, at most
        // 4096 sets; with more, the scan and the step read the index array pset)
        hm[i] = make_meta((uint32_t)len[i], wnt, elig, dis, nin, (uint32_t)pset[i] & (MAX_SETS - 1));
    }
    std::vector<uint8_t> hin(e->B, 0);
    if (!cfg->brokers_nil)
        for (int64_t k = 0; k < cfg->n_brokers; k++) hin[dense_of(cfg->brokers[k])] = 1;
    // broker -> sets containing it (incremental set-record upkeep)
    std::vector<int32_t> hbo(e->B + 1, 0), hbi;
    {
        std::vector<std::vector<int32_t>> bs(e->B);
        for (int64_t s = 0; s < e->nsets; s++) {
            std::vector<int> u = sets[s];
            std::sort(u.begin(), u.end());
            u.erase(std::unique(u.begin(), u.end()), u.end());
            for (int b : u) bs[b].push_back((int32_t)s);
        }
        for (int64_t b = 0; b < e->B; b++) hbo[b + 1] = hbo[b] + (int32_t)bs[b].size();
        hbi.reserve(hbo[e->B]);
        for (int64_t b = 0; b < e->B; b++) hbi.insert(hbi.end(), bs[b].begin(), bs[b].end());
    }

    // per-broker partition lists (non-integral mode), sorted by partition index
    std::vector<uint32_t> hls, hll, hlc, hle;
    if (!e->integral) {
        uint32_t slack = cfg->list_slack > 0 ? (uint32_t)cfg->list_slack : 1024u;
        e->list_slack = slack;
        hls.resize(e->B); hll.resize(e->B); hlc.resize(e->B);
        uint64_t off = 0;
        for (int64_t b = 0; b < e->B; b++) {
            hls[b] = (uint32_t)off; hll[b] = 0; hlc[b] = (uint32_t)cn[b] + slack;
            off += hlc[b];
        }
        if (off >= (1ull << 32)) {
            e->last_err = "broker lists exceed 2^32 entries";
            *out = e;
            return KB_ERR_UNSUPPORTED;
        }
        hle.resize(off ? off : 1, 0);
        for (int64_t i = 0; i < n; i++)
            for (int k = 0; k < len[i]; k++) {
                int b = dense[c->replica_off[i] - c->replica_off[0] + k];
                hle[hls[b] + hll[b]++] = (uint32_t)i;
            }
    }

    // device
    if (hipSetDevice(e->dev) != hipSuccess) { e->last_err = "hipSetDevice failed (no GPU?)"; *out = e; return KB_ERR_HIP; }
    int ncu = 256;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, e->dev);
    if (ncu <= 0) ncu = 256;
    const size_t rbytes = (size_t)e->B * 16;          // (r, f(r)) pairs
    const size_t setbytes = (size_t)e->nsets * e->units * 16;
    const size_t dedup = (size_t)DEDUP_SCAN * (4 + 8 + 8);
    // past MAXB brokers the scan reads the broker tables (and the set records) from memory
    // (L2-resident) and k_step keeps its per-broker tables in a memory scratch
    e->gb = e->B > MAXB;
    e->lds_sets = !e->gb && setbytes <= (size_t)LDS_SETS_MAX;
    const size_t pbytes = ((size_t)e->B * 2 + 15) & ~(size_t)15;
    e->scan_lds = (e->gb ? 0 : rbytes + 2 * pbytes) + (e->lds_sets ? setbytes : 0) + dedup;
    // (room for the in-stream refresh's two fold buffers: ScanArgs.rfpass)
    e->rf_stream = !e->integral;
    if (const char* v = diag_getenv("KB_RF_STREAM")) if (*v == '0') e->rf_stream = false;   // diagnostic
    if (e->rf_stream) e->scan_lds = std::max(e->scan_lds, (size_t)RF_LDS_BYTES);
    // one wave of resident workgroups; each loops over its tiles
    int per_cu = scan_blocks_per_cu(e->rc_dev, e->lds_sets, e->gb, e->scan_lds);
    if (per_cu < 1) per_cu = 1;
    // a tile is twaves blocks of BLK partitions, one per scoring wave: the full 16 when the
    // shard fills every resident workgroup slot with whole tiles, fewer on small shards
    // (c2's 10k partitions: 79 workgroups of one scoring wave instead of 5 of 16 -- the
    // census walks of an all-ties cluster spread over 79 CUs)
    {
        const int64_t nblk = (e->shard_end - e->shard_begin + BLK - 1) / BLK;
        const int64_t slots = (int64_t)per_cu * ncu;
        e->twaves = (int)std::max<int64_t>(1, std::min<int64_t>(SCAN_THREADS / 64, nblk / std::max<int64_t>(slots, 1)));
        if (const char* v = diag_getenv("KB_TWAVES")) if (atoi(v) > 0) e->twaves = std::min(atoi(v), SCAN_THREADS / 64);  // diagnostic
        e->ntiles = (nblk + e->twaves - 1) / e->twaves;
    }
    // eager refolds (thousands of brokers, non-integral loads: the decisions there need exact
    // folds often, and each then waited for a refresh of the approximate loads): EGW extra
    // workgroups per scan launch, kept co-resident with the scan's (and its list workgroup)
    e->eager = e->rf_stream && e->B >= 2048;
    // (fewer brokers: lazy loads, refreshed when a decision needs them exact; a plan whose
    // decisions keep needing them switches to eager refolds, switch_to_eager)
    e->eager_auto = e->rf_stream && !e->eager && !e->gb;
    if (const char* v = diag_getenv("KB_EAGER")) { e->eager = e->rf_stream && *v == '1'; e->eager_auto = false; }  // diagnostic
    if (const char* v = diag_getenv("KB_EAGER_AUTO")) e->eager_auto = e->eager_auto && *v != '0';               // A/B
    e->slots_scan = (int64_t)per_cu * ncu;
    e->nscan = std::min<int64_t>(e->ntiles, std::max<int64_t>(1, (int64_t)per_cu * ncu - (e->eager ? EGW + 1 : 0)));
    if (const char* v = diag_getenv("KB_NSCAN")) if (atoi(v) > 0) e->nscan = std::min<int64_t>(e->ntiles, atoi(v));  // diagnostic
    e->nscan = std::min<int64_t>(e->nscan, SUM_RECS);     // (a rank summary reads one record per thread)
    if (const char* v = diag_getenv("KB_DEBUG_SCAN")) e->dbg_scan = atoi(v);                                   // diagnostic
    {
        // k_step's LDS: static tables + per-broker arrays (+ every set's words when they fit)
        const int st_lds = step_static_lds(e->gb);
        if (st_lds < 0) { e->last_err = "k_step attributes unavailable"; *out = e; return KB_ERR_HIP; }
        const int lim = 160 * 1024;
        const int sbw = (int)e->nsets * e->W64;
        e->sb_lds = (!e->gb && sbw * 8 <= STEP_SB_MAX && st_lds + step_lds((int)e->B, e->NP2, sbw).total <= lim) ? 1 : 0;
        if (const char* v = diag_getenv("KB_STEP_SB")) if (*v == '0') e->sb_lds = 0;                           // diagnostic
        e->step_lds_bytes = e->gb ? 0 : step_lds((int)e->B, e->NP2, e->sb_lds ? sbw : 0).total;
        // the deferred prep's region (bl positions, one 16-B record per set; DESIGN.md "Deferred
        // prep"): set words resident, one-unit records, at most 1024 sets (its set list lives in
        // the step's mark words)
        e->fp_lds = 0;
        e->fp_bk = 0;
        const int fpb = (((int)e->B * 4 + 15) & ~15) + (int)e->nsets * 16 * e->units;
        const int fpk = (int)std::min<int64_t>(e->nscan, STEP_THREADS) * 2 * (int)sizeof(Contender);
        bool fp = !e->gb && e->sb_lds && e->units <= FP_MAXU && e->nsets <= 1024 &&
                  st_lds + e->step_lds_bytes + fpb <= lim;
        if (const char* v = diag_getenv("KB_FP")) fp = fp && *v != '0';                           // A/B
        if (fp) {
            e->fp_lds = e->step_lds_bytes;
            e->step_lds_bytes += fpb;
            // (the records' best keys too, for the fast prep's upper bound: it then defers only
            // with at most STEP_THREADS records)
            if (e->nscan <= STEP_THREADS && st_lds + e->step_lds_bytes + fpk <= lim) { e->fp_bk = 1; e->step_lds_bytes += fpk; }
        }
        if (st_lds + e->step_lds_bytes > lim) { e->last_err = "too many brokers for k_step's LDS"; *out = e; return KB_ERR_UNSUPPORTED; }
    }
    {
        // fused pairs (k_pair): the scan's grid plus one resident step workgroup, which then
        // takes a scan workgroup's slot; the scan keeps its kernel for the bound passes, the
        // incremental mode and the multi-GPU summaries
        const bool full_shard = e->shard_begin == 0 && e->shard_end == n;
        // (small shards -- scan tiles of fewer than 16 scoring waves, c2's 10k partitions --
        // keep two launches: there the hand-off measured slower than the launch boundary,
        // 0.0427 vs 0.0389 ms/step at c2, profiles/r04_c)
        // (small shards too -- scan tiles of fewer than 16 scoring waves, c2's 10k partitions --
        // since the fast / deferred prep runs in the fused step only: c2 0.0410 -> 0.0388 ms/step
        // on one box, round 6; round 4 had measured the hand-off slower there without it)
        bool small_fuse = true;
        if (const char* v = diag_getenv("KB_FUSE_SMALL")) small_fuse = *v != '0';                  // A/B
        e->fuse = !e->gb && pair_supported(e->rc_dev) && e->nsets <= (int64_t)MAX_SETS &&
                  full_shard && e->nscan > 1 && (e->twaves == SCAN_THREADS / 64 || small_fuse);
        if (const char* v = diag_getenv("KB_FUSE")) e->fuse = e->fuse && *v != '0';                      // A/B
        if (const char* v = diag_getenv("KB_FUSE_PRE")) e->fuse_pre = *v != '0';                          // diagnostic
        if (const char* v = diag_getenv("KB_PAIR_WAIT_TICKS")) e->pair_wait_ticks = strtoull(v, nullptr, 10);   // tests
        if (e->fuse) {
            e->pair_lds = std::max(e->scan_lds, (size_t)e->step_lds_bytes);
            int pst = 0;
            const int pcu = pair_blocks_per_cu(e->rc_dev, e->lds_sets, e->pair_lds, &pst);
            e->slots_pair = (int64_t)pcu * ncu;
            if (pcu < 1 || pst + e->pair_lds > 160 * 1024) e->fuse = false;
            // (every workgroup of the grid resident at once: the scan's, the list workgroup, the
            // eager ones and the step workgroup)
            else e->nscan = std::min<int64_t>(e->ntiles, std::max<int64_t>(1, (int64_t)pcu * ncu -
                                              (e->eager ? EGW + 1 : (e->integral ? 0 : 1)) - 1));
        }
        // the sharded protocol's scan + rank summary as one launch (k_scansum): the scan's
        // grid plus one resident summary workgroup; every workgroup resident at once, as in
        // k_pair (an engine whose k_pair grid would have to shrink for it keeps two launches)
        e->fuse_sum = !e->gb && pair_supported(e->rc_dev) && e->nsets <= (int64_t)MAX_SETS && e->nscan > 1;
        if (const char* v = diag_getenv("KB_FUSE_SUM")) e->fuse_sum = e->fuse_sum && *v != '0';          // A/B
        if (e->fuse_sum) {
            int sst = 0;
            const int scu = scansum_blocks_per_cu(e->rc_dev, e->lds_sets, e->scan_lds, &sst);
            e->slots_sum = (int64_t)scu * ncu;
            const int64_t cap = (int64_t)scu * ncu - (e->eager ? EGW + 1 : (e->integral ? 0 : 1)) - 1;
            // (the summary workgroup stages r in the scan's dynamic LDS)
            // (a fused engine never shrinks its scan grid for the summary workgroup; an unfused
            // one -- small shards, whose grids are far below the cap -- may)
            if (scu < 1 || sst + e->scan_lds > 160 * 1024 || cap < 1 || (e->fuse && cap < e->nscan) ||
                e->scan_lds < (size_t)e->B * 8) e->fuse_sum = false;
            else e->nscan = std::min<int64_t>(e->nscan, cap);
        }
        // (after every grid sizing above: a rank summary reads one record per thread)
        e->nscan = std::min<int64_t>(e->nscan, SUM_RECS);
    }
    HIPCHK(hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking));
    e->own_st = true;
    if (const char* v = diag_getenv("KB_WGT")) {                 // diagnostic: scan workgroup timeline
        e->wgt_path = v;
        HIPCHK(dalloc(&e->wgt, 6 * (size_t)std::max<int64_t>(e->nscan, 1)));
        HIPCHK(hipMemset(e->wgt, 0, 6 * (size_t)std::max<int64_t>(e->nscan, 1) * 8));
    }
    HIPCHK(dalloc(&e->w, e->Ppad));
    HIPCHK(dalloc(&e->meta, e->Ppad));
    HIPCHK(dalloc(&e->rep, (size_t)e->rc_dev * e->Ppad));
    HIPCHK(dalloc(&e->nc, e->Ppad));
    // (+16 B on the arrays k_step stages by LDS-DMA: it copies whole 16-B granules)
    HIPCHK(dalloc(&e->load, e->B + 2));
    HIPCHK(dalloc(&e->lerr, e->B));
    if (e->gb) HIPCHK(dalloc(&e->gscr, (size_t)step_lds((int)e->B, e->NP2, 0).total));
    HIPCHK(dalloc(&e->pair_cnt, PAIR_SHARDS * PAIR_STRIDE));
    HIPCHK(hipMemset(e->pair_cnt, 0, PAIR_SHARDS * PAIR_STRIDE * 4));
    HIPCHK(dalloc(&e->eb, e->B + 2));
    HIPCHK(dalloc(&e->bfl, e->B + 16));
    HIPCHK(dalloc(&e->cnt, e->B));
    HIPCHK(dalloc(&e->setbits, (size_t)e->nsets * e->W64 + 2));   // (+2: k_step reads whole 16-B words)
    HIPCHK(dalloc(&e->setrec, (size_t)e->nsets * e->units));
    HIPCHK(dalloc(&e->order, e->B + 4));
    HIPCHK(dalloc(&e->posu, e->B));
    HIPCHK(dalloc(&e->blm, e->B));
    HIPCHK(dalloc(&e->posm, e->B));
    HIPCHK(dalloc(&e->r, e->B));
    HIPCHK(dalloc(&e->bset_off, e->B + 1));
    HIPCHK(dalloc(&e->bset_ids, hbi.size()));
    HIPCHK(dalloc(&e->recs, (size_t)std::max<int64_t>(e->nscan, 1) * WGREC_BYTES));
    if (const char* v = diag_getenv("KB_CONT_CAP")) e->cont_cap = (uint32_t)std::max(1, atoi(v));   // tests: growth path
    HIPCHK(dalloc(&e->cont, e->cont_cap));
    HIPCHK(dalloc(&e->ctl, 1));
    HIPCHK(dalloc(&e->bdesc, std::max<size_t>(hbd.size(), 1)));
    {
        // bound-pass block list: [0, 2 * max(nscan, STEP_THREADS)) the blocks of the last
        // records' best keys (k_step writes them; -1: none), then the heaviest blocks by
        // weight up to one block per scan wave
        const size_t kr = 2 * (size_t)std::max<int64_t>(e->nscan, STEP_THREADS);
        const size_t tot = std::max<size_t>(kr, (size_t)e->nscan * (SCAN_THREADS / 64));
        std::vector<BlockDesc> hub(tot);
        for (size_t i = 0; i < tot; i++) {
            const size_t j = i - kr;
            if (i >= kr && j < hbd.size()) hub[i] = hbd[j];
            else { hub[i].wmax = -1.0; hub[i].blk = 0; }
        }
        e->nubdesc = (int64_t)tot;
        HIPCHK(dalloc(&e->ubdesc, tot));
        HIPCHK(hipMemcpy(e->ubdesc, hub.data(), tot * sizeof(BlockDesc), hipMemcpyHostToDevice));
    }
    if (!hbd.empty()) HIPCHK(hipMemcpy(e->bdesc, hbd.data(), hbd.size() * sizeof(BlockDesc), hipMemcpyHostToDevice));
    e->logcap = 1024;
    HIPCHK(dalloc(&e->log, e->logcap));
    // the pinned mirror of the control block (fine-grained and mapped: k_xfer writes and
    // reads it directly) and k_xfer's sequence word
    HIPCHK(hipHostMalloc((void**)&e->h_ctl, sizeof(DevCtl), hipHostMallocCoherent | hipHostMallocMapped));
    HIPCHK(hipHostGetDevicePointer((void**)&e->h_ctl_d, e->h_ctl, 0));
    HIPCHK(hipHostMalloc((void**)&e->h_flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    HIPCHK(hipHostGetDevicePointer((void**)&e->h_flag_d, e->h_flag, 0));
    *e->h_flag = 0;
    if (const char* v = diag_getenv("KB_XFER")) e->xfer = std::min(2, std::max(0, atoi(v)));      // A/B
    HIPCHK(hipMemcpy(e->w, hw.data(), hw.size() * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->meta, hm.data(), hm.size() * 4, hipMemcpyHostToDevice));
    if (!e->lds_sets) {
        std::vector<uint32_t> hp(e->Ppad, 0u);
        for (int64_t i = 0; i < n; i++) hp[i] = (uint32_t)pset[i];
        HIPCHK(dalloc(&e->pset, e->Ppad));
        HIPCHK(hipMemcpy(e->pset, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
    }
    HIPCHK(hipMemcpy(e->rep, hr.data(), hr.size() * 2, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->nc, hnc.data(), hnc.size() * 4, hipMemcpyHostToDevice));
    if (e->B) {
        // flags: bit0 present (holds a replica), bit1 listed in -broker-ids (BF_* in kernels.hip)
        std::vector<uint8_t> fl(e->B, 0);
        for (int64_t b = 0; b < e->B; b++) fl[b] = (uint8_t)((cn[b] > 0 ? 1 : 0) | (hin[b] ? 2 : 0));
        std::vector<double> zero(e->B, 0.0);
        HIPCHK(hipMemcpy(e->load, ld.data(), ld.size() * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(e->lerr, le.data(), le.size() * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(e->eb, zero.data(), zero.size() * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(e->bfl, fl.data(), fl.size(), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(e->cnt, cn.data(), cn.size() * 4, hipMemcpyHostToDevice));
    }
    HIPCHK(hipMemcpy(e->bset_off, hbo.data(), hbo.size() * 4, hipMemcpyHostToDevice));
    if (!hbi.empty()) HIPCHK(hipMemcpy(e->bset_ids, hbi.data(), hbi.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->setbits, hsb.data(), hsb.size() * 8, hipMemcpyHostToDevice));
    if (!e->integral) {
        HIPCHK(dalloc(&e->L.lstart, e->B));
        HIPCHK(dalloc(&e->L.llen, e->B));
        HIPCHK(dalloc(&e->L.lcap, e->B));
        HIPCHK(dalloc(&e->L.lent, hle.size()));
        if (e->B) {
            HIPCHK(hipMemcpy(e->L.lstart, hls.data(), hls.size() * 4, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(e->L.llen, hll.data(), hll.size() * 4, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(e->L.lcap, hlc.data(), hlc.size() * 4, hipMemcpyHostToDevice));
        }
        HIPCHK(hipMemcpy(e->L.lent, hle.data(), hle.size() * 4, hipMemcpyHostToDevice));
        {
            // fold checkpoints of the initial loads: every 64th partial sum of each list's
            // in-order fold (the loads above are the same folds)
            std::vector<double> hck(hle.size(), 0.0);
            for (int64_t b = 0; b < e->B; b++) {
                double acc = 0.0;
                for (uint32_t k = 0; k < hll[b]; k++) {
                    const int64_t i = hle[hls[b] + k];
                    int slot = 0;
                    while (slot < len[i] && dn(i, slot) != (int)b) slot++;
                    acc += slot == 0 ? wt[i] * (double)(len[i] + ncon[i]) : wt[i];
                    if ((k + 1) % 64 == 0) hck[hls[b] + k] = acc;
                }
            }
            HIPCHK(dalloc(&e->L.ck, hck.size()));
            HIPCHK(hipMemcpy(e->L.ck, hck.data(), hck.size() * 8, hipMemcpyHostToDevice));
            HIPCHK(dalloc(&e->L.dpos, std::max<int64_t>(e->B, 1)));
            HIPCHK(hipMemset(e->L.dpos, 0xFF, std::max<int64_t>(e->B, 1) * 4));
        }
        if (const int rc = upload_rf(e); rc != KB_OK) { *out = e; return rc; }
    }
    DevCtl z;
    memset(&z, 0, sizeof z);
    z.logcap = e->logcap;
    z.full_prep = 1;
    z.stop_part = -1;
    z.tk_on = e->time_kernels;
    z.step_mask = SM_ALL;
    z.ts_beg = NONE64;
    HIPCHK(hipMemcpy(e->ctl, &z, sizeof z, hipMemcpyHostToDevice));
    HIPCHK(hipEventCreate(&e->ev0));
    HIPCHK(hipEventCreate(&e->ev1));
    e->scan_bytes = (e->shard_end - e->shard_begin) * (int64_t)(8 + 4 + 2 * e->rc_dev);
    // thousands of brokers with -allow-leader: a move rarely leaves a best key whose brokers
    // it did not touch, so the next step's census bound is open; the conditional bound pass
    // runs from the first step (else the second step's census spills once, ~1 s at c5 in
    // round 2).  Plans without -allow-leader carry every scored wave's bound key (BK), which
    // keeps the bound closed: there the pass waits for a first retry (c5: none in 200 steps,
    // 0.1006 -> 0.0962 ms/step without the pass's two launches per step)
    e->ub_mode = e->B >= 2048 && e->allow_leader;
    if (const char* v = diag_getenv("KB_UB_MODE")) e->ub_mode = *v == '1';                      // diagnostic
    if (const char* v = diag_getenv("KB_UB_STICKY")) e->ub_sticky = *v != '0';                   // diagnostic
    *out = e;
    return KB_OK;
}

// ---------------------------------------------------------- step launch

static void fill_refresh_args(kb_engine* e, RefreshArgs& ra) {
    ra.ctl = e->ctl; ra.w = e->w; ra.rep = e->rep; ra.meta = e->meta; ra.nc = e->nc;
    ra.load = e->load; ra.lerr = e->lerr; ra.eb = e->eb; ra.bfl = e->bfl; ra.B = (int)e->B;
    ra.L = e->L;
}

// the refresh arguments as the in-stream refresh reads them (after create and relist)
static int upload_rf(kb_engine* e) {
    if (e->integral) return KB_OK;
    RefreshArgs ra;
    fill_refresh_args(e, ra);
    if (!e->rf_dev) HIPCHK(dalloc(&e->rf_dev, 1));
    HIPCHK(hipMemcpy(e->rf_dev, &ra, sizeof ra, hipMemcpyHostToDevice));
    return KB_OK;
}

static void fill_scan_args(kb_engine* e, ScanArgs& s) {
    s.ctl = e->ctl; s.w = e->w; s.rep = e->rep; s.meta = e->meta;
    s.Ppad = e->Ppad; s.shard_begin = e->shard_begin; s.shard_end = e->shard_end;
    s.ntiles = (int)e->ntiles; s.nscan = (int)e->nscan; s.twaves = e->twaves;
    s.B = (int)e->B; s.nsets = (int)e->nsets; s.W64 = e->W64; s.units = e->units;
    s.setbits = e->setbits; s.setrec = e->setrec; s.r = e->r; s.blm = e->blm; s.posm = e->posm;
    s.allow_leader = e->allow_leader; s.rebalance = e->rebalance; s.sem_go = e->sem == KB_SEM_GO;
    s.R = scan_recs(e->recs, (int)e->nscan); s.cont = e->cont; s.cont_cap = e->cont_cap;
    s.ncont = &e->ctl->ncont; s.cont_ovf = &e->ctl->cont_overflow;
    s.listwg = e->integral ? 0 : 1;
    s.dbg = e->dbg_scan;
    s.ubpass = 0;
    s.L = e->L;
    s.incr = e->incr; s.nblk = (int)e->nblk; s.bdesc = e->bdesc;
    s.pset = e->pset;
    s.rfpass = 0;
    s.rf = e->rf_dev;
    s.eager = e->eager && e->nscan > 0 ? EGW : 0;
    s.gt = e->gb ? 1 : 0;
    s.done = e->pair_cnt;
    s.wgt = e->wgt;
    s.pred = 0;                       // (enqueue_pair sets it for k_pair)
    s.dyn_lds = (int)e->scan_lds;
}

static void fill_step_args(kb_engine* e, StepArgs& a, const Recs& R, int use_spill) {
    a.ctl = e->ctl; a.w = e->w; a.rep = e->rep; a.meta = e->meta; a.nc = e->nc; a.Ppad = e->Ppad;
    a.RC = e->rc_dev; a.KR = e->KR; a.K = e->K; a.units = e->units; a.W64 = e->W64; a.B = (int)e->B;
    a.nsets = (int)e->nsets; a.NP2 = e->NP2;
    a.sb_lds = e->sb_lds; a.lds_bytes = e->step_lds_bytes;
    a.gscr = e->gscr;
    a.wait_cnt = e->pair_cnt; a.wait_n = 0; a.fuse_pre = 1; a.wait_ticks = e->pair_wait_ticks;
    a.setbits = e->setbits; a.setrec = e->setrec;
    a.order = e->order; a.posu = e->posu; a.blm = e->blm; a.posm = e->posm; a.r = e->r;
    a.load = e->load; a.lerr = e->lerr; a.eb = e->eb; a.bfl = e->bfl; a.cnt = e->cnt;
    a.bset_off = e->bset_off; a.bset_ids = e->bset_ids;
    a.R = R;
    a.cont = e->cont; a.cont_cap = e->cont_cap; a.use_spill = use_spill;
    a.allow_leader = e->allow_leader; a.rebalance = e->rebalance; a.sem_go = e->sem == KB_SEM_GO;
    a.integral = e->integral ? 1 : 0; a.exact_unb = e->exact_unb;
    a.minrep = e->minrep; a.min_unbalance = e->min_unb; a.wmax = e->wmax;
    a.log = e->log; a.L = e->L;
    a.incr = e->incr && use_spill;
    a.ubdesc = e->ubdesc;
    a.ub_heavy = e->nubdesc > 2 * std::max<int64_t>(e->nscan, STEP_THREADS) ? 1 : 0;
    a.pset = e->pset;
    a.rf_final = 0;
    a.eager = e->eager && e->nscan > 0 ? 1 : 0;
    // deferred prep (DevCtl.fp): its LDS region whenever the engine has one (a pending one is
    // finished by whichever step runs next); a step may defer only in the fused single-GPU path
    a.fp_lds = e->fp_lds;
    a.fp_bk = e->fp_bk && R.n <= STEP_THREADS ? 1 : 0;
    a.fp_ok = e->fp_lds && e->fuse && use_spill && !a.incr && !a.eager && !e->rebalance ? 1 : 0;
}

static const int kStepBatch = 64;
static const int64_t kLogChunk = 16384;   // steps per device step log (kb_engine_plan chunks)

static void mark(kb_engine* e, int kind_next) {
    if (!e->time_kernels) return;
    // mode 1: k_scan / k_step are device-clock timed (no events between them); mode 2:
    // HIP events around every launch (dispatch included, the interval rocprofv3 reports)
    if (e->time_kernels == 1 && (kind_next == TK_SCAN || kind_next == TK_STEP || kind_next == TK_BOUND)) return;
    if (e->tev.empty()) {
        e->tev.resize((size_t)kStepBatch * 4 + 16);
        e->tkind.resize(e->tev.size());
        for (auto& v : e->tev) hipEventCreate(&v);
    }
    if (e->tev_used < (int)e->tev.size()) {
        e->tkind[e->tev_used] = kind_next;
        hipEventRecord(e->tev[e->tev_used++], e->st);
    }
}

// accumulate the durations of the marks recorded since the last harvest
static void harvest(kb_engine* e) {
    if (!e->time_kernels || e->tev_used == 0) return;
    hipEventSynchronize(e->tev[e->tev_used - 1]);
    for (int i = 0; i + 1 < e->tev_used; i++) {
        const int k = e->tkind[i];
        if (k < 0 || k >= TK_N) continue;
        float ms = 0;
        if (hipEventElapsedTime(&ms, e->tev[i], e->tev[i + 1]) == hipSuccess) {
            e->kms[k] += ms;
            e->klaunch[k]++;
        }
    }
    e->tev_used = 0;
}

static void enqueue_scan(kb_engine* e, bool rf = false) {
    if (e->nscan == 0 && e->integral) return;
    ScanArgs s;
    fill_scan_args(e, s);
    s.rfpass = rf && e->rf_stream && e->nscan > 0;
    if (e->nscan == 0) s.listwg = 1;
    launch_scan(s, e->rc_dev, e->lds_sets, e->scan_lds, e->st);
}

// the first step after a full prep has no best keys to bound its minimum: a
// census-free scan (no list op) plus k_ubinit sets ub to the step's own minima
static void enqueue_ubinit(kb_engine* e, bool rf = false, bool tighten = false) {
    if (e->nscan == 0) return;
    mark(e, TK_BOUND);
    ScanArgs s;
    fill_scan_args(e, s);
    s.rfpass = rf && e->rf_stream;
    s.listwg = 0;
    s.eager = 0;                      // (the main scan launch refolds)
    s.dbg |= 1;
    s.ubpass = tighten ? 2 : 1;
    // (set records in LDS: the block-list kernel, which scans only the blocks of the last
    // records' best keys when k_step left them, DevCtl.ub_sub)
    s.incr = e->lds_sets ? 1 : 0;
    s.bdesc = e->ubdesc;
    s.nblk = (int)e->nubdesc;
    launch_scan(s, e->rc_dev, e->lds_sets, e->scan_lds, e->st);
    launch_ubinit(e->ctl, scan_recs(e->recs, (int)e->nscan), e->allow_leader, tighten ? 1 : 0, e->st);
}

static void enqueue_step(kb_engine* e, bool rf = false) {
    StepArgs a;
    fill_step_args(e, a, scan_recs(e->recs, (int)e->nscan), 1);
    a.rf_final = rf && e->rf_stream && e->nscan > 0;
    launch_step(a, e->st);
}

// one Balance(): scan (if prepped) then resolve + apply + prep of the next step
// (rf: this pair may follow a step halted for exact loads: the pair's first scan launch
// refolds the loads and its k_step resumes; rf_scan: the main scan is that first launch)
static void enqueue_pair(kb_engine* e, bool rf = false, bool rf_scan = false) {
    if (e->fuse && !e->incr) {
        // one launch: the scan's grid and the step workgroup (k_pair)
        mark(e, TK_SCAN);
        ScanArgs s;
        fill_scan_args(e, s);
        s.rfpass = rf && rf_scan && e->rf_stream;
        s.pred = 1;
        StepArgs a;
        fill_step_args(e, a, scan_recs(e->recs, (int)e->nscan), 1);
        a.rf_final = rf && e->rf_stream;
        a.wait_n = s.nscan + (s.listwg ? 1 : 0) + s.eager;
        s.dyn_lds = (int)e->pair_lds;
        a.fuse_pre = e->fuse_pre;
        launch_pair(s, a, e->rc_dev, e->lds_sets, e->pair_lds, e->st);
        return;
    }
    mark(e, TK_SCAN);
    enqueue_scan(e, rf && rf_scan);
    mark(e, TK_STEP);
    enqueue_step(e, rf);
}

// Lay the per-broker partition lists out again from the device's partition words
// (partition order, the getBrokerLoad fold order) with twice the slack: a list ran
// out of room (ctl.list_overflow).  Every applied change is already in the
// partition words, so a pending list edit is dropped with the old lists.
static int relist(kb_engine* e) {
    const int64_t P = e->P;
    std::vector<uint16_t> hr((size_t)e->rc_dev * e->Ppad);
    std::vector<uint32_t> hm((size_t)e->Ppad);
    HIPCHK(hipMemcpy(hr.data(), e->rep, hr.size() * 2, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hm.data(), e->meta, hm.size() * 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> cnt(e->B, 0);
    for (int64_t i = 0; i < P; i++) {
        const int nr = (int)meta_nrep(hm[i]);
        for (int k = 0; k < nr && k < e->rc_dev; k++) cnt[hr[(size_t)k * e->Ppad + i]]++;
    }
    e->list_slack = e->list_slack < (1u << 30) ? 2 * e->list_slack : e->list_slack;
    std::vector<uint32_t> hls(e->B), hll(e->B, 0), hlc(e->B);
    uint64_t off = 0;
    for (int64_t b = 0; b < e->B; b++) { hls[b] = (uint32_t)off; hlc[b] = cnt[b] + e->list_slack; off += hlc[b]; }
    if (off >= (1ull << 32)) { e->last_err = "broker lists exceed 2^32 entries"; return KB_ERR_CAPACITY; }
    std::vector<uint32_t> hle(off ? off : 1, 0);
    for (int64_t i = 0; i < P; i++) {
        const int nr = (int)meta_nrep(hm[i]);
        for (int k = 0; k < nr && k < e->rc_dev; k++) {
            const int b = hr[(size_t)k * e->Ppad + i];
            hle[hls[b] + hll[b]++] = (uint32_t)i;
        }
    }
    uint32_t* nent = nullptr;
    HIPCHK(dalloc(&nent, hle.size()));
    hipFree(e->L.lent);
    e->L.lent = nent;
    // (the checkpoints follow the new layout; every broker is refolded from its start)
    double* nck = nullptr;
    HIPCHK(dalloc(&nck, hle.size()));
    hipFree(e->L.ck);
    e->L.ck = nck;
    HIPCHK(hipMemset(e->L.dpos, 0, std::max<int64_t>(e->B, 1) * 4));
    HIPCHK(hipMemcpy(e->L.lent, hle.data(), hle.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->L.lstart, hls.data(), hls.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->L.llen, hll.data(), hll.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->L.lcap, hlc.data(), hlc.size() * 4, hipMemcpyHostToDevice));
    // every broker holding a replica is refolded from the new lists by the refresh that
    // follows (a load folded from an edit the old lists dropped must not survive them)
    if (e->B) {
        std::vector<uint8_t> fl(e->B);
        HIPCHK(hipMemcpy(fl.data(), e->bfl, e->B, hipMemcpyDeviceToHost));
        for (int64_t b = 0; b < e->B; b++) if (cnt[b] > 0) fl[b] |= 4;   // BF_DIRTY (kernels.hip)
        HIPCHK(hipMemcpy(e->bfl, fl.data(), e->B, hipMemcpyHostToDevice));
    }
    if (const int rc = upload_rf(e); rc != KB_OK) return rc;
    e->relists++;
    return KB_OK;
}

// exact refolds of the approximate loads (k_refresh), then a full prep
static int refresh(kb_engine* e) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }            // (the device block changes behind the host copy)
    roctxMark("kb:refresh (exact refolds of the approximate loads)");
    if (e->integral) return KB_OK;
    mark(e, -1);
    launch_listop(e->ctl, e->L, e->st);
    HIPCHK(hipMemcpyAsync(e->h_ctl, e->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    if (e->h_ctl->list_overflow) {
        if (const int rc = relist(e); rc != KB_OK) return rc;   // (a capacity limit stays one)
        DevCtl c = *e->h_ctl;
        c.list_overflow = 0;
        c.pending_list = 0;
        HIPCHK(hipMemcpy(e->ctl, &c, sizeof c, hipMemcpyHostToDevice));
    }
    RefreshArgs ra;
    fill_refresh_args(e, ra);
    mark(e, TK_REFRESH);
    launch_refresh(ra, e->st);
    mark(e, -1);
    HIPCHK(hipGetLastError());
    // halted (if NEED_EXACT) -> run, prepped = 0, full_prep = 1, ndirty = 0
    HIPCHK(hipMemcpyAsync(e->h_ctl, e->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    DevCtl c = *e->h_ctl;
    if (c.halted == H_NEED_EXACT) c.halted = H_RUN;
    c.prepped = 0; c.full_prep = 1; c.ndirty = 0; c.want_refresh = 0;
    c.eg_n = 0;
    c.fp = 0;                                        // (the full prep rebuilds what a deferred one would)
    HIPCHK(hipMemcpyAsync(e->ctl, &c, sizeof c, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    e->refreshes++;
    return KB_OK;
}

static int reset_ctl(kb_engine* e, int64_t budget_steps) {
    if (!e->ctl_mirror) {          // (after a plan, the host copy is current: no round trip)
        HIPCHK(hipMemcpyAsync(e->h_ctl, e->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipStreamSynchronize(e->st));
    }
    e->ctl_mirror = false;
    DevCtl c = *e->h_ctl;
    if (c.halted == H_NEED_EXACT) {
        if (const int rc = refresh(e); rc != KB_OK) return rc;
        c = *e->h_ctl;
        c.halted = H_RUN; c.prepped = 0; c.full_prep = 1; c.ndirty = 0; c.want_refresh = 0;
        c.fp = 0;
    }
    c.halted = H_RUN;
    c.logpos = 0;
    c.logcap = e->logcap;
    c.stop_part = e->stop_part;
    c.step_mask = e->step_mask;
    if (!e->reuse_now) { c.ncont = 0; c.cont_overflow = 0; }   // (a scan runs first: an empty spill)
    e->recs_fresh = false;
    const long long bud = (long long)c.steps + budget_steps;
    c.budget = bud > 0x7FFFFFFF ? 0x7FFFFFFF : (int32_t)bud;
    *e->h_ctl = c;
    if (e->xfer) {
        // (k_xfer reads the mirror when it runs: nothing writes it before the batch's end)
        XferArgs x{};
        x.src[0] = (const uint32_t*)e->h_ctl_d; x.dst[0] = (uint32_t*)e->ctl; x.n[0] = (int)(sizeof(DevCtl) / 4);
        launch_xfer(x, e->st);
    } else {
        HIPCHK(hipMemcpyAsync(e->ctl, e->h_ctl, sizeof c, hipMemcpyHostToDevice, e->st));
    }
    return KB_OK;
}

static int convert(kb_engine* e, const ChangeDev& d, kb_change* o) {
    memset(o, 0, sizeof *o);
    o->step = d.step;
    o->kind = d.kind;
    o->slot = d.slot;
    o->partition = d.part;
    o->from_broker = d.from >= 0 ? e->ids[d.from] : -1;
    o->to_broker = d.to >= 0 ? e->ids[d.to] : -1;
    o->unbalance_before = d.su;
    o->unbalance_after = d.cu;
    o->exact = d.exact;
    o->err_code = d.err_code;
    o->err_broker = d.err_broker >= 0 ? e->ids[d.err_broker] : -1;
    if (d.status == 1) { o->status = KB_CHANGE; return KB_CHANGE; }
    if (d.status == 0) { o->status = KB_NOCHANGE; return KB_NOCHANGE; }
    // error: format the reference message
    std::vector<int64_t> reps;
    std::string ps;
    if (d.part >= 0 && d.part < e->P) { read_replicas(e, d.part, reps); ps = part_string(e, d.part, reps); }
    std::string step = d.step >= 0 && d.step < 9 ? kStepNames[d.step] : "Balance";
    int rc = KB_ERR_STEP;
    switch (d.err_code) {
        case E_DUP: e->last_err = step + ": partition " + ps + " has duplicated replicas"; break;
        case E_REMOVE: e->last_err = step + ": partition " + ps + " unable to pick replica to remove"; break;
        case E_ADD: e->last_err = step + ": partition " + ps + " unable to pick replica to add"; break;
        case E_DIS:
            e->last_err = step + ": partition " + ps + " unable to pick replica to replace broker " +
                          std::to_string((long long)o->err_broker);
            break;
        case E_PANIC:
            e->last_err = step + ": panic: the reference Go code panics on this input" +
                          (ps.empty() ? std::string() : " (" + ps + ")");
            rc = KB_ERR_PANIC;
            break;
        case E_CONT_OVERFLOW: e->last_err = step + ": engine capacity: near-tie buffer overflow"; rc = KB_ERR_CAPACITY; break;
        case E_LIST_OVERFLOW: e->last_err = step + ": engine capacity: broker list overflow"; rc = KB_ERR_CAPACITY; break;
        case E_DUP_UNSUP:
            e->last_err = step + ": engine: partition " + ps + " holds duplicated replicas (Go aliasing after a "
                          "remove) and ValidateReplicas is not in the step mask; the engine's loads assume "
                          "distinct replicas";
            rc = KB_ERR_UNSUPPORTED;
            break;
        case E_PAIR_TIMEOUT:
            e->last_err = "engine: the fused scan + step launch timed out waiting for the scan workgroups";
            rc = KB_ERR_HIP;
            break;
        default: e->last_err = step + ": error"; break;
    }
    o->status = rc;
    return rc;
}

static int pending_result(kb_engine* e, kb_change* o) {
    memset(o, 0, sizeof *o);
    o->status = e->pending;
    o->step = e->pending_step;
    o->partition = -1;
    o->from_broker = o->to_broker = -1;
    e->last_err = e->pending_msg;
    return e->pending;
}

// grow the device step log to hold max_steps entries (the new buffer first: a failed
// allocation leaves the old one and its capacity in place)
static int ensure_log(kb_engine* e, int64_t max_steps) {
    if (max_steps <= e->logcap) return KB_OK;
    const int cap = (int)std::min<int64_t>(max_steps, 1 << 30);
    ChangeDev* nl = nullptr;
    if (dalloc(&nl, cap) != hipSuccess) {
        e->last_err = "cannot allocate the step log";
        return KB_ERR_HIP;
    }
    hipFree(e->log);
    e->log = nl;
    e->logcap = cap;
    return KB_OK;
}

// The near-tie spill buffer overflowed with the census bound already at the step
// minimum (exact ties over many brokers): 8x the capacity, up to kContMax, and the
// halted step runs again.  Only past kContMax is it a capacity error.
static const uint32_t kContMax = 1u << 26;   // 64M candidates (2 GiB)
static int grow_spill(kb_engine* e) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }            // (the device block changes behind the host copy)
    roctxMark("kb:grow_spill (near-tie buffer x8, step runs again)");
    if (e->cont_cap >= kContMax) {
        e->last_err = "engine capacity: more than " + std::to_string(kContMax) + " near-tied candidates in one step";
        return KB_ERR_CAPACITY;
    }
    const uint32_t cap = std::min<uint32_t>(kContMax, e->cont_cap * 8u);
    Contender* nc = nullptr;
    if (dalloc(&nc, cap) != hipSuccess) {
        e->last_err = "cannot allocate the near-tie spill buffer";
        return KB_ERR_CAPACITY;
    }
    HIPCHK(hipStreamSynchronize(e->st));
    hipFree(e->cont);
    e->cont = nc;
    e->cont_cap = cap;
    e->spill_grows++;
    DevCtl c = *e->h_ctl;
    c.halted = H_RUN;
    c.ncont = 0;
    c.cont_overflow = 0;
    HIPCHK(hipMemcpyAsync(e->ctl, &c, sizeof c, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    *e->h_ctl = c;
    return KB_OK;
}

// run up to max_steps Balance() calls device-resident; returns the number of
// log entries written (changes + the terminating no-change / error)
// Lazy loads (fewer than 2048 brokers) cost a halt, a refresh and a re-run whenever a
// decision needs exact folds, and the approximate loads' error widens eps and with it the
// census; on a balanced cluster without -allow-leader that is a quarter of the steps (c3nl
// past its 300th step: 0.118 ms/step lazy, 0.051 eager).  Once the halts reach one per 16
// steps over the last 64-128 steps (at least 4 of them) the plan switches to eager refolds
// (the next launches refold the touched brokers
// beside the scan): the grids shrink by the eager workgroups so every workgroup of a fused
// launch stays resident.  Switched between batches, where no list edit is in flight but the
// last step's (which the next launch's list workgroup applies, the eager workgroups having
// no brokers yet).  The decisions do not depend on the mode.
static void maybe_switch_to_eager(kb_engine* e, const DevCtl& c) {
    if (!e->eager_auto || e->eager) return;
    const unsigned long long st = (unsigned long long)std::max(c.steps, 0), h = c.total_exact_halts;
    const unsigned long long ds = st - std::min(st, e->w0_steps), dh = h - std::min(h, e->w0_halts);
    if (dh < 4 || 16 * dh < ds) {
        if (st >= e->w1_steps + 64) {
            e->w0_steps = e->w1_steps; e->w0_halts = e->w1_halts;
            e->w1_steps = st; e->w1_halts = h;
        }
        return;
    }
    const int64_t lw = EGW + 1;                       // the eager workgroups and the list workgroup
    int64_t n = std::min<int64_t>(e->nscan, std::max<int64_t>(1, e->slots_scan - lw));
    if (e->fuse) n = std::min<int64_t>(n, std::max<int64_t>(1, e->slots_pair - lw - 1));
    if (e->fuse_sum) n = std::min<int64_t>(n, std::max<int64_t>(1, e->slots_sum - lw - 1));
    e->nscan = n;
    e->eager = true;
    e->recs_fresh = false;
    e->eager_switches++;
}

static int run_steps(kb_engine* e, int64_t max_steps) {
    if (ensure_log(e, max_steps) != KB_OK) return KB_ERR_HIP;
    if (e->h_logcap < e->logcap) {
        if (e->h_log) hipHostFree(e->h_log);
        e->h_log = nullptr;
        e->h_logcap = 0;
        HIPCHK(hipHostMalloc((void**)&e->h_log, (size_t)e->logcap * sizeof(ChangeDev),
                             hipHostMallocCoherent | hipHostMallocMapped));
        HIPCHK(hipHostGetDevicePointer((void**)&e->h_log_d, e->h_log, 0));
        e->h_logcap = e->logcap;
    }
    // (kb_engine_step: the scan records of a masked step that changed nothing describe the
    // state still; the first pair reuses them)
    bool reuse = e->reuse_now && e->h_ctl->prepped;
    const double t_r0 = now_us();
    if (const int rc = reset_ctl(e, max_steps); rc != KB_OK) { e->reuse_now = false; return rc; }
    e->host_us[0] += now_us() - t_r0;
    e->reuse_now = false;
    reuse = reuse && e->h_ctl->prepped && e->h_ctl->halted == H_RUN;
    const int steps0 = e->h_ctl->steps;
    bool prepped = e->h_ctl->prepped != 0;
    bool fresh = false;                 // h_ctl holds the device block after the last batch
    HIPCHK(hipEventRecord(e->ev0, e->st));
    for (;;) {
        const int64_t done = e->h_ctl->steps - steps0;
        if (done >= max_steps) break;
        const int64_t pairs = std::min<int64_t>(e->batch, max_steps - done + (prepped ? 0 : 1));
        const int lp0 = e->h_ctl->logpos;
        const int st0 = e->h_ctl->steps;
        const double t_b0 = now_us();
        roctxRangePush("kb:batch (scan + step pairs)");
        for (int64_t s = 0; s < pairs; s++) {
            // pair 0 ran the full prep; once a step had to re-scan (no surviving best
            // keys bound the next minimum), every scan gets the conditional bound pass
            // (a halt for exact loads in pair s - 1 is refolded by pair s's first scan launch)
            const bool ubp = (s == 1 && !prepped) || (e->ub_mode && (s > 0 || prepped));
            const bool rf = s > 0;
            if (s == 0 && reuse) {           // kb_engine_step: the last masked step's records
                mark(e, TK_STEP);
                enqueue_step(e);
                continue;
            }
            if (ubp) enqueue_ubinit(e, rf);
            enqueue_pair(e, rf, !ubp);
        }
        mark(e, -1);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(e->ev1, e->st));
        // the control block and this batch's log entries (at most one per pair) come
        // back with one synchronisation
        const int64_t ln = std::min<int64_t>(pairs, (int64_t)e->logcap - lp0);
        const double t_enq = now_us();
        if (e->xfer) {
            XferArgs x{};
            x.src[0] = (const uint32_t*)e->ctl; x.dst[0] = (uint32_t*)e->h_ctl_d; x.n[0] = (int)(sizeof(DevCtl) / 4);
            if (ln > 0) {
                x.src[1] = (const uint32_t*)(e->log + lp0); x.dst[1] = (uint32_t*)(e->h_log_d + lp0);
                x.n[1] = (int)(ln * (int64_t)(sizeof(ChangeDev) / 4));
            }
            if (e->xfer == 2) { x.flag = e->h_flag_d; x.seq = ++e->xseq; }
            launch_xfer(x, e->st);
            HIPCHK(hipGetLastError());
            if (e->xfer == 2) {
                // poll the sequence word k_xfer stores after its copies (system-scope release);
                // past 2 ms of polling (long batches, or a failed launch) wait on the stream
                const double t0 = now_us();
                bool seen = false;
                for (int it = 0;; it++) {
                    if (__atomic_load_n(e->h_flag, __ATOMIC_ACQUIRE) == x.seq) { seen = true; break; }
                    if ((it & 255) == 255 && now_us() - t0 > 2000.0) break;
                }
                if (!seen) HIPCHK(hipStreamSynchronize(e->st));
            } else {
                HIPCHK(hipStreamSynchronize(e->st));
            }
        } else {
            HIPCHK(hipMemcpyAsync(e->h_ctl, e->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, e->st));
            if (ln > 0)
                HIPCHK(hipMemcpyAsync(e->h_log + lp0, e->log + lp0, (size_t)ln * sizeof(ChangeDev),
                                      hipMemcpyDeviceToHost, e->st));
            HIPCHK(hipStreamSynchronize(e->st));
        }
        e->host_us[1] += t_enq - t_b0;
        e->host_us[2] += now_us() - t_enq;
        roctxRangePop();
        if (e->h_ctl->logpos > lp0 && e->h_ctl->logpos <= e->logcap &&
            e->h_log[e->h_ctl->logpos - 1].err_code == E_PAIR_TIMEOUT) {
            // (the error is returned with this batch's log)
            if (const int r = poison_after_timeout(e); r != KB_OK) return r;
        }
        fresh = true;
        reuse = false;
        harvest(e);
        const DevCtl& c = *e->h_ctl;
        if (c.total_retries > 0 && e->ub_sticky) e->ub_mode = true;
        // adaptive batch: the pairs enqueued behind a halted step run as no-ops (a launch
        // each), so after a halt the next batch is about twice the steps that ran before
        // it; full batches double it again, up to kStepBatch
        if (c.halted == H_NEED_EXACT || c.halted == H_NEED_SPILL || c.want_refresh)
            e->batch = (int)std::max<int64_t>(4, std::min<int64_t>(kStepBatch, 2 * (int64_t)(c.steps - st0) + 2));
        else if (c.steps - st0 >= pairs - 1)
            e->batch = std::min(kStepBatch, 2 * e->batch);
        if (c.halted == H_DONE) break;
        if (c.steps >= c.budget) break;              // (kb_engine_plan_until's stop, whatever the halt)
        if (c.halted == H_NEED_SPILL) {
            // more near-tied candidates than the spill buffer holds: grow it, run the step again
            const int rc = grow_spill(e);
            if (rc != KB_OK) return rc;
            fresh = false;
            continue;
        }
        if (c.halted == H_NEED_EXACT || (c.want_refresh && c.steps - steps0 < max_steps)) {
            if (const int rc = refresh(e); rc != KB_OK) return rc;
            // refresh() cleared halted; the step log position is kept
            maybe_switch_to_eager(e, c);
            prepped = false;
            fresh = false;
            continue;
        }
        maybe_switch_to_eager(e, c);
        prepped = c.prepped != 0;
    }
    float ms = 0;
    hipEventElapsedTime(&ms, e->ev0, e->ev1);
    e->last_ms += ms;
    if (!fresh) {
        HIPCHK(hipStreamSynchronize(e->st));
        HIPCHK(hipMemcpy(e->h_ctl, e->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost));
    }
    e->ctl_mirror = true;
    return (int)std::min<int64_t>(e->h_ctl->logpos, e->logcap);
}

extern "C" int kb_engine_balance(kb_engine* e, kb_change* out) {
    if (!e || !out) return KB_ERR_INVALID;
    return kb_engine_step(e, KB_STEPS_ALL, out);
}

// One Balance() restricted to the steps in step_mask (bit k = kb_step k, in the reference's
// order, balancer.go:34-44): a Go steps table whose entries are cgo calls
// calls it once per entry.  ValidateWeights and FillDefaults ran at create (the weights and
// defaults never change on the device); ValidateReplicas can fail later only under Go
// aliasing (a remove duplicates a replica), so under KB_SEM_APPLIED it is host
// work too.  A masked step that changes nothing keeps the prep and its scan records, and the
// next masked step resolves them again without a scan (the state has not changed).
extern "C" int kb_engine_step(kb_engine* e, uint32_t step_mask, kb_change* out) {
    if (!e || !out || (step_mask & ~(uint32_t)KB_STEPS_ALL)) return KB_ERR_INVALID;
    auto nochange = [&]() {
        memset(out, 0, sizeof *out);
        out->status = KB_NOCHANGE; out->step = -1; out->partition = -1;
        out->from_broker = out->to_broker = out->err_broker = -1;
        return KB_NOCHANGE;
    };
    if (e->dead) return dead_result(e);
    if (e->pending) {
        // a validation error (create): returned by its own step and by every later one (the
        // engine holds no state past a failed validation); earlier steps change nothing
        if (step_mask >> e->pending_step) return pending_result(e, out);
        return nochange();
    }
    // the steps that could change something: ValidateWeights / FillDefaults never (create
    // ran them), ValidateReplicas only under Go aliasing, ReassignLeaders / MoveLeaders
    // only with their flags (steps.go:292-307 return nil, nil otherwise); with the records
    // of an unchanged state at hand, a first-index step whose predicate no partition
    // holds (the last resolve's DevCtl.last_fm) changes nothing either
    uint32_t dev = step_mask & ~(uint32_t)(SM_VALIDATE_WEIGHTS | SM_FILL_DEFAULTS);
    if (e->sem != KB_SEM_GO) dev &= ~(uint32_t)SM_VALIDATE_REPLICAS;
    if (!e->rebalance) dev &= ~(uint32_t)SM_REASSIGN;
    if (!e->allow_leader) dev &= ~(uint32_t)SM_MOVE_LEADERS;
    if (e->recs_fresh) {
        const uint32_t fm = e->h_ctl->last_fm;
        if (!(fm & (1u << F_DUP))) dev &= ~(uint32_t)SM_VALIDATE_REPLICAS;
        if (!(fm & (1u << F_REMOVE))) dev &= ~(uint32_t)SM_REMOVE;
        if (!(fm & (1u << F_ADD))) dev &= ~(uint32_t)SM_ADD;
        if (!(fm & (1u << F_DIS))) dev &= ~(uint32_t)SM_DISALLOWED;
    }
    if (!dev) return nochange();                  // (no device work: the records stay)
    e->last_ms = 0;
    e->step_mask = step_mask;                     // (k_step never tests bits 0 and 2)
    dev = step_mask;
    e->reuse_now = e->recs_fresh;
    const int nlog = run_steps(e, 1);
    e->step_mask = SM_ALL;
    if (nlog < 0) return nlog;
    if (nlog == 0) return nochange();
    const ChangeDev& d = e->h_log[0];
    const int rc = convert(e, d, out);
    // the records stay valid for the next masked step when this one changed nothing
    e->recs_fresh = dev != SM_ALL && d.status == 0 && e->h_ctl->halted == H_DONE && e->h_ctl->prepped;
    return rc;
}

extern "C" int kb_engine_plan(kb_engine* e, int64_t max_steps, kb_change* out, int64_t* n_out) {
    if (!e || !n_out || max_steps < 0) return KB_ERR_INVALID;
    *n_out = 0;
    if (max_steps == 0) return KB_NOCHANGE;
    if (e->pending) { if (out) pending_result(e, out); *n_out = 1; return e->pending; }
    if (e->dead) return dead_result(e);
    e->host_us[4] += 1;
    for (int k = 0; k < TK_N; k++) { e->kms[k] = 0; e->klaunch[k] = 0; }
    e->tev_used = 0;
    e->last_ms = 0;
    // chunks of at most kLogChunk steps: the device step log stays bounded whatever
    // max_steps asks for (the caller's `out` holds max_steps entries)
    int rc = KB_NOCHANGE;
    int64_t k = 0;
    while (k < max_steps) {
        const int64_t m = std::min<int64_t>(max_steps - k, kLogChunk);
        const int nlog = run_steps(e, m);
        if (nlog < 0) { *n_out = k; return nlog; }
        const double t_c0 = now_us();
        for (int64_t i = 0; i < nlog; i++) {         // (run_steps copied the log entries)
            kb_change tmp;
            kb_change* o = out ? &out[k] : &tmp;
            rc = convert(e, e->h_log[i], o);
            k++;
            if (rc != KB_CHANGE) { *n_out = k; e->host_us[3] += now_us() - t_c0; return rc; }
            if (e->stop_part >= 0 && o->partition != e->stop_part) {   // (kb_engine_plan_until)
                *n_out = k; e->host_us[3] += now_us() - t_c0; return rc;
            }
        }
        e->host_us[3] += now_us() - t_c0;
        if (nlog < m) break;
    }
    *n_out = k;
    return rc;
}

// run()'s -complete-partition loop device-resident (kafkabalancer.go:193-221): once
// -max-reassign changes are out, the reference keeps calling Balance() while the change is on
// the completing partition and stops after the first one that is not (it is applied: the
// probe).  The same as kb_engine_plan with that stop on the device: 64 steps per host round
// trip instead of one Balance() call per change.
extern "C" int kb_engine_plan_until(kb_engine* e, int64_t max_steps, int64_t stop_part, kb_change* out, int64_t* n_out) {
    if (!e || !n_out || max_steps < 0) return KB_ERR_INVALID;
    e->stop_part = stop_part < 0 ? -1 : stop_part;
    const int rc = kb_engine_plan(e, max_steps, out, n_out);
    e->stop_part = -1;
    return rc;
}

extern "C" int64_t kb_engine_replicas(kb_engine* e, int64_t i, int64_t* buf, int64_t cap) {
    if (!e || i < 0 || i >= e->P) return KB_ERR_INVALID;
    std::vector<int64_t> r;
    if (read_replicas(e, i, r) < 0) return KB_ERR_HIP;
    for (int64_t k = 0; k < (int64_t)r.size() && k < cap; k++) buf[k] = r[k];
    return (int64_t)r.size();
}

// make every load the exact fold again (before reading them out)
static int make_exact(kb_engine* e) {
    if (e->integral) return KB_OK;
    HIPCHK(hipMemcpyAsync(e->h_ctl, e->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    if (e->h_ctl->ndirty == 0 && !e->h_ctl->pending_list) return KB_OK;
    return refresh(e);
}

extern "C" int64_t kb_engine_loads(kb_engine* e, int64_t* ids, double* loads, int64_t cap) {
    if (!e) return KB_ERR_INVALID;
    if (make_exact(e) != KB_OK) return KB_ERR_HIP;
    std::vector<double> ld(e->B);
    if (e->B && hipMemcpy(ld.data(), e->load, e->B * 8, hipMemcpyDeviceToHost) != hipSuccess) return KB_ERR_HIP;
    for (int64_t k = 0; k < e->B && k < cap; k++) { if (ids) ids[k] = e->ids[k]; if (loads) loads[k] = ld[k]; }
    return e->B;
}

extern "C" double kb_engine_unbalance(kb_engine* e) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }            // (the device block changes behind the host copy)
    if (!e || e->B == 0) return 0.0;
    if (make_exact(e) != KB_OK) return NAN;
    std::vector<double> ld(e->B);
    std::vector<uint8_t> fl(e->B);
    hipMemcpy(ld.data(), e->load, e->B * 8, hipMemcpyDeviceToHost);
    hipMemcpy(fl.data(), e->bfl, e->B, hipMemcpyDeviceToHost);
    std::vector<int> bl;
    for (int64_t b = 0; b < e->B; b++) if (fl[b] & 3) bl.push_back((int)b);
    std::sort(bl.begin(), bl.end(), [&](int x, int y) { return ld[x] != ld[y] ? ld[x] < ld[y] : x < y; });
    double S = 0;
    for (int b : bl) S += ld[b];
    double avg = S / (double)bl.size(), U = 0;
    for (int b : bl) {
        double r = ld[b] / avg - 1.0;
        if (r > 0) U += r * r; else U += r * r / 2;
    }
    return U;
}

extern "C" int kb_engine_stats(kb_engine* e, kb_stats* o) {
    if (!e || !o) return KB_ERR_INVALID;
    memset(o, 0, sizeof *o);
    DevCtl c;
    HIPCHK(hipMemcpy(&c, e->ctl, sizeof c, hipMemcpyDeviceToHost));
    o->steps = c.steps;
    o->candidates = (int64_t)c.total_cand;
    o->contenders = (int64_t)c.total_cont;
    o->exact_folds = (int64_t)c.total_folds;
    o->scan_bytes = e->scan_bytes;
    o->device_ms = e->last_ms;
    o->n_brokers = e->B;
    o->n_sets = e->nsets;
    o->integral = e->integral ? 1 : 0;
    o->max_replicas = e->rc_dev;
    o->refreshes = e->refreshes + (int64_t)c.total_rf_stream;
    o->exact_halts = (int64_t)c.total_exact_halts;
    o->scan_workgroups = e->nscan;
    o->retries = (int64_t)c.total_retries;
    o->spill_grows = e->spill_grows;
    o->blocks_scanned = (int64_t)c.total_blocks;
    o->relists = e->relists;
    o->fused_pairs = e->fuse && !e->incr ? 1 : 0;
    o->fused_summaries = e->fuse_sum ? 1 : 0;
    o->eager = e->eager ? 1 : 0;
    o->eager_switches = e->eager_switches;
    o->fast_preps = (int64_t)e->h_ctl->total_fp;
    return KB_OK;
}

// incremental mode: see include/kbengine.h.  Switching (either way)
// clears the device's permission flag, so the next scan is a full one and refreshes
// the cached candidate counts.
extern "C" int kb_engine_set_incremental(kb_engine* e, int32_t on) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }            // (the device block changes behind the host copy)
    if (!e) return KB_ERR_INVALID;
    if (on && !e->lds_sets) {       // (the incremental scan kernel keeps the set records in LDS)
        e->last_err = "incremental mode needs the allowed-set records in LDS (too many sets or brokers)";
        return KB_ERR_UNSUPPORTED;
    }
    HIPCHK(hipStreamSynchronize(e->st));
    e->incr = on ? 1 : 0;
    DevCtl c;
    HIPCHK(hipMemcpy(&c, e->ctl, sizeof c, hipMemcpyDeviceToHost));
    c.incr_ok = 0;
    c.wskip = 0.0;
    HIPCHK(hipMemcpy(e->ctl, &c, sizeof c, hipMemcpyHostToDevice));
    *e->h_ctl = c;
    return KB_OK;
}

// k_step / k_scan durations come from the device clock (100 MHz): each scan workgroup
// stamps its start and end, k_step folds the scan's interval and its own into
// ctl->tk_*; k_refresh (rare) is timed with events around its launches
extern "C" int kb_engine_timings(kb_engine* e, double* ms, int64_t* launches, int n) {
    if (!e) return KB_ERR_INVALID;
    DevCtl c;
    HIPCHK(hipStreamSynchronize(e->st));
    HIPCHK(hipMemcpy(&c, e->ctl, sizeof c, hipMemcpyDeviceToHost));
    const double tick_ms = 1e-5;
    double kms[TK_N + 5];
    int64_t kn[TK_N + 5];
    for (int k = 0; k < TK_N; k++) { kms[k] = e->kms[k]; kn[k] = e->klaunch[k]; }
    for (int k = TK_N; k < TK_N + 5; k++) { kms[k] = 0; kn[k] = 0; }
    if (e->time_kernels == 1) {
        // spans (dispatch included, rocprofv3's interval) and the inner device-clock
        // intervals (first workgroup start .. last end)
        kms[TK_STEP] = (double)c.tk_span[1] * tick_ms; kn[TK_STEP] = (int64_t)c.tk_span_n[1];
        kms[TK_SCAN] = (double)c.tk_span[0] * tick_ms; kn[TK_SCAN] = (int64_t)c.tk_span_n[0];
        kms[TK_N] = (double)c.tk_sum[1] * tick_ms; kn[TK_N] = (int64_t)c.tk_n[1];
        kms[TK_N + 1] = (double)c.tk_sum[0] * tick_ms; kn[TK_N + 1] = (int64_t)c.tk_n[0];
        kms[TK_N + 2] = (double)c.tk_pair * tick_ms; kn[TK_N + 2] = (int64_t)c.tk_pair_n;
        kms[TK_N + 3] = (double)c.tk_eg * tick_ms; kn[TK_N + 3] = (int64_t)c.tk_eg_n;
        kms[TK_N + 4] = (double)c.tk_eg_edit * tick_ms; kn[TK_N + 4] = (int64_t)c.tk_eg_n;
    }
    for (int k = 0; k < TK_N + 5 && k < n; k++) {
        if (ms) ms[k] = kms[k];
        if (launches) launches[k] = kn[k];
    }
    return TK_N + 5;
}

// diagnostic: the control block's scalars (after a plan: the prep of the next step):
// [0..1] ub per kind, [2] eps, [3] U0, [4] V, [5] avg, [6] rlo, [7] rhi, [8] E, [9] S
extern "C" int kb_engine_ctl_scalars(kb_engine* e, double* out, int n) {
    if (!e || !out) return KB_ERR_INVALID;
    DevCtl c;
    HIPCHK(hipStreamSynchronize(e->st));
    HIPCHK(hipMemcpy(&c, e->ctl, sizeof c, hipMemcpyDeviceToHost));
    const double v[10] = {c.ub[0], c.ub[1], c.eps, c.U0, c.V, c.avg, c.rlo, c.rhi, c.E, c.S};
    for (int k = 0; k < 10 && k < n; k++) out[k] = v[k];
    return 10;
}

// diagnostic: the last scan's record headers (RecHdr, include/kbengine.h does not describe
// them: kafkabalancer_amd/csrc/engine_dev.h); returns the record count
extern "C" int64_t kb_engine_debug_records(kb_engine* e, void* out, int64_t cap) {
    if (!e) return KB_ERR_INVALID;
    const int64_t n = std::min<int64_t>(e->nscan, cap);
    HIPCHK(hipStreamSynchronize(e->st));
    if (out && n > 0) HIPCHK(hipMemcpy(out, e->recs, (size_t)n * sizeof(RecHdr), hipMemcpyDeviceToHost));
    return e->nscan;
}

// diagnostic: cumulative host phases of the plan calls since the last kb_engine_set_timing
// (us): [0] reset_ctl, [1] enqueue of the batches, [2] waiting for them (the batch-end
// transfer included), [3] log conversion, [4] kb_engine_plan calls
extern "C" int kb_engine_host_timings(kb_engine* e, double* us, int n) {
    if (!e || !us) return KB_ERR_INVALID;
    for (int k = 0; k < 5 && k < n; k++) us[k] = e->host_us[k];
    return 5;
}

extern "C" int kb_engine_set_timing(kb_engine* e, int32_t on) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }            // (the device block changes behind the host copy)
    if (!e) return KB_ERR_INVALID;
    for (double& v : e->host_us) v = 0;
    HIPCHK(hipStreamSynchronize(e->st));
    e->tev_used = 0;
    for (int k = 0; k < TK_N; k++) { e->kms[k] = 0; e->klaunch[k] = 0; }
    e->time_kernels = on == 2 ? 2 : (on ? 1 : 0);
    DevCtl c;
    HIPCHK(hipMemcpy(&c, e->ctl, sizeof c, hipMemcpyDeviceToHost));
    c.tk_on = e->time_kernels == 1;                 // (mode 2: events only, production kernels)
    c.tk_sum[0] = c.tk_sum[1] = c.tk_n[0] = c.tk_n[1] = 0;
    c.tk_span[0] = c.tk_span[1] = c.tk_span_n[0] = c.tk_span_n[1] = 0;
    c.tk_pair = c.tk_pair_n = 0;
    c.tk_eg = c.tk_eg_edit = c.tk_eg_n = 0;
    c.ts_beg = NONE64;
    c.ts_end = 0;
    c.ts_prev_end = 0;
    HIPCHK(hipMemcpy(e->ctl, &c, sizeof c, hipMemcpyHostToDevice));
    *e->h_ctl = c;
    return KB_OK;
}

extern "C" int kb_engine_stamps(kb_engine* e, uint64_t* out, int n) {
    if (!e || !out) return KB_ERR_INVALID;
    DevCtl c;
    HIPCHK(hipMemcpy(&c, e->ctl, sizeof c, hipMemcpyDeviceToHost));
    for (int k = 0; k < 32 && k < n; k++) out[k] = c.stamps[k];
    return 32;
}

// Diagnostic: average device time of k_scan over `iters` back-to-back launches on
// the current prepped state (the scan only writes its records and spill buffer).
extern "C" int kb_engine_bench_scan(kb_engine* e, int iters, double* avg_us) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }            // (the device block changes behind the host copy)
    if (!e || iters < 1 || !avg_us) return KB_ERR_INVALID;
    if (e->pending) return e->pending;
    if (const int rc = reset_ctl(e, 1); rc != KB_OK) return rc;
    if (!e->h_ctl->prepped) {
        enqueue_step(e);                              // prep only
        HIPCHK(hipStreamSynchronize(e->st));
    }
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    if (e->ub_mode) enqueue_ubinit(e);                // an open census bound: close it first
    const int incr = e->incr;
    e->incr = 0;                                      // (always the full scan)
    enqueue_scan(e);                                  // warm
    // KB_PROBE_INTERLEAVE (diagnostic): 1 = an empty one-workgroup kernel between the
    // scans, 2 = one that rewrites the scan's tables (as k_step does); each scan is
    // then timed on its own
    int il = 0;
    if (const char* v = diag_getenv("KB_PROBE_INTERLEAVE")) il = atoi(v);
    float ms = 0;
    if (il) {
        hipEvent_t c, d;
        HIPCHK(hipEventCreate(&c));
        HIPCHK(hipEventCreate(&d));
        double tot = 0;
        for (int i = 0; i < iters; i++) {
            launch_touch(e->r, il == 2 ? (int)e->B : 0, e->blm, e->posm, e->setrec,
                         il == 2 ? (int)e->nsets * e->units : 0, e->st);
            HIPCHK(hipEventRecord(c, e->st));
            enqueue_scan(e);
            HIPCHK(hipEventRecord(d, e->st));
            HIPCHK(hipEventSynchronize(d));
            float x = 0;
            hipEventElapsedTime(&x, c, d);
            tot += x;
        }
        ms = (float)tot;
        hipEventDestroy(c);
        hipEventDestroy(d);
    } else {
        HIPCHK(hipEventRecord(a, e->st));
        for (int i = 0; i < iters; i++) enqueue_scan(e);
        HIPCHK(hipEventRecord(b, e->st));
        HIPCHK(hipEventSynchronize(b));
        hipEventElapsedTime(&ms, a, b);
    }
    *avg_us = 1e3 * ms / iters;
    hipEventDestroy(a);
    hipEventDestroy(b);
    e->incr = incr;
    // forget the spills of the repeated scans
    HIPCHK(hipMemsetAsync(&e->ctl->ncont, 0, 8, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    return KB_OK;
}

// Diagnostic: k_step alone on one fixed input: the state k_step mutates is snapshotted
// after a scan and restored before every launch, and HIP events time the launch alone.
// Run on -DKB_STOP_AT=k builds (kernels.hip, KB_STOP: return after phase k), the
// cumulative times give the phase costs without instrumenting the production kernel.
extern "C" int kb_engine_bench_step(kb_engine* e, int iters, double* avg_us) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }
    if (!e || iters < 1 || !avg_us) return KB_ERR_INVALID;
    if (e->pending) return e->pending;
    if (const int rc = reset_ctl(e, 1); rc != KB_OK) return rc;
    if (!e->h_ctl->prepped) {
        enqueue_step(e);                              // prep only
        HIPCHK(hipStreamSynchronize(e->st));
    }
    if (e->ub_mode) enqueue_ubinit(e);
    enqueue_scan(e);                                  // the records k_step resolves
    struct Arr { void* p; size_t bytes; void* snap; };
    std::vector<Arr> arrs = {
        {e->ctl, sizeof(DevCtl), nullptr}, {e->load, (size_t)e->B * 8, nullptr}, {e->lerr, (size_t)e->B * 8, nullptr},
        {e->eb, (size_t)e->B * 8, nullptr}, {e->bfl, (size_t)e->B, nullptr}, {e->cnt, (size_t)e->B * 4, nullptr},
        {e->order, (size_t)e->B * 4, nullptr}, {e->posu, (size_t)e->B * 4, nullptr}, {e->blm, (size_t)e->B * 4, nullptr},
        {e->posm, (size_t)e->B * 4, nullptr}, {e->r, (size_t)e->B * 8, nullptr},
        {e->rep, (size_t)e->rc_dev * e->Ppad * 2, nullptr}, {e->meta, (size_t)e->Ppad * 4, nullptr},
        {e->setrec, (size_t)e->nsets * e->units * 16, nullptr}};
    if (e->ubdesc) arrs.push_back({e->ubdesc, (size_t)e->nubdesc * sizeof(BlockDesc), nullptr});
    for (auto& x : arrs) {
        if (!x.bytes) continue;
        HIPCHK(hipMalloc(&x.snap, x.bytes));
        HIPCHK(hipMemcpyAsync(x.snap, x.p, x.bytes, hipMemcpyDeviceToDevice, e->st));
    }
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    StepArgs sa;
    fill_step_args(e, sa, scan_recs(e->recs, (int)e->nscan), 1);
    double tot = 0;
    for (int i = 0; i <= iters; i++) {               // (the first launch warms up)
        for (auto& x : arrs)
            if (x.bytes) HIPCHK(hipMemcpyAsync(x.p, x.snap, x.bytes, hipMemcpyDeviceToDevice, e->st));
        HIPCHK(hipEventRecord(a, e->st));
        launch_step(sa, e->st);
        HIPCHK(hipEventRecord(b, e->st));
        HIPCHK(hipEventSynchronize(b));
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        if (i) tot += ms;
    }
    *avg_us = 1e3 * tot / iters;
    for (auto& x : arrs)                              // (leave the engine as it was after the scan)
        if (x.bytes) { HIPCHK(hipMemcpyAsync(x.p, x.snap, x.bytes, hipMemcpyDeviceToDevice, e->st)); }
    HIPCHK(hipStreamSynchronize(e->st));
    for (auto& x : arrs) if (x.snap) hipFree(x.snap);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return KB_OK;
}

extern "C" int kb_engine_last_error(kb_engine* e, char* buf, size_t n) {
    if (!e || !buf || n == 0) return KB_ERR_INVALID;
    snprintf(buf, n, "%s", e->last_err.c_str());
    return (int)e->last_err.size();
}

extern "C" void kb_engine_destroy(kb_engine* e) {
    if (!e) return;
    if (e->wgt) {
        // diagnostic (KB_WGT=path): the last scan launch's {start, scored, record written}
        // per workgroup (100 MHz device clock), appended as one JSON line
        std::vector<unsigned long long> h(6 * (size_t)std::max<int64_t>(e->nscan, 1));
        hipStreamSynchronize(e->st);
        hipMemcpy(h.data(), e->wgt, h.size() * 8, hipMemcpyDeviceToHost);
        if (FILE* f = fopen(e->wgt_path.c_str(), "a")) {
            fprintf(f, "{\"nscan\": %lld, \"wg\": [", (long long)e->nscan);
            for (size_t i = 0; i < h.size(); i++) fprintf(f, "%s%llu", i ? ", " : "", h[i]);
            fprintf(f, "]}\n");
            fclose(f);
        }
        hipFree(e->wgt);
    }
    void* ptrs[] = {e->w, e->rep, e->meta, e->pset, e->nc, e->load, e->lerr, e->eb, e->bfl, e->cnt,
                    e->setbits, e->setrec, e->order, e->posu, e->blm, e->posm, e->r,
                    e->bset_off, e->bset_ids, e->gscr, e->pair_cnt, e->recs, e->cont, e->ctl, e->log, e->bdesc, e->ubdesc,
                    e->L.lstart, e->L.llen, e->L.lcap, e->L.lent, e->L.ck, e->L.dpos, e->rf_dev};
    for (void* p : ptrs) if (p) hipFree(p);
    if (e->gath_buf) hipFree(e->gath_buf);         // (sum_buf is a slot of it)
    if (e->comm) { hipStreamSynchronize(e->st); rccl_api().comm_destroy(e->comm); }
    if (e->h_ctl) hipHostFree(e->h_ctl);
    if (e->h_flag) hipHostFree(e->h_flag);
    if (e->h_log) hipHostFree(e->h_log);
    if (e->ev0) hipEventDestroy(e->ev0);
    if (e->ev1) hipEventDestroy(e->ev1);
    for (auto v : e->tev) hipEventDestroy(v);
    if (e->own_st && e->st) hipStreamDestroy(e->st);
    delete e;
}

// ----------------------------------------------------- multi-GPU phases

extern "C" int64_t kb_engine_summary_bytes(kb_engine* e) {
    return e ? (int64_t)summary_bytes(e->sum_keys) : (int64_t)summary_bytes(SUMMARY_KEYS);
}

// A rank summary overflowed (more near-tie keys than it carries) or the scan's spill
// buffer did: every rank sees the same gathered flags and halts the same step; each
// grows its summaries 8x (up to SUMMARY_KEYS_MAX) and, if its scan spilled past it, its
// spill buffer; the caller re-allocates the exchange buffers (kb_engine_summary_bytes)
// and runs the step again.  Past both limits it is a capacity error.
static int grow_summary(kb_engine* e) {
    HIPCHK(hipStreamSynchronize(e->st));
    DevCtl c;
    HIPCHK(hipMemcpy(&c, e->ctl, sizeof c, hipMemcpyDeviceToHost));
    // The decision depends only on state every rank shares (sum_keys, identical on all
    // ranks, and the gathered summaries' flags): no rank re-enters the collective alone.
    // Below the summary limit every rank grows its summaries alike (the gathered layout
    // needs one size) and the spill buffer only where this rank's scan overflowed it.
    // At the limit the step runs again only if some rank reported a spill overflow it
    // can still grow (summary flag bit 2, k_summary); otherwise every rank returns the
    // capacity error.
    bool any_growable = false;
    if (e->gath && e->gath_n > 0) {
        const Recs G = summary_recs((unsigned char*)e->gath, e->gath_n, e->sum_keys);
        for (int i = 0; i < e->gath_n && !any_growable; i++) {
            uint32_t fl = 0;
            HIPCHK(hipMemcpy(&fl, &G.h(i)->flags, 4, hipMemcpyDeviceToHost));
            any_growable = (fl & 4u) != 0;
        }
    }
    if (e->sum_keys >= SUMMARY_KEYS_MAX && !any_growable) {
        e->last_err = "engine capacity: more than " + std::to_string(SUMMARY_KEYS_MAX) +
                      " near-tied candidates in one rank summary";
        return KB_ERR_CAPACITY;
    }
    // (an open census bound spilled on some rank -- the gathered flags, alike on every rank:
    // bound passes from now on; a pass only ever tightens this rank's own census)
    if (c.cont_overflow || any_growable) e->ub_mode = true;
    if (c.cont_overflow && e->cont_cap < kContMax) {
        const int rc = grow_spill(e);
        if (rc != KB_OK) return rc;
        HIPCHK(hipMemcpy(&c, e->ctl, sizeof c, hipMemcpyDeviceToHost));
    }
    e->sum_keys = std::min(SUMMARY_KEYS_MAX, 8 * e->sum_keys);
    c.halted = H_RUN;
    c.ncont = 0;
    c.cont_overflow = 0;
    HIPCHK(hipMemcpy(e->ctl, &c, sizeof c, hipMemcpyHostToDevice));
    *e->h_ctl = c;
    e->ctl_mirror = false;
    return KB_GROW;
}

extern "C" int kb_engine_set_stream(kb_engine* e, void* s) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }            // (the device block changes behind the host copy)
    if (!e) return KB_ERR_INVALID;
    if (e->own_st && e->st) hipStreamDestroy(e->st);
    e->st = (hipStream_t)s;
    e->own_st = false;
    return KB_OK;
}

// this rank's scan and its summary into summary_dev: one k_scansum launch (the summary
// workgroup waits in the scan's grid), or k_scan then k_summary
static int enqueue_scan_summary(kb_engine* e, void* summary_dev) {
    // the tightening bound pass (a census-free scan, then ub = min(ub, this shard's minima)):
    // a rank's prep bounds the next minimum with its one gathered summary's few keys, which
    // at thousands of brokers either share a broker with the applied move (an open bound)
    // or sit far above the minimum -- either way most waves then pass the census gate and
    // spill (c5 at world size 1: 64M spilled keys through the summary workgroup, ~0.2-0.5 s
    // per step, before this pass).  The rank's own minima are a valid census bound for its
    // own scan (its summary holds the keys within 4 eps of its own minima); the resolve
    // reads ub only for its -inf state, which the pass leaves alone.
    if (e->ub_mode || e->B >= 2048) enqueue_ubinit(e, false, true);
    SumArgs s;
    s.ctl = e->ctl; s.R = scan_recs(e->recs, (int)e->nscan); s.cont = e->cont; s.cont_cap = e->cont_cap;
    s.r = e->r; s.B = (int)e->B; s.out = summary_recs((unsigned char*)summary_dev, 1, e->sum_keys);
    s.spill_growable = e->cont_cap < kContMax ? 1 : 0;
    s.wait_cnt = e->pair_cnt; s.wait_n = 0; s.wait_ticks = e->pair_wait_ticks; s.log = e->log;
    if (e->fuse_sum) {
        ScanArgs a;
        fill_scan_args(e, a);
        s.wait_n = a.nscan + (a.listwg ? 1 : 0) + a.eager;
        launch_scansum(a, s, e->rc_dev, e->lds_sets, e->scan_lds, e->st);
    } else {
        enqueue_scan(e);
        launch_summary(s, e->st);
    }
    HIPCHK(hipGetLastError());
    return KB_OK;
}

extern "C" int kb_engine_step_begin(kb_engine* e, void* summary_dev) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }            // (the device block changes behind the host copy)
    if (!e || !summary_dev) return KB_ERR_INVALID;
    if (e->dead) return dead_result(e);
    if (e->pending) return e->pending;
    if (const int rc = reset_ctl(e, 1); rc != KB_OK) return rc;
    if (!e->h_ctl->prepped) enqueue_step(e);       // prep only (nothing to resolve yet)
    return enqueue_scan_summary(e, summary_dev);
}

// ---- batched multi-GPU steps: the host enqueues several (scan, summary, all-gather,
// resolve) rounds without a host round trip; a halted step turns the rest into no-ops
extern "C" int kb_engine_sharded_reset(kb_engine* e, int64_t budget_steps) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }            // (the device block changes behind the host copy)
    if (!e || budget_steps < 1) return KB_ERR_INVALID;
    if (e->dead) return dead_result(e);
    if (e->pending) return e->pending;
    if (const int rc = reset_ctl(e, budget_steps); rc != KB_OK) return rc;
    if (!e->h_ctl->prepped) enqueue_step(e);       // prep only (nothing to resolve yet)
    HIPCHK(hipGetLastError());
    return KB_OK;
}

extern "C" int kb_engine_sharded_scan(kb_engine* e, void* summary_dev) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }            // (the device block changes behind the host copy)
    if (!e || !summary_dev) return KB_ERR_INVALID;
    if (e->dead) return dead_result(e);
    return enqueue_scan_summary(e, summary_dev);
}

extern "C" int kb_engine_sharded_resolve(kb_engine* e, const void* gathered_dev, int32_t n_ranks) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }            // (the device block changes behind the host copy)
    if (!e || !gathered_dev || n_ranks < 1) return KB_ERR_INVALID;
    StepArgs a;
    fill_step_args(e, a, summary_recs((unsigned char*)gathered_dev, n_ranks, e->sum_keys), 0);
    launch_step(a, e->st);
    HIPCHK(hipGetLastError());
    e->gath = gathered_dev; e->gath_n = n_ranks;
    return KB_OK;
}

extern "C" int kb_engine_sharded_collect(kb_engine* e, kb_change* out, int64_t cap, int64_t* n_out) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }            // (the device block changes behind the host copy)
    if (!e || !n_out || cap < 0) return KB_ERR_INVALID;
    *n_out = 0;
    HIPCHK(hipMemcpyAsync(e->h_ctl, e->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    const DevCtl c = *e->h_ctl;
    const int nlog = (int)std::min<int64_t>(std::min<int64_t>(c.logpos, e->logcap), cap);
    std::vector<ChangeDev> logv((size_t)nlog);
    if (nlog) HIPCHK(hipMemcpy(logv.data(), e->log, (size_t)nlog * sizeof(ChangeDev), hipMemcpyDeviceToHost));
    int rc = KB_CHANGE;
    int64_t k = 0;
    for (int i = 0; i < nlog; i++)
        if (logv[i].err_code == E_PAIR_TIMEOUT)
            if (const int r = poison_after_timeout(e); r != KB_OK) return r;
    for (int i = 0; i < nlog; i++) {
        kb_change tmp;
        const int r = convert(e, logv[i], out ? &out[k] : &tmp);
        k++;
        if (r != KB_CHANGE) { rc = r; break; }
    }
    *n_out = k;
    if (rc != KB_CHANGE) return rc;                   // no change / error: the plan ends
    if (c.halted == H_NEED_SPILL) return grow_summary(e);   // bigger summaries, step again
    // exact loads needed (the resolve could not decide, or the load error grew):
    // every rank reaches the same verdict on the same state -- refold, then go on
    if (c.halted == H_NEED_EXACT || c.want_refresh) {
        if (const int rc = refresh(e); rc != KB_OK) return rc;
        return KB_RETRY;
    }
    return KB_CHANGE;
}

extern "C" int kb_engine_step_finish(kb_engine* e, const void* gathered_dev, int32_t n_ranks, kb_change* out) {
    if (e) { e->ctl_mirror = false; e->recs_fresh = false; }            // (the device block changes behind the host copy)
    if (!e || !gathered_dev || n_ranks < 1 || !out) return KB_ERR_INVALID;
    if (e->pending) return pending_result(e, out);
    StepArgs a;
    fill_step_args(e, a, summary_recs((unsigned char*)gathered_dev, n_ranks, e->sum_keys), 0);
    launch_step(a, e->st);
    HIPCHK(hipGetLastError());
    e->gath = gathered_dev; e->gath_n = n_ranks;
    HIPCHK(hipMemcpyAsync(e->h_ctl, e->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    const DevCtl c = *e->h_ctl;
    if (c.logpos > 0) {
        // the step committed (a change, no change or an error); a NEED_EXACT raised by
        // the prep that followed the apply only asks for exact loads before the next step
        ChangeDev d;
        HIPCHK(hipMemcpy(&d, e->log, sizeof d, hipMemcpyDeviceToHost));
        if (d.err_code == E_PAIR_TIMEOUT)
            if (const int r = poison_after_timeout(e); r != KB_OK) return r;
        const int rc = convert(e, d, out);
        if (rc == KB_CHANGE && (c.halted == H_NEED_EXACT || c.want_refresh))
            if (const int rc = refresh(e); rc != KB_OK) return rc;
        return rc;
    }
    if (c.halted == H_NEED_SPILL) {                   // bigger summaries, then the step again
        const int rc = grow_summary(e);
        memset(out, 0, sizeof *out);
        out->status = rc;
        return rc;
    }
    // the resolve could not certify its decision from the bounds: every rank reaches
    // the same verdict on the same state -- refold, then redo the step
    if (c.halted == H_NEED_EXACT) { if (const int rc = refresh(e); rc != KB_OK) return rc; }
    memset(out, 0, sizeof *out);
    out->status = KB_RETRY;
    return KB_RETRY;
}

// ----------------------------------------------------- RCCL-driven sharded plan

extern "C" int kb_comm_unique_id(unsigned char* id) {
    if (!id) return KB_ERR_INVALID;
    RcclApi& R = rccl_api();
    if (!R.get_unique_id) return KB_ERR_UNSUPPORTED;
    ncclUniqueId u;
    if (R.get_unique_id(&u) != ncclSuccess) return KB_ERR_HIP;
    static_assert(sizeof(ncclUniqueId) == KB_COMM_ID_BYTES, "RCCL unique id size");
    memcpy(id, &u, sizeof u);
    return KB_OK;
}

extern "C" int kb_engine_comm_init(kb_engine* e, int32_t n_ranks, int32_t rank, const unsigned char* id) {
    if (!e || !id || n_ranks < 1 || rank < 0 || rank >= n_ranks) return KB_ERR_INVALID;
    RcclApi& R = rccl_api();
    if (!R.comm_init_rank) { e->last_err = R.err; return KB_ERR_UNSUPPORTED; }
    if (e->comm) { HIPCHK(hipStreamSynchronize(e->st)); R.comm_destroy(e->comm); e->comm = nullptr; }
    HIPCHK(hipSetDevice(e->dev));
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    const ncclResult_t r = R.comm_init_rank(&e->comm, n_ranks, u, rank);
    if (r != ncclSuccess) {
        e->comm = nullptr;
        e->last_err = std::string("ncclCommInitRank: ") + R.error_string(r);
        return KB_ERR_HIP;
    }
    e->nranks = n_ranks;
    e->rank = rank;
    // (a new communicator may change the world size or this rank's slot: the exchange
    // buffers are sized and offset for the old one, so the next plan reallocates them)
    HIPCHK(hipStreamSynchronize(e->st));
    if (e->gath_buf) hipFree(e->gath_buf);
    e->gath_buf = e->sum_buf = nullptr;
    e->xbuf_bytes = 0;
    return KB_OK;
}

// (re-)size the exchange buffers to the current summary size (it grows after a KB_GROW,
// alike on every rank)
static int ensure_xbufs(kb_engine* e) {
    const int64_t sb = (int64_t)summary_bytes(e->sum_keys);
    if (sb == e->xbuf_bytes && e->sum_buf) return KB_OK;
    HIPCHK(hipStreamSynchronize(e->st));
    if (e->gath_buf) hipFree(e->gath_buf);
    e->sum_buf = e->gath_buf = nullptr;
    // in-place all-gather: this rank's summary is its own slot of the gathered buffer
    HIPCHK(hipMalloc((void**)&e->gath_buf, (size_t)sb * e->nranks));
    HIPCHK(hipMemset(e->gath_buf, 0, (size_t)sb * e->nranks));
    e->sum_buf = e->gath_buf + (size_t)sb * e->rank;
    e->xbuf_bytes = sb;
    return KB_OK;
}

// The whole -max-reassign plan of a partition-sharded engine, driven from C: batches of up
// to 64 rounds (scan + rank summary, ncclAllGather of the summaries on the engine's stream,
// the identical resolve + apply + prep on every rank) per host round trip; a halted round
// turns the rest of the batch into no-ops on every rank alike.  Every rank calls it with
// the same max_steps; the changes are the same on every rank.  Same result convention as
// kb_engine_plan.
extern "C" int kb_engine_sharded_plan(kb_engine* e, int64_t max_steps, kb_change* out, int64_t* n_out) {
    if (!e || !n_out || max_steps < 0) return KB_ERR_INVALID;
    *n_out = 0;
    if (!e->comm) { e->last_err = "kb_engine_sharded_plan: no communicator (kb_engine_comm_init)"; return KB_ERR_INVALID; }
    if (max_steps == 0) return KB_NOCHANGE;
    if (e->pending) { if (out) pending_result(e, out); *n_out = 1; return e->pending; }
    if (e->dead) return dead_result(e);
    RcclApi& R = rccl_api();
    e->last_ms = 0;
    HIPCHK(hipEventRecord(e->ev0, e->st));
    std::vector<kb_change> tmp;
    int64_t k = 0;
    int rc = KB_CHANGE;
    while (k < max_steps) {
        if (const int r = ensure_xbufs(e); r != KB_OK) { *n_out = k; return r; }
        const int64_t b = std::min<int64_t>(kStepBatch, max_steps - k);
        if (const int r = kb_engine_sharded_reset(e, b); r < 0) { *n_out = k; return r; }
        for (int64_t i = 0; i < b; i++) {
            if (const int r = kb_engine_sharded_scan(e, e->sum_buf); r < 0) { *n_out = k; return r; }
            const ncclResult_t nr = R.all_gather(e->sum_buf, e->gath_buf, (size_t)e->xbuf_bytes, ncclUint8, e->comm, e->st);
            if (nr != ncclSuccess) {
                e->last_err = std::string("ncclAllGather: ") + R.error_string(nr);
                *n_out = k;
                return KB_ERR_HIP;
            }
            if (const int r = kb_engine_sharded_resolve(e, e->gath_buf, e->nranks); r < 0) { *n_out = k; return r; }
        }
        tmp.resize((size_t)b + 1);
        int64_t n = 0;
        rc = kb_engine_sharded_collect(e, tmp.data(), b + 1, &n);
        for (int64_t i = 0; i < n && k < max_steps; i++, k++)
            if (out) out[k] = tmp[(size_t)i];
        if (rc == KB_CHANGE || rc == KB_RETRY || rc == KB_GROW) { rc = KB_CHANGE; continue; }
        break;                                        // no change / error: the plan ends
    }
    HIPCHK(hipEventRecord(e->ev1, e->st));
    HIPCHK(hipEventSynchronize(e->ev1));
    float ms = 0;
    hipEventElapsedTime(&ms, e->ev0, e->ev1);
    e->last_ms = ms;
    *n_out = k;
    return rc;
}
