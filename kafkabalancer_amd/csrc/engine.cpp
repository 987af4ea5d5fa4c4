// engine.cpp -- host half of the MI355X kafkabalancer engine: the C ABI declared
// in include/kbengine.h.  Marshals the reference's PartitionList
// (kafkabalancer.go:40-58) into the device SoA layout, performs the one-time
// ValidateWeights / ValidateReplicas / FillDefaults (steps.go:7-66), and drives
// the per-step kernels of kernels.hip.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (host folds must
// round exactly like Go on amd64: no FMA contraction).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
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

struct kb_engine {
    int dev = 0;
    hipStream_t st = nullptr;
    bool own_st = false;
    int64_t P = 0, Ppad = 0, B = 0, nsets = 0, tiles = 0;
    int rcap = 0, rc_dev = 1, K = 3, W64 = 1, NP2 = 64;
    int sem = KB_SEM_APPLIED, allow_leader = 0, rebalance = 0;
    int64_t minrep = 2;
    double min_unb = 0.01;
    int64_t shard_begin = 0, shard_end = 0;
    bool integral = false;
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
    int32_t* nc = nullptr;
    double* load = nullptr;
    int32_t* cnt = nullptr;
    uint8_t* incfg = nullptr;
    uint64_t* setbits = nullptr;
    int32_t* lists = nullptr;
    unsigned char* setrec = nullptr;
    int32_t* order = nullptr;
    int32_t* blm = nullptr;
    int32_t* posm = nullptr;
    double* r = nullptr;
    BlockRec* blockrec = nullptr;
    Contender* cont = nullptr;
    uint32_t cont_cap = 1u << 20;
    uint32_t *lstart = nullptr, *llen = nullptr, *lcap = nullptr, *lent = nullptr;
    DevCtl* ctl = nullptr;
    ChangeDev* log = nullptr;
    int logcap = 0;
    DevCtl* h_ctl = nullptr;          // pinned
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0;
    int64_t scan_bytes = 0;
    int exact_unb = 0;
    // per-kernel timing (cfg->time_kernels): one event ring per batch of steps
    int time_kernels = 0;
    std::vector<hipEvent_t> tev;      // 6 events per step
    int tev_used = 0;
    double kms[6] = {0, 0, 0, 0, 0, 0};
    int64_t klaunch[6] = {0, 0, 0, 0, 0, 0};
    std::string last_err;
};

// ------------------------------------------------------------ helpers

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

static const int kRcChoices[] = {1, 2, 3, 4, 6, 8, 12, 16};

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

    // dense broker universe = sorted unique ids (so dense order == BrokerID order)
    std::vector<int64_t> all;
    int64_t nrep_total = n ? c->replica_off[n] - c->replica_off[0] : 0;
    all.reserve((size_t)nrep_total + 64);
    for (int64_t i = 0; i < nrep_total; i++) all.push_back(c->replica_ids[c->replica_off[0] + i]);
    if (c->n_sets > 0 && c->set_off)
        for (int64_t i = c->set_off[0]; i < c->set_off[c->n_sets]; i++) all.push_back(c->set_ids[i]);
    if (!cfg->brokers_nil)
        for (int64_t i = 0; i < cfg->n_brokers; i++) all.push_back(cfg->brokers[i]);
    std::sort(all.begin(), all.end());
    all.erase(std::unique(all.begin(), all.end()), all.end());
    if ((int64_t)all.size() > MAXB) {
        e->last_err = "engine supports at most 4096 distinct brokers";
        *out = e;
        return KB_ERR_UNSUPPORTED;
    }
    e->ids = all;
    e->B = (int64_t)all.size();
    std::unordered_map<int64_t, int> idmap;
    idmap.reserve(all.size() * 2 + 1);
    for (size_t i = 0; i < all.size(); i++) idmap[all[i]] = (int)i;

    // replicas as dense ids, per partition
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
        for (int64_t i = 0; i < n && !e->pending; i++) {
            std::vector<int64_t> r = reps_of(i);
            std::sort(r.begin(), r.end());
            if (std::adjacent_find(r.begin(), r.end()) != r.end()) {
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
        for (int64_t k = c->set_off[s]; k < c->set_off[s + 1]; k++) sets[s].push_back(idmap[c->set_ids[k]]);
    int64_t def_set = -1;
    if (need_default) {
        def_set = nsets_in;
        if (!cfg->brokers_nil) {
            for (int64_t k = 0; k < cfg->n_brokers; k++) sets[def_set].push_back(idmap[cfg->brokers[k]]);
        } else {
            // getBrokerList (utils.go:49-64): every broker holding a replica
            std::vector<char> seen(e->B, 0);
            for (int64_t i = 0; i < nrep_total; i++) seen[idmap[c->replica_ids[c->replica_off[0] + i]]] = 1;
            for (int64_t b = 0; b < e->B; b++) if (seen[b]) sets[def_set].push_back((int)b);
        }
    }
    e->nsets = (int64_t)sets.size();
    if (e->nsets == 0) { sets.emplace_back(); e->nsets = 1; }
    if ((uint64_t)e->nsets >= MAX_SETS) {
        e->last_err = "engine supports at most 32767 distinct broker lists";
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
    std::vector<uint16_t> dense((size_t)nrep_total);
    for (int64_t i = 0; i < n; i++) {
        for (int k = 0; k < len[i]; k++) {
            int b = idmap[rid(i, k)];
            dense[c->replica_off[i] - c->replica_off[0] + k] = (uint16_t)b;
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

    // shard
    e->shard_begin = cfg->shard_begin;
    e->shard_end = (cfg->shard_begin == 0 && cfg->shard_end == 0) ? n : cfg->shard_end;
    if (e->shard_begin < 0 || e->shard_end > n || e->shard_begin > e->shard_end ||
        ((e->shard_begin % TILE) != 0 && e->shard_begin != e->shard_end)) {
        e->last_err = "shard_begin must be a multiple of 1024 and 0 <= begin <= end <= n";
        delete e;
        return KB_ERR_INVALID;
    }
    e->tiles = (e->shard_end - e->shard_begin + TILE - 1) / TILE;
    e->Ppad = ((n + TILE - 1) / TILE) * TILE + TILE;

    // host SoA images
    std::vector<double> hw(e->Ppad, 0.0);
    std::vector<uint32_t> hm(e->Ppad, 0u);
    std::vector<uint16_t> hr((size_t)e->rc_dev * e->Ppad, 0);
    std::vector<int32_t> hnc(e->Ppad, 0);
    for (int64_t i = 0; i < n; i++) {
        hw[i] = wt[i];
        uint32_t elig = want[i] >= e->minrep ? 1u : 0u;
        uint32_t wnt = want[i] < 0 ? 0u : (uint32_t)std::min<int64_t>(want[i], 31);
        for (int k = 0; k < len[i]; k++) hr[(size_t)k * e->Ppad + i] = dense[c->replica_off[i] - c->replica_off[0] + k];
        hnc[i] = (int32_t)ncon[i];
    }
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
        hm[i] = make_meta((uint32_t)len[i], wnt, elig, dis, nin, (uint32_t)pset[i]);
    }
    std::vector<uint8_t> hin(e->B, 0);
    if (!cfg->brokers_nil)
        for (int64_t k = 0; k < cfg->n_brokers; k++) hin[idmap[cfg->brokers[k]]] = 1;

    // per-broker partition lists (non-integral mode), sorted by partition index
    std::vector<uint32_t> hls, hll, hlc, hle;
    if (!e->integral) {
        uint32_t slack = cfg->list_slack > 0 ? (uint32_t)cfg->list_slack : 1024u;
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
    HIPCHK(hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking));
    e->own_st = true;
    HIPCHK(dalloc(&e->w, e->Ppad));
    HIPCHK(dalloc(&e->meta, e->Ppad));
    HIPCHK(dalloc(&e->rep, (size_t)e->rc_dev * e->Ppad));
    HIPCHK(dalloc(&e->nc, e->Ppad));
    HIPCHK(dalloc(&e->load, e->B));
    HIPCHK(dalloc(&e->cnt, e->B));
    HIPCHK(dalloc(&e->incfg, e->B));
    HIPCHK(dalloc(&e->setbits, (size_t)e->nsets * e->W64));
    HIPCHK(dalloc(&e->lists, (size_t)e->nsets * 2 * e->K));
    HIPCHK(dalloc(&e->setrec, (size_t)e->nsets * sr_stride(e->K)));
    HIPCHK(dalloc(&e->order, e->B));
    HIPCHK(dalloc(&e->blm, e->B));
    HIPCHK(dalloc(&e->posm, e->B));
    HIPCHK(dalloc(&e->r, e->B));
    HIPCHK(dalloc(&e->blockrec, e->tiles));
    HIPCHK(dalloc(&e->cont, e->cont_cap));
    HIPCHK(dalloc(&e->ctl, 1));
    e->logcap = 1024;
    HIPCHK(dalloc(&e->log, e->logcap));
    HIPCHK(hipHostMalloc((void**)&e->h_ctl, sizeof(DevCtl), hipHostMallocDefault));
    HIPCHK(hipMemcpy(e->w, hw.data(), hw.size() * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->meta, hm.data(), hm.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->rep, hr.data(), hr.size() * 2, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->nc, hnc.data(), hnc.size() * 4, hipMemcpyHostToDevice));
    if (e->B) {
        HIPCHK(hipMemcpy(e->load, ld.data(), ld.size() * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(e->cnt, cn.data(), cn.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(e->incfg, hin.data(), hin.size(), hipMemcpyHostToDevice));
    }
    HIPCHK(hipMemcpy(e->setbits, hsb.data(), hsb.size() * 8, hipMemcpyHostToDevice));
    if (!e->integral) {
        HIPCHK(dalloc(&e->lstart, e->B));
        HIPCHK(dalloc(&e->llen, e->B));
        HIPCHK(dalloc(&e->lcap, e->B));
        HIPCHK(dalloc(&e->lent, hle.size()));
        if (e->B) {
            HIPCHK(hipMemcpy(e->lstart, hls.data(), hls.size() * 4, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(e->llen, hll.data(), hll.size() * 4, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(e->lcap, hlc.data(), hlc.size() * 4, hipMemcpyHostToDevice));
        }
        HIPCHK(hipMemcpy(e->lent, hle.data(), hle.size() * 4, hipMemcpyHostToDevice));
    }
    DevCtl z;
    memset(&z, 0, sizeof z);
    z.logcap = e->logcap;
    HIPCHK(hipMemcpy(e->ctl, &z, sizeof z, hipMemcpyHostToDevice));
    HIPCHK(hipEventCreate(&e->ev0));
    HIPCHK(hipEventCreate(&e->ev1));
    e->scan_bytes = (e->shard_end - e->shard_begin) * (int64_t)(8 + 4 + 2 * e->rc_dev);
    *out = e;
    return KB_OK;
}

// ---------------------------------------------------------- step launch

static void fill_scan_args(kb_engine* e, ScanArgs& s) {
    s.ctl = e->ctl; s.w = e->w; s.rep = e->rep; s.meta = e->meta;
    s.Ppad = e->Ppad; s.shard_begin = e->shard_begin; s.shard_end = e->shard_end;
    s.K = e->K; s.W64 = e->W64; s.stride = sr_stride(e->K); s.setbits = e->setbits; s.setrec = e->setrec;
    s.r = e->r; s.blm = e->blm; s.posm = e->posm;
    s.allow_leader = e->allow_leader; s.rebalance = e->rebalance; s.sem_go = e->sem == KB_SEM_GO;
    s.blockrec = e->blockrec; s.cont = e->cont; s.cont_cap = e->cont_cap;
}

static void fill_resolve_args(kb_engine* e, ResolveArgs& r) {
    r.ctl = e->ctl; r.w = e->w; r.rep = e->rep; r.meta = e->meta; r.nc = e->nc; r.Ppad = e->Ppad;
    r.RC = e->rc_dev; r.K = e->K; r.W64 = e->W64; r.B = (int)e->B;
    r.setbits = e->setbits; r.lists = e->lists; r.blm = e->blm; r.posm = e->posm; r.r = e->r;
    r.load = e->load; r.cnt = e->cnt; r.cont = e->cont; r.cont_cap = e->cont_cap;
    r.allow_leader = e->allow_leader; r.rebalance = e->rebalance; r.sem_go = e->sem == KB_SEM_GO;
    r.integral = e->integral ? 1 : 0; r.minrep = e->minrep; r.min_unbalance = e->min_unb;
    r.exact_unb = e->exact_unb;
    r.lstart = e->lstart; r.llen = e->llen; r.lcap = e->lcap; r.lent = e->lent; r.log = e->log;
}

static const int kStepBatch = 64;

static void mark(kb_engine* e, int k) {
    if (!e->time_kernels) return;
    if (e->tev.empty()) {
        e->tev.resize((size_t)kStepBatch * 7 + 14);
        for (auto& v : e->tev) hipEventCreate(&v);
    }
    if (e->tev_used < (int)e->tev.size()) hipEventRecord(e->tev[e->tev_used++], e->st);
    (void)k;
}

// accumulate the durations of the marks recorded since the last harvest
static void harvest(kb_engine* e) {
    if (!e->time_kernels || e->tev_used == 0) return;
    hipEventSynchronize(e->tev[e->tev_used - 1]);
    for (int s = 0; s + 6 < e->tev_used; s += 7) {
        for (int k = 0; k < 6; k++) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, e->tev[s + k], e->tev[s + k + 1]) == hipSuccess) {
                e->kms[k] += ms;
                e->klaunch[k]++;
            }
        }
    }
    e->tev_used = 0;
}

// prep + setlists + scan (the local half of a step)
static void enqueue_front(kb_engine* e) {
    PrepArgs pa;
    pa.ctl = e->ctl; pa.load = e->load; pa.cnt = e->cnt; pa.incfg = e->incfg;
    pa.B = (int)e->B; pa.NP2 = e->NP2; pa.order = e->order; pa.blm = e->blm; pa.posm = e->posm;
    pa.r = e->r; pa.rmax_w = e->wmax;
    mark(e, 0);
    launch_prep(pa, e->st);
    mark(e, 1);
    SetArgs sa;
    sa.ctl = e->ctl; sa.nsets = (int)e->nsets; sa.B = (int)e->B; sa.W64 = e->W64; sa.K = e->K;
    sa.stride = sr_stride(e->K); sa.setbits = e->setbits; sa.order = e->order; sa.posm = e->posm;
    sa.cnt = e->cnt; sa.r = e->r; sa.setrec = e->setrec; sa.lists = e->lists;
    launch_setlists(sa, e->st);
    if (e->tiles > 0) {
        ScanArgs s;
        fill_scan_args(e, s);
        mark(e, 2);
        launch_scan(s, e->rc_dev, (int)e->tiles, e->st);
        mark(e, 3);
        ReduceArgs ra;
        ra.ctl = e->ctl; ra.blockrec = e->blockrec; ra.tiles = (int)e->tiles;
        launch_reduce(ra, e->st);
        mark(e, 4);
        launch_census(s, e->rc_dev, (int)e->tiles, e->st);
    } else {
        mark(e, 2);
        mark(e, 3);
        mark(e, 4);
    }
}

static void enqueue_step(kb_engine* e) {
    enqueue_front(e);
    ResolveArgs r;
    fill_resolve_args(e, r);
    mark(e, 5);
    launch_resolve(r, e->st);
    mark(e, 6);
}

static int reset_ctl(kb_engine* e, int logcap) {
    // halted = 0, logpos = 0, logcap
    int32_t hdr[4];
    HIPCHK(hipMemcpyAsync(hdr, e->ctl, sizeof hdr, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    hdr[0] = 0; hdr[2] = 0; hdr[3] = logcap;
    HIPCHK(hipMemcpyAsync(e->ctl, hdr, sizeof hdr, hipMemcpyHostToDevice, e->st));
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

extern "C" int kb_engine_balance(kb_engine* e, kb_change* out) {
    if (!e || !out) return KB_ERR_INVALID;
    if (e->pending) return pending_result(e, out);
    if (reset_ctl(e, e->logcap) != KB_OK) return KB_ERR_HIP;
    HIPCHK(hipEventRecord(e->ev0, e->st));
    enqueue_step(e);
    HIPCHK(hipEventRecord(e->ev1, e->st));
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->st));
    harvest(e);
    float ms = 0;
    hipEventElapsedTime(&ms, e->ev0, e->ev1);
    e->last_ms = ms;
    ChangeDev d;
    HIPCHK(hipMemcpy(&d, e->log, sizeof d, hipMemcpyDeviceToHost));
    return convert(e, d, out);
}

extern "C" int kb_engine_plan(kb_engine* e, int64_t max_steps, kb_change* out, int64_t* n_out) {
    if (!e || !n_out || max_steps < 0) return KB_ERR_INVALID;
    *n_out = 0;
    if (max_steps == 0) return KB_NOCHANGE;
    if (e->pending) { if (out) pending_result(e, out); *n_out = 1; return e->pending; }
    if (max_steps > e->logcap) {
        hipFree(e->log);
        e->logcap = (int)std::min<int64_t>(max_steps, 1 << 30);
        HIPCHK(dalloc(&e->log, e->logcap));
    }
    if (reset_ctl(e, e->logcap) != KB_OK) return KB_ERR_HIP;
    for (int k = 0; k < 6; k++) { e->kms[k] = 0; e->klaunch[k] = 0; }
    e->tev_used = 0;
    HIPCHK(hipEventRecord(e->ev0, e->st));
    int64_t done = 0;
    const int64_t batch = kStepBatch;
    while (done < max_steps) {
        int64_t nb = std::min<int64_t>(batch, max_steps - done);
        for (int64_t s = 0; s < nb; s++) enqueue_step(e);
        done += nb;
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(e->h_ctl, e->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipStreamSynchronize(e->st));
        harvest(e);
        if (e->h_ctl->halted) break;
    }
    HIPCHK(hipEventRecord(e->ev1, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    float ms = 0;
    hipEventElapsedTime(&ms, e->ev0, e->ev1);
    e->last_ms = ms;
    HIPCHK(hipMemcpy(e->h_ctl, e->ctl, sizeof(DevCtl), hipMemcpyDeviceToHost));
    int64_t nlog = std::min<int64_t>(e->h_ctl->logpos, e->logcap);
    std::vector<ChangeDev> logv((size_t)nlog);
    if (nlog) HIPCHK(hipMemcpy(logv.data(), e->log, (size_t)nlog * sizeof(ChangeDev), hipMemcpyDeviceToHost));
    int rc = KB_NOCHANGE;
    int64_t k = 0;
    for (int64_t i = 0; i < nlog; i++) {
        kb_change tmp;
        rc = convert(e, logv[i], out ? &out[k] : &tmp);
        k++;
        if (rc != KB_CHANGE) break;
    }
    *n_out = k;
    return rc;
}

extern "C" int64_t kb_engine_replicas(kb_engine* e, int64_t i, int64_t* buf, int64_t cap) {
    if (!e || i < 0 || i >= e->P) return KB_ERR_INVALID;
    std::vector<int64_t> r;
    if (read_replicas(e, i, r) < 0) return KB_ERR_HIP;
    for (int64_t k = 0; k < (int64_t)r.size() && k < cap; k++) buf[k] = r[k];
    return (int64_t)r.size();
}

extern "C" int64_t kb_engine_loads(kb_engine* e, int64_t* ids, double* loads, int64_t cap) {
    if (!e) return KB_ERR_INVALID;
    std::vector<double> ld(e->B);
    if (e->B && hipMemcpy(ld.data(), e->load, e->B * 8, hipMemcpyDeviceToHost) != hipSuccess) return KB_ERR_HIP;
    for (int64_t k = 0; k < e->B && k < cap; k++) { if (ids) ids[k] = e->ids[k]; if (loads) loads[k] = ld[k]; }
    return e->B;
}

extern "C" double kb_engine_unbalance(kb_engine* e) {
    if (!e || e->B == 0) return 0.0;
    std::vector<double> ld(e->B);
    std::vector<int32_t> cn(e->B);
    std::vector<uint8_t> in(e->B);
    hipMemcpy(ld.data(), e->load, e->B * 8, hipMemcpyDeviceToHost);
    hipMemcpy(cn.data(), e->cnt, e->B * 4, hipMemcpyDeviceToHost);
    hipMemcpy(in.data(), e->incfg, e->B, hipMemcpyDeviceToHost);
    std::vector<int> bl;
    for (int64_t b = 0; b < e->B; b++) if (cn[b] > 0 || in[b]) bl.push_back((int)b);
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
    return KB_OK;
}

extern "C" int kb_engine_timings(kb_engine* e, double* ms, int64_t* launches, int n) {
    if (!e) return KB_ERR_INVALID;
    for (int k = 0; k < 6 && k < n; k++) {
        if (ms) ms[k] = e->kms[k];
        if (launches) launches[k] = e->klaunch[k];
    }
    return 6;
}

extern "C" int kb_engine_stamps(kb_engine* e, uint64_t* out, int n) {
    if (!e || !out) return KB_ERR_INVALID;
    DevCtl c;
    HIPCHK(hipMemcpy(&c, e->ctl, sizeof c, hipMemcpyDeviceToHost));
    for (int k = 0; k < 16 && k < n; k++) out[k] = c.stamps[k];
    return 16;
}

extern "C" int kb_engine_last_error(kb_engine* e, char* buf, size_t n) {
    if (!e || !buf || n == 0) return KB_ERR_INVALID;
    snprintf(buf, n, "%s", e->last_err.c_str());
    return (int)e->last_err.size();
}

extern "C" void kb_engine_destroy(kb_engine* e) {
    if (!e) return;
    void* ptrs[] = {e->w, e->rep, e->meta, e->nc, e->load, e->cnt, e->incfg, e->setbits, e->lists,
                    e->setrec, e->order, e->blm, e->posm, e->r, e->blockrec, e->cont, e->ctl,
                    e->log, e->lstart, e->llen, e->lcap, e->lent};
    for (void* p : ptrs) if (p) hipFree(p);
    if (e->h_ctl) hipHostFree(e->h_ctl);
    if (e->ev0) hipEventDestroy(e->ev0);
    if (e->ev1) hipEventDestroy(e->ev1);
    for (auto v : e->tev) hipEventDestroy(v);
    if (e->own_st && e->st) hipStreamDestroy(e->st);
    delete e;
}

// ----------------------------------------------------- multi-GPU phases

extern "C" int64_t kb_engine_summary_bytes(kb_engine* e) { (void)e; return (int64_t)sizeof(Summary); }

extern "C" int kb_engine_set_stream(kb_engine* e, void* s) {
    if (!e) return KB_ERR_INVALID;
    if (e->own_st && e->st) hipStreamDestroy(e->st);
    e->st = (hipStream_t)s;
    e->own_st = false;
    return KB_OK;
}

extern "C" int kb_engine_step_begin(kb_engine* e, void* summary_dev) {
    if (!e || !summary_dev) return KB_ERR_INVALID;
    if (e->pending) return e->pending;
    if (reset_ctl(e, e->logcap) != KB_OK) return KB_ERR_HIP;
    enqueue_front(e);
    SumArgs s;
    s.ctl = e->ctl; s.cont = e->cont; s.cont_cap = e->cont_cap; s.out = (Summary*)summary_dev;
    launch_summary(s, e->st);
    HIPCHK(hipGetLastError());
    return KB_OK;
}

extern "C" int kb_engine_step_finish(kb_engine* e, const void* gathered_dev, int32_t n_ranks, kb_change* out) {
    if (!e || !gathered_dev || n_ranks < 1 || !out) return KB_ERR_INVALID;
    if (e->pending) return pending_result(e, out);
    MergeArgs m;
    m.ctl = e->ctl; m.all = (const Summary*)gathered_dev; m.nranks = n_ranks; m.cont = e->cont;
    m.cont_cap = e->cont_cap; m.r = e->r;
    launch_merge(m, e->st);
    ResolveArgs r;
    fill_resolve_args(e, r);
    launch_resolve(r, e->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->st));
    ChangeDev d;
    HIPCHK(hipMemcpy(&d, e->log, sizeof d, hipMemcpyDeviceToHost));
    return convert(e, d, out);
}
