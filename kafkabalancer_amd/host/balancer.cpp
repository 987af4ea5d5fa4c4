// balancer.cpp -- host side of the boundary: marshals the PartitionList into
// kb_cluster, drives kb_engine_* and mirrors each change into pl with the
// reference's slice semantics (utils.go:166-202).
#include "balancer.hpp"

#include <algorithm>
#include <unordered_set>
#include <map>

namespace kbh {

static const char* kSteps[9] = {"ValidateWeights", "ValidateReplicas", "FillDefaults",
                                "RemoveExtraReplicas", "AddMissingReplicas", "MoveDisallowedReplicas",
                                "ReassignLeaders", "MoveLeaders", "MoveNonLeaders"};

Planner::Planner(PartitionList& pl, const RebalanceConfig& cfg, int semantics, int device)
    : pl_(pl), cfg_(cfg), sem_(semantics) {
    const size_t n = pl.partitions.size();
    std::vector<int64_t> rep, roff(n + 1, 0), nr(n), ncons(n), pid(n), sidx(n, -1), sids, soff{0}, toff(n + 1, 0);
    std::vector<double> w(n);
    std::string blob;
    std::map<std::vector<int64_t>, int64_t> sets;
    for (size_t i = 0; i < n; i++) {
        const Partition& p = pl.partitions[i];
        for (size_t k = 0; k < p.replicas.len; k++) rep.push_back(p.replicas.at(k));
        roff[i + 1] = (int64_t)rep.size();
        w[i] = p.weight;
        nr[i] = p.num_replicas;
        ncons[i] = p.num_consumers;
        pid[i] = p.partition;
        blob += p.topic;
        toff[i + 1] = (int64_t)blob.size();
        if (!p.brokers.nil()) {
            std::vector<int64_t> b = p.brokers.values();
            auto it = sets.find(b);
            if (it == sets.end()) {
                it = sets.emplace(b, (int64_t)sets.size()).first;
                sids.insert(sids.end(), b.begin(), b.end());
                soff.push_back((int64_t)sids.size());
            }
            sidx[i] = it->second;
        }
    }
    if (rep.empty()) rep.push_back(0);
    if (sids.empty()) sids.push_back(0);
    kb_cluster c{};
    c.n_partitions = (int64_t)n;
    c.replica_ids = rep.data();
    c.replica_off = roff.data();
    c.weight = w.data();
    c.num_replicas = nr.data();
    c.num_consumers = ncons.data();
    c.n_sets = (int64_t)sets.size();
    c.set_ids = sids.data();
    c.set_off = soff.data();
    c.set_idx = sidx.data();
    c.topic_blob = blob.c_str();
    c.topic_off = toff.data();
    c.partition_id = pid.data();
    kb_config k{};
    k.allow_leader = cfg.allow_leader;
    k.rebalance_leaders = cfg.rebalance_leaders;
    k.min_replicas = cfg.min_replicas;
    k.min_unbalance = cfg.min_unbalance;
    k.brokers = cfg.brokers.empty() ? nullptr : cfg.brokers.data();
    k.n_brokers = (int64_t)cfg.brokers.size();
    k.brokers_nil = cfg.brokers_nil;
    k.semantics = semantics;
    k.device = device;
    int rc = kb_engine_create(&c, &k, &eng_);
    if (rc < 0) {
        char buf[1024] = {0};
        if (eng_) kb_engine_last_error(eng_, buf, sizeof buf);
        create_err_ = std::string("engine: ") + (buf[0] ? buf : "kb_engine_create failed") +
                      " (code " + std::to_string(rc) + ")";
        if (eng_) kb_engine_destroy(eng_);
        eng_ = nullptr;
    }
}

Planner::~Planner() {
    if (eng_) kb_engine_destroy(eng_);
}

// FillDefaults (steps.go:39-66) on the host mirror; the engine did the same
void Planner::fill_defaults() {
    if (filled_ || pl_.partitions.empty()) return;
    filled_ = true;
    if (pl_.partitions[0].weight == 0)
        for (auto& p : pl_.partitions) p.weight = 1.0;
    // (the default list only when some partition has none: c3's partitions all carry
    // their own, and collecting + sorting every replica id cost 0.1 s of the plan)
    bool need = false;
    for (auto& p : pl_.partitions) if (p.brokers.nil()) { need = true; break; }
    Slice brokers;
    if (need && !cfg_.brokers_nil) {
        brokers = Slice::of(cfg_.brokers);
    } else if (need) {
        std::unordered_set<int64_t> seen;
        for (auto& p : pl_.partitions)
            for (size_t k = 0; k < p.replicas.len; k++) seen.insert(p.replicas.at(k));
        std::vector<int64_t> all(seen.begin(), seen.end());
        std::sort(all.begin(), all.end());
        if (!all.empty()) brokers = Slice::of(all);           // getBrokerList: nil when empty
    }
    if (need)
        for (auto& p : pl_.partitions)
            if (p.brokers.nil()) p.brokers = brokers;
    for (auto& p : pl_.partitions)
        if (p.num_replicas == 0) p.num_replicas = (int64_t)p.replicas.len;
}

StepResult Planner::apply(const kb_change& ch, int rc) {
    StepResult r;
    r.status = rc;
    r.change = ch;
    r.step = ch.step >= 0 && ch.step < 9 ? kSteps[ch.step] : "";
    if (rc < 0) {
        char buf[2048] = {0};
        kb_engine_last_error(eng_, buf, sizeof buf);
        r.err = buf;
        return r;
    }
    fill_defaults();
    if (rc == KB_NOCHANGE) return r;
    Partition& p = pl_.partitions[(size_t)ch.partition];
    Partition ret = p;                                         // Go passes Partition by value
    const size_t slot = (size_t)ch.slot;
    switch (ch.kind) {
        case KB_KIND_REPLACE:                                  // utils.go:186-190
            p.replicas.at(slot) = ch.to_broker;
            break;
        case KB_KIND_SWAP: {                                   // utils.go:179-185
            size_t ex = 0;
            for (size_t k = 0; k < p.replicas.len; k++) if (p.replicas.at(k) == ch.to_broker) { ex = k; break; }
            int64_t old = p.replicas.at(slot);
            p.replicas.at(slot) = ch.to_broker;
            p.replicas.at(ex) = old;
            break;
        }
        case KB_KIND_REMOVE:                                   // utils.go:176-178 (in-place shift)
            for (size_t k = slot; k + 1 < p.replicas.len; k++) p.replicas.at(k) = p.replicas.at(k + 1);
            ret.replicas.len = p.replicas.len - 1;
            if (sem_ == KB_SEM_APPLIED) p.replicas.len -= 1;
            break;
        case KB_KIND_ADD: {                                    // utils.go:199-202
            std::vector<int64_t> v = p.replicas.values();
            v.push_back(ch.to_broker);
            ret.replicas = Slice::of(v);
            if (sem_ == KB_SEM_APPLIED) p.replicas = ret.replicas;
            break;
        }
        default:
            break;
    }
    if (ch.kind != KB_KIND_REMOVE && ch.kind != KB_KIND_ADD) ret.replicas = p.replicas;
    else if (ch.kind == KB_KIND_REMOVE) ret.replicas.arr = p.replicas.arr;
    ret.weight = p.weight;
    ret.num_replicas = p.num_replicas;
    ret.brokers = p.brokers;
    r.part = ret;
    return r;
}

StepResult Planner::Step() {
    kb_change ch{};
    int rc = kb_engine_balance(eng_, &ch);
    return apply(ch, rc);
}

std::vector<StepResult> Planner::Plan(int64_t n) { return PlanUntil(n, -1); }

std::vector<StepResult> Planner::PlanUntil(int64_t n, int64_t pidx) {
    // in chunks: the change buffer stays bounded whatever -max-reassign asks for
    // (the reference loops until no change, kafkabalancer.go:177-233)
    constexpr int64_t kChunk = 4096;
    std::vector<StepResult> out;
    std::vector<kb_change> chs((size_t)std::min<int64_t>(std::max<int64_t>(n, 0), kChunk));
    while (n > 0) {
        const int64_t m = std::min<int64_t>(n, kChunk);
        int64_t got = 0;
        int rc = kb_engine_plan_until(eng_, m, pidx, chs.data(), &got);
        for (int64_t i = 0; i < got; i++) {
            int s = chs[(size_t)i].status;
            int r = s == KB_CHANGE ? KB_CHANGE : (s == KB_NOCHANGE ? KB_NOCHANGE : rc);
            out.push_back(apply(chs[(size_t)i], r));
            if (r != KB_CHANGE) return out;
            if (pidx >= 0 && chs[(size_t)i].partition != pidx) return out;
        }
        if (got == 0) {
            if (rc < 0) {
                kb_change z{};
                z.status = rc;
                out.push_back(apply(z, rc));
            }
            return out;
        }
        n -= got;
    }
    return out;
}

StepResult Balance(PartitionList& pl, const RebalanceConfig& cfg, int semantics) {
    Planner pln(pl, cfg, semantics);
    if (!pln.ok()) {
        StepResult r;
        r.status = KB_ERR_HIP;
        r.err = pln.error();
        return r;
    }
    return pln.Step();
}

}  // namespace kbh
