// balancer.hpp -- Balance() (balancer.go:49-65) and run()'s plan loop on top of
// the MI355X engine's C ABI (include/kbengine.h).
#pragma once
#include <string>
#include <vector>

#include "../../include/kbengine.h"
#include "model.hpp"

namespace kbh {

struct StepResult {
    int status = 0;             // KB_CHANGE / KB_NOCHANGE / < 0 error
    std::string step;           // step that produced the change or the error
    Partition part;             // the returned partition (aliases pl like the reference)
    std::string err;            // "<Step>: <message>" (Balance error text)
    kb_change change{};
};

// The resident engine for one PartitionList.  pl is mutated exactly as the
// reference mutates it: FillDefaults (steps.go:39-66) and the aliasing writes
// of replacepl/addpl (utils.go:166-202) per the chosen semantics.
class Planner {
public:
    Planner(PartitionList& pl, const RebalanceConfig& cfg, int semantics, int device = 0);
    ~Planner();
    bool ok() const { return eng_ != nullptr; }
    const std::string& error() const { return create_err_; }
    // one Balance() call
    StepResult Step();
    // up to n Balance() calls device-resident; stops after a no-change or error
    std::vector<StepResult> Plan(int64_t n);
    // ... and after the first change on a partition other than pidx (kb_engine_plan_until:
    // the -complete-partition loop, kafkabalancer.go:193-221)
    std::vector<StepResult> PlanUntil(int64_t n, int64_t pidx);

private:
    StepResult apply(const kb_change& ch, int rc);
    void fill_defaults();
    PartitionList& pl_;
    RebalanceConfig cfg_;
    int sem_;
    kb_engine* eng_ = nullptr;
    bool filled_ = false;
    std::string create_err_;
};

// Balance(pl, cfg): one step on a fresh engine (faithful to the reference API,
// which takes the list each call); the resident Planner is the fast path.
StepResult Balance(PartitionList& pl, const RebalanceConfig& cfg, int semantics = KB_SEM_GO);

}  // namespace kbh
