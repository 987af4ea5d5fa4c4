// kb_cpu_engine.cpp -- the engine's algorithm on the host CPU (OpenMP), the
// "optimised CPU" baseline of BASELINE.md / SURVEY.md 8(d).  MEASUREMENT
// INFRASTRUCTURE: bench.py's cpu_baseline leg times it; tests/test_cpu_engine.py
// checks its plans against the oracle.  Never used by the product.
//
// Same algorithm as the GPU path (DESIGN.md "Exactness"), restated for a CPU:
//   * loads are the exact getBrokerLoad folds (utils.go:92-105), kept by refolding the
//     touched brokers from partition-ordered per-broker lists after each change;
//   * every (partition, slot) of the step's kind is scored with the O(1) delta
//     d = [f(r_s - delta) - f(r_s)] + [f(r_t + delta) - f(r_t)] against its first
//     allowed non-replica target in bl order (steps.go:167-222), in parallel;
//   * every candidate within 4 eps of the minimum (the rigorous bound of DESIGN.md,
//     exact loads: E = 0) is refolded exactly in the reference's order and the
//     lexicographic (U, iteration index) minimum wins (steps.go:211);
//   * MoveLeaders then MoveNonLeaders (steps.go:284-298), cu < su - MinUnbalance.
//   * the first-index stages before move() (steps.go:70-143): the first partition whose
//     replica count differs from NumReplicas (RemoveExtraReplicas / AddMissingReplicas) or
//     that holds a replica outside its allowed list (MoveDisallowedReplicas), found by a
//     parallel first-index search, then the reference's pick over the allowed list sorted by
//     (load, id) (utils.go:66-90).
// Scope: applied semantics, no ReassignLeaders (create refuses a cluster with an error
// stage: an empty replica list).
#include <omp.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace {

inline double fsq(double r) { const double q = r * r; return r > 0 ? q : q / 2; }

struct Cand {
    double d;
    int32_t s, t;            // dense brokers
    double w;
    uint64_t iter;           // (p << 21) | (slot << 16) | bl position of t
};

struct Engine {
    int64_t P = 0;
    int B = 0, RC = 0;
    std::vector<int64_t> ids;                // dense -> broker id
    std::vector<int32_t> rep;                // [P][RC]
    std::vector<int8_t> nrep;
    std::vector<double> w;
    std::vector<int32_t> nc;
    std::vector<uint8_t> elig;
    std::vector<int32_t> want;               // NumReplicas (after FillDefaults)
    std::vector<int32_t> pset;               // set index
    std::vector<std::vector<uint8_t>> setmask;   // [nsets][B]
    std::vector<uint8_t> incfg;              // -broker-ids member
    std::vector<double> load;
    std::vector<int32_t> cnt;
    std::vector<std::vector<int64_t>> lists; // partition-ordered per-broker lists
    int allow_leader = 0;
    double min_unb = 0.01;
    int threads = 1;
    int64_t cand_total = 0;
};

void refold(Engine& e, int b) {
    double acc = 0.0;
    for (int64_t p : e.lists[b]) {
        const int32_t* r = &e.rep[(size_t)p * e.RC];
        acc += r[0] == b ? e.w[p] * (double)(e.nrep[p] + e.nc[p]) : e.w[p];
    }
    e.load[b] = acc;
}

}  // namespace

extern "C" {

// flat cluster as kb_cluster (include/kbengine.h) after FillDefaults: weights filled,
// num_replicas filled; set_idx < 0 = the default set (cfg brokers or every broker
// holding a replica).  Returns nullptr when the cluster is outside the scope above.
void* cpu_engine_create(int64_t n, const int64_t* rid, const int64_t* roff, const double* weight,
                        const int64_t* num_replicas, const int64_t* num_consumers, int64_t nsets,
                        const int64_t* set_ids, const int64_t* set_off, const int64_t* set_idx,
                        const int64_t* brokers, int64_t nbrokers, int brokers_nil, int allow_leader,
                        int64_t min_replicas, double min_unbalance, int threads) {
    Engine* e = new Engine();
    e->P = n;
    e->allow_leader = allow_leader;
    e->min_unb = min_unbalance;
    e->threads = threads > 0 ? threads : omp_get_max_threads();
    std::vector<int64_t> all(rid, rid + (n ? roff[n] : 0));
    if (nsets > 0) all.insert(all.end(), set_ids, set_ids + set_off[nsets]);
    if (!brokers_nil) all.insert(all.end(), brokers, brokers + nbrokers);
    std::sort(all.begin(), all.end());
    all.erase(std::unique(all.begin(), all.end()), all.end());
    e->ids = all;
    e->B = (int)all.size();
    std::unordered_map<int64_t, int> dm;
    for (int i = 0; i < e->B; i++) dm[all[i]] = i;
    int rc = 1;
    for (int64_t i = 0; i < n; i++)
        rc = std::max<int>(rc, (int)std::max<int64_t>(roff[i + 1] - roff[i], num_replicas[i]));   // (room for adds)
    if (rc > 64) { delete e; return nullptr; }
    e->RC = rc;
    e->rep.assign((size_t)n * rc, -1);
    e->nrep.resize(n); e->w.assign(weight, weight + n); e->nc.assign(n, 0);
    e->elig.resize(n); e->pset.resize(n); e->want.resize(n);
    for (int64_t i = 0; i < n; i++) {
        e->nrep[i] = (int8_t)(roff[i + 1] - roff[i]);
        if (e->nrep[i] == 0) { delete e; return nullptr; }               // (a panic path: not in scope)
        for (int k = 0; k < e->nrep[i]; k++) e->rep[(size_t)i * rc + k] = dm[rid[roff[i] + k]];
        if (num_consumers) e->nc[i] = (int32_t)num_consumers[i];
        e->elig[i] = num_replicas[i] >= min_replicas;
        e->want[i] = (int32_t)num_replicas[i];
    }
    e->incfg.assign(e->B, 0);
    if (!brokers_nil) for (int64_t k = 0; k < nbrokers; k++) e->incfg[dm[brokers[k]]] = 1;
    e->setmask.assign((size_t)nsets + 1, std::vector<uint8_t>(e->B, 0));
    for (int64_t s = 0; s < nsets; s++)
        for (int64_t k = set_off[s]; k < set_off[s + 1]; k++) e->setmask[s][dm[set_ids[k]]] = 1;
    e->load.assign(e->B, 0.0); e->cnt.assign(e->B, 0); e->lists.assign(e->B, {});
    for (int64_t i = 0; i < n; i++)
        for (int k = 0; k < e->nrep[i]; k++) { const int b = e->rep[(size_t)i * rc + k]; e->cnt[b]++; e->lists[b].push_back(i); }
    for (int b = 0; b < e->B; b++) {
        if (!brokers_nil) { if (e->incfg[b]) e->setmask[nsets][b] = 1; }
        else if (e->cnt[b]) e->setmask[nsets][b] = 1;                  // getBrokerList (utils.go:49-64)
        refold(*e, b);
    }
    for (int64_t i = 0; i < n; i++) e->pset[i] = set_idx && set_idx[i] >= 0 ? (int32_t)set_idx[i] : (int32_t)nsets;
    return e;
}

void cpu_engine_destroy(void* h) { delete (Engine*)h; }

int64_t cpu_engine_candidates(void* h) { return ((Engine*)h)->cand_total; }

// One Balance() of the move() steps; returns 1 change (out: kind step 7/8, partition,
// slot, from id, to id, su, cu), 0 no change.
// the brokers of a partition's allowed list sorted by (load, id), brokers absent from the
// load map at 0 (getBrokerListByLoad, utils.go:66-79), or only those holding a replica
// (getBrokerListByLoadBL over getBL, utils.go:81-90)
static std::vector<int> by_load(const Engine& e, int set, bool present_only) {
    std::vector<int> v;
    for (int b = 0; b < e.B; b++)
        if (e.setmask[set][b] && (!present_only || e.cnt[b])) v.push_back(b);
    std::sort(v.begin(), v.end(), [&](int x, int y) {
        const double lx = e.cnt[x] ? e.load[x] : 0.0, ly = e.cnt[y] ? e.load[y] : 0.0;
        return lx != ly ? lx < ly : x < y;
    });
    return v;
}

// the partition's replica list changed: move it between the per-broker lists and refold
// every broker whose contribution changed (the leader's is W * (len(R) + NumConsumers))
static void relist_partition(Engine& e, int64_t p, const std::vector<int>& before) {
    const int32_t* rp = &e.rep[(size_t)p * e.RC];
    std::vector<int> after(rp, rp + e.nrep[p]);
    for (int b : before)
        if (std::find(after.begin(), after.end(), b) == after.end()) {
            auto& l = e.lists[b];
            l.erase(std::lower_bound(l.begin(), l.end(), p));
            e.cnt[b]--;
        }
    for (int b : after)
        if (std::find(before.begin(), before.end(), b) == before.end()) {
            auto& l = e.lists[b];
            l.insert(std::lower_bound(l.begin(), l.end(), p), p);
            e.cnt[b]++;
        }
    std::vector<int> touched(before);
    touched.insert(touched.end(), after.begin(), after.end());
    std::sort(touched.begin(), touched.end());
    touched.erase(std::unique(touched.begin(), touched.end()), touched.end());
    for (int b : touched) refold(e, b);
}

// RemoveExtraReplicas / AddMissingReplicas / MoveDisallowedReplicas (steps.go:70-143):
// 1 = a change (out as cpu_engine_step), 0 = none of them applies, -1 = the reference's error
static int first_index_stages(Engine& e, int64_t* out_i, double* out_d) {
    const int64_t P = e.P;
    int64_t fr = P, fa = P, fd = P;
#pragma omp parallel for num_threads(e.threads) reduction(min : fr, fa, fd) schedule(static)
    for (int64_t p = 0; p < P; p++) {
        if (e.want[p] < e.nrep[p]) fr = std::min(fr, p);
        if (e.want[p] > e.nrep[p]) fa = std::min(fa, p);
        const std::vector<uint8_t>& m = e.setmask[e.pset[p]];
        const int32_t* rp = &e.rep[(size_t)p * e.RC];
        for (int k = 0; k < e.nrep[p]; k++) if (!m[rp[k]]) { fd = std::min(fd, p); break; }
    }
    out_d[0] = out_d[1] = 0.0;
    auto emit = [&](int step, int64_t p, int slot, int from, int to) {
        out_i[0] = step; out_i[1] = p; out_i[2] = slot;
        out_i[3] = from >= 0 ? e.ids[from] : -1; out_i[4] = to >= 0 ? e.ids[to] : -1;
        return 1;
    };
    if (fr < P) {                                    // steps.go:70-89: the lightest allowed replica
        const int64_t p = fr;
        int32_t* rp = &e.rep[(size_t)p * e.RC];
        const std::vector<int> before(rp, rp + e.nrep[p]);
        for (int b : by_load(e, e.pset[p], false)) {
            int slot = -1;
            for (int k = 0; k < e.nrep[p] && slot < 0; k++) if (rp[k] == b) slot = k;
            if (slot < 0) continue;
            for (int k = slot; k + 1 < e.nrep[p]; k++) rp[k] = rp[k + 1];   // replacepl(-1): the first slot
            rp[--e.nrep[p]] = -1;
            relist_partition(e, p, before);
            return emit(3, p, slot, b, -1);
        }
        return -1;
    }
    if (fa < P) {                                    // steps.go:93-113: the heaviest allowed non-replica
        const int64_t p = fa;
        int32_t* rp = &e.rep[(size_t)p * e.RC];
        const std::vector<int> before(rp, rp + e.nrep[p]);
        const std::vector<int> v = by_load(e, e.pset[p], false);
        for (int i = (int)v.size() - 1; i >= 0; i--) {
            const int b = v[i];
            if (std::find(before.begin(), before.end(), b) != before.end()) continue;
            if (e.nrep[p] >= e.RC) return -1;
            rp[e.nrep[p]++] = b;                     // addpl
            relist_partition(e, p, before);
            return emit(4, p, e.nrep[p] - 1, -1, b);
        }
        return -1;
    }
    if (fd < P) {                                    // steps.go:117-143: the heaviest allowed holder
        const int64_t p = fd;
        int32_t* rp = &e.rep[(size_t)p * e.RC];
        const std::vector<int> before(rp, rp + e.nrep[p]);
        const std::vector<int> v = by_load(e, e.pset[p], true);
        const std::vector<uint8_t>& m = e.setmask[e.pset[p]];
        int slot = -1;
        for (int k = 0; k < e.nrep[p] && slot < 0; k++) if (!m[rp[k]] || !e.cnt[rp[k]]) slot = k;
        for (int i = (int)v.size() - 1; i >= 0; i--) {
            const int b = v[i];
            if (std::find(before.begin(), before.end(), b) != before.end()) continue;
            const int from = rp[slot];
            rp[slot] = b;                            // replacepl at the slot
            relist_partition(e, p, before);
            return emit(5, p, slot, from, b);
        }
        return -1;
    }
    return 0;
}

int cpu_engine_step(void* h, int64_t* out_i, double* out_d) {
    Engine& e = *(Engine*)h;
    if (const int r = first_index_stages(e, out_i, out_d); r != 0) return r;
    const int B = e.B, RC = e.RC;
    // bl: brokers in the load map or in -broker-ids (steps.go:150-157), by (load, id)
    std::vector<int> bl;
    for (int b = 0; b < B; b++) if (e.cnt[b] || e.incfg[b]) bl.push_back(b);
    std::sort(bl.begin(), bl.end(), [&](int x, int y) { return e.load[x] != e.load[y] ? e.load[x] < e.load[y] : x < y; });
    const int n = (int)bl.size();
    std::vector<int> pos(B, -1);
    for (int i = 0; i < n; i++) pos[bl[i]] = i;
    std::vector<double> Lm(n);
    for (int i = 0; i < n; i++) Lm[i] = e.load[bl[i]];
    double S = 0;
    for (int i = 0; i < n; i++) S += Lm[i];
    const double avg = S / (double)n;
    double su = 0;
    for (int i = 0; i < n; i++) { const double r = Lm[i] / avg - 1.0; su += r > 0 ? r * r : r * r / 2; }
    const double iav = 1.0 / avg;
    std::vector<double> r(B, 0.0), fr(B, 0.0);
    double V = 0, Rm = 0, U0 = 0, wmax = 0;
    for (int b : bl) {
        r[b] = e.load[b] * iav - 1.0; fr[b] = fsq(r[b]); U0 += fr[b];
        const double ar = std::fabs(r[b]); V += ar * (1 + ar); Rm = std::max(Rm, ar);
    }
    for (int64_t p = 0; p < e.P; p++) wmax = std::max(wmax, e.w[p]);
    const double u = DBL_EPSILON / 2, R = Rm + wmax * iav;
    double eps = 64.0 * u * ((n + 8.0) * (U0 + 2.0 * V) + 4.0 * (1.0 + R) * (1.0 + R));
    if (!(eps > 1e-300)) eps = 1e-300;
    // first members of every set in bl order (the move targets)
    const int nsets = (int)e.setmask.size(), KR = RC + 1;
    std::vector<int> rec((size_t)nsets * KR, -1), nelig(nsets, 0);
    for (int s = 0; s < nsets; s++) {
        int k = 0;
        for (int i = 0; i < n; i++) {
            if (!e.setmask[s][bl[i]]) continue;
            if (k < KR) rec[(size_t)s * KR + k] = bl[i];
            k++;
        }
        nelig[s] = k;
    }
    for (int kind = e.allow_leader ? 0 : 1; kind < 2; kind++) {
        const int T = e.threads;
        std::vector<double> tmin(T, HUGE_VAL);
        std::vector<std::vector<Cand>> tc(T);
        std::vector<int64_t> tcnt(T, 0);
#pragma omp parallel num_threads(T)
        {
            const int t = omp_get_thread_num();
            double mn = HUGE_VAL;
            int64_t cc = 0;
            std::vector<Cand> L;                       // thread-private (no false sharing)
#pragma omp for schedule(static)
            for (int64_t p = 0; p < e.P; p++) {
                if (!e.elig[p] || e.nrep[p] == 0) continue;
                const int32_t* rp = &e.rep[(size_t)p * RC];
                const int s0 = e.pset[p];
                const std::vector<uint8_t>& m = e.setmask[s0];
                int nin = 0;
                for (int k = 0; k < e.nrep[p]; k++) nin += m[rp[k]];
                const int ne = nelig[s0] - nin;
                const double delta = e.w[p] * iav;
                const int lo = kind == 0 ? 0 : 1, hi = kind == 0 ? 1 : e.nrep[p];
                for (int slot = lo; slot < hi; slot++) {
                    cc += ne > 0 ? ne : 0;
                    const int src = rp[slot];
                    const double ds = fsq(r[src] - delta) - fr[src];
                    // walk the set in bl order: first target, then any near-tied ones
                    const int* rr = &rec[(size_t)s0 * KR];
                    int i = 0, k = 0, b = -1;
                    for (;;) {
                        if (k < KR) { b = rr[k]; if (b < 0) break; }
                        else {                                  // past the record: continue in bl order
                            int q = (b >= 0 ? pos[b] : -1) + 1;
                            while (q < n && !m[bl[q]]) q++;
                            if (q >= n) break;
                            b = bl[q];
                        }
                        k++;
                        bool isrep = false;
                        for (int x = 0; x < e.nrep[p]; x++) isrep |= rp[x] == b;
                        if (isrep) continue;
                        const double d = ds + (fsq(r[b] + delta) - fr[b]);
                        i++;
                        if (d < mn) {
                            mn = d;
                            L.erase(std::remove_if(L.begin(), L.end(), [&](const Cand& c) { return c.d > mn + 4 * eps; }), L.end());
                        }
                        if (d <= mn + 4 * eps)
                            L.push_back(Cand{d, src, b, e.w[p], ((uint64_t)p << 21) | ((uint64_t)slot << 16) | (uint64_t)pos[b]});
                        if (d > mn + 8 * eps) break;            // monotone in the target load up to 2 eps
                    }
                    (void)i;
                }
            }
            tmin[t] = mn;
            tcnt[t] = cc;
            tc[t].swap(L);
        }
        double g = HUGE_VAL;
        for (int t = 0; t < T; t++) { g = std::min(g, tmin[t]); e.cand_total += tcnt[t]; }
        // contenders: exact folds in the reference's order (utils.go:119-147), one per key
        double bu = su;
        Cand best{0, -1, -1, 0, ~0ull};
        bool improved = false;
        std::map<std::tuple<int32_t, int32_t, uint64_t>, double> seen;    // (s, t, w bits) -> exact U
        std::vector<Cand> all;
        for (auto& L : tc) for (auto& c : L) if (c.d <= g + 4 * eps) all.push_back(c);
        std::sort(all.begin(), all.end(), [](const Cand& a, const Cand& b) { return a.iter < b.iter; });
        for (const Cand& c : all) {
            uint64_t wb; std::memcpy(&wb, &c.w, 8);
            const auto key = std::make_tuple(c.s, c.t, wb);
            double U;
            auto it = seen.find(key);
            if (it != seen.end()) U = it->second;
            else {
                const int ps = pos[c.s], pt = pos[c.t];
                double S2 = 0;
                for (int i2 = 0; i2 < n; i2++) S2 += i2 == ps ? Lm[i2] - c.w : (i2 == pt ? Lm[i2] + c.w : Lm[i2]);
                const double a2 = S2 / (double)n;
                U = 0;
                for (int i2 = 0; i2 < n; i2++) {
                    const double L2 = i2 == ps ? Lm[i2] - c.w : (i2 == pt ? Lm[i2] + c.w : Lm[i2]);
                    const double rr2 = L2 / a2 - 1.0;
                    U += rr2 > 0 ? rr2 * rr2 : rr2 * rr2 / 2;
                }
                seen.emplace(key, U);
            }
            if (U < bu) { bu = U; best = c; improved = true; }   // strict <: first minimum in order
        }
        const double cu = bu;
        if (cu < su - e.min_unb && improved) {
            const int64_t p = (int64_t)(best.iter >> 21);
            const int slot = (int)((best.iter >> 16) & 31);
            int32_t* rp = &e.rep[(size_t)p * RC];
            const int from = rp[slot], to = best.t;
            rp[slot] = to;                                       // replacepl (utils.go:186-190)
            auto& lf = e.lists[from];
            lf.erase(std::lower_bound(lf.begin(), lf.end(), p));
            auto& lt = e.lists[to];
            lt.insert(std::lower_bound(lt.begin(), lt.end(), p), p);
            e.cnt[from]--; e.cnt[to]++;
            refold(e, from); refold(e, to);
            out_i[0] = kind == 0 ? 7 : 8; out_i[1] = p; out_i[2] = slot; out_i[3] = e.ids[from]; out_i[4] = e.ids[to];
            out_d[0] = su; out_d[1] = cu;
            return 1;
        }
    }
    return 0;
}

}  // extern "C"
