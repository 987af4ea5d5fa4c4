/*
 * kb_oracle.c -- CPU restatement of the kjelle/kafkabalancer balancer.
 *
 * TEST INFRASTRUCTURE ONLY (see kb_oracle.h).  Follows, line by line in
 * behaviour, the reference Go sources:
 *   utils.go:19-28   byBrokerLoad order (load asc, id asc)
 *   utils.go:39-47   inBrokerList (linear)
 *   utils.go:49-64   getBrokerList
 *   utils.go:66-90   getBrokerListByLoad / getBrokerListByLoadBL
 *   utils.go:92-105  getBrokerLoad (fold in partition order)
 *   utils.go:107-117 getBL
 *   utils.go:119-147 getUnbalanceBL (sequential folds, IEEE division)
 *   utils.go:149-202 emptypl / singlepl / findBrokerPos / replacepl / addpl
 *   steps.go:7-307   the nine steps, move() and distributeLeaders()
 *   balancer.go:34-65 steps table and Balance()
 *   kafkabalancer.go:177-233 run() main loop; codecs.go:67-93 filter/write
 *
 * Build with -O2 -ffp-contract=off (no FMA contraction, no fast-math) so that
 * every float64 operation rounds exactly like Go on amd64 (GOAMD64=v1).
 */
#include "kb_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

/* ------------------------------------------------------------------ slices */

static or_slice sl_make(int64_t len, int64_t cap) {
    or_slice s; s.len = len; s.cap = cap < len ? len : cap;
    s.a = (int64_t *)calloc((size_t)(s.cap ? s.cap : 1), sizeof(int64_t));
    return s;
}

/* Go append() of one element (growth => fresh backing array) */
static or_slice sl_append(or_slice s, int64_t v) {
    if (s.a != NULL && s.len < s.cap) { s.a[s.len] = v; s.len++; return s; }
    int64_t ncap = s.cap < 4 ? 4 : s.cap * 2;
    or_slice n = sl_make(s.len + 1, ncap);
    if (s.len) memcpy(n.a, s.a, (size_t)s.len * sizeof(int64_t));
    n.a[s.len] = v;
    return n;
}

/* ----------------------------------------------------------- formatting */

/* Partition.String() = fmt.Sprintf("Partition(%s,%d,%+v)") (kafkabalancer.go:64-66) */
static void part_string(const or_partition *p, char *buf, size_t n) {
    size_t o = (size_t)snprintf(buf, n, "Partition(%s,%lld,[", p->topic, (long long)p->partition);
    for (int64_t i = 0; i < p->replicas.len && o < n; i++)
        o += (size_t)snprintf(buf + o, n - o, i ? " %lld" : "%lld", (long long)p->replicas.a[i]);
    if (o < n) snprintf(buf + o, n - o, "])");
}

static const char *step_names[9] = {
    "ValidateWeights", "ValidateReplicas", "FillDefaults", "RemoveExtraReplicas",
    "AddMissingReplicas", "MoveDisallowedReplicas", "ReassignLeaders",
    "MoveLeaders", "MoveNonLeaders"};

/* --------------------------------------------------------- broker loads */

typedef struct { int64_t id; double load; } bload;

typedef struct {            /* tiny open-addressing map BrokerID -> slot */
    int64_t *keys; int32_t *vals; int64_t cap;
    int64_t *ids; double *loads; int64_t n, ncap;
} lmap;

static void lm_init(lmap *m, int64_t hint) {
    int64_t cap = 64; while (cap < hint * 2) cap <<= 1;
    m->cap = cap; m->keys = (int64_t *)malloc((size_t)cap * sizeof(int64_t));
    m->vals = (int32_t *)malloc((size_t)cap * sizeof(int32_t));
    for (int64_t i = 0; i < cap; i++) m->vals[i] = -1;
    m->ncap = 16; m->n = 0;
    m->ids = (int64_t *)malloc((size_t)m->ncap * sizeof(int64_t));
    m->loads = (double *)malloc((size_t)m->ncap * sizeof(double));
}
static void lm_free(lmap *m) { free(m->keys); free(m->vals); free(m->ids); free(m->loads); }
static uint64_t hmix(uint64_t x) { x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33; return x; }
static void lm_grow(lmap *m);
static int32_t lm_find(const lmap *m, int64_t id) {
    uint64_t h = hmix((uint64_t)id) & (uint64_t)(m->cap - 1);
    for (;;) {
        if (m->vals[h] < 0) return -1;
        if (m->keys[h] == id) return m->vals[h];
        h = (h + 1) & (uint64_t)(m->cap - 1);
    }
}
/* returns slot, inserting load 0 if absent (Go map zero value) */
static int32_t lm_slot(lmap *m, int64_t id) {
    int32_t f = lm_find(m, id);
    if (f >= 0) return f;
    if ((m->n + 1) * 2 > m->cap) lm_grow(m);
    uint64_t h = hmix((uint64_t)id) & (uint64_t)(m->cap - 1);
    while (m->vals[h] >= 0) h = (h + 1) & (uint64_t)(m->cap - 1);
    if (m->n == m->ncap) {
        m->ncap *= 2;
        m->ids = (int64_t *)realloc(m->ids, (size_t)m->ncap * sizeof(int64_t));
        m->loads = (double *)realloc(m->loads, (size_t)m->ncap * sizeof(double));
    }
    m->keys[h] = id; m->vals[h] = (int32_t)m->n;
    m->ids[m->n] = id; m->loads[m->n] = 0.0;
    return (int32_t)m->n++;
}
static void lm_grow(lmap *m) {
    int64_t ncap = m->cap * 2;
    free(m->keys); free(m->vals);
    m->cap = ncap; m->keys = (int64_t *)malloc((size_t)ncap * sizeof(int64_t));
    m->vals = (int32_t *)malloc((size_t)ncap * sizeof(int32_t));
    for (int64_t i = 0; i < ncap; i++) m->vals[i] = -1;
    for (int64_t i = 0; i < m->n; i++) {
        uint64_t h = hmix((uint64_t)m->ids[i]) & (uint64_t)(ncap - 1);
        while (m->vals[h] >= 0) h = (h + 1) & (uint64_t)(ncap - 1);
        m->keys[h] = m->ids[i]; m->vals[h] = (int32_t)i;
    }
}

/* getBrokerLoad (utils.go:92-105): per-broker fold in partition order */
static void get_broker_load(const or_plist *pl, lmap *m) {
    lm_init(m, 64);
    for (int64_t i = 0; i < pl->n; i++) {
        const or_partition *p = &pl->parts[i];
        for (int64_t k = 0; k < p->replicas.len; k++) {
            int32_t s = lm_slot(m, p->replicas.a[k]);
            if (k == 0)
                m->loads[s] += p->weight * (double)(p->replicas.len + p->num_consumers);
            else
                m->loads[s] += p->weight;
        }
    }
}

static int bload_less(const bload *a, const bload *b) {   /* utils.go:23-28 */
    if (a->load != b->load) return a->load < b->load;
    return a->id < b->id;
}
static int bload_cmp(const void *x, const void *y) {
    const bload *a = (const bload *)x, *b = (const bload *)y;
    if (bload_less(a, b)) return -1;
    if (bload_less(b, a)) return 1;
    return 0;
}

/* getBL (utils.go:107-117) */
static bload *get_bl(const lmap *m, int64_t *n) {
    bload *bl = (bload *)malloc((size_t)(m->n ? m->n : 1) * sizeof(bload));
    for (int64_t i = 0; i < m->n; i++) { bl[i].id = m->ids[i]; bl[i].load = m->loads[i]; }
    qsort(bl, (size_t)m->n, sizeof(bload), bload_cmp);
    *n = m->n;
    return bl;
}

/* getUnbalanceBL (utils.go:119-147) */
static double unbalance_bl(const bload *bl, int64_t n) {
    double sum = 0, maxl = 0;
    for (int64_t i = 0; i < n; i++) { sum += bl[i].load; if (maxl < bl[i].load) maxl = bl[i].load; }
    double avg = sum / (double)n;
    double u = 0;
    for (int64_t i = 0; i < n; i++) {
        double r = bl[i].load / avg - 1.0;
        if (r > 0) u += r * r;
        else u += r * r / 2;
    }
    (void)maxl;
    return u;
}

double or_unbalance(const double *loads, int64_t n) {
    double sum = 0;
    for (int64_t i = 0; i < n; i++) sum += loads[i];
    double avg = sum / (double)n, u = 0;
    for (int64_t i = 0; i < n; i++) {
        double r = loads[i] / avg - 1.0;
        if (r > 0) u += r * r; else u += r * r / 2;
    }
    return u;
}

static int in_list(const int64_t *h, int64_t n, int64_t needle) {   /* utils.go:39-47 */
    for (int64_t i = 0; i < n; i++) if (h[i] == needle) return 1;
    return 0;
}

/* getBrokerListByLoad (utils.go:66-79): p.Brokers sorted by (loads[id] or 0, id) */
static int64_t *by_load(const lmap *m, const or_slice *brokers) {
    int64_t n = brokers->len;
    bload *b = (bload *)malloc((size_t)(n ? n : 1) * sizeof(bload));
    for (int64_t i = 0; i < n; i++) {
        int32_t s = lm_find(m, brokers->a[i]);
        b[i].id = brokers->a[i]; b[i].load = s >= 0 ? m->loads[s] : 0.0;
    }
    qsort(b, (size_t)n, sizeof(bload), bload_cmp);
    int64_t *r = (int64_t *)malloc((size_t)(n ? n : 1) * sizeof(int64_t));
    for (int64_t i = 0; i < n; i++) r[i] = b[i].id;
    free(b);
    return r;
}

/* ------------------------------------------------------ result builders */

static void set_err(or_result *res, int step, const char *msg) {
    res->status = -1; res->step = step;
    snprintf(res->err, sizeof res->err, "%s: %s", step_names[step], msg);
}

/* replacepl (utils.go:166-197) on the Go value copy *p (shares the backing
 * array with pl); then, for OR_SEM_APPLIED, make pl's header follow. */
static int replacepl(or_plist *pl, int64_t pidx, int64_t orig, int64_t repl, int sem,
                     or_result *res, int step, int kind) {
    or_partition p = pl->parts[pidx];          /* Go passes Partition by value */
    for (int64_t idx = 0; idx < p.replicas.len; idx++) {
        if (p.replicas.a[idx] != orig) continue;
        res->slot = idx;
        if (repl == -1) {
            /* p.Replicas = append(p.Replicas[:idx], p.Replicas[idx+1:]...) : in-place shift */
            for (int64_t k = idx; k + 1 < p.replicas.len; k++) p.replicas.a[k] = p.replicas.a[k + 1];
            p.replicas.len -= 1;
            if (sem == OR_SEM_APPLIED) pl->parts[pidx].replicas.len -= 1;
            kind = OR_REMOVE;
        } else {
            int64_t existing = -1;
            for (int64_t k = 0; k < p.replicas.len; k++) if (p.replicas.a[k] == repl) { existing = k; break; }
            if (existing > -1) {
                int64_t e = p.replicas.a[idx];
                p.replicas.a[idx] = repl;
                p.replicas.a[existing] = e;
                kind = OR_SWAP;
            } else {
                p.replicas.a[idx] = repl;
            }
        }
        res->status = 1; res->step = step; res->pidx = pidx; res->kind = kind;
        res->from = orig; res->to = repl; res->part = p;
        return 1;
    }
    /* panic(fmt.Sprintf("partition %v replicas don't contain %d")) */
    char ps[512]; part_string(&p, ps, sizeof ps);
    char m[700]; snprintf(m, sizeof m, "panic: partition %s replicas don't contain %lld", ps, (long long)orig);
    set_err(res, step, m);
    return -1;
}

static int addpl(or_plist *pl, int64_t pidx, int64_t b, int sem, or_result *res, int step) {
    or_partition p = pl->parts[pidx];
    p.replicas = sl_append(p.replicas, b);           /* utils.go:199-202 */
    if (sem == OR_SEM_APPLIED) pl->parts[pidx].replicas = p.replicas;
    res->status = 1; res->step = step; res->pidx = pidx; res->kind = OR_ADD;
    res->from = -1; res->to = b; res->slot = p.replicas.len - 1; res->part = p;
    return 1;
}

/* ------------------------------------------------------------- the steps */

static int g_threads = 1;                 /* see or_set_threads (move_impl) */
void or_set_threads(int n) { g_threads = n < 1 ? 1 : n; }

static int validate_weights(or_plist *pl, or_result *res) {      /* steps.go:7-23 */
    char ps[512], m[700];
    int has = pl->parts[0].weight != 0;
    for (int64_t i = 0; i < pl->n; i++) {
        const or_partition *p = &pl->parts[i];
        if (has && p->weight == 0) {
            part_string(p, ps, sizeof ps); snprintf(m, sizeof m, "partition %s has no weight", ps);
            set_err(res, 0, m); return -1;
        }
        if (!has && p->weight != 0) {
            part_string(&pl->parts[0], ps, sizeof ps); snprintf(m, sizeof m, "partition %s has no weight", ps);
            set_err(res, 0, m); return -1;
        }
        if (p->weight < 0) {
            part_string(p, ps, sizeof ps); snprintf(m, sizeof m, "partition %s has negative weight", ps);
            set_err(res, 0, m); return -1;
        }
    }
    return 0;
}

static int validate_replicas(or_plist *pl, or_result *res) {     /* steps.go:27-36 */
    for (int64_t i = 0; i < pl->n; i++) {
        const or_partition *p = &pl->parts[i];
        int64_t distinct = 0;
        for (int64_t a = 0; a < p->replicas.len; a++) {
            int dup = 0;
            for (int64_t b = 0; b < a; b++) if (p->replicas.a[b] == p->replicas.a[a]) { dup = 1; break; }
            if (!dup) distinct++;
        }
        if (distinct != p->replicas.len) {
            char ps[512], m[700]; part_string(p, ps, sizeof ps);
            snprintf(m, sizeof m, "partition %s has duplicated replicas", ps);
            set_err(res, 1, m); return -1;
        }
    }
    return 0;
}

static int cmp_i64(const void *x, const void *y) {
    int64_t a = *(const int64_t *)x, b = *(const int64_t *)y;
    return a < b ? -1 : a > b;
}

static void fill_defaults(or_plist *pl, const or_config *cfg) {   /* steps.go:39-66 */
    if (pl->parts[0].weight == 0)
        for (int64_t i = 0; i < pl->n; i++) pl->parts[i].weight = 1.0;
    int any_nil = 0;
    for (int64_t i = 0; i < pl->n && !any_nil; i++) any_nil = pl->parts[i].brokers.a == NULL;
    if (!any_nil) goto num_replicas;
    or_slice brokers;
    if (!cfg->brokers_nil) {
        /* Go shares cfg.Brokers' backing array (alive for the whole run); the caller's
         * or_config may not outlive this call, so the list owns a copy */
        brokers = sl_make(cfg->nbrokers, cfg->nbrokers);
        if (cfg->nbrokers) memcpy(brokers.a, cfg->brokers, (size_t)cfg->nbrokers * sizeof(int64_t));
    } else {                                          /* getBrokerList (utils.go:49-64) */
        lmap m; lm_init(&m, 64);
        for (int64_t i = 0; i < pl->n; i++)
            for (int64_t k = 0; k < pl->parts[i].replicas.len; k++) lm_slot(&m, pl->parts[i].replicas.a[k]);
        if (m.n == 0) { brokers.a = NULL; brokers.len = brokers.cap = 0; }
        else {
            brokers = sl_make(m.n, m.n);
            memcpy(brokers.a, m.ids, (size_t)m.n * sizeof(int64_t));
            qsort(brokers.a, (size_t)m.n, sizeof(int64_t), cmp_i64);
        }
        lm_free(&m);
    }
    for (int64_t i = 0; i < pl->n; i++)
        if (pl->parts[i].brokers.a == NULL) pl->parts[i].brokers = brokers;
num_replicas:
    for (int64_t i = 0; i < pl->n; i++)
        if (pl->parts[i].num_replicas == 0) pl->parts[i].num_replicas = pl->parts[i].replicas.len;
}

static int remove_extra(or_plist *pl, int sem, or_result *res) {  /* steps.go:70-89 */
    lmap m; get_broker_load(pl, &m);
    int rc = 0;
    for (int64_t i = 0; i < pl->n && rc == 0; i++) {
        or_partition *p = &pl->parts[i];
        if (p->num_replicas >= p->replicas.len) continue;
        int64_t *bb = by_load(&m, &p->brokers);
        int64_t b = 0; int found = 0;
        for (int64_t k = 0; k < p->brokers.len; k++)
            if (in_list(p->replicas.a, p->replicas.len, bb[k])) { b = bb[k]; found = 1; break; }
        free(bb);
        if (found) rc = replacepl(pl, i, b, -1, sem, res, 3, OR_REMOVE);
        else {
            char ps[512], msg[700]; part_string(p, ps, sizeof ps);
            snprintf(msg, sizeof msg, "partition %s unable to pick replica to remove", ps);
            set_err(res, 3, msg); rc = -1;
        }
    }
    lm_free(&m);
    return rc;
}

static int add_missing(or_plist *pl, int sem, or_result *res) {   /* steps.go:93-113 */
    lmap m; get_broker_load(pl, &m);
    int rc = 0;
    for (int64_t i = 0; i < pl->n && rc == 0; i++) {
        or_partition *p = &pl->parts[i];
        if (p->num_replicas <= p->replicas.len) continue;
        int64_t *bb = by_load(&m, &p->brokers);
        int64_t b = 0; int found = 0;
        for (int64_t k = p->brokers.len - 1; k >= 0; k--)
            if (!in_list(p->replicas.a, p->replicas.len, bb[k])) { b = bb[k]; found = 1; break; }
        free(bb);
        if (found) rc = addpl(pl, i, b, sem, res, 4);
        else {
            char ps[512], msg[700]; part_string(p, ps, sizeof ps);
            snprintf(msg, sizeof msg, "partition %s unable to pick replica to add", ps);
            set_err(res, 4, msg); rc = -1;
        }
    }
    lm_free(&m);
    return rc;
}

static int g_window;                      /* see or_set_window (move_window) */

/* The first partition holding a replica outside getBrokerListByLoadBL(loads, p.Brokers)
 * (utils.go:81-90): a replica always has a load, so that is a replica outside p.Brokers.
 * One hash set per distinct Brokers slice; O(P R) instead of the list intersections. */
static int64_t first_disallowed(const or_plist *pl) {
    /* dense ids of every broker named by a Brokers slice, one bitmap per distinct slice
       (keyed by its backing array: partitions share the slice FillDefaults gave them) */
    lmap ids; lm_init(&ids, 64);
    lmap keys; lm_init(&keys, 64);
    for (int64_t i = 0; i < pl->n; i++) {
        const or_partition *p = &pl->parts[i];
        if (lm_find(&keys, (int64_t)(intptr_t)p->brokers.a) >= 0) continue;
        lm_slot(&keys, (int64_t)(intptr_t)p->brokers.a);
        for (int64_t q = 0; q < p->brokers.len; q++) lm_slot(&ids, p->brokers.a[q]);
    }
    const int64_t W = (ids.n + 63) / 64 + 1;
    uint64_t *bits = (uint64_t *)calloc((size_t)(keys.n * W + 1), sizeof(uint64_t));
    for (int64_t i = 0; i < pl->n; i++) {
        const or_partition *p = &pl->parts[i];
        const int32_t j = lm_find(&keys, (int64_t)(intptr_t)p->brokers.a);
        uint64_t *b = bits + (int64_t)j * W;
        if (b[W - 1]) continue;                       /* (word W-1: this slice is done) */
        for (int64_t q = 0; q < p->brokers.len; q++) {
            const int64_t k = lm_find(&ids, p->brokers.a[q]);
            b[k >> 6] |= 1ull << (k & 63);
        }
        b[W - 1] = 1;
    }
    int64_t first = pl->n;
    for (int64_t i = 0; i < pl->n && first == pl->n; i++) {
        const or_partition *p = &pl->parts[i];
        const uint64_t *b = bits + (int64_t)lm_find(&keys, (int64_t)(intptr_t)p->brokers.a) * W;
        for (int64_t r = 0; r < p->replicas.len; r++) {
            const int64_t k = lm_find(&ids, p->replicas.a[r]);
            if (k < 0 || !((b[k >> 6] >> (k & 63)) & 1ull)) { first = i; break; }
        }
    }
    free(bits); lm_free(&ids); lm_free(&keys);
    return first;
}

static int move_disallowed(or_plist *pl, int sem, or_result *res) { /* steps.go:117-143 */
    lmap m; get_broker_load(pl, &m);
    int64_t nbl; bload *bl = get_bl(&m, &nbl);
    int64_t *A = (int64_t *)malloc((size_t)(nbl ? nbl : 1) * sizeof(int64_t));
    int rc = 0;
    int64_t i_start = 0;
    if (g_window) {
        /* (golden generation: the partitions before the first hit pass untouched) */
        i_start = first_disallowed(pl);
    } else if (g_threads > 1 && pl->n > 1) {
        /* the first partition holding a replica outside getBrokerListByLoadBL's list
         * (every earlier one passes untouched); the loop below starts there */
        int64_t first = pl->n;
#pragma omp parallel num_threads(g_threads)
        {
            int64_t *A2 = (int64_t *)malloc((size_t)(nbl ? nbl : 1) * sizeof(int64_t));
            int64_t mine = pl->n;
#pragma omp for schedule(static)
            for (int64_t i = 0; i < pl->n; i++) {
                if (i >= mine) continue;
                const or_partition *p = &pl->parts[i];
                int64_t na = 0;
                for (int64_t k = 0; k < nbl; k++)
                    if (in_list(p->brokers.a, p->brokers.len, bl[k].id)) A2[na++] = bl[k].id;
                for (int64_t r = 0; r < p->replicas.len; r++)
                    if (!in_list(A2, na, p->replicas.a[r])) { mine = i; break; }
            }
#pragma omp critical
            if (mine < first) first = mine;
            free(A2);
        }
        i_start = first;
    }
    for (int64_t i = i_start; i < pl->n && rc == 0; i++) {
        or_partition *p = &pl->parts[i];
        int64_t na = 0;                       /* getBrokerListByLoadBL (utils.go:81-90) */
        for (int64_t k = 0; k < nbl; k++)
            if (in_list(p->brokers.a, p->brokers.len, bl[k].id)) A[na++] = bl[k].id;
        for (int64_t r = 0; r < p->replicas.len && rc == 0; r++) {
            int64_t id = p->replicas.a[r];
            if (in_list(A, na, id)) continue;
            int64_t pick = 0; int found = 0;
            for (int64_t k = na - 1; k >= 0; k--) {
                if (in_list(p->replicas.a, p->replicas.len, A[k])) continue;
                pick = A[k]; found = 1; break;
            }
            if (found) rc = replacepl(pl, i, id, pick, sem, res, 5, OR_REPLACE);
            else {
                char ps[512], msg[760]; part_string(p, ps, sizeof ps);
                snprintf(msg, sizeof msg, "partition %s unable to pick replica to replace broker %lld",
                         ps, (long long)id);
                set_err(res, 5, msg); rc = -1;
            }
        }
    }
    free(A); free(bl); lm_free(&m);
    return rc;
}

/* loads + zero-filled cfg.Brokers (steps.go:215-220 / 300-305) */
static bload *loads_with_cfg(const or_plist *pl, const or_config *cfg, int64_t *nbl) {
    lmap m; get_broker_load(pl, &m);
    for (int64_t k = 0; k < cfg->nbrokers; k++) lm_slot(&m, cfg->brokers[k]);
    bload *bl = get_bl(&m, nbl);
    lm_free(&m);
    return bl;
}

static int distribute_leaders(or_plist *pl, const or_config *cfg, int sem, or_result *res) {
    int64_t n; bload *bl = loads_with_cfg(pl, cfg, &n);  /* steps.go:234-282 */
    double su = unbalance_bl(bl, n);
    int rc = 0;
    if (!(su < cfg->min_unbalance)) {
        if (n == 0) { set_err(res, 6, "panic: index out of range"); free(bl); return -1; }
        int64_t heavy = bl[n - 1].id;
        /* pp is built over EVERY partition first (steps.go:257-262): p.Replicas[0]
         * panics on any empty list, wherever it sits relative to the first pick */
        for (int64_t i = 0; i < pl->n; i++)
            if (pl->parts[i].replicas.len == 0) {
                set_err(res, 6, "panic: index out of range");
                free(bl);
                return -1;
            }
        for (int64_t i = 0; i < pl->n; i++) {
            or_partition *p = &pl->parts[i];
            if (p->replicas.a[0] != heavy) continue;
            if (p->num_replicas < cfg->min_replicas) continue;
            rc = replacepl(pl, i, p->replicas.a[0], bl[0].id, sem, res, 6, OR_REPLACE);
            res->su = su;
            break;
        }
    }
    free(bl);
    return rc;
}

/* Threads used by move() and MoveDisallowedReplicas' first-hit search (default 1:
 * the plain sequential restatement).  With T > 1 the partitions are split into T
 * contiguous chunks in order; every chunk runs the reference's own loop on a
 * private copy of bl, and the chunk results are merged in chunk order, which
 * yields exactly the sequential result: move() keeps the FIRST strict minimum in
 * (partition, slot, bl) order starting from cu = su (steps.go:163,211), i.e. the
 * lexicographic minimum of (u, iteration index) over the candidates with u < su,
 * and a panic is the one the sequential loop meets first.  Used to generate the
 * large golden plans (tests/golden/gen_scale.py); tests/test_oracle.py checks it
 * against T = 1. */

/* one chunk [i0, i1) of move()'s partition loop on bl (restored on return).
 * Returns 0, or the step error (1 = slice bounds panic, 2 = assertion) with the
 * partition in *ep. */
static int move_chunk(const or_plist *pl, const or_config *cfg, int leaders, bload *bl, int64_t n,
                      int64_t i0, int64_t i1, double *cu, int64_t *cp, int64_t *cr, int64_t *cb,
                      int64_t *cnt, int64_t *ep) {
    for (int64_t i = i0; i < i1; i++) {
        const or_partition *p = &pl->parts[i];
        if (p->num_replicas < cfg->min_replicas) continue;
        int64_t lo = 1, hi = p->replicas.len;
        if (leaders) { lo = 0; hi = 1; }
        if (p->replicas.len < lo || p->replicas.len < hi) { *ep = i; return 1; }  /* Go slice bounds panic */
        for (int64_t s = lo; s < hi; s++) {
            int64_t r = p->replicas.a[s];
            int64_t ridx = -1; double rload = 0;
            for (int64_t k = 0; k < n; k++)
                if (bl[k].id == r) { ridx = k; rload = bl[k].load; bl[k].load -= p->weight; }
            if (ridx == -1) { *ep = i; return 2; }
            for (int64_t k = 0; k < n; k++) {
                if (!in_list(p->brokers.a, p->brokers.len, bl[k].id)) continue;
                if (in_list(p->replicas.a, p->replicas.len, bl[k].id)) continue;
                double bload_ = bl[k].load;
                bl[k].load += p->weight;
                double u = unbalance_bl(bl, n);
                (*cnt)++;
                if (u < *cu) { *cu = u; *cp = i; *cr = r; *cb = bl[k].id; }
                bl[k].load = bload_;
            }
            bl[ridx].load = rload;
        }
    }
    return 0;
}

/* ------------------------------------------------ windowed exact move()
 * or_set_window(1) (golden generation only, tests/golden/gen_scale.py): the same result
 * as move_chunk's literal loop at a fraction of its cost on thousands of brokers.  Every
 * candidate is first scored in O(1): U~ = su + [f((L_r - w)/avg - 1) - f(r_r)] +
 * [f((L_t + w)/avg - 1) - f(r_t)] with avg and r_i = L_i/avg - 1 of the unchanged bl.  The
 * reference's U of a candidate (getUnbalanceBL over bl with two loads changed, two
 * sequential folds, utils.go:119-147) differs from the real value of the same expression
 * by at most ~2 n u (|U| + V), u = 2^-53, V = sum |r_i|(1 + |r_i|): recursive summation
 * errs by at most (n - 1) u sum|t_i| (Higham 4.2), the load sum's error moves every
 * r_i by at most (n - 1) u (1 + |r_i|), i.e. a term by ~2 |r_i| (1 + |r_i|) n u; moving w
 * between two brokers leaves the real load sum unchanged, so U~ (the unchanged bl's fold
 * plus two exact-to-rounding term deltas) is within eps = 16 n u (|su| + V + 1) of the
 * reference's U -- a window eight times the bound.  Any candidate with U~ > min U~ + 2 eps then has a
 * larger U than the U~-minimum, so the reference's first strict minimum (steps.go:211,
 * the lexicographic minimum of (U, iteration order) below su) lies among the candidates
 * within 2 eps of min U~: those, and only those, are folded exactly like move_chunk does,
 * in iteration order.  tests/test_oracle.py checks it against the literal loop. */
static int g_window = 0;
void or_set_window(int on) { g_window = on ? 1 : 0; }
/* target walks the early stop below ended (n >= 64), summed over move_window calls: the
   tests check that the walk's branch is exercised (tests/test_oracle.py) */
static int64_t g_walk_stops = 0;
int64_t or_walk_stops(void) { return g_walk_stops; }
void or_reset_walk_stops(void) { g_walk_stops = 0; }

typedef struct { double ua; int64_t i, s, k, ridx; } wcand;
typedef struct { wcand *v; int64_t n, cap; double best; } wlist;

static void wl_push(wlist *L, wcand c) {
    if (L->n == L->cap) { L->cap = L->cap ? 2 * L->cap : 1024; L->v = (wcand *)realloc(L->v, (size_t)L->cap * sizeof(wcand)); }
    L->v[L->n++] = c;
}
static double f_unb(double r) { return r > 0 ? r * r : r * r / 2; }

static int move_window(const or_plist *pl, const or_config *cfg, int leaders, bload *bl, int64_t n, double su,
                       int64_t np, double *cu, int64_t *cp, int64_t *cr, int64_t *cb, int64_t *cnt_out) {
    double sum = 0;
    for (int64_t k = 0; k < n; k++) sum += bl[k].load;
    const double avg = sum / (double)n;
    double *fr = (double *)malloc((size_t)(n ? n : 1) * sizeof(double));
    double V = 0;
    for (int64_t k = 0; k < n; k++) {
        const double r = bl[k].load / avg - 1.0;
        fr[k] = f_unb(r);
        V += fabs(r) * (1.0 + fabs(r));
    }
    const double eps = 16.0 * (double)(n + 1) * 0x1p-53 * (V + fabs(su) + 1.0);
    /* bl position of every broker id, and one bitmap over bl positions per distinct
       Brokers slice (partitions share the slice FillDefaults gave them) */
    lmap pos; lm_init(&pos, n);
    for (int64_t k = 0; k < n; k++) { int32_t q = lm_slot(&pos, bl[k].id); pos.loads[q] = (double)k; }
    const int64_t W = (n + 63) / 64;
    int32_t *sidx = (int32_t *)malloc((size_t)(np ? np : 1) * sizeof(int32_t));
    uint64_t *bits = NULL;
    const int64_t **skey = NULL;
    int64_t nset = 0, setcap = 0, last = -1;
    lmap kmap; lm_init(&kmap, 64);                  /* slice backing array -> set index */
    for (int64_t i = 0; i < np; i++) {
        const int64_t *key = pl->parts[i].brokers.a;
        int64_t j = last >= 0 && skey[last] == key ? last : -1;
        if (j < 0) {
            const int32_t q = lm_find(&kmap, (int64_t)(intptr_t)key);
            if (q >= 0) j = (int64_t)kmap.loads[q];
        }
        if (j < 0) {
            const int32_t q = lm_slot(&kmap, (int64_t)(intptr_t)key);
            kmap.loads[q] = (double)nset;
            if (nset == setcap) {
                setcap = setcap ? 2 * setcap : 16;
                skey = (const int64_t **)realloc((void *)skey, (size_t)setcap * sizeof(int64_t *));
                bits = (uint64_t *)realloc(bits, (size_t)(setcap * (W ? W : 1)) * sizeof(uint64_t));
            }
            j = nset++;
            skey[j] = key;
            uint64_t *b = bits + j * W;
            memset(b, 0, (size_t)(W ? W : 1) * sizeof(uint64_t));
            const or_partition *p = &pl->parts[i];
            for (int64_t q = 0; q < p->brokers.len; q++) {
                const int32_t m = lm_find(&pos, p->brokers.a[q]);
                if (m >= 0) { const int64_t k = (int64_t)pos.loads[m]; b[k >> 6] |= 1ull << (k & 63); }
            }
        }
        sidx[i] = (int32_t)j;
        last = j;
    }
    int64_t *setcnt = (int64_t *)malloc((size_t)(nset ? nset : 1) * sizeof(int64_t));
    for (int64_t j = 0; j < nset; j++) {
        setcnt[j] = 0;
        for (int64_t q = 0; q < W; q++) setcnt[j] += __builtin_popcountll(bits[j * W + q]);
    }
    /* Early stop of a slot's target walk (n >= 64 only).  For a fixed source the real value
       of the O(1) score is h(L_t) = f((L_t + w)/avg - 1) - f(L_t/avg - 1) plus constants, and
       h is nondecreasing in L_t (f is convex); targets come in bl order, i.e. ascending L_t.
       The computed score is within d of that real value: w/avg <= L_s/avg = 1 + r_s, so
       every term is at most 3 (V + 1) and its argument errs by ~2 u (|x| + 1); with the four
       adds d <= 100 u (V + |su| + 1) < eps / 2 once n >= 64 (eps is 16 (n + 1) u
       (V + |su| + 1) >= 1040 u (...)).  So a computed score above best + 3 eps puts the real
       value of this and every later target above best + 2.5 eps and their computed scores
       above best + 2 eps: outside the window (best only falls, so the thread's running best
       is conservative). */
    const int walk = n >= 64;
    int T = g_threads < 1 ? 1 : g_threads;
    if (T > np) T = np > 0 ? (int)np : 1;
    wlist *TL = (wlist *)calloc((size_t)T, sizeof(wlist));
    int64_t *tcnt = (int64_t *)calloc((size_t)T, sizeof(int64_t));
    int64_t *tstop = (int64_t *)calloc((size_t)T, sizeof(int64_t));
    int *terr = (int *)calloc((size_t)T, sizeof(int));
#pragma omp parallel for num_threads(T) schedule(static, 1)
    for (int t = 0; t < T; t++) {
        wlist *L = &TL[t];
        L->best = HUGE_VAL;
        const int64_t i0 = np * t / T, i1 = np * (t + 1) / T;
        int64_t rk[64];
        for (int64_t i = i0; i < i1 && !terr[t]; i++) {
            const or_partition *p = &pl->parts[i];
            if (p->num_replicas < cfg->min_replicas) continue;
            int64_t lo = 1, hi = p->replicas.len;
            if (leaders) { lo = 0; hi = 1; }
            if (p->replicas.len < lo || p->replicas.len < hi) { terr[t] = 1; break; }
            const int64_t nr = p->replicas.len < 64 ? p->replicas.len : 64;
            for (int64_t q = 0; q < nr; q++) {
                const int32_t m = lm_find(&pos, p->replicas.a[q]);
                rk[q] = m >= 0 ? (int64_t)pos.loads[m] : -1;
            }
            const uint64_t *b = bits + (int64_t)sidx[i] * W;
            const double w = p->weight;
            /* candidates of one slot = set members minus the partition's replicas (distinct:
               ValidateReplicas ran) */
            int64_t nin = 0;
            for (int64_t q = 0; q < nr; q++) nin += rk[q] >= 0 && ((b[rk[q] >> 6] >> (rk[q] & 63)) & 1ull);
            for (int64_t s = lo; s < hi; s++) {
                const int64_t ridx = s < 64 ? rk[s] : -1;
                if (ridx < 0) { terr[t] = 2; break; }
                const double ds = f_unb((bl[ridx].load - w) / avg - 1.0) - fr[ridx];
                tcnt[t] += setcnt[sidx[i]] - nin;
                /* targets in bl order = ascending load: set bits word by word */
                for (int64_t wd = 0, stop = 0; wd < W && !stop; wd++) {
                    uint64_t m = b[wd];
                    while (m) {
                        const int64_t k = wd * 64 + __builtin_ctzll(m);
                        m &= m - 1;
                        int isrep = 0;
                        for (int64_t q = 0; q < nr; q++) isrep |= rk[q] == k;
                        if (isrep) continue;
                        const double ua = su + ds + (f_unb((bl[k].load + w) / avg - 1.0) - fr[k]);
                        if (ua <= L->best + 2 * eps) {
                            wcand c = {ua, i, s, k, ridx};
                            wl_push(L, c);
                            if (ua < L->best) L->best = ua;
                        } else if (walk && ua > L->best + 3 * eps) {
                            stop = 1;          /* every later target scores above the window */
                            tstop[t]++;
                            break;
                        }
                    }
                }
            }
        }
    }
    int err = 0;
    double best = HUGE_VAL;
    for (int t = 0; t < T; t++) g_walk_stops += tstop[t];
    free(tstop);
    for (int t = 0; t < T && !err; t++) {
        *cnt_out += tcnt[t];
        if (terr[t]) { err = terr[t]; break; }          /* the first panic in order */
        if (TL[t].best < best) best = TL[t].best;
    }
    if (!err) {
        bload *b2 = (bload *)malloc((size_t)(n ? n : 1) * sizeof(bload));
        if (n) memcpy(b2, bl, (size_t)n * sizeof(bload));
        for (int t = 0; t < T; t++)
            for (int64_t c = 0; c < TL[t].n; c++) {
                const wcand x = TL[t].v[c];
                if (!(x.ua <= best + 2 * eps)) continue;
                const or_partition *p = &pl->parts[x.i];
                const double rl = b2[x.ridx].load, tl = b2[x.k].load;
                b2[x.ridx].load -= p->weight;                 /* as move_chunk does, in order */
                b2[x.k].load += p->weight;
                const double u = unbalance_bl(b2, n);
                b2[x.ridx].load = rl; b2[x.k].load = tl;
                if (u < *cu) { *cu = u; *cp = x.i; *cr = p->replicas.a[x.s]; *cb = b2[x.k].id; }
            }
        free(b2);
    }
    if (getenv("KB_ORACLE_WINDOW_DEBUG")) {
        int64_t tot = 0, in = 0;
        for (int t = 0; t < T; t++) { tot += TL[t].n; for (int64_t c = 0; c < TL[t].n; c++) in += TL[t].v[c].ua <= best + 2 * eps; }
        fprintf(stderr, "window: eps %.3g best %.17g listed %lld folded %lld\n", eps, best, (long long)tot, (long long)in);
    }
    for (int t = 0; t < T; t++) free(TL[t].v);
    free(TL); free(tcnt); free(terr); free(fr); free(bits); free(setcnt); lm_free(&kmap); free((void *)skey); free(sidx); lm_free(&pos);
    return err;
}

/* move (steps.go:145-232).  limit < 0 => all partitions. */
static int move_impl(or_plist *pl, const or_config *cfg, int leaders, int sem, or_result *res,
                     int64_t limit, int64_t *ncand, double *cu_out) {
    int64_t n; bload *bl = loads_with_cfg(pl, cfg, &n);
    double su = unbalance_bl(bl, n), cu = su;
    int64_t cp = -1, cr = 0, cb = 0, cnt = 0;
    int64_t np = limit < 0 || limit > pl->n ? pl->n : limit;
    int err = 0;
    int T = g_threads;
    if (T > np) T = np > 0 ? (int)np : 1;
    if (g_window && limit < 0 && n > 0) {
        err = move_window(pl, cfg, leaders, bl, n, su, np, &cu, &cp, &cr, &cb, &cnt);
    } else if (T <= 1) {
        int64_t ep = -1;
        err = move_chunk(pl, cfg, leaders, bl, n, 0, np, &cu, &cp, &cr, &cb, &cnt, &ep);
    } else {
        double *tcu = (double *)malloc((size_t)T * sizeof(double));
        int64_t *tv = (int64_t *)malloc((size_t)T * 5 * sizeof(int64_t));
        int *terr = (int *)calloc((size_t)T, sizeof(int));
#pragma omp parallel for num_threads(T) schedule(static, 1)
        for (int t = 0; t < T; t++) {
            bload *b2 = (bload *)malloc((size_t)(n ? n : 1) * sizeof(bload));
            if (n) memcpy(b2, bl, (size_t)n * sizeof(bload));
            int64_t i0 = np * t / T, i1 = np * (t + 1) / T;
            int64_t *v = tv + 5 * t;     /* cp, cr, cb, cnt, ep */
            tcu[t] = su; v[0] = -1; v[1] = v[2] = v[3] = 0; v[4] = -1;
            terr[t] = move_chunk(pl, cfg, leaders, b2, n, i0, i1, &tcu[t], &v[0], &v[1], &v[2], &v[3], &v[4]);
            free(b2);
        }
        for (int t = 0; t < T && !err; t++) {
            int64_t *v = tv + 5 * t;
            cnt += v[3];
            if (terr[t]) { err = terr[t]; break; }          /* the first panic in order */
            if (v[0] >= 0 && tcu[t] < cu) { cu = tcu[t]; cp = v[0]; cr = v[1]; cb = v[2]; }
        }
        free(tcu); free(tv); free(terr);
    }
    free(bl);
    if (err) {
        set_err(res, leaders ? 7 : 8, err == 1 ? "panic: slice bounds out of range"
                                                : "assertion failed: replica not in broker loads");
        return -1;
    }
    if (ncand) *ncand = cnt;
    if (cu_out) *cu_out = cu;
    if (limit >= 0) return 0;
    res->su = su; res->cu = cu;
    if (cu < su - cfg->min_unbalance)
        return replacepl(pl, cp, cr, cb, sem, res, leaders ? 7 : 8, OR_REPLACE);
    return 0;
}

int or_balance(or_plist *pl, const or_config *cfg, int sem, or_result *res) {
    memset(res, 0, sizeof *res);
    res->pidx = -1;
    if (pl->n == 0) { set_err(res, 0, "panic: index out of range"); return -1; }
    int rc;
    if ((rc = validate_weights(pl, res)) != 0) return rc;
    if ((rc = validate_replicas(pl, res)) != 0) return rc;
    fill_defaults(pl, cfg);
    if ((rc = remove_extra(pl, sem, res)) != 0) return rc;
    if ((rc = add_missing(pl, sem, res)) != 0) return rc;
    if ((rc = move_disallowed(pl, sem, res)) != 0) return rc;
    if (cfg->rebalance_leaders && (rc = distribute_leaders(pl, cfg, sem, res)) != 0) return rc;
    if (cfg->allow_leader && (rc = move_impl(pl, cfg, 1, sem, res, -1, NULL, NULL)) != 0) return rc;
    if ((rc = move_impl(pl, cfg, 0, sem, res, -1, NULL, NULL)) != 0) return rc;
    res->status = 0;
    return 0;
}

/* One Balance() over the steps whose bit is set in mask (bit k = steps table entry k,
 * balancer.go:34-44), in table order; the first non-nil result wins (balancer.go:49-65).
 * mask = 0x1FF is or_balance. */
int or_step(or_plist *pl, const or_config *cfg, int sem, unsigned mask, or_result *res) {
    memset(res, 0, sizeof *res);
    res->pidx = -1;
    int rc;
    if (mask & 1u) {
        if (pl->n == 0) { set_err(res, 0, "panic: index out of range"); return -1; }
        if ((rc = validate_weights(pl, res)) != 0) return rc;
    }
    if ((mask & 2u) && (rc = validate_replicas(pl, res)) != 0) return rc;
    if (mask & 4u) fill_defaults(pl, cfg);
    if ((mask & 8u) && (rc = remove_extra(pl, sem, res)) != 0) return rc;
    if ((mask & 16u) && (rc = add_missing(pl, sem, res)) != 0) return rc;
    if ((mask & 32u) && (rc = move_disallowed(pl, sem, res)) != 0) return rc;
    if ((mask & 64u) && cfg->rebalance_leaders && (rc = distribute_leaders(pl, cfg, sem, res)) != 0) return rc;
    if ((mask & 128u) && cfg->allow_leader && (rc = move_impl(pl, cfg, 1, sem, res, -1, NULL, NULL)) != 0) return rc;
    if ((mask & 256u) && (rc = move_impl(pl, cfg, 0, sem, res, -1, NULL, NULL)) != 0) return rc;
    res->status = 0;
    return 0;
}

int64_t or_move_sample(or_plist *pl, const or_config *cfg, int leaders, int64_t max_parts, double *cu) {
    or_result res; memset(&res, 0, sizeof res);
    int64_t cnt = 0;
    move_impl(pl, cfg, leaders, OR_SEM_APPLIED, &res, max_parts < 0 ? 0 : max_parts, &cnt, cu);
    return cnt;
}

/* ------------------------------------------------------------- JSON out */

/* Go encoding/json floatEncoder: strconv 'f' (or 'e' outside [1e-6,1e21)), shortest digits */
void or_format_float(double x, char *buf) {
    if (x == 0) { strcpy(buf, signbit(x) ? "-0" : "0"); return; }
    char tmp[64];
    int prec;
    for (prec = 1; prec <= 17; prec++) {
        snprintf(tmp, sizeof tmp, "%.*e", prec - 1, x);
        if (strtod(tmp, NULL) == x) break;
    }
    /* tmp = [-]d.ddde[+-]XX ; extract digits and exponent */
    char digits[32]; int nd = 0; const char *q = tmp; int neg = 0;
    if (*q == '-') { neg = 1; q++; }
    while (*q && *q != 'e') { if (*q != '.') digits[nd++] = *q; q++; }
    digits[nd] = 0;
    int e10 = atoi(q + 1);              /* value = d.ddd * 10^e10 */
    while (nd > 1 && digits[nd - 1] == '0') digits[--nd] = 0;
    char *o = buf;
    if (neg) *o++ = '-';
    double ax = fabs(x);
    if (ax < 1e-6 || ax >= 1e21) {
        *o++ = digits[0];
        if (nd > 1) { *o++ = '.'; memcpy(o, digits + 1, (size_t)nd - 1); o += nd - 1; }
        int ee = e10;
        *o++ = 'e'; *o++ = ee < 0 ? '-' : '+';
        if (ee < 0) ee = -ee;
        if (ee < 10 && e10 >= 0) { *o++ = '0'; *o++ = (char)('0' + ee); }   /* e+0X keeps the zero */
        else o += sprintf(o, "%d", ee);                                       /* e-0X -> e-X cleanup */
        *o = 0;
        return;
    }
    int pointpos = e10 + 1;             /* digits before the decimal point */
    if (pointpos <= 0) {
        *o++ = '0'; *o++ = '.';
        for (int i = 0; i < -pointpos; i++) *o++ = '0';
        memcpy(o, digits, (size_t)nd); o += nd;
    } else if (pointpos >= nd) {
        memcpy(o, digits, (size_t)nd); o += nd;
        for (int i = nd; i < pointpos; i++) *o++ = '0';
    } else {
        memcpy(o, digits, (size_t)pointpos); o += pointpos;
        *o++ = '.';
        memcpy(o, digits + pointpos, (size_t)(nd - pointpos)); o += nd - pointpos;
    }
    *o = 0;
}

typedef struct { char *b; size_t n, cap; } sbuf;
static void sb_put(sbuf *s, const char *t, size_t n) {
    if (s->n + n + 1 > s->cap) {
        while (s->n + n + 1 > s->cap) s->cap = s->cap ? s->cap * 2 : 4096;
        s->b = (char *)realloc(s->b, s->cap);
    }
    memcpy(s->b + s->n, t, n); s->n += n; s->b[s->n] = 0;
}
static void sb_str(sbuf *s, const char *t) { sb_put(s, t, strlen(t)); }

static void json_string(sbuf *s, const char *t) {
    static const char hx[] = "0123456789abcdef";
    sb_put(s, "\"", 1);
    for (const unsigned char *c = (const unsigned char *)t; *c; c++) {
        char e[8];
        if (*c == '"' || *c == '\\') { e[0] = '\\'; e[1] = (char)*c; sb_put(s, e, 2); }
        else if (*c == '\n') sb_str(s, "\\n");
        else if (*c == '\r') sb_str(s, "\\r");
        else if (*c == '\t') sb_str(s, "\\t");
        else if (*c == '\b') sb_str(s, "\\b");
        else if (*c == '\f') sb_str(s, "\\f");
        else if (*c < 0x20 || *c == '<' || *c == '>' || *c == '&') {
            e[0] = '\\'; e[1] = 'u'; e[2] = '0'; e[3] = '0'; e[4] = hx[*c >> 4]; e[5] = hx[*c & 15];
            sb_put(s, e, 6);
        } else sb_put(s, (const char *)c, 1);
    }
    sb_put(s, "\"", 1);
}

static void json_ints(sbuf *s, const or_slice *v) {
    if (v->a == NULL) { sb_str(s, "null"); return; }
    sb_str(s, "[");
    char t[32];
    for (int64_t i = 0; i < v->len; i++) { snprintf(t, sizeof t, i ? ",%lld" : "%lld", (long long)v->a[i]); sb_str(s, t); }
    sb_str(s, "]");
}

static void json_partition(sbuf *s, const or_partition *p) {
    char t[64];
    sb_str(s, "{\"topic\":"); json_string(s, p->topic);
    snprintf(t, sizeof t, ",\"partition\":%lld,\"replicas\":", (long long)p->partition); sb_str(s, t);
    json_ints(s, &p->replicas);
    if (p->weight != 0) { sb_str(s, ",\"weight\":"); or_format_float(p->weight, t); sb_str(s, t); }
    if (p->num_replicas != 0) { snprintf(t, sizeof t, ",\"num_replicas\":%lld", (long long)p->num_replicas); sb_str(s, t); }
    if (p->brokers.a != NULL && p->brokers.len > 0) { sb_str(s, ",\"brokers\":"); json_ints(s, &p->brokers); }
    if (p->num_consumers != 0) { snprintf(t, sizeof t, ",\"num_consumers\":%lld", (long long)p->num_consumers); sb_str(s, t); }
    sb_str(s, "}");
}

static void json_plist(sbuf *s, const or_partition *ps, int64_t n, int nil) {
    sb_str(s, "{\"version\":1,\"partitions\":");
    if (nil) sb_str(s, "null");
    else {
        sb_str(s, "[");
        for (int64_t i = 0; i < n; i++) { if (i) sb_str(s, ","); json_partition(s, &ps[i]); }
        sb_str(s, "]");
    }
    sb_str(s, "}\n");
}

/* ----------------------------------------------------------- run() loop */

int or_run_plan(or_plist *pl, const or_config *cfg, int64_t max_reassign, int complete_partition,
                int full_output, int unique, int sem, char **out, char *err, size_t errlen,
                int64_t *nsteps_out) {
    int64_t cap = 16, n = 0, nsteps = 0;
    or_partition *opl = (or_partition *)malloc((size_t)cap * sizeof(or_partition));
    int completing = 0;
    or_partition cpart; memset(&cpart, 0, sizeof cpart);
    int64_t r = max_reassign;
    const int64_t guard = max_reassign + 100000;   /* the reference would loop forever */
    *out = NULL;
    while (r > 0) {
        or_result res;
        int rc = or_balance(pl, cfg, sem, &res);
        nsteps++;
        if (rc < 0) {
            snprintf(err, errlen, "failed optimizing distribution: %s", res.err);
            free(opl); if (nsteps_out) *nsteps_out = nsteps; return 3;
        }
        if (res.status == 0) break;
        or_partition p = res.part;
        if (sem == OR_SEM_APPLIED) {                 /* snapshot the entry */
            or_slice c = sl_make(p.replicas.len, p.replicas.len);
            if (p.replicas.len) memcpy(c.a, p.replicas.a, (size_t)p.replicas.len * sizeof(int64_t));
            p.replicas = c;
        }
        if (completing) {
            if (!(strcmp(cpart.topic, p.topic) == 0 && cpart.partition == p.partition)) break;
        }
        if (n == cap) { cap *= 2; opl = (or_partition *)realloc(opl, (size_t)cap * sizeof(or_partition)); }
        opl[n++] = p;
        r--;
        if (r == 0 && complete_partition) {
            r = 1;
            if (!completing) { cpart = p; completing = 1; }
        }
        if (nsteps > guard) {
            snprintf(err, errlen, "reference does not terminate (complete-partition loop)");
            free(opl); if (nsteps_out) *nsteps_out = nsteps; return 99;
        }
    }
    if (nsteps_out) *nsteps_out = nsteps;
    or_partition *ps = opl; int64_t np = n; int nil = n == 0;
    if (full_output) { ps = pl->parts; np = pl->n; nil = pl->parts == NULL; }
    or_partition *filt = NULL;
    if (unique) {                                   /* FilterPartitionList (codecs.go:67-82) */
        filt = (or_partition *)malloc((size_t)(np ? np : 1) * sizeof(or_partition));
        int64_t k = 0;
        for (int64_t i = 0; i < np; i++) {
            int seen = 0;
            for (int64_t j = 0; j < k; j++)
                if (strcmp(filt[j].topic, ps[i].topic) == 0 && filt[j].partition == ps[i].partition) { seen = 1; break; }
            if (!seen) filt[k++] = ps[i];
        }
        ps = filt; np = k; nil = k == 0;
    }
    sbuf s = {0, 0, 0};
    json_plist(&s, ps, np, nil);
    *out = s.b;
    free(filt); free(opl);
    return 0;
}

void or_free(void *p) { free(p); }

/* ------------------------------------------------ construction helpers */

or_plist *or_plist_build(int64_t n, const char *topic_blob, const int64_t *topic_off,
                         const int64_t *partition, const int64_t *rep_flat, const int64_t *rep_off,
                         const int8_t *rep_nil, const double *weight, const int64_t *num_replicas,
                         int64_t nsets, const int64_t *set_flat, const int64_t *set_off,
                         const int64_t *set_idx, const int64_t *num_consumers) {
    or_plist *pl = (or_plist *)calloc(1, sizeof(or_plist));
    pl->version = 1; pl->n = n;
    pl->parts = (or_partition *)calloc((size_t)(n ? n : 1), sizeof(or_partition));
    or_slice *sets = (or_slice *)calloc((size_t)(nsets ? nsets : 1), sizeof(or_slice));
    for (int64_t s = 0; s < nsets; s++) {
        int64_t len = set_off[s + 1] - set_off[s];
        sets[s] = sl_make(len, len);
        if (len) memcpy(sets[s].a, set_flat + set_off[s], (size_t)len * sizeof(int64_t));
    }
    for (int64_t i = 0; i < n; i++) {
        or_partition *p = &pl->parts[i];
        int64_t tl = topic_off[i + 1] - topic_off[i];
        char *t = (char *)malloc((size_t)tl + 1);
        memcpy(t, topic_blob + topic_off[i], (size_t)tl); t[tl] = 0;
        p->topic = t;
        p->partition = partition[i];
        int64_t rl = rep_off[i + 1] - rep_off[i];
        if (rep_nil && rep_nil[i]) { p->replicas.a = NULL; p->replicas.len = p->replicas.cap = 0; }
        else {
            p->replicas = sl_make(rl, rl);
            if (rl) memcpy(p->replicas.a, rep_flat + rep_off[i], (size_t)rl * sizeof(int64_t));
        }
        p->weight = weight[i];
        p->num_replicas = num_replicas[i];
        if (set_idx[i] < 0) { p->brokers.a = NULL; p->brokers.len = p->brokers.cap = 0; }
        else p->brokers = sets[set_idx[i]];
        p->num_consumers = num_consumers[i];
    }
    free(sets);
    return pl;
}

int64_t or_plist_replicas(const or_plist *pl, int64_t i, int64_t *buf, int64_t cap) {
    const or_slice *s = &pl->parts[i].replicas;
    for (int64_t k = 0; k < s->len && k < cap; k++) buf[k] = s->a[k];
    return s->len;
}

int64_t or_plist_len(const or_plist *pl) { return pl->n; }
