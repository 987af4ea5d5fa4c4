/*
 * shim_test.c -- drives the C ABI (include/kbengine.h) exactly as the cgo shim of
 * INTEGRATION.md does: every array the engine reads is malloc'd C memory (no host
 * language memory crosses the boundary), KB_SEM_GO (the reference's slice aliasing),
 * kb_engine_last_error for the "<Step>: <msg>" text, kb_engine_destroy.
 *
 * Like the shim it keeps a host mirror of the partition list (what the Go side's own
 * replacepl / addpl / FillDefaults do to pl, utils.go:166-202, steps.go:39-66) and one
 * engine per (partition list, config): a call with a different config destroys the
 * engine and creates a new one from the mirror, as the Go caller passing a new
 * RebalanceConfig (balancer.go:49) would have the shim do.
 *
 * Two bindings of Balance() (balancer.go:49-65):
 *   mode 0: one kb_engine_balance per Balance() call (the whole steps table on the device);
 *   mode 1: the reference's steps table walked on the host, each entry one
 *           kb_engine_step(e, KB_STEP_BIT(k)) call, the first change or error wins.
 *
 * Input (whitespace separated, written by tests/test_shim_c.py):
 *   n_partitions
 *   per partition: topic partition nrep r_1..r_nrep weight num_replicas num_consumers nb b_1..b_nb
 *                  (nb = -1: nil Brokers)
 *   ncfg, then ncfg lines: allow_leader rebalance_leaders min_replicas min_unbalance brokers_nil
 *                          n_brokers b_1..b_n
 *   steps mode            (Balance() call s uses config s % ncfg)
 * Output: one line per Balance() call: "change <step> <pidx> <kind> <from> <to> <slot>",
 * "nochange", or "error <rc> <message>"; then "engines <created> <destroyed>".
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "kbengine.h"

static void *xmalloc(size_t n) {
    void *p = malloc(n ? n : 1);
    if (!p) { fprintf(stderr, "out of memory\n"); exit(2); }
    return p;
}

#define MAXREP 16

/* the host mirror of pl (the Go side's PartitionList) */
typedef struct {
    char topic[256];
    long long part, rep[MAXREP], nrep, want, cons, nb;   /* nb < 0: nil Brokers */
    double w;
    long long *brokers;
} Part;

typedef struct {
    int al, rl, bnil;
    long long mr, nbk;
    double mu;
    long long *brokers;
} Cfg;

static int cmp_ll(const void *a, const void *b) {
    long long x = *(const long long *)a, y = *(const long long *)b;
    return x < y ? -1 : x > y;
}

/* FillDefaults (steps.go:39-66) on the mirror */
static void fill_defaults(Part *P, long long n, const Cfg *c) {
    if (n == 0) return;
    if (P[0].w == 0) for (long long i = 0; i < n; i++) P[i].w = 1.0;
    long long *def = NULL, ndef = 0;
    int need = 0;
    for (long long i = 0; i < n; i++) if (P[i].nb < 0) need = 1;
    if (need) {
        if (!c->bnil) {
            def = xmalloc(sizeof(long long) * (size_t)(c->nbk + 1));
            memcpy(def, c->brokers, sizeof(long long) * (size_t)c->nbk);
            ndef = c->nbk;
        } else {                        /* getBrokerList (utils.go:49-64): sorted, unique */
            long long tot = 0;
            for (long long i = 0; i < n; i++) tot += P[i].nrep;
            def = xmalloc(sizeof(long long) * (size_t)(tot + 1));
            for (long long i = 0; i < n; i++) for (long long k = 0; k < P[i].nrep; k++) def[ndef++] = P[i].rep[k];
            qsort(def, (size_t)ndef, sizeof(long long), cmp_ll);
            long long m = 0;
            for (long long k = 0; k < ndef; k++) if (m == 0 || def[m - 1] != def[k]) def[m++] = def[k];
            ndef = m;
        }
        for (long long i = 0; i < n; i++)
            if (P[i].nb < 0) {
                P[i].brokers = xmalloc(sizeof(long long) * (size_t)(ndef + 1));
                memcpy(P[i].brokers, def, sizeof(long long) * (size_t)ndef);
                P[i].nb = ndef;
            }
        free(def);
    }
    for (long long i = 0; i < n; i++) if (P[i].want == 0) P[i].want = P[i].nrep;
}

/* replacepl / addpl with Go's aliasing (utils.go:166-202): a remove shifts the shared
 * array and pl keeps its length, an append is not visible through pl */
static void apply_change(Part *P, const kb_change *ch) {
    Part *p = &P[ch->partition];
    if (ch->kind == KB_KIND_ADD) return;
    for (long long i = 0; i < p->nrep; i++) {
        if (p->rep[i] != ch->from_broker) continue;
        if (ch->kind == KB_KIND_REMOVE) {
            for (long long k = i; k + 1 < p->nrep; k++) p->rep[k] = p->rep[k + 1];
        } else {
            long long ex = -1;
            for (long long k = 0; k < p->nrep && ex < 0; k++) if (p->rep[k] == ch->to_broker) ex = k;
            if (ex >= 0) { long long t = p->rep[i]; p->rep[i] = ch->to_broker; p->rep[ex] = t; }
            else p->rep[i] = ch->to_broker;
        }
        return;
    }
}

static int created = 0, destroyed = 0;

/* kb_engine_create from the mirror (the shim's newGPUEngine): C memory only */
static kb_engine *make_engine(const Part *P, long long n, const Cfg *c, char *msg) {
    int64_t *rep = xmalloc(sizeof(int64_t) * (size_t)(MAXREP * n + 1));
    int64_t *roff = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    double *w = xmalloc(sizeof(double) * (size_t)(n + 1));
    int64_t *nr = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t *nc = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t *pid = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t *sidx = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t *toff = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t *soff = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    size_t sn = 0, tn = 0, nsets = 0;
    for (long long i = 0; i < n; i++) { sn += P[i].nb > 0 ? (size_t)P[i].nb : 0; tn += strlen(P[i].topic); }
    int64_t *sids = xmalloc(sizeof(int64_t) * (sn + 1));
    char *blob = xmalloc(tn + 1);
    roff[0] = 0; toff[0] = 0; soff[0] = 0; sn = 0; tn = 0;
    for (long long i = 0; i < n; i++) {
        const size_t tl = strlen(P[i].topic);
        memcpy(blob + tn, P[i].topic, tl); tn += tl; toff[i + 1] = (int64_t)tn;
        pid[i] = P[i].part;
        for (long long k = 0; k < P[i].nrep; k++) rep[roff[i] + k] = P[i].rep[k];
        roff[i + 1] = roff[i] + P[i].nrep;
        w[i] = P[i].w; nr[i] = P[i].want; nc[i] = P[i].cons;
        if (P[i].nb < 0) { sidx[i] = -1; continue; }
        /* one set per listed Brokers slice (the shim deduplicates by content; a set per
           partition is equally valid input) */
        for (long long k = 0; k < P[i].nb; k++) sids[sn++] = P[i].brokers[k];
        sidx[i] = (int64_t)nsets;
        soff[++nsets] = (int64_t)sn;
    }
    int64_t *brokers = xmalloc(sizeof(int64_t) * (size_t)(c->nbk + 1));
    for (long long k = 0; k < c->nbk; k++) brokers[k] = c->brokers[k];
    kb_config *cfg = xmalloc(sizeof *cfg);
    memset(cfg, 0, sizeof *cfg);
    cfg->allow_leader = c->al; cfg->rebalance_leaders = c->rl; cfg->min_replicas = c->mr;
    cfg->min_unbalance = c->mu; cfg->brokers = brokers; cfg->n_brokers = c->nbk; cfg->brokers_nil = c->bnil;
    cfg->semantics = KB_SEM_GO;
    kb_cluster *cl = xmalloc(sizeof *cl);
    memset(cl, 0, sizeof *cl);
    cl->n_partitions = n; cl->replica_ids = rep; cl->replica_off = roff; cl->weight = w;
    cl->num_replicas = nr; cl->num_consumers = nc; cl->n_sets = (int64_t)nsets; cl->set_ids = sids;
    cl->set_off = soff; cl->set_idx = sidx; cl->topic_blob = blob; cl->topic_off = toff;
    cl->partition_id = pid;
    kb_engine *e = NULL;
    const int rc = kb_engine_create(cl, cfg, &e);
    /* the engine copied everything: the arena goes now (as the shim's defer does) */
    free(rep); free(roff); free(w); free(nr); free(nc); free(pid); free(sidx); free(toff);
    free(sids); free(soff); free(blob); free(brokers); free(cfg); free(cl);
    if (rc < 0) {
        msg[0] = 0;
        if (e) kb_engine_last_error(e, msg, 4096);
        printf("create-error %d %s\n", rc, msg);
        kb_engine_destroy(e);
        return NULL;
    }
    created++;
    return e;
}

/* one Balance() call: kb_engine_balance, or the steps table one kb_engine_step per entry */
static int balance_call(kb_engine *e, int mode, kb_change *ch) {
    if (mode == 0) return kb_engine_balance(e, ch);
    for (int k = KB_STEP_VALIDATE_WEIGHTS; k <= KB_STEP_MOVE_NON_LEADERS; k++) {
        const int rc = kb_engine_step(e, KB_STEP_BIT(k), ch);
        if (rc != KB_NOCHANGE) return rc;
    }
    return KB_NOCHANGE;
}

int main(int argc, char **argv) {
    FILE *f = argc > 1 ? fopen(argv[1], "r") : stdin;
    if (!f) { perror("input"); return 2; }
    long long n;
    if (fscanf(f, "%lld", &n) != 1 || n < 0) return 2;
    Part *P = xmalloc(sizeof(Part) * (size_t)(n + 1));
    memset(P, 0, sizeof(Part) * (size_t)(n + 1));
    for (long long i = 0; i < n; i++) {
        Part *p = &P[i];
        if (fscanf(f, "%255s %lld %lld", p->topic, &p->part, &p->nrep) != 3 || p->nrep < 0 || p->nrep > MAXREP)
            return 2;
        for (long long j = 0; j < p->nrep; j++) if (fscanf(f, "%lld", &p->rep[j]) != 1) return 2;
        if (fscanf(f, "%lf %lld %lld %lld", &p->w, &p->want, &p->cons, &p->nb) != 4) return 2;
        if (p->nb >= 0) {
            p->brokers = xmalloc(sizeof(long long) * (size_t)(p->nb + 1));
            for (long long j = 0; j < p->nb; j++) if (fscanf(f, "%lld", &p->brokers[j]) != 1) return 2;
        }
    }
    int ncfg;
    if (fscanf(f, "%d", &ncfg) != 1 || ncfg < 1) return 2;
    Cfg *C = xmalloc(sizeof(Cfg) * (size_t)ncfg);
    for (int c = 0; c < ncfg; c++) {
        if (fscanf(f, "%d %d %lld %lf %d %lld", &C[c].al, &C[c].rl, &C[c].mr, &C[c].mu, &C[c].bnil, &C[c].nbk) != 6)
            return 2;
        C[c].brokers = xmalloc(sizeof(long long) * (size_t)(C[c].nbk + 1));
        for (long long j = 0; j < C[c].nbk; j++) if (fscanf(f, "%lld", &C[c].brokers[j]) != 1) return 2;
    }
    long long steps;
    int mode;
    if (fscanf(f, "%lld %d", &steps, &mode) != 2) return 2;
    if (f != stdin) fclose(f);

    char *msg = xmalloc(4096);
    kb_engine *e = NULL;
    int cur = -1;
    for (long long s = 0; s < steps; s++) {
        const int ci = (int)(s % ncfg);
        if (ci != cur) {                     /* a new RebalanceConfig: a new engine from pl */
            if (e) { kb_engine_destroy(e); destroyed++; }
            e = make_engine(P, n, &C[ci], msg);
            if (!e) return 1;
            cur = ci;
        }
        kb_change ch;
        const int rc = balance_call(e, mode, &ch);
        /* the Go side: FillDefaults ran (unless a validation step failed), then the
           returned partition was built with replacepl / addpl on pl */
        if (rc >= 0 || ch.step > KB_STEP_FILL_DEFAULTS) fill_defaults(P, n, &C[ci]);
        if (rc == KB_NOCHANGE) { printf("nochange\n"); break; }
        if (rc < 0) {
            kb_engine_last_error(e, msg, 4096);
            printf("error %d %s\n", rc, msg);
            break;
        }
        apply_change(P, &ch);
        printf("change %d %lld %d %lld %lld %d\n", ch.step, (long long)ch.partition, ch.kind,
               (long long)ch.from_broker, (long long)ch.to_broker, ch.slot);
    }
    if (e) { kb_engine_destroy(e); destroyed++; }
    printf("engines %d %d\n", created, destroyed);
    free(msg);
    return 0;
}
