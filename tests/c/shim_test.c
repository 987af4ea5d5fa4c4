/*
 * shim_test.c -- drives the C ABI (include/kbengine.h) exactly as the cgo shim of
 * INTEGRATION.md does: every array the engine reads is malloc'd C memory (no host
 * language memory crosses the boundary), one kb_engine_create per partition list,
 * then one kb_engine_balance per Balance() call (balancer.go:49-65) with
 * KB_SEM_GO (the reference's slice aliasing), kb_engine_last_error for the
 * "<Step>: <msg>" text, kb_engine_destroy.
 *
 * Input (whitespace separated, written by tests/test_shim_c.py):
 *   n_partitions
 *   per partition: topic partition nrep r_1..r_nrep weight num_replicas num_consumers nb b_1..b_nb
 *                  (nb = -1: nil Brokers)
 *   allow_leader rebalance_leaders min_replicas min_unbalance brokers_nil n_brokers b_1..b_n
 *   steps
 * Output: one line per Balance() call: "change <step> <pidx> <kind> <from> <to> <slot>",
 * "nochange", or "error <rc> <message>".
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

int main(int argc, char **argv) {
    FILE *f = argc > 1 ? fopen(argv[1], "r") : stdin;
    if (!f) { perror("input"); return 2; }
    long long n;
    if (fscanf(f, "%lld", &n) != 1 || n < 0) return 2;
    /* the shim's arena: C memory only */
    int64_t *rep = xmalloc(sizeof(int64_t) * (size_t)(16 * n + 1));
    int64_t *roff = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    double *w = xmalloc(sizeof(double) * (size_t)(n + 1));
    int64_t *nr = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t *nc = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t *pid = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t *sidx = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t *toff = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    size_t scap = 1024, sn = 0, nsets = 0, tcap = 1024, tn = 0;
    int64_t *sids = xmalloc(sizeof(int64_t) * scap);
    int64_t *soff = xmalloc(sizeof(int64_t) * (size_t)(n + 1));
    char *blob = xmalloc(tcap);
    roff[0] = 0; toff[0] = 0; soff[0] = 0;
    for (long long i = 0; i < n; i++) {
        char topic[256];
        long long part, k, nb;
        if (fscanf(f, "%255s %lld %lld", topic, &part, &k) != 3 || k < 0 || k > 16) return 2;
        size_t tl = strlen(topic);
        if (tn + tl > tcap) { tcap = 2 * (tn + tl); blob = realloc(blob, tcap); }
        memcpy(blob + tn, topic, tl); tn += tl; toff[i + 1] = (int64_t)tn;
        pid[i] = part;
        for (long long j = 0; j < k; j++) {
            long long r;
            if (fscanf(f, "%lld", &r) != 1) return 2;
            rep[roff[i] + j] = r;
        }
        roff[i + 1] = roff[i] + k;
        long long want, cons;
        if (fscanf(f, "%lf %lld %lld %lld", &w[i], &want, &cons, &nb) != 4) return 2;
        nr[i] = want; nc[i] = cons;
        if (nb < 0) { sidx[i] = -1; continue; }
        /* one set per listed Brokers slice (the shim deduplicates by content; a set per
           partition is equally valid input) */
        if (sn + (size_t)nb > scap) { scap = 2 * (sn + (size_t)nb); sids = realloc(sids, sizeof(int64_t) * scap); }
        for (long long j = 0; j < nb; j++) {
            long long b;
            if (fscanf(f, "%lld", &b) != 1) return 2;
            sids[sn++] = b;
        }
        sidx[i] = (int64_t)nsets;
        soff[++nsets] = (int64_t)sn;
    }
    kb_config *cfg = xmalloc(sizeof *cfg);
    memset(cfg, 0, sizeof *cfg);
    int al, rl, bnil;
    long long mr, nbk, steps;
    double mu;
    if (fscanf(f, "%d %d %lld %lf %d %lld", &al, &rl, &mr, &mu, &bnil, &nbk) != 6) return 2;
    int64_t *brokers = xmalloc(sizeof(int64_t) * (size_t)(nbk + 1));
    for (long long j = 0; j < nbk; j++) {
        long long b;
        if (fscanf(f, "%lld", &b) != 1) return 2;
        brokers[j] = b;
    }
    if (fscanf(f, "%lld", &steps) != 1) return 2;
    if (f != stdin) fclose(f);
    cfg->allow_leader = al; cfg->rebalance_leaders = rl; cfg->min_replicas = mr;
    cfg->min_unbalance = mu; cfg->brokers = brokers; cfg->n_brokers = nbk; cfg->brokers_nil = bnil;
    cfg->semantics = KB_SEM_GO;

    kb_cluster *cl = xmalloc(sizeof *cl);
    memset(cl, 0, sizeof *cl);
    cl->n_partitions = n; cl->replica_ids = rep; cl->replica_off = roff; cl->weight = w;
    cl->num_replicas = nr; cl->num_consumers = nc; cl->n_sets = (int64_t)nsets; cl->set_ids = sids;
    cl->set_off = soff; cl->set_idx = sidx; cl->topic_blob = blob; cl->topic_off = toff;
    cl->partition_id = pid;

    char *msg = xmalloc(4096);
    kb_engine *e = NULL;
    int rc = kb_engine_create(cl, cfg, &e);
    if (rc < 0) {
        msg[0] = 0;
        if (e) kb_engine_last_error(e, msg, 4096);
        printf("create-error %d %s\n", rc, msg);
        kb_engine_destroy(e);
        return 1;
    }
    /* the engine copied everything: the arena may go now (as the shim's defer does) */
    free(rep); free(roff); free(w); free(nr); free(nc); free(pid); free(sidx); free(toff);
    free(sids); free(soff); free(blob); free(brokers); free(cfg); free(cl);
    for (long long s = 0; s < steps; s++) {
        kb_change ch;
        rc = kb_engine_balance(e, &ch);
        if (rc == KB_NOCHANGE) { printf("nochange\n"); break; }
        if (rc < 0) {
            kb_engine_last_error(e, msg, 4096);
            printf("error %d %s\n", rc, msg);
            break;
        }
        printf("change %d %lld %d %lld %lld %d\n", ch.step, (long long)ch.partition, ch.kind,
               (long long)ch.from_broker, (long long)ch.to_broker, ch.slot);
    }
    free(msg);
    kb_engine_destroy(e);
    return 0;
}
