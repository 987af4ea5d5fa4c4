/*
 * kb_oracle.h -- CPU restatement of the kjelle/kafkabalancer balancer.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in kafkabalancer_amd/ (the product) may
 * include, link or call this.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, and only as the checker.
 *
 * Parity pin: the 16 TestBalancing cases (reference balancer_test.go:36-186)
 * and the CLI exit-code cases (kafkabalancer_test.go:11-166), stored as data
 * under tests/golden/.  The reference is Go; no Go toolchain exists here or on
 * the GPU box, so the reference itself cannot be run.
 *
 * Data model mirrors kafkabalancer.go:16-58.  Replica and broker lists are Go
 * slices {ptr,len,cap}; replacepl()/addpl() keep Go's aliasing behaviour
 * (utils.go:166-202) when OR_SEM_GO is selected.
 */
#ifndef KB_ORACLE_H
#define KB_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { int64_t *a; int64_t len, cap; } or_slice;  /* a == NULL => nil */

typedef struct {
    const char *topic;          /* TopicName */
    int64_t partition;          /* PartitionID */
    or_slice replicas;          /* []BrokerID */
    double weight;              /* Weight */
    int64_t num_replicas;       /* NumReplicas */
    or_slice brokers;           /* Brokers (nil = default) */
    int64_t num_consumers;      /* NumConsumers */
} or_partition;

typedef struct {
    int64_t version;
    or_partition *parts;
    int64_t n;
} or_plist;

typedef struct {
    int allow_leader;           /* AllowLeaderRebalancing */
    int rebalance_leaders;      /* RebalanceLeaders */
    int64_t min_replicas;       /* MinReplicasForRebalancing */
    double min_unbalance;       /* MinUnbalance */
    int complete_partition;     /* CompletePartition */
    int64_t *brokers;           /* Brokers (NULL + nbrokers_nil=1 => nil) */
    int64_t nbrokers;
    int brokers_nil;
} or_config;

/* change kinds */
enum { OR_NONE = 0, OR_REPLACE = 1, OR_REMOVE = 2, OR_ADD = 3, OR_SWAP = 4 };
/* semantics of how a returned change reaches pl */
enum { OR_SEM_GO = 0, OR_SEM_APPLIED = 1 };

typedef struct {
    int status;                 /* 0 = no change, 1 = change, -1 = error */
    int step;                   /* index into the steps table (balancer.go:34-44) */
    int64_t pidx;               /* partition index in pl */
    int kind;
    int64_t from, to;           /* broker ids (to=-1 for removes) */
    int64_t slot;               /* replica slot touched */
    or_partition part;          /* the returned partition (Go value copy; replicas may alias pl) */
    double su, cu;              /* unbalance before / chosen (move steps only) */
    char err[1024];             /* "<StepName>: <message>" */
} or_result;

int  or_balance(or_plist *pl, const or_config *cfg, int semantics, or_result *res);
/* Balance() over the steps in mask only (bit k = steps table entry k); 0x1FF = or_balance */
int  or_step(or_plist *pl, const or_config *cfg, int semantics, unsigned mask, or_result *res);

/* run() main loop (kafkabalancer.go:177-233) after parsing.  Writes the
 * output JSON (Go encoding/json format, trailing newline) into *out (malloc'd)
 * or an error message into err.  Returns the CLI exit code (0 or 3). */
int  or_run_plan(or_plist *pl, const or_config *cfg, int64_t max_reassign,
                 int complete_partition, int full_output, int unique, int semantics,
                 char **out, char *err, size_t errlen, int64_t *nsteps_out);

/* Bounded timing sample of move() (steps.go:210-297): scores the candidates of
 * the first max_parts partitions exactly as the reference does. Returns the
 * number of candidates scored; best unbalance in *cu. */
int64_t or_move_sample(or_plist *pl, const or_config *cfg, int leaders,
                       int64_t max_parts, double *cu);

/* getUnbalanceBL on an explicit (ids, loads) list in the given order (utils.go:119-147) */
double or_unbalance(const double *loads, int64_t n);

/* Go encoding/json float64 formatting (shortest round trip). buf >= 40 */
void or_format_float(double x, char *buf);

void or_free(void *p);

/* Worker threads of move() / MoveDisallowedReplicas' search (default 1).  Any
 * count gives the identical result (chunked in order, merged in order). */
void or_set_threads(int n);

/* Golden generation only: move() scores every candidate in O(1) first and folds exactly
 * (the reference's getUnbalanceBL) only those within a window that provably holds the
 * reference's choice -- the same result as the literal loop (kb_oracle.c: move_window;
 * tests/test_oracle.py checks it).  Default off. */
void or_set_window(int on);
int64_t or_walk_stops(void);
void or_reset_walk_stops(void);

/* Build a partition list from flat arrays.  Brokers lists are deduplicated
 * into sets; partitions with the same set_idx share one slice (as FillDefaults
 * makes them share in Go).  set_idx < 0 => nil Brokers. rep_nil may be NULL. */
or_plist *or_plist_build(int64_t n, const char *topic_blob, const int64_t *topic_off,
                         const int64_t *partition, const int64_t *rep_flat, const int64_t *rep_off,
                         const int8_t *rep_nil, const double *weight, const int64_t *num_replicas,
                         int64_t nsets, const int64_t *set_flat, const int64_t *set_off,
                         const int64_t *set_idx, const int64_t *num_consumers);
int64_t or_plist_replicas(const or_plist *pl, int64_t i, int64_t *buf, int64_t cap);
int64_t or_plist_len(const or_plist *pl);

#ifdef __cplusplus
}
#endif
#endif
