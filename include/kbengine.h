/*
 * kbengine.h -- C ABI of the MI355X kafkabalancer move-search engine.
 *
 * This is the drop-in boundary for the reference's step pipeline
 * (balancer.go:34-65).  The reference seam is the step signature
 *     func(*PartitionList, RebalanceConfig) (*PartitionList, error)
 * dispatched by Balance() (balancer.go:49-65).  A host (the cgo shim shown in
 * INTEGRATION.md, the C++ host library in kafkabalancer_amd/host, or the
 * Python mirror) marshals a PartitionList into kb_cluster once, then asks the
 * engine for one Balance() step at a time (kb_engine_balance) or for a whole
 * -max-reassign plan that stays resident on the GPU (kb_engine_plan).
 *
 * All entry points are plain C: pointers + sizes, no HIP or torch types.
 * Return values: >= 0 success (status), < 0 a KB_ERR_* code; the text of the
 * last error is available from kb_engine_last_error().
 */
#ifndef KBENGINE_H
#define KBENGINE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KB_ABI_VERSION 11

/* step indices == position in the reference's steps table (balancer.go:34-44) */
enum kb_step {
    KB_STEP_VALIDATE_WEIGHTS = 0,     /* steps.go:7-23 */
    KB_STEP_VALIDATE_REPLICAS = 1,    /* steps.go:27-36 */
    KB_STEP_FILL_DEFAULTS = 2,        /* steps.go:39-66 */
    KB_STEP_REMOVE_EXTRA = 3,         /* steps.go:70-89 */
    KB_STEP_ADD_MISSING = 4,          /* steps.go:93-113 */
    KB_STEP_MOVE_DISALLOWED = 5,      /* steps.go:117-143 */
    KB_STEP_REASSIGN_LEADERS = 6,     /* steps.go:301-307 -> distributeLeaders :234-282 */
    KB_STEP_MOVE_LEADERS = 7,         /* steps.go:292-298 -> move(leaders=true) */
    KB_STEP_MOVE_NON_LEADERS = 8      /* steps.go:286-288 -> move(leaders=false) */
};
/* step masks of kb_engine_step: bit (1u << kb_step) per entry of the steps table */
#define KB_STEP_BIT(s) (1u << (s))
#define KB_STEPS_ALL 0x1FFu

/* kb_change.status / return value of kb_engine_balance */
enum { KB_NOCHANGE = 0, KB_CHANGE = 1,
       KB_RETRY = 2 /* kb_engine_step_finish only: loads were refolded exactly, redo the step */,
       KB_GROW = 3  /* sharded steps: a rank summary overflowed; kb_engine_summary_bytes grew,
                       re-allocate the exchange buffers and redo the step */ };

/* kinds of change (what replacepl/addpl did, utils.go:166-202) */
enum { KB_KIND_NONE = 0, KB_KIND_REPLACE = 1, KB_KIND_REMOVE = 2, KB_KIND_ADD = 3, KB_KIND_SWAP = 4 };

/* how a change reaches the partition list */
enum {
    KB_SEM_APPLIED = 0,   /* every change is applied to the state (default) */
    KB_SEM_GO = 1         /* emulate Go slice aliasing: a remove shifts in place and keeps
                             the slice length (duplicates the last replica), an add is not
                             visible to the next call (utils.go:178,199-202) */
};

/* error codes */
enum {
    KB_OK = 0,
    KB_ERR_INVALID = -1,        /* bad arguments */
    KB_ERR_HIP = -2,            /* HIP runtime error / no device */
    KB_ERR_UNSUPPORTED = -3,    /* outside the engine's sizing limits */
    KB_ERR_STEP = -4,           /* a step returned an error (Balance() error); see last_error */
    KB_ERR_CAPACITY = -5,       /* a per-broker list or the contender buffer overflowed */
    KB_ERR_PANIC = -6           /* input on which the reference Go code panics */
};

/* Cluster state, the marshalled PartitionList (kafkabalancer.go:40-58).
 * Arrays are host memory; the engine copies them to the device once. */
typedef struct {
    int64_t n_partitions;
    const int64_t *replica_ids;     /* concatenated Replicas of all partitions */
    const int64_t *replica_off;     /* [n_partitions + 1] offsets into replica_ids */
    const double *weight;           /* [n] Weight (0 = absent) */
    const int64_t *num_replicas;    /* [n] NumReplicas (0 = absent) */
    const int64_t *num_consumers;   /* [n] NumConsumers (may be NULL => all 0) */
    int64_t n_sets;                 /* distinct Brokers lists */
    const int64_t *set_ids;         /* concatenated Brokers lists */
    const int64_t *set_off;         /* [n_sets + 1] */
    const int64_t *set_idx;         /* [n] index of the partition's Brokers list, -1 = nil */
    /* optional, used only to format error messages like the reference */
    const char *topic_blob;         /* concatenated topic names (may be NULL) */
    const int64_t *topic_off;       /* [n + 1] */
    const int64_t *partition_id;    /* [n] PartitionID (may be NULL) */
} kb_cluster;

/* RebalanceConfig (balancer.go:12-20) plus engine options */
typedef struct {
    int32_t allow_leader;           /* AllowLeaderRebalancing */
    int32_t rebalance_leaders;      /* RebalanceLeaders */
    int64_t min_replicas;           /* MinReplicasForRebalancing */
    double min_unbalance;           /* MinUnbalance */
    const int64_t *brokers;         /* Brokers (explicit -broker-ids) */
    int64_t n_brokers;
    int32_t brokers_nil;            /* 1 => Brokers == nil ("auto") */
    int32_t semantics;              /* KB_SEM_* */
    int32_t device;                 /* HIP device ordinal */
    int32_t list_slack;             /* extra entries per broker list (0 = default 1024) */
    int64_t shard_begin;            /* partitions [shard_begin, shard_end) scanned by this */
    int64_t shard_end;              /*   engine; 0,0 = all (multi-GPU sharding) */
    int32_t exact_unbalance;        /* 1 => unbalance_after is always the exact sequential
                                       fold (costs one O(B) fold per step); 0 => exact only
                                       when a near tie needed it, else within eps */
    int32_t time_kernels;           /* 1 => HIP events around every launch (kb_engine_timings) */
} kb_config;

/* One step's result: the change Balance() would return (balancer.go:49-65). */
typedef struct {
    int32_t status;                 /* KB_NOCHANGE / KB_CHANGE / < 0 error */
    int32_t step;                   /* kb_step that produced it (or failed) */
    int32_t kind;                   /* KB_KIND_* */
    int32_t slot;                   /* replica slot that changed */
    int64_t partition;              /* index into the cluster's partition list */
    int64_t from_broker;            /* broker id replaced/removed (-1 for add) */
    int64_t to_broker;              /* broker id placed/added (-1 for remove) */
    double unbalance_before;        /* su: getUnbalanceBL before the step (move steps) */
    double unbalance_after;         /* cu: scored unbalance of the chosen move */
    int32_t exact;                  /* 1 if unbalance_after is the exact sequential fold */
    int32_t err_code;               /* engine-internal error detail */
    int64_t err_broker;             /* broker id named in the error message */
} kb_change;

typedef struct {
    int64_t steps;                  /* steps executed */
    int64_t candidates;             /* (partition, slot, target) moves scored (SURVEY 8d metric 1) */
    int64_t contenders;             /* near-tie candidates verified with exact folds */
    int64_t exact_folds;            /* exact getUnbalanceBL evaluations */
    int64_t scan_bytes;             /* algorithmic bytes read by the scan kernel, last step */
    double device_ms;               /* device time of the last kb_engine_plan (HIP events) */
    int64_t n_brokers;              /* dense broker universe size */
    int64_t n_sets;
    int32_t integral;               /* 1 => loads are exact under incremental updates */
    int32_t max_replicas;           /* replica slots per partition on the device */
    int64_t refreshes;              /* exact refolds of the approximate loads (k_refresh) */
    int64_t exact_halts;            /* steps that needed exact loads to decide */
    int64_t scan_workgroups;        /* k_scan workgroups (one record each) */
    int64_t retries;                /* steps re-scanned with the census bound tightened to the
                                       step minimum after a near-tie spill overflow (ABI 3) */
    int64_t spill_grows;            /* near-tie spill buffer growths (exact ties over many
                                       brokers; the step ran again, ABI 5) */
    int64_t blocks_scanned;         /* incremental mode: 128-partition blocks the scans read
                                       (kb_engine_set_incremental, ABI 6) */
    int64_t relists;                /* per-broker partition lists laid out again after one ran
                                       out of slack (kb_config.list_slack, ABI 8) */
    int64_t fused_pairs;            /* 1: a plan's scan + step run as one launch (k_pair, ABI 8) */
    int64_t fused_summaries;        /* 1: a sharded scan and its rank summary run as one launch
                                       (k_scansum, ABI 10) */
    int64_t eager;                  /* 1: touched brokers are refolded beside the next scan
                                       (eager refolds; ABI 10) */
    int64_t eager_switches;         /* plans switched from lazy loads to eager refolds (ABI 10) */
    int64_t fast_preps;             /* steps whose order / positions / set records were left to the
                                       next launch (the deferred prep, ABI 11) */
} kb_stats;

typedef struct kb_engine kb_engine;

/* ABI version of the loaded library (== KB_ABI_VERSION) */
int kb_abi_version(void);

/* Diagnostics opt-in (process-wide, default off).  Only after kb_set_diagnostics(1) does the
 * library read its A/B and diagnostic switches from the environment at kb_engine_create
 * (KB_FUSE, KB_EAGER, KB_PAIR_WAIT_TICKS, ...: the list is in INTEGRATION.md); a drop-in host
 * never calls it, so an inherited environment cannot change the engine's kernel paths.  The
 * test suite and the bench scripts opt in (kafkabalancer_amd/engine.py: KB_DIAGNOSTICS=1). */
void kb_set_diagnostics(int on);
int kb_diagnostics_enabled(void);

/* Validates + fills defaults like ValidateWeights/ValidateReplicas/FillDefaults
 * (steps.go:7-66) and uploads the SoA state.  A validation error does not fail
 * creation: it is returned by the first kb_engine_balance(), like Balance(). */
int kb_engine_create(const kb_cluster *cluster, const kb_config *cfg, kb_engine **out);

/* One Balance() call: runs the fused step pipeline on the device, applies the
 * change to the device state (per cfg->semantics), returns KB_CHANGE /
 * KB_NOCHANGE or < 0.  Equivalent of balancer.go:49-65 + the aliasing write.
 * Same as kb_engine_step(e, KB_STEPS_ALL, out). */
int kb_engine_balance(kb_engine *e, kb_change *out);

/* One Balance() restricted to the steps whose bit is set in step_mask, in the reference's
 * order (balancer.go:34-44): with a single bit it is that step function alone, e.g.
 * KB_STEP_BIT(KB_STEP_MOVE_NON_LEADERS) = MoveNonLeaders(pl, cfg) (steps.go:286-288), so a
 * host that keeps the reference's steps table and Balance() binds each entry to one call
 * (INTEGRATION.md).  Returns KB_CHANGE (out = the change, applied on the device per
 * cfg->semantics), KB_NOCHANGE (the step returned nil, nil) or < 0 ("<Step>: <msg>" in
 * kb_engine_last_error).  ValidateWeights / FillDefaults ran at create: their bits change
 * nothing (a create-time validation error is returned by its own step and every later
 * one).  After a KB_NOCHANGE the next call resolves the same scan of the unchanged state
 * (no second scan): a host walking the table pays one scan per Balance(). */
int kb_engine_step(kb_engine *e, uint32_t step_mask, kb_change *out);

/* Device-resident plan: up to max_steps Balance() calls without host
 * round trips (run()'s loop with -complete-partition=false,
 * kafkabalancer.go:181-221).  Stops after the first no-change or error.
 * Writes the changes to out[0..*n_out).  Returns the last status. */
int kb_engine_plan(kb_engine *e, int64_t max_steps, kb_change *out, int64_t *n_out);

/* kb_engine_plan that also stops after the first applied change whose partition is not
 * stop_part (that change is applied and returned last): run()'s -complete-partition loop
 * (kafkabalancer.go:193-221) -- past -max-reassign the reference keeps calling Balance() while
 * the change is on the completing partition, and the first change that does not compare ends
 * the loop (applied: the probe).  stop_part < 0: kb_engine_plan.  (ABI 11) */
int kb_engine_plan_until(kb_engine *e, int64_t max_steps, int64_t stop_part, kb_change *out, int64_t *n_out);

/* Current replicas of partition i (after applied changes); returns the count. */
int64_t kb_engine_replicas(kb_engine *e, int64_t i, int64_t *buf, int64_t cap);

/* Exact broker loads (getBrokerLoad, utils.go:92-105) for the dense universe;
 * ids[k], loads[k] for k < return value. */
int64_t kb_engine_loads(kb_engine *e, int64_t *ids, double *loads, int64_t cap);

/* getUnbalanceBL (utils.go:119-147) of the current state over bl_move order */
double kb_engine_unbalance(kb_engine *e);

int kb_engine_stats(kb_engine *e, kb_stats *out);

/* Per-kernel device time of the plans since kb_engine_set_timing: ms[k] = summed duration
 * of kernel k, launches[k] = count, for k in {0 k_step (resolve + apply + prep), 1 k_scan,
 * 2 k_refresh, 3 the conditional bound pass (k_scan ubpass + k_ubinit; mode 2 only),
 * 4 k_step and 5 k_scan first-workgroup-start .. last-end (mode 1 only)}.  In mode 1,
 * k = 0 / 1 are device-clock spans from the end of the kernel before (dispatch included:
 * the interval rocprofv3 --kernel-trace reports), over back-to-back launches; 6 (mode 1, fused
 * pairs) k_pair from its first workgroup's start to the step workgroup's end; 7 / 8 (mode 1)
 * an eager refold workgroup's start .. end / start .. its list edit done.  Returns 9. */
int kb_engine_timings(kb_engine *e, double *ms, int64_t *launches, int n);

/* Kernel timing for the following plans (resets the sums): 0 off; 1 k_scan / k_step from
 * the device clock (workgroups stamp the 100 MHz clock; no events between them), the rest
 * from HIP events; 2 HIP events around every launch (each event adds its own ~2-3 us to
 * the interval around a launch). */
int kb_engine_set_timing(kb_engine *e, int32_t on);

/* Diagnostic (ABI 9): host phases of the kb_engine_plan calls since kb_engine_set_timing, in
 * microseconds: us[0] control-block reset, [1] enqueue of the batches, [2] waiting for them
 * (the batch-end control-block / log transfer included), [3] log conversion, [4] the
 * number of calls.  Returns 5. */
int kb_engine_host_timings(kb_engine *e, double *us, int n);

/* Incremental rescoring mode (single GPU, off by default): after a
 * move() step (MoveLeaders / MoveNonLeaders, steps.go:145-232) the next scan reads only
 * the partition blocks a lower-bound certificate cannot exclude from the step's
 * near-tie window, and reuses the last full scan's candidate counts.  Results are
 * identical to the full scan (same changes, same loads); only the bytes read differ
 * (kb_stats.blocks_scanned).  Returns KB_OK. */
int kb_engine_set_incremental(kb_engine *e, int32_t on);

/* Diagnostic: accumulated in-kernel phase stamps (100 MHz ticks) of k_step
 * phases and scan event counts (up to 32 slots, returns the slot count);
 * non-zero only in a -DKB_STAMPS build. */
int kb_engine_stamps(kb_engine *e, uint64_t *out, int n);

/* Diagnostic: average device time (us) of the scan kernel over `iters`
 * back-to-back launches on the current state (nothing is applied). */
int kb_engine_bench_scan(kb_engine *e, int iters, double *avg_us);
/* Diagnostic: k_step alone on a fixed input (state snapshotted after a scan, restored
 * before each launch); HIP-event time per launch in *avg_us.  The engine is left as it
 * was after the scan.  (Phase costs: run it on -DKB_STOP_AT=k builds.) */
int kb_engine_bench_step(kb_engine *e, int iters, double *avg_us);

/* Reference-format message of the last error ("<Step>: partition Partition(t,p,[..]) ..."). */
int kb_engine_last_error(kb_engine *e, char *buf, size_t n);

void kb_engine_destroy(kb_engine *e);

/* ---- multi-GPU step phases (one engine per rank, partitions sharded) ----
 * A step is:  begin (local scan) -> exchange of fixed-size summaries between
 * ranks (all-gather, done by the caller over RCCL) -> finish (identical
 * resolution on every rank).  `summary` and `gathered` are DEVICE pointers. */
/* bytes of one rank summary: 1936 (56 near-tie keys) to start with; after a KB_GROW it
 * is 8x the keys (up to 2048), the same on every rank */
int64_t kb_engine_summary_bytes(kb_engine *e);
int kb_engine_step_begin(kb_engine *e, void *summary_dev);
int kb_engine_step_finish(kb_engine *e, const void *gathered_dev, int32_t n_ranks, kb_change *out);
/* hipStream_t on which all engine work is enqueued (NULL = engine-owned stream) */
int kb_engine_set_stream(kb_engine *e, void *hip_stream);

/* Batched multi-GPU steps (no host round trip per step): sharded_reset(budget) once,
 * then per step sharded_scan(summary) -> all-gather -> sharded_resolve(gathered, n),
 * then sharded_collect: the steps' changes (the log of the batch, at most cap), and
 * KB_CHANGE (go on), KB_RETRY (loads were refolded exactly; go on), or the plan's last
 * status (KB_NOCHANGE / error) as the last entry.  Steps after a halt are no-ops. */
int kb_engine_sharded_reset(kb_engine *e, int64_t budget_steps);
int kb_engine_sharded_scan(kb_engine *e, void *summary_dev);
int kb_engine_sharded_resolve(kb_engine *e, const void *gathered_dev, int32_t n_ranks);
int kb_engine_sharded_collect(kb_engine *e, kb_change *out, int64_t cap, int64_t *n_out);

/* ---- RCCL-driven sharded plan (ABI 9): the per-step exchange without a host in the loop.
 * Rank 0 calls kb_comm_unique_id and the caller broadcasts the KB_COMM_ID_BYTES bytes to
 * every rank (any channel: torch.distributed, MPI, a file); each rank then binds its engine
 * (created with its shard in kb_config.shard_begin / shard_end) to the communicator and
 * calls kb_engine_sharded_plan with the same max_steps.  Per step: the shard's scan and
 * rank summary, ncclAllGather of the fixed-size summaries on the engine's stream, the
 * identical resolve + apply + prep on every rank; 64 steps per host round trip.  RCCL is
 * bound at run time (KB_ERR_UNSUPPORTED without it).  Result convention of kb_engine_plan;
 * every rank returns the same changes. */
#define KB_COMM_ID_BYTES 128
int kb_comm_unique_id(unsigned char *id);
int kb_engine_comm_init(kb_engine *e, int32_t n_ranks, int32_t rank, const unsigned char *id);
int kb_engine_sharded_plan(kb_engine *e, int64_t max_steps, kb_change *out, int64_t *n_out);

#ifdef __cplusplus
}
#endif
#endif
