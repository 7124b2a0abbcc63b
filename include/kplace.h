/*
 * kplace.h — C-ABI of the MI355X-native batch placement engine (libkplace.so).
 *
 * This is the drop-in boundary for kubeinfer's placement hot path. The
 * reference (Moore-Z/Kubernetes-Native-Distributed-AI-Job-Scheduler, Go module
 * github.com/Moore-Z/kubeinfer) has no FFI and no placement code of its own:
 *   - its per-job driver is LLMServiceReconciler.Reconcile
 *     (internal/controller/llmservice_controller.go:66-174), one CR at a time;
 *   - it builds one Deployment per CR with Spec.Replicas identical pods
 *     (desiredDeployment, llmservice_controller.go:182-313) and leaves the node
 *     choice of each pod to the external kube-scheduler (Filter/Score/selectHost).
 * Every entry point below replaces that per-pod Filter/Score/Bind pass with one
 * batched solve of the whole pending queue; the Go caller a maintainer would add
 * (pkg/placement, cgo) is shown in INTEGRATION.md. The placement semantics are
 * frozen in DESIGN.md §2 ("Placement spec"), restated on the CPU in oracle/.
 *
 * Conventions (all entry points):
 *   - SoA, row-major by dimension: req[d*J + j], cap[d*N + n], used[d*N + n].
 *   - Caller owns every buffer; the library copies what it needs and retains
 *     no caller pointer after return.
 *   - Errors are negative int codes (KP_E*), never aborts or C++ exceptions.
 *   - One call at a time per kp_ctx (internal mutex). Every entry calls
 *     hipSetDevice itself, so calls may come from any OS thread (cgo hops
 *     threads between calls).
 */
#ifndef KPLACE_H
#define KPLACE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KP_ABI_VERSION 8  /* 4: kp_last_error_r; 5: kp_timing.incr_rounds;
                              6: kp_score_dev, kp_timing.score_form / score_classes;
                              7: kp_timing phase split (cand/xchg/pass_ms,
                                 kp_set_profiling level 2); kp_load_running and
                                 kp_preempt are collective on world_size > 1
                                 contexts (every rank calls them, in the same
                                 order as its kp_solve calls);
                              8: kp_timing.rccl_calls (was padding),
                                 kp_last_timing_shards; kp_last_timing on a
                                 kp_create_multi context = max over shards */

/* ---- limits ------------------------------------------------------------ */
#define KP_MAX_DIMS 8       /* resource dimensions per job/node               */
#define KP_MAX_CAND 32       /* top-K candidate nodes kept per unit per round  */
#define KP_MAX_GANG 64      /* members of one all-or-nothing gang             */
#define KP_MAX_VALUE ((int64_t)1 << 56) /* bound on req/cap/used entries       */

/* ---- error codes -------------------------------------------------------- */
#define KP_OK 0
#define KP_EINVAL (-1)   /* malformed snapshot / params / arguments            */
#define KP_EHIP (-2)     /* HIP runtime error                                  */
#define KP_ERCCL (-3)    /* RCCL error (multi-GPU contexts)                    */
#define KP_ENOMEM (-4)   /* host or device allocation failed                   */
#define KP_ESTATE (-5)   /* call order violated (e.g. solve before load)       */
#define KP_ENODEV (-6)   /* no usable gfx950 device                            */

/* ---- score modes -------------------------------------------------------- */
#define KP_SCORE_MOST_ALLOCATED 0  /* bin-pack (kube-scheduler MostAllocated)  */
#define KP_SCORE_LEAST_ALLOCATED 1 /* spread  (kube-scheduler LeastAllocated) */

/* ---- node tie-break modes ------------------------------------------------ */
/* Both act on the node's canonical position pos(n): its rank when the nodes
   are sorted by capacity vector (dim 0 first), then by index (DESIGN.md
   §2.3). With one capacity vector for all nodes pos(n) = n. */
#define KP_TIE_NODE_INDEX 0 /* equal scores: lowest canonical position wins    */
#define KP_TIE_ROTATED 1    /* equal scores: per-job Weyl rotation of the
                               canonical position (deterministic stand-in for
                               kube-scheduler's random selectHost)            */

/* ---- score sentinels ---------------------------------------------------- */
#define KP_SCORE_INFEASIBLE (-1) /* score-matrix entry of an infeasible pair  */
#define KP_SCORE_NONE (-1)       /* score_of_job of an unplaced job           */

/* ---- status of a job after a solve -------------------------------------- */
#define KP_JOB_PLACED 0
#define KP_JOB_NO_FIT 1      /* no node can host it (or its gang) any more    */
#define KP_JOB_ROUND_LIMIT 2 /* still unresolved when max_rounds ran out      */

/*
 * Snapshot of the pending queue and the node table.
 * Job side, from the LLMService CRD (api/v1/llmservice_types.go:25-52): one
 * job = one replica; the Spec.Replicas replicas of one CR form one gang
 * (contiguous job indices, identical req/prio, all-or-nothing).
 */
typedef struct kp_snapshot {
  int32_t J, N, D;
  const int64_t *req;          /* [D*J] >= 0                                  */
  const int64_t *cap;          /* [D*N] >= 0                                  */
  const int64_t *used;         /* [D*N] 0 <= used <= cap; NULL = all zero     */
  const int32_t *prio;         /* [J] higher first; NULL = all 0              */
  const int32_t *gang_id;      /* [J] <0 = singleton; NULL = all singletons   */
  const int32_t *gang_size;    /* [J] checked against the run length; NULL ok */
  const int32_t *topo_domain;  /* [N] >= 0 (rack / xGMI island); NULL = n     */
  /* [J] topo domain this job prefers, -1 = none; NULL = all -1. The
     CacheStrategy "shared" term (api/v1/llmservice_types.go:42-44): the
     domain of the node running the CR's Status.CacheCoordinator (:60), so
     replicas that fetch the model from the coordinator stay on its xGMI
     island / rack (docs/PROJECT_ROADMAP.md:173-174). Equal within a gang. */
  const int32_t *affinity;
} kp_snapshot;

/* Scoring / assignment knobs (manager flags in the Go host). */
typedef struct kp_params {
  int32_t w_dim[KP_MAX_DIMS]; /* per-dim utilisation weight, 0..65535         */
  int32_t score_mode;         /* KP_SCORE_*                                   */
  int32_t gpu_dim;            /* dim holding the GPU count, -1 = none         */
  int32_t w_gpu_fit;          /* bonus when a job takes exactly the node's
                                 remaining free GPUs, 0..2^20                 */
  int32_t w_spread;           /* penalty per same-gang member already planned
                                 into the node's topo domain, 0..2^20         */
  int32_t tie_mode;           /* KP_TIE_*                                     */
  uint32_t tie_seed;          /* salt of the rotated tie-break                */
  int32_t max_rounds;         /* 0 = until every unit is resolved             */
  int32_t n_cand;             /* top-K candidates per unit, 1..KP_MAX_CAND    */
  int32_t util_scale;         /* per-dim utilisation scale S, 1..1024
                                 (100 = kube-scheduler MaxNodeScore)          */
  int32_t max_passes;         /* acceptance passes per round, 1..64           */
  int32_t w_affinity;         /* bonus when the node's topo domain equals the
                                 job's affinity domain, 0..2^20               */
} kp_params;

/* Fills *p with the documented defaults. */
void kp_params_default(kp_params *p);

typedef struct kp_result {
  int32_t *node_of_job;  /* [J] node index, -1 = unplaced                     */
  int32_t *score_of_job; /* [J] snapshot score of the chosen node, -1 = none  */
  int32_t *status_of_job;/* [J] KP_JOB_*; NULL = not wanted                   */
  int64_t *used_out;     /* [D*N] node usage after commit; NULL = not wanted  */
  /* filled by the library: */
  int32_t rounds;        /* auction rounds executed                           */
  int32_t passes;        /* acceptance passes executed (all rounds)           */
  int32_t placed_jobs;
  int32_t unplaced_jobs;
  int32_t units;         /* gangs + singletons                                */
  int64_t pairs_scored;  /* sum over rounds of (active units x N)             */
} kp_result;

/* ---- context ------------------------------------------------------------- */
typedef struct kp_ctx kp_ctx;

typedef struct kp_config {
  int32_t device;        /* HIP device ordinal (-1 = current)                 */
  int32_t world_size;    /* 1 = single GPU; >1 = one process per GPU          */
  int32_t rank;          /* this process' rank in [0, world_size)             */
  const void *nccl_id;   /* 128-byte ncclUniqueId from kp_dist_unique_id on
                            rank 0, broadcast by the caller; NULL if world 1,
                            or for a host-staged exchange (kp_set_allgather) */
  int64_t max_pairs_matrix; /* cap on score-matrix entries per chunk
                               (0 = library default)                         */
} kp_config;

int kp_create(kp_ctx **out, const kp_config *cfg);
/*
 * One context over n_gpus GPUs of this node, for a single manager process
 * (cmd/manager/main.go:157-200 runs ONE process with one reconciler,
 * :181-187): the library runs one worker thread per GPU, each owning a
 * row shard of the pending units, and exchanges candidates
 * over RCCL (communicators from ncclCommInitAll inside the library) when the
 * ids are distinct, or through host memory when an id repeats (one GPU
 * driving several shards: testing). Every other entry point accepts the
 * returned context unchanged; outputs come from shard 0 (all shards commit
 * identical placements). cfg: only max_pairs_matrix is read (may be NULL).
 */
int kp_create_multi(kp_ctx **out, const int32_t *gpu_ids, int32_t n_gpus,
                    const kp_config *cfg);
void kp_destroy(kp_ctx *ctx);
/* Generic text of an error code (static storage). */
const char *kp_strerror(int code);
/* Detailed text of the last error returned on this context (the HIP/RCCL
   call and its message), "" if none. Kept per context, not per thread (cgo
   hops OS threads). The pointer stays valid for the context's lifetime; a
   later failing call on ctx may overwrite the text while it is read, so a
   caller with concurrent calls on one context uses kp_last_error_r. */
const char *kp_last_error(kp_ctx *ctx);
/* The same text copied into buf (NUL-terminated, truncated to len - 1 bytes)
   under the context lock. Returns the full length of the message. */
int kp_last_error_r(kp_ctx *ctx, char *buf, size_t len);
int kp_abi_version(void);
/* Writes the 128-byte RCCL unique id for a multi-process context. */
int kp_dist_unique_id(void *out128);
/* Host-staged candidate exchange for a multi-process context created without
 * an RCCL id: `fn` all-gathers `bytes` from every rank into `recv` (rank-major,
 * world_size * bytes) and returns 0 on success. It is called on the thread that
 * calls kp_solve; the library stages device buffers through host memory around
 * it. Meant for transports other than RCCL and for testing the sharded solve
 * with several processes on one GPU (RCCL needs one GPU per rank). */
typedef int (*kp_allgather_fn)(void *user, const void *send, size_t bytes, void *recv);
int kp_set_allgather(kp_ctx *ctx, kp_allgather_fn fn, void *user);

/*
 * One-shot placement: validate + upload the snapshot, solve, download, under
 * ONE acquisition of the context lock (concurrent kp_place calls on one
 * context never interleave their snapshots). Synchronous. Replaces one
 * kube-scheduler cycle per pending pod. A failed load leaves the context
 * with no snapshot loaded (later kp_solve/kp_fetch return KP_ESTATE).
 */
int kp_place(kp_ctx *ctx, const kp_snapshot *s, const kp_params *p,
             kp_result *r);

/* ---- staged interface (device-resident snapshot, streaming churn) -------- */
/* Upload the node table; it stays resident and is updated by every solve. */
int kp_load_nodes(kp_ctx *ctx, int32_t N, int32_t D, const int64_t *cap,
                  const int64_t *used, const int32_t *topo_domain);
/* Upload (validate, group into gangs, rank) the pending queue. */
int kp_load_jobs(kp_ctx *ctx, int32_t J, const int64_t *req,
                 const int32_t *prio, const int32_t *gang_id,
                 const int32_t *gang_size, const int32_t *affinity);
/* Solve the loaded queue against the resident node table and commit the
   accepted placements into it. Inputs must already be resident. */
int kp_solve(kp_ctx *ctx, const kp_params *p, kp_result *stats);
/* Copy the last solve's per-job outputs (and optionally node usage) out. */
int kp_fetch(kp_ctx *ctx, kp_result *r);
/* Streaming churn: used[d][node_idx[k]] += delta[d*K + k] (negative = job
   completion). Fails with KP_EINVAL if a node would leave [0, cap]. */
int kp_apply_delta(kp_ctx *ctx, const int32_t *node_idx, const int64_t *delta,
                   int32_t K);
/* Restore the resident node usage to what the last kp_load_nodes uploaded
   (device-side copy; for repeated what-if solves on one snapshot). */
int kp_reset_nodes(kp_ctx *ctx);

/*
 * Filter + score pass only (the materialised outputs the north_star names):
 * for jobs [job_lo, job_hi) of the loaded queue against the resident node
 * table, writes score[(j-job_lo)*N + n] (KP_SCORE_INFEASIBLE if the job does
 * not fit) and the feasibility bitmask mask[(j-job_lo)*ceil(N/64) + n/64]
 * bit n%64. Either output may be NULL.
 */
int kp_score(kp_ctx *ctx, const kp_params *p, int32_t job_lo, int32_t job_hi,
             int32_t *score, uint64_t *mask);

/*
 * The same filter + score pass into DEVICE memory that the caller owns on the
 * context's GPU (e.g. a consumer that keeps the matrix in HBM for its own
 * kernels): rows [job_lo, job_hi) with the padded row stride Ns =
 * round_up(N, 64): score_dev[(j-job_lo)*Ns + n] (padding columns
 * KP_SCORE_INFEASIBLE) and mask_dev[(j-job_lo)*(Ns/64) + n/64]. Either may be
 * NULL. Complete on return; with kp_set_profiling on, kp_last_timing reports
 * the kernels' time (score_ms: the capacity-class kernel's own start / end
 * stamps through hipExtLaunchKernel, HIP events around the launch for the
 * other forms) and algorithmic bytes (score_bytes).
 * Not available on a kp_create_multi context (KP_EINVAL).
 */
int kp_score_dev(kp_ctx *ctx, const kp_params *p, int32_t job_lo, int32_t job_hi,
                 int32_t *score_dev, uint64_t *mask_dev);

/*
 * Preemption candidates (BASELINE config #4).
 *
 * The running jobs of the resident node table form the victim pool: running
 * job r uses req[d*R + r] on node[r] with priority prio[r]; its usage must
 * already be part of the loaded `used` (per node and dim the running requests
 * sum to <= used), else KP_EINVAL. kp_load_nodes clears the pool.
 *
 * COLLECTIVE on a multi-process context (kp_create with world_size > 1):
 * every rank loads the whole pool, and kp_preempt scores its own block of the
 * preemptor list and all-gathers the nominations, so every
 * rank must call kp_load_running and kp_preempt, like kp_solve; a call on one
 * rank alone blocks in the exchange. kp_create_multi contexts drive their
 * shards themselves (one call from the host).
 */
int kp_load_running(kp_ctx *ctx, int32_t R, const int32_t *node, const int64_t *req,
                    const int32_t *prio);

typedef struct kp_preemption {
  int32_t *node_of_job;    /* [J] nominated node, -1 = none                   */
  int32_t *victims_of_job; /* [J] running jobs to evict there, 0 = none       */
  int64_t *cost_of_job;    /* [J] sum of the victims' priorities, 0 = none    */
  /* filled by the library: */
  int32_t preemptors;      /* NO_FIT singleton jobs scored                     */
  int32_t nominated;       /* preemptors with a candidate node                 */
  int64_t pairs_scored;    /* preemptors x N                                   */
} kp_preemption;

/*
 * After kp_solve: for every NO_FIT job that is a singleton unit (gang size 1)
 * with priority p, pick the node whose eviction set is smallest when only
 * running jobs of priority < p may be evicted (kube-scheduler's
 * selectVictimsOnNode "reprieve" order: priority desc, running index asc),
 * against the post-solve usage; ties by lower sum of victim priorities, then
 * lower node index. Nominations are independent per job (nothing is evicted);
 * any output array may be NULL.
 */
int kp_preempt(kp_ctx *ctx, kp_preemption *out);

/* Timing of the last kp_solve, measured with HIP events on the solve stream
 * (kp_set_profiling(ctx, 1)): the filter+score launches are bracketed; the
 * select is not (select_ms = 0, select_bytes still counted) and accept_ms is
 * the rest of the solve. Level 2 (kp_set_profiling(ctx, 2)) adds event records
 * at every round's phase boundaries (a few us each: diagnosis, not the timed
 * steps) and fills the phase split; the phases sum to solve_ms up to the
 * solve's first and last launches. */
typedef struct kp_timing {
  double solve_ms;          /* whole device solve (first launch .. last)     */
  double score_ms;          /* sum of filter+score kernel time               */
  double select_ms;         /* sum of top-K select kernel time               */
  double accept_ms;         /* plan + exchange + acceptance + commit         */
  int64_t score_launches;
  int64_t score_bytes;      /* algorithmic bytes of the filter+score kernels */
  int64_t select_bytes;     /* algorithmic bytes of the select kernels       */
  int32_t fused;            /* 1: fused filter+score+top-K (no score matrix;
                               score_* then time/count k_score_topk)         */
  int32_t score_form;       /* kp_score / kp_score_dev / the materialised solve
                               path: 1 = the capacity-class form (k_score32c),
                               0 = the per-wave uniform / mixed form */
  int32_t score_classes;    /* capacity classes of the node table (0: more than
                               the class form handles) */
  int32_t rccl_calls;       /* ncclAllGather calls since the last kp_solve
                               started (its rounds' exchanges + any kp_preempt
                               after it); 0 without an RCCL communicator.
                               Counted at every profiling level.             */
  /* level 2 only (else 0), summed over the solve's rounds: */
  double cand_ms;           /* candidate phase: round start (active-unit
                               compaction, node pack) + filter/score/top-K +
                               candidate merge of this rank's units          */
  double xchg_ms;           /* candidate exchange of a multi-rank solve: pack
                               + all-gather + unpack (0 on one GPU)          */
  double pass_ms;           /* bidder index + plan/accept passes + commit    */
} kp_timing;
/* On a kp_create_multi context: every time field is the slowest shard's (the
   max per field), score_launches / score_bytes / select_bytes the sum over
   shards, the other fields shard 0's. */
int kp_last_timing(kp_ctx *ctx, kp_timing *t);
/* Per-shard timing: fills t[0 .. min(n, shards) - 1] in shard order and
   returns the number of shards (1 for a one-GPU / one-rank context; n = 0
   only asks for the count). Negative KP_E* on failure. */
int kp_last_timing_shards(kp_ctx *ctx, kp_timing *t, int32_t n);

/* HIP-event timing: 0 off (default), 1 the filter+score launches, 2 also the
   per-round phase split (kp_timing.cand/xchg/pass_ms). Both add event records
   between launches. */
int kp_set_profiling(kp_ctx *ctx, int level);

/* Host-side helper for the snapshot packer: parses an LLMService GPUMemory
   string (CRD pattern ^\d+(Gi|Mi)$, ai.ruijie.io_llmservices.yaml:48-51) into
   MiB. "" -> 0. Returns KP_EINVAL on pattern mismatch or int64 overflow. */
int kp_parse_gpu_memory(const char *s, int64_t *mib);

#ifdef __cplusplus
}
#endif
#endif /* KPLACE_H */
