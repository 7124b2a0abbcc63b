/*
 * kp_oracle.h — CPU restatement of the kplace placement spec.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this code, and only as the checker /
 * the timed CPU baseline. The product path (libkplace.so) never links it.
 *
 * PARITY STATUS: "parity unpinned" for the placement itself. The reference
 * (Moore-Z/Kubernetes-Native-Distributed-AI-Job-Scheduler) contains no
 * filter/score/assign code; its de-facto placer is the external
 * kube-scheduler (absent from go.mod:5-101, not in this container). The
 * semantics restated here are this build's own spec. What IS
 * pinned to the reference: the job model (one CR -> Spec.Replicas identical
 * replicas = one gang, llmservice_controller.go:182-203; CRD defaults and the
 * GPUMemory pattern, api/v1/llmservice_types.go:25-52,
 * config/crd/bases/ai.ruijie.io_llmservices.yaml:39-71), checked against the
 * reference's own sample CRs in tests/golden/.
 */
#ifndef KP_ORACLE_H
#define KP_ORACLE_H

#include "../include/kplace.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Full placement. nthreads<=0 -> 1. Same validation
   rules and error codes as kp_place. */
int kpo_place(const kp_snapshot *s, const kp_params *p, kp_result *r,
              int nthreads);

/* Filter + score matrix for jobs [job_lo, job_hi) against s->used
   (DESIGN.md §2.3). Either output may be NULL. */
int kpo_score(const kp_snapshot *s, const kp_params *p, int32_t job_lo,
              int32_t job_hi, int32_t *score, uint64_t *mask);

/* Placement (as kpo_place, outputs into *res if non-NULL) followed by the
   preemption candidates of DESIGN.md §2.9 against the post-solve usage; the
   running jobs are (node[r], req[d*R + r], prio[r]). Same validation as
   kp_load_running. */
int kpo_preempt(const kp_snapshot *s, const kp_params *p, int32_t R, const int32_t *node,
                const int64_t *req, const int32_t *prio, kp_result *res,
                kp_preemption *pr, int nthreads);
int kpo_check_running(const kp_snapshot *s, int32_t R, const int32_t *node,
                      const int64_t *req, const int32_t *prio);

/* ---- stepwise interface (world_size>1 protocol tests, tests/test_dist) ---- */
typedef struct kpo_state kpo_state;

int kpo_state_new(const kp_snapshot *s, const kp_params *p, kpo_state **out);
void kpo_state_free(kpo_state *st);
int32_t kpo_state_units(const kpo_state *st);
int32_t kpo_state_active(const kpo_state *st);
int32_t kpo_state_unit_leader(const kpo_state *st, int32_t u);
int32_t kpo_state_unit_size(const kpo_state *st, int32_t u);
/* §2.4 candidate phase (the J x N part) for the units at rank positions
   [unit_lo, unit_hi): writes n_cand node indices per unit (best first,
   -1 padded; all -1 = no node fits one member; PLACED/NO_FIT units get all
   -1 too) to cand[(u - unit_lo) * n_cand + k]. Pure: the state is not
   modified. */
int kpo_round_candidates(const kpo_state *st, int32_t unit_lo, int32_t unit_hi,
                         int32_t *cand, int nthreads);
/* §2.5 passes of one round given every unit's candidates (cand[U*n_cand]).
   Commits the accepted placements. Returns the number of still-active
   units. */
int32_t kpo_round_run(kpo_state *st, const int32_t *cand);
/* Write outputs; may be called after any round. */
int kpo_state_result(const kpo_state *st, kp_result *r);

#ifdef __cplusplus
}
#endif
#endif
