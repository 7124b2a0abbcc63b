// kp_internal.hpp — shared definitions of libkplace (host orchestration +
// gfx950 kernels). Not part of the ABI; include/kplace.h is.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/kplace.h"

namespace kp {

// Weyl multiplier of the rotated tie-break and its inverse
// modulo 2^32 (decodes a node index back out of a packed candidate key).
constexpr uint32_t kTieMul = 0x9E3779B1u;
constexpr uint32_t inv32(uint32_t a) {
  uint32_t x = a;  // Newton iteration: x = x * (2 - a x), 5 steps reach 32 bits
  for (int i = 0; i < 5; ++i) x *= 2u - a * x;
  return x;
}
constexpr uint32_t kTieMulInv = inv32(kTieMul);
static_assert(kTieMul * kTieMulInv == 1u, "tie multiplier must be invertible");

enum UnitStatus : int32_t { kActive = 0, kPlaced = 1, kNoFit = 2 };

// k_score32's class form (kp_score.hip): node tables with at most this many
// distinct capacity vectors get per-(row, class) thresholds staged in LDS
constexpr int kScoreClasses = 8;
// k_score_topk workgroup: kFzWaves waves x 128 columns; the fused
// candidate phase's layout is padded to whole tiles
constexpr int kFzWaves = 8;
constexpr int kFzTileMax = 128 * kFzWaves;

// d.pass_flag layout: [0, 64) productive-pass flags of the current round
constexpr int kPassFlagWords = 128;
// d.counters words: [0] this rank's active units, [1] the global count, [32]
// bid nodes of the round, [33] bidder entries, [40, 56) launch probes

// Solve statistics accumulated on the device (no per-round host round trip):
// rounds with active units, sum of active units over rounds (x N = pairs
// scored) and productive passes.
struct SolveStats {
  int64_t rounds, active_sum, passes, pad;
};

// The per-round work of k_csr_keys (kp_pass.hip) done by the fused
// candidate merge (k_merge_tour) in counting mode on one GPU: open the slots,
// set the slot bitmap bits, re-initialise the pass state (one launch fewer
// per round). enabled = 0: k_csr_keys runs instead.
struct RoundKeys {
  int32_t enabled, A, K, N, D;
  int64_t nwin, Wb, init_n;
  uint32_t *bm, *bms, *bid;  // bms: one bit per nonzero bm word (Ws words per row)
  int64_t Ws;
  int64_t *bmin;
  int32_t *win, *seg_start, *pass_flag, *node_flag, *nl_count, *status;
  uint8_t *open;
  const int32_t *A_dev;
  struct SolveStats *st;
};

// Scoring constants copied into kernel arguments (wave-uniform -> SGPRs).
struct ScoreParams {
  int32_t D;
  int32_t N;
  int32_t w[KP_MAX_DIMS];
  int32_t most_allocated;  // 1 = MostAllocated, 0 = LeastAllocated
  int32_t gpu_dim;         // -1 = none
  int32_t w_gpu_fit;
  int32_t w_spread;
  int32_t tie_rotated;
  int32_t n_cand;
  int32_t S;           // util_scale
  int32_t w_affinity;  // CacheStrategy "shared" bonus
};

// Device buffers of one context. Node table SoA [D][N]; units in rank order.
struct DevState {
  // node table (resident across solves; `used` is committed into)
  int64_t *cap = nullptr, *used = nullptr, *used0 = nullptr;  // used0: as loaded
  uint32_t *R32 = nullptr, *K32 = nullptr;  // [D][N] exact-division tables (div_prep)
  int64_t *base = nullptr;  // LeastAllocated base: sum of w*S over dims with cap > 0
  int32_t *topo = nullptr;
  int32_t *perm = nullptr;  // [N] canonical order: nodes sorted by (cap vector, index)
  uint32_t *np32 = nullptr;  // [5*D+4][cap_P] 32-bit score tile planes
  // capacity classes (distinct capacity vectors) when there are at most
  // kScoreClasses of them: class of each node, and the classes' capacities
  uint32_t *ncls = nullptr;  // [N]
  uint32_t *ccap = nullptr;  // [kScoreClasses][D]
  // fused solve layout: canonical order with every capacity
  // class starting on a 128-column wave tile; column -> node (-1 = padding)
  // and per wave tile the canonical position of its first column minus that
  // column (pos = column - wshift[column / 128])
  int32_t *colnode = nullptr;  // [fz_P]
  int32_t *wshift = nullptr;   // [fz_P / 128]
  // fused solve: capacity class of every 128-column wave tile ([fz_P / 128],
  // 0 for padding-only tiles), the classes' capacities ([nfc][D]) and the
  // per-(unit, class) row records of k_score_topk ([U][nfc][RW], once per solve)
  int32_t *tcls = nullptr;
  uint32_t *fccap = nullptr;
  uint32_t *crec = nullptr;
  uint64_t *part = nullptr;    // [rows][fz_P / 1024][K] per-tile top-K keys
  uint64_t *fz_prof = nullptr; // [16] phase clocks of a KP_FZ_PROFILE build (KP_FZ_PROF=1)
  // units (rank order), job outputs
  int64_t *q = nullptr;  // [D][U]
  int32_t *leader = nullptr, *size = nullptr, *status = nullptr;
  int32_t *aff = nullptr;  // [U] affinity topo domain, -1 = none
  uint32_t *salt = nullptr;
  int32_t *job_node = nullptr, *job_score = nullptr, *job_status = nullptr;
  // round scratch
  int32_t *act = nullptr;       // [U] active unit ids of this round (global order)
  int32_t *act_local = nullptr; // [U] this rank's active units
  int32_t *cand = nullptr;      // [U*K] candidate nodes per active slot
  int32_t *cand_local = nullptr;// [U*K]
  int32_t *score = nullptr;     // [rows*N] materialised score matrix (chunk)
  uint64_t *mask = nullptr;     // [rows*ceil(N/64)]
  int32_t *rowmap = nullptr;    // [rows] row -> unit of kp_score_dev's single launch
  uint8_t *open = nullptr;      // [U] per active slot
  int32_t *flag = nullptr;      // [U] active flags (compaction input)
  // pass state: per bidder entry e (node-sorted order) the pass-start score and
  // a pass-tagged bid; a flag per 64-entry window; per multi-node gang slot its
  // parts {node, members, member offset, score} in candidate order, the part
  // count and an arrival counter (the last accepted part commits the gang)
  int32_t *s0 = nullptr;        // [U*K]
  uint32_t *bid = nullptr;      // [U*K] (pass << 8) | members
  // per 64-entry bidder window: the last pass with a bid of a short bidder
  // row in it, the smallest request per dim of its entries (once per round),
  // and [D][P/64 + 64] the smallest bid (members x request) of the long
  // rows' bids of the current pass, tagged (pass + 1) << 48 | (2^48 - 1 -
  // min) by the plan's atomicMax (0 = none this round)
  int32_t *win = nullptr;       // [P/64 + 128]
  int64_t *winmin = nullptr;    // [D][P/64 + 64]
  int64_t *bmin = nullptr;      // [D][P/64 + 64]
  int4 *gpart = nullptr;        // [U*K]
  int32_t *nparts = nullptr;    // [U]
  int32_t *arrive = nullptr;    // [U]
  // node -> (slot, candidate) inverse index, rebuilt once per round
  uint32_t *csr_kin = nullptr, *csr_vin = nullptr, *csr_keys = nullptr, *csr_vals = nullptr;
  int32_t *inv = nullptr;       // [U*K] (slot, candidate) -> entry
  int32_t *ent_unit = nullptr;  // [U*K] entry -> unit id
  int32_t *ent_slot = nullptr, *ent_size = nullptr, *ent_lead = nullptr;  // [U*K]
  int64_t *ent_q = nullptr;     // [D][U*K] request of the entry's unit
  int32_t *seg_start = nullptr, *seg_end = nullptr;  // [N]
  int32_t *node_flag = nullptr; // [N] last pass in which the node received a bid
  int32_t *node_list = nullptr; // [N] nodes with bidders this round (count: counters[32])
  int4 *nrec = nullptr;
  uint32_t *nst = nullptr;      // [N][16] static plan record (D <= 4, fits32): cap, R, K per dim, base, topo         // [N] per node_list entry {node, seg_start, seg_end, 0} (plan pass 0)
  int32_t *pass_flag = nullptr; // [kPassFlagWords] pass p produced proposals
  // preemption: unit priorities, victim-pool CSR sorted
  // (node, prio desc, running index asc) with per-node suffix sums, outputs
  int32_t *uprio = nullptr;     // [U]
  int32_t *plist = nullptr;     // [U] preemptor units of the last kp_preempt
  int32_t *pre_send = nullptr, *pre_recv = nullptr;  // multi-rank preemption blocks
  int32_t *roff = nullptr;      // [N+1]
  int64_t *rreq = nullptr, *rsuf = nullptr;  // [D][R]
  int32_t *rprio = nullptr;     // [R]
  int32_t *pre_node = nullptr, *pre_vict = nullptr;  // [J]
  int64_t *pre_cost = nullptr;  // [J]
  // streaming churn (kp_apply_delta)
  int32_t *dl_node = nullptr;   // [K]
  int64_t *dl_delta = nullptr;  // [D][K]
  int32_t *dl_bad = nullptr;    // [16] violation flag (allocated at kp_create)
  int32_t *counters = nullptr;  // small device counters
  SolveStats *stats = nullptr;  // [1]
  // counting-mode CSR (kp_pass.hip): [N][ceil(A/32)] slot bitmap (all-zero
  // between rounds), its summary [N][ceil(A/1024)] (bit w of a row: bm word w
  // is nonzero), per word {rank of its first bit in the row, bits}, row lengths
  uint32_t *bm = nullptr;
  uint32_t *bms = nullptr;
  uint2 *rowinfo = nullptr;
  int32_t *cnt = nullptr;
  void *temp = nullptr;         // rocprim temporary storage
  size_t temp_bytes = 0;
  // dist exchange
  int32_t *xg_counts = nullptr; // [world]
  int32_t *xg_send = nullptr;   // [Umax*(K+1)]
  int32_t *xg_recv = nullptr;   // [world*Umax*(K+1)]
};

}  // namespace kp

namespace kp {
struct Multi;  // kp_multi.cpp: one context over several GPUs (kp_create_multi)
}

struct kp_ctx {
  std::mutex mu;
  kp::Multi *multi = nullptr;  // non-null: this context forwards to its shards
  int device = 0;
  int world = 1, rank = 0;
  void *nccl_comm = nullptr;  // ncclComm_t
  // the solve runs the multi-rank form (act/cand exchanged once per round,
  // preemption rows all-gathered): world > 1, or a one-rank RCCL communicator
  // (KP_RCCL_SOLO=1, tests: the RCCL exchange executed on a one-GPU box)
  bool xchg = false;
  int32_t rccl_calls = 0;  // ncclAllGather calls of the current / last solve
  // host-staged exchange (kp_set_allgather) when world > 1 without RCCL
  kp_allgather_fn allgather = nullptr;
  void *allgather_user = nullptr;
  std::vector<int32_t> h_xg_send, h_xg_recv;
  // kp_create_multi shard: set by the multi context when a peer shard's call
  // failed; the shard's waits on its exchange poll it instead of blocking, so a
  // peer that never joins a collective cannot hang this shard
  const std::atomic<int> *peer_failed = nullptr;
  bool in_collective = false;  // this solve enqueued an RCCL collective
  // KP_TEST_FAIL_SOLVE (test knob): the next solve on this rank fails with
  // KP_ENOMEM at its first exchange (the peer-failure path of kp_create_multi)
  int32_t test_fail_solve = 0;
  int64_t max_pairs_matrix = 0;
  hipStream_t stream = nullptr;
  int profiling = 0;  // kp_set_profiling level (0 off, 1 filter+score events, 2 + phase split)
  // kp_score_dev under profiling: the events hipExtLaunchKernel stamps at the
  // start and end of the next k_score32c launch (kernel time only)
  hipEvent_t score_ev0 = nullptr, score_ev1 = nullptr;
  hipEvent_t fz_end_event = nullptr;  // profiling: recorded right after k_score_topk
  // test knobs, read from the environment at kp_create (never set in
  // production): KP_SELECT_LDS_CAP shrinks the threshold select's survivor
  // buffer (forces its threshold-raise path), KP_SELECT_GENERIC=1 forces the
  // generic per-lane top-K select
  int32_t select_lds_cap = 0;
  bool select_generic = false;
  int32_t select_bs = 0;  // KP_SELECT_BS: preferred threshold-select block size
  // score launch geometry (tuning knobs): target workgroups per launch and
  // the smallest number of job rows per workgroup
  int32_t score_wg_target = 4096, score_min_rpb = 4, score_npl = 2;
  int32_t fz_wg_target = 4096;  // KP_FZ_WG_TARGET: target workgroups of k_score_topk (r06: 2048 -> 4096, config #3 -2.7 %)
  bool fz_h16 = true;     // KP_FZ_H16=0: 32-bit LDS scores in k_score_topk
  int32_t fz_tie_bits = 0;  // KP_FZ_TIE_BITS=b (tests): b select-phase tie bits, forces collisions
  // KP_ACC_WAVES: largest k_accept grid in waves, grid-stride over the rest (0 =
  // one per node); 2,048: config #5 batches -2 %, config #3 neutral (tools/ab_*env.sh)
  int32_t acc_waves = 2048;
  int32_t acc_list = 1;  // KP_ACC_LIST=0: k_accept walks every node while entries >= nodes
  // KP_COMPACT_MAX: largest unit range compacted by the one-workgroup kernel
  int32_t compact_max = 65536;
  bool preempt32 = true;  // KP_PREEMPT32=0: the 64-bit per-row preemption kernel on 32-bit tables too
  // the victim pool's (victims, priority sum, node) fits one ordered 64-bit
  // key (N < 2^20, < 2^11 running jobs per node, |sum of their priorities| < 2^31)
  bool pre_key_ok = false;
  int32_t round_serial = 0;  // rounds enqueued on this context (< 2^30, then reset)
  int32_t cur_serial = 0;    // this round's serial (the host-followed pass tags)
  bool round_begin = true;  // KP_ROUND_BEGIN=0: round start + compaction as two launches
  // KP_KEYS_MERGE=0: k_csr_keys as its own launch; keys_in_merge: this
  // round's merge did its work
  bool keys_merge_enabled = true, keys_in_merge = false;
  // node -> bidder index by counting (KP_CSR_SORT=1: rocprim radix sort)
  bool csr_count_enabled = true, bm_dirty = false;
  int32_t csr_mode = 0;  // the current round's index: 1 counting, 0 sort
  // counting mode while the round's bitmap (N x ceil(A/32) words, 12 B each
  // with its row info) has at most this many words (KP_CSR_BM_MAX, 3 GB);
  // larger rounds, or a bitmap that cannot be allocated, use the radix sort
  int64_t csr_bm_max = int64_t{1} << 28;
  int64_t cap_bm_words = 0;
  int32_t cap_cnt_N = 0;
  // sizes
  int32_t N = 0, D = 0, J = 0, U = 0, R = 0, cap_R = 0, cap_delta = 0;
  int64_t cap_pre_xg = 0;  // int32 entries of d.pre_send (d.pre_recv: world x that)
  int32_t cap_N = 0, cap_U = 0, cap_J = 0, cap_rows = 0, cap_props = 0, cap_K = 0;
  int32_t mat_Ns = 0;          // row stride the score matrix was allocated for
  int64_t cap_P = 0;           // columns of d.np32
  int64_t cap_part = 0;        // entries of d.part
  int64_t cap_fz = 0;          // columns of d.colnode
  int64_t cap_tcls = 0, cap_fccap = 0;  // entries of d.tcls / d.fccap
  // fused score + top-K (k_score_topk): columns of the class-aligned layout,
  // whether that layout is compact enough to use, KP_FUSED=0 disables it
  int32_t fz_P = 0;
  int32_t n_classes = 0;  // capacity classes of the node table (0: more than kScoreClasses)
  bool score_classes = true;  // KP_SCORE_CLASSES=0: k_score32 without the class form
  bool fz_layout_ok = false, fused_enabled = true;
  int64_t max_cap = 0, max_req = 0;  // largest cap / request of the loaded tables
  int32_t cap_mask_rows = 0;   // rows of d.mask (kp_score only)
  int64_t cap_rowmap = 0;      // entries of d.rowmap (kp_score_dev only)
  int32_t nfc = 0;             // capacity classes of the fused layout (d.fccap)
  int64_t cap_crec = 0;        // words of d.crec
  bool crec_ok = false;        // this solve's row records are in d.crec (k_score_topk PRE form)
  bool crec_enabled = true;    // KP_FZ_CREC=0: thresholds inside k_score_topk (A/B)
  int64_t crec_max_bytes = (int64_t)512 << 20;  // larger tables: in-kernel thresholds
  int64_t cap_q = 0;           // int64 entries of d.q
  int32_t u_lo = 0, u_hi = 0;  // this rank's shard of units (rank positions)
  bool nodes_loaded = false, jobs_loaded = false, solved = false;
  // every cap and every req < 2^32: the filter+score pass may run in 32-bit
  bool caps32 = false, reqs32 = false, fits32 = false;
  int32_t util_scale_loaded = 0;  // S the R table was built for
  int32_t mode_loaded = -1;
  int32_t w_loaded[KP_MAX_DIMS] = {0};
  // host mirrors
  std::vector<int64_t> h_cap, h_used;
  std::vector<int32_t> h_topo;
  std::vector<int32_t> h_leader, h_size, h_prio, h_aff;
  std::vector<int64_t> h_q;
  // pinned host scratch
  int32_t *pinned = nullptr;  // small counters
  // coherent pinned word the compaction kernel stores the round's active
  // count into (KP_COUNT_DIRECT=0: copy it with hipMemcpyAsync instead)
  int32_t *pinned_coh = nullptr;  // [0]: round count; [32, 96): per-pass flags (hpass)
  // host-followed passes (one GPU): the host keeps pass_follow passes enqueued
  // ahead of the last pass whose flag k_accept stored into hpass, and stops at
  // the first pass without proposals (0 = every round enqueues max_passes)
  int32_t *hpass = nullptr;
  int32_t pass_follow = 2;
  // KP_BMIN_WIN: bidder rows spanning at least this many 64-entry windows get
  // per-pass window bid minima (plan atomics) on top of the round's request
  // minima; shorter rows only flags
  int32_t bmin_windows = 64;
  // dims with per-pass bid minima (bit d); 0 = automatic (kp_pass.hip
  // bmin_dims_of: the two most contended), KP_BMIN_DIMS overrides
  int32_t bmin_dims = 0;
  // per-dim totals of the loaded tables (capacity, usage at load, pending
  // requests): the automatic choice of bid-minima dims
  double cap_sum[KP_MAX_DIMS] = {0}, used_sum[KP_MAX_DIMS] = {0}, req_sum[KP_MAX_DIMS] = {0};
  int32_t acc_big_ratio = 48;  // k_accept's long-row form when A*K >= ratio * N (0: never)
  bool hpass_on = false;
  void *stage = nullptr;  // pinned staging of kp_load_jobs' unit arrays
  size_t stage_bytes = 0;
  bool count_direct = true;
  bool host_prof = false;  // KP_HOST_PROF=1: host enqueue / wait split per solve on stderr
  kp::DevState d;
  // what the next node-plane pack builds: the solve's canonical column order
  // (scores by perm[column]) or kp_score's node order, for these params
  kp::ScoreParams pack_sp{};
  bool pack_canonical = false;
  bool pack_fused = false;  // the fused layout (colnode), else perm / identity
  bool pack_full = true;    // the next pack also writes the capacity planes
  bool last_fused = false;  // the last solve ran the fused candidate phase
  std::vector<int32_t> h_perm;
  kp_result last{};
  kp_timing timing{};
  std::string last_error;  // detail of the last failed call (kp_last_error)
  // what kp_last_error returns: a copy of last_error taken under the lock,
  // in storage that later calls overwrite but never free
  char last_error_buf[512] = {0};
};

// Kernel launchers (kp_score.hip, kp_pass.hip).
namespace kp {
int launch_prep_nodes(kp_ctx *c, int32_t S, int most_allocated, const int32_t *w);
// 32-bit node planes (d.np32) of the current usage; k_score32 reads them, so
// every caller of launch_score packs first (the solve does it in the fused
// round-start kernel of launch_active / launch_active_async)
// order-preserving compaction of flags[0, n) into out (lo + index), count ->
// counters[0] (and *host_count when given)
int launch_compact_to(kp_ctx *c, const int32_t *flag, int32_t lo, int32_t n, int32_t *out,
                      int32_t *host_count);
int launch_pack(kp_ctx *c);
// Kernels that take a device count pointer (rows_dev / A_dev, nullable) size
// their grid by the host bound and clamp to the device count, so a round can
// be enqueued before the host knows its exact number of active units.
// (sstride / mstride: row strides of score / mask in elements, 0 = the
// internal layout Ns / Ns / 64; the non-class forms take the internal one only)
int launch_score(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit,
                 int32_t rows, int32_t *score, uint64_t *mask, const int64_t *q,
                 int32_t qstride, const int32_t *rows_dev = nullptr, int64_t sstride = 0,
                 int64_t mstride = 0);
int launch_select(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit,
                  int32_t rows, const int32_t *score, int32_t *cand,
                  const int32_t *rows_dev = nullptr);
// fused filter + score + top-K of the solve (kp_topk.hip): candidates of
// `rows` rows (act_local order) straight into cand, no score matrix
// (init_wgs: the merge's extra workgroups re-initialise the round state when
// it does k_csr_keys' work)
// the per-(unit, class) row records of the fused candidate phase (thresholds
// c - rho, WQ and the row's request / GPU / affinity words), once per solve
int launch_unit_rec(kp_ctx *c, const ScoreParams &sp);
int launch_score_topk(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit, int32_t rows,
                      int32_t ksh, int32_t *cand, const int32_t *rows_dev, bool init_wgs);
int launch_csr_build(kp_ctx *c, int32_t A, int32_t K, const int32_t *A_dev = nullptr);
// this round's index form (counting or sort) and its bitmap; called by
// launch_csr_build, or before the candidate merge when that does k_csr_keys' work
int csr_prepare(kp_ctx *c, int32_t A, int32_t K);
int csr_reserve(kp_ctx *c, int32_t Amax);
RoundKeys round_keys_args(kp_ctx *c, int32_t A, int32_t K, const int32_t *A_dev);
int launch_plan(kp_ctx *c, const ScoreParams &sp, int32_t A, int32_t pass,
                const int32_t *A_dev = nullptr);
// direct (nullable): in, request the count stored by the compaction kernel
// into c->pinned_coh (out: whether it was); else copied to count_host
int launch_active_async(kp_ctx *c, int32_t lo, int32_t hi, int32_t *count_host,
                        bool *direct = nullptr);
int launch_accept(kp_ctx *c, const ScoreParams &sp, int32_t pass, int32_t A);
// the static per-node plan records d.nst (every solve, after the division tables)
int launch_node_rec(kp_ctx *c);
void launch_probe(kp_ctx *c, const ScoreParams &sp, int32_t A);
int launch_active(kp_ctx *c, int32_t lo, int32_t hi, int32_t *A_host);
// unit status, job outputs and the per-unit tie-break salts of a solve
int launch_reset_units(kp_ctx *c, uint32_t tie_seed);
int launch_finalize(kp_ctx *c);
// multi-GPU exchange blocks: [count, (unit, K candidates) x B] per rank; pack
// reads the device count counters[0], unpack writes the global count to
// counters[1]
int launch_pack_exchange(kp_ctx *c, int32_t B, int32_t K);
int launch_unpack_exchange(kp_ctx *c, int32_t world, int32_t B, int32_t K);
size_t rocprim_temp_bytes(int32_t max_items);
// preemptor compaction + the scoring of this rank's rows [*lo, *hi) of them
int launch_preempt(kp_ctx *c, int32_t *P_host, int32_t *lo, int32_t *hi);
// multi-rank preemption: this rank's rows -> blocks of 4 int32 per row, and
// every rank's blocks (B rows each) -> the preemptors' jobs
int launch_preempt_pack(kp_ctx *c, int32_t lo, int32_t hi, int32_t *send);
int launch_preempt_unpack(kp_ctx *c, int32_t P, int32_t B, const int32_t *recv);
int launch_delta(kp_ctx *c, int32_t K, int32_t *bad_host);

// the value of a tuning / test knob: read only under KP_DEBUG_KNOBS=1, else NULL
const char *knob(const char *name);
// context over one GPU (kp_api.cpp); nccl_comm, if given, is adopted
int create_one(kp_ctx **out, int device, int world, int rank, const void *nccl_id,
               void *nccl_comm, int64_t max_pairs);
// kp_create_multi (kp_multi.cpp): one context over n GPUs, one worker thread
// per GPU, each with its own single-GPU shard context
int multi_create(kp_ctx **out, const int32_t *gpu_ids, int32_t n, int64_t max_pairs);
void multi_destroy(kp_ctx *c);
// Runs fn(shard, index) on every shard's worker thread (all) or on shard 0
// only, under the multi context's lock; returns the first failure (by shard
// index) and copies that shard's kp_last_error text.
int multi_run(kp_ctx *c, const std::function<int(kp_ctx *, int)> &fn, bool all);
}  // namespace kp

#define KP_HIP(expr)                                                \
  do {                                                              \
    hipError_t e_ = (expr);                                         \
    if (e_ != hipSuccess) {                                         \
      kp_set_error(#expr, e_);                                      \
      return KP_EHIP;                                               \
    }                                                               \
  } while (0)

void kp_set_error(const char *what, hipError_t e);
// detail text for a non-HIP failure of the current call (kp_last_error)
void kp_set_error_msg(const std::string &msg);

#define KP_TRY(expr)              \
  do {                            \
    int rc_ = (expr);             \
    if (rc_ != KP_OK) return rc_; \
  } while (0)

namespace kp {
// columns of one k_score_topk workgroup tile (one per-row top-K list each)
inline int fz_tile(const kp_ctx *) { return kFzTileMax; }
}  // namespace kp
