// kp_api.cpp — C-ABI entry points and host orchestration of libkplace.
//
// The boundary replaces kubeinfer's one-CR-at-a-time driver
// (LLMServiceReconciler.Reconcile, internal/controller/llmservice_controller.go:66-174)
// and the external kube-scheduler's per-pod Filter/Score/selectHost/Bind with
// one batched solve. Host code here validates, groups the queue
// into gangs (one LLMService CR = Spec.Replicas identical replicas,
// llmservice_controller.go:182-203), ranks units, and drives the round/pass
// loop; every data-parallel step runs in the gfx950 kernels of kp_score.hip /
// kp_pass.hip / kp_preempt.hip. There is no CPU fallback: without a gfx950
// device kp_create fails with KP_ENODEV.
//
// Threading contract (include/kplace.h): every entry point takes the
// context's mutex for its whole duration (kp_place included: one acquisition
// for load + solve + fetch) and calls hipSetDevice itself. The detail text of
// a failure is kept per context (kp_last_error), because cgo callers hop OS
// threads between calls.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>

#include "kp_internal.hpp"

namespace {
thread_local std::string g_err;           // last HIP/RCCL detail on this thread
thread_local kp_ctx *g_cur = nullptr;     // context of the entry point running here
}  // namespace

void kp_set_error(const char *what, hipError_t e) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  if (g_cur) g_cur->last_error = g_err;
}

void kp_set_error_msg(const std::string &msg) {
  if (g_cur) g_cur->last_error = msg;
}

namespace kp {
constexpr int kProfWords = 16 + 64 + 4 * 1024;  // fz_prof: fused phases + pass profile

// Entry guard of every public call: the context lock for the whole call, the
// per-context error slot, and the context's device on this thread.
struct Entry {
  kp_ctx *c;
  std::unique_lock<std::mutex> lk;
  kp_ctx *prev;
  explicit Entry(kp_ctx *ctx) : c(ctx), lk(ctx->mu), prev(g_cur) {
    g_cur = ctx;
    ctx->last_error.clear();
  }
  ~Entry() { g_cur = prev; }
};

// KP_DEBUG_KNOBS=1 is the only environment variable the product reads; the
// tuning / A/B / test knobs below it are ignored without it
const char *knob(const char *name) {
  const char *on = std::getenv("KP_DEBUG_KNOBS");
  return on && std::strcmp(on, "1") == 0 ? std::getenv(name) : nullptr;
}

static int fail(int code, const char *fmt, ...) {
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  kp_set_error_msg(buf);
  return code;
}


// ---- validation, identical to oracle/kp_oracle.c check_params/check_nodes ----
static int check_params(const kp_params *p, int32_t D) {
  if (!p) return fail(KP_EINVAL, "params: NULL");
  for (int d = 0; d < KP_MAX_DIMS; ++d)
    if (p->w_dim[d] < 0 || p->w_dim[d] > 65535) return fail(KP_EINVAL, "params: w_dim[%d]", d);
  if (p->score_mode != KP_SCORE_MOST_ALLOCATED && p->score_mode != KP_SCORE_LEAST_ALLOCATED)
    return fail(KP_EINVAL, "params: score_mode");
  if (p->gpu_dim < -1 || p->gpu_dim >= D) return fail(KP_EINVAL, "params: gpu_dim");
  if (p->w_gpu_fit < 0 || p->w_gpu_fit > (1 << 20)) return fail(KP_EINVAL, "params: w_gpu_fit");
  if (p->w_spread < 0 || p->w_spread > (1 << 20)) return fail(KP_EINVAL, "params: w_spread");
  if (p->tie_mode != KP_TIE_NODE_INDEX && p->tie_mode != KP_TIE_ROTATED)
    return fail(KP_EINVAL, "params: tie_mode");
  if (p->max_rounds < 0) return fail(KP_EINVAL, "params: max_rounds");
  if (p->n_cand < 1 || p->n_cand > KP_MAX_CAND) return fail(KP_EINVAL, "params: n_cand");
  if (p->util_scale < 1 || p->util_scale > 1024) return fail(KP_EINVAL, "params: util_scale");
  if (p->max_passes < 1 || p->max_passes > 64) return fail(KP_EINVAL, "params: max_passes");
  if (p->w_affinity < 0 || p->w_affinity > (1 << 20)) return fail(KP_EINVAL, "params: w_affinity");
  return KP_OK;
}

template <typename T>
static int dalloc(T **p, size_t n) {
  if (*p) {
    (void)hipFree(*p);
    *p = nullptr;
  }
  if (n == 0) n = 1;
  if (hipMalloc(reinterpret_cast<void **>(p), n * sizeof(T)) != hipSuccess) {
    *p = nullptr;
    return fail(KP_ENOMEM, "hipMalloc of %zu bytes", n * sizeof(T));
  }
  return KP_OK;
}

static int ensure_nodes(kp_ctx *c, int32_t N, int32_t D) {
  if (N <= c->cap_N && D == c->D && c->d.cap) return KP_OK;
  c->cap_N = 0;  // a failed (re)allocation leaves no usable node buffers
  const int32_t n = std::max(N, 64);
  KP_TRY(dalloc(&c->d.cap, (size_t)D * n));
  KP_TRY(dalloc(&c->d.used, (size_t)D * n));
  KP_TRY(dalloc(&c->d.used0, (size_t)D * n));
  KP_TRY(dalloc(&c->d.R32, (size_t)D * n));
  KP_TRY(dalloc(&c->d.K32, (size_t)D * n));
  KP_TRY(dalloc(&c->d.base, (size_t)n));
  KP_TRY(dalloc(&c->d.topo, (size_t)n));
  KP_TRY(dalloc(&c->d.seg_start, (size_t)n));
  KP_TRY(dalloc(&c->d.seg_end, (size_t)n));
  KP_TRY(dalloc(&c->d.roff, (size_t)n + 1));
  KP_TRY(dalloc(&c->d.node_flag, (size_t)n));
  // +16: k_accept's list mode reads a record for up to KP_ACC_WPB - 1 padding waves
  KP_TRY(dalloc(&c->d.node_list, (size_t)n + 16));
  KP_TRY(dalloc(&c->d.nrec, (size_t)n + 16));
  KP_TRY(dalloc(&c->d.nst, (size_t)n * 16));
  KP_TRY(dalloc(&c->d.perm, (size_t)n));
  KP_TRY(dalloc(&c->d.ncls, (size_t)n));
  KP_TRY(dalloc(&c->d.ccap, (size_t)kScoreClasses * KP_MAX_DIMS));
  c->cap_N = n;
  return KP_OK;
}

// 32-bit node planes: [5*D+3][cols], cols = the widest layout in use (the
// fused solve's class-aligned columns or round_up(N, 1024))
static int ensure_np32(kp_ctx *c, int64_t cols, int32_t D) {
  const int64_t need = (int64_t)(5 * D + 4) * std::max<int64_t>(cols, 1024);
  if (c->d.np32 && need <= c->cap_P) return KP_OK;
  c->cap_P = 0;
  KP_TRY(dalloc(&c->d.np32, (size_t)need));
  c->cap_P = need;
  return KP_OK;
}

// per-tile top-K lists of the fused solve: rows x tiles x K keys
static int ensure_part(kp_ctx *c, int64_t entries) {
  if (c->d.part && entries <= c->cap_part) return KP_OK;
  c->cap_part = 0;
  KP_TRY(dalloc(&c->d.part, (size_t)std::max<int64_t>(entries, 64)));
  c->cap_part = entries;
  return KP_OK;
}

static int ensure_units(kp_ctx *c, int32_t U, int32_t J) {
  const int32_t K = KP_MAX_CAND;
  if (U > c->cap_U) {
    c->cap_U = 0;
    const size_t u = (size_t)std::max(U, 64);
    KP_TRY(dalloc(&c->d.leader, u));
    KP_TRY(dalloc(&c->d.size, u));
    KP_TRY(dalloc(&c->d.status, u));
    KP_TRY(dalloc(&c->d.salt, u));
    KP_TRY(dalloc(&c->d.aff, u));
    KP_TRY(dalloc(&c->d.act_local, u));
    KP_TRY(dalloc(&c->d.cand_local, u * K));
    KP_TRY(dalloc(&c->d.open, u));
    KP_TRY(dalloc(&c->d.flag, u));
    const size_t pm = u * K;  // (slot, candidate) pairs of a round
    KP_TRY(dalloc(&c->d.s0, pm));
    KP_TRY(dalloc(&c->d.bid, pm));
    KP_TRY(dalloc(&c->d.gpart, pm));
    KP_TRY(dalloc(&c->d.win, pm / 64 + 128));
    KP_TRY(dalloc(&c->d.winmin, (pm / 64 + 128) * KP_MAX_DIMS));
    KP_TRY(dalloc(&c->d.bmin, (pm / 64 + 128) * KP_MAX_DIMS));
    KP_TRY(dalloc(&c->d.nparts, u));
    KP_TRY(dalloc(&c->d.arrive, u));
    KP_TRY(dalloc(&c->d.uprio, u));
    KP_TRY(dalloc(&c->d.plist, u));
    KP_TRY(dalloc(&c->d.inv, pm));
    KP_TRY(dalloc(&c->d.ent_unit, pm));
    KP_TRY(dalloc(&c->d.ent_slot, pm));
    KP_TRY(dalloc(&c->d.ent_size, pm));
    KP_TRY(dalloc(&c->d.ent_lead, pm));
    KP_TRY(dalloc(&c->d.ent_q, pm * KP_MAX_DIMS));
    KP_TRY(dalloc(&c->d.csr_kin, pm));
    KP_TRY(dalloc(&c->d.csr_vin, pm));
    KP_TRY(dalloc(&c->d.csr_keys, pm));
    KP_TRY(dalloc(&c->d.csr_vals, pm));
    KP_TRY(dalloc(&c->d.pass_flag, kPassFlagWords));
    KP_TRY(dalloc(&c->d.counters, 64));
    KP_TRY(dalloc(&c->d.stats, 1));
    c->d.temp_bytes = rocprim_temp_bytes((int32_t)std::min<size_t>(pm, INT32_MAX));
    KP_TRY(dalloc(reinterpret_cast<uint8_t **>(&c->d.temp), c->d.temp_bytes));
    if (c->xchg) {
      KP_TRY(dalloc(&c->d.act, u));
      KP_TRY(dalloc(&c->d.cand, u * K));
      KP_TRY(dalloc(&c->d.xg_counts, (size_t)c->world));
      KP_TRY(dalloc(&c->d.xg_send, 1 + u * (K + 1)));
      KP_TRY(dalloc(&c->d.xg_recv, (size_t)c->world * (1 + u * (K + 1))));
    } else {
      c->d.act = c->d.act_local;
      c->d.cand = c->d.cand_local;
    }
    c->cap_U = (int32_t)u;
  }
  if (J > c->cap_J) {
    c->cap_J = 0;
    const size_t j = (size_t)std::max(J, 64);
    KP_TRY(dalloc(&c->d.job_node, j));
    KP_TRY(dalloc(&c->d.job_score, j));
    KP_TRY(dalloc(&c->d.job_status, j));
    KP_TRY(dalloc(&c->d.pre_node, j));
    KP_TRY(dalloc(&c->d.pre_vict, j));
    KP_TRY(dalloc(&c->d.pre_cost, j));
    c->cap_J = (int32_t)j;
  }
  return KP_OK;
}

static int ensure_q(kp_ctx *c, int32_t U, int32_t D) {
  const int64_t n = (int64_t)D * std::max(U, 64);
  if (n <= c->cap_q && c->d.q) return KP_OK;  // grows only
  c->cap_q = 0;
  KP_TRY(dalloc(&c->d.q, (size_t)n));
  c->cap_q = n;
  return KP_OK;
}

// Score matrix of the solve: `rows` rows of stride Ns = round_up(N, 64). Kept
// across solves and node-table reloads while the stride does not change (a
// resident ~1 GB buffer at config #3; no hipMalloc/hipFree in the solve).
static int ensure_matrix(kp_ctx *c, int32_t rows) {
  const int32_t Ns = (c->N + 63) & ~63;
  if (c->d.score && Ns == c->mat_Ns && rows <= c->cap_rows) return KP_OK;
  c->cap_rows = 0;
  KP_TRY(dalloc(&c->d.score, (size_t)rows * std::max(Ns, 64)));
  c->cap_rows = rows;
  c->mat_Ns = Ns;
  return KP_OK;
}

// Feasibility bitmask rows of kp_score (never allocated by a solve).
static int ensure_mask(kp_ctx *c, int32_t rows) {
  const int32_t words = std::max((c->N + 63) / 64, 1);
  if (c->d.mask && (int64_t)rows * words <= (int64_t)c->cap_mask_rows) return KP_OK;
  c->cap_mask_rows = 0;
  KP_TRY(dalloc(&c->d.mask, (size_t)rows * words));
  c->cap_mask_rows = (int32_t)std::min<int64_t>((int64_t)rows * words, INT32_MAX);
  return KP_OK;
}

static ScoreParams make_sp(const kp_ctx *c, const kp_params *p) {
  ScoreParams sp{};
  sp.D = c->D;
  sp.N = c->N;
  for (int d = 0; d < KP_MAX_DIMS; ++d) sp.w[d] = p->w_dim[d];
  sp.most_allocated = p->score_mode == KP_SCORE_MOST_ALLOCATED;
  sp.gpu_dim = p->gpu_dim;
  sp.w_gpu_fit = p->w_gpu_fit;
  sp.w_spread = p->w_spread;
  sp.tie_rotated = p->tie_mode == KP_TIE_ROTATED;
  sp.n_cand = p->n_cand;
  sp.S = p->util_scale;
  sp.w_affinity = p->w_affinity;
  return sp;
}

// Division tables and LeastAllocated base depend on (S, mode, weights):
// rebuild on change
static int prep_for(kp_ctx *c, const kp_params *p) {
  bool same = c->util_scale_loaded == p->util_scale && c->mode_loaded == p->score_mode;
  for (int d = 0; d < KP_MAX_DIMS; ++d) same = same && c->w_loaded[d] == p->w_dim[d];
  if (same) return KP_OK;
  KP_TRY(launch_prep_nodes(c, p->util_scale, p->score_mode == KP_SCORE_MOST_ALLOCATED,
                           p->w_dim));
  c->util_scale_loaded = p->util_scale;
  c->mode_loaded = p->score_mode;
  for (int d = 0; d < KP_MAX_DIMS; ++d) c->w_loaded[d] = p->w_dim[d];
  return KP_OK;
}

static int64_t rows_per_chunk(const kp_ctx *c) {
  const int64_t Ns = (c->N + 63) & ~63;
  int64_t maxp = c->max_pairs_matrix > 0 ? c->max_pairs_matrix : (int64_t)1 << 30;
  int64_t r = std::max<int64_t>(1, maxp / std::max<int64_t>(Ns, 64));
  return std::min<int64_t>(r, INT32_MAX / std::max<int64_t>(Ns, 64));
}

// HIP events of one solve, destroyed on every exit path
struct Events {
  std::vector<hipEvent_t> ev;
  ~Events() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
  int make(hipEvent_t *e, unsigned flags) {
    KP_HIP(hipEventCreateWithFlags(e, flags));
    ev.push_back(*e);
    return KP_OK;
  }
};

// ---------------------------------------------------------------------------
// context creation (one GPU)
// ---------------------------------------------------------------------------
int create_one(kp_ctx **out, int device, int world, int rank, const void *nccl_id,
               void *nccl_comm, int64_t max_pairs) {
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return KP_ENODEV;
  int dev = device;
  if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return KP_ENODEV;
  if (dev >= ndev) return KP_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return KP_ENODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return KP_ENODEV;
  kp_ctx *c = new (std::nothrow) kp_ctx();
  if (!c) return KP_ENOMEM;
  c->device = dev;
  c->world = world;
  c->rank = rank;
  c->max_pairs_matrix = max_pairs;
  // A/B and test knobs: honoured only under KP_DEBUG_KNOBS=1, so that a
  // manager process's inherited environment cannot switch kernels or key
  // encodings; the defaults below are the product
  if (const char *e = knob("KP_SELECT_LDS_CAP")) c->select_lds_cap = std::atoi(e);
  if (const char *e = knob("KP_SELECT_GENERIC")) c->select_generic = std::atoi(e) != 0;
  if (const char *e = knob("KP_SELECT_BS")) c->select_bs = std::atoi(e);
  if (const char *e = knob("KP_FZ_CREC")) c->crec_enabled = std::atoi(e) != 0;
  if (const char *e = knob("KP_SCORE_WG_TARGET")) c->score_wg_target = std::max(64, std::atoi(e));
  if (const char *e = knob("KP_SCORE_MIN_RPB")) c->score_min_rpb = std::max(1, std::atoi(e));
  if (const char *e = knob("KP_SCORE_NPL")) c->score_npl = std::atoi(e) == 4 ? 4 : 2;
  if (const char *e = knob("KP_COMPACT_MAX")) c->compact_max = std::atoi(e);
  if (const char *e = knob("KP_FUSED")) c->fused_enabled = std::atoi(e) != 0;
  if (const char *e = knob("KP_SCORE_CLASSES")) c->score_classes = std::atoi(e) != 0;
  if (const char *e = knob("KP_PREEMPT32")) c->preempt32 = std::atoi(e) != 0;
  if (const char *e = knob("KP_ACC_LIST")) c->acc_list = std::atoi(e);
  if (const char *e = knob("KP_ACC_BIG_RATIO")) c->acc_big_ratio = std::max(0, std::atoi(e));
  if (const char *e = knob("KP_BMIN_WIN")) c->bmin_windows = std::max(1, std::atoi(e));
  if (const char *e = knob("KP_BMIN_DIMS")) c->bmin_dims = (int32_t)std::strtol(e, nullptr, 0);
  if (const char *e = knob("KP_PASS_FOLLOW")) c->pass_follow = std::max(0, std::min(64, std::atoi(e)));
  if (const char *e = knob("KP_KEYS_MERGE")) c->keys_merge_enabled = std::atoi(e) != 0;
  if (const char *e = knob("KP_ROUND_BEGIN")) c->round_begin = std::atoi(e) != 0;
  if (const char *e = knob("KP_CSR_SORT")) c->csr_count_enabled = std::atoi(e) == 0;
  if (const char *e = knob("KP_CSR_BM_MAX")) c->csr_bm_max = std::atoll(e);
  if (const char *e = knob("KP_ACC_WAVES")) c->acc_waves = std::max(0, std::atoi(e));
  if (const char *e = knob("KP_FZ_WG_TARGET")) c->fz_wg_target = std::max(64, std::atoi(e));
  if (const char *e = knob("KP_COUNT_DIRECT")) c->count_direct = std::atoi(e) != 0;
  if (const char *e = knob("KP_HOST_PROF")) c->host_prof = std::atoi(e) != 0;
  if (const char *e = knob("KP_FZ_H16")) c->fz_h16 = std::atoi(e) != 0;
  if (const char *e = knob("KP_TEST_FAIL_SOLVE"))  // tests: rank e fails its next solve
    c->test_fail_solve = world > 1 && std::atoi(e) == rank;
  if (const char *e = knob("KP_FZ_TIE_BITS")) c->fz_tie_bits = std::max(0, std::min(31, std::atoi(e)));
  if (const char *e = knob("KP_FZ_PROF"))  // phase clocks (KP_FZ_PROFILE builds only)
    if (std::atoi(e) != 0 && hipMalloc(reinterpret_cast<void **>(&c->d.fz_prof), kProfWords * 8) == hipSuccess) {
      // [16 + 64 + 4 L + {0, 2}]: minima of the pass-profile launch stamps
      std::vector<uint64_t> h(kProfWords, 0);
      for (int L = 0; L < 1024; ++L) h[16 + 64 + 4 * L] = h[16 + 64 + 4 * L + 2] = ~0ull;
      (void)hipMemcpy(c->d.fz_prof, h.data(), kProfWords * 8, hipMemcpyHostToDevice);
    }
  if (hipSetDevice(dev) != hipSuccess ||
      hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void **>(&c->pinned), 4096, hipHostMallocDefault) !=
          hipSuccess ||
      hipHostMalloc(reinterpret_cast<void **>(&c->pinned_coh), 512,
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipMalloc(reinterpret_cast<void **>(&c->d.dl_bad), 16 * sizeof(int32_t)) != hipSuccess) {
    kp_destroy(c);
    return KP_EHIP;
  }
  c->hpass = c->pinned_coh + 32;
  for (int i = 0; i < 64; ++i) c->hpass[i] = -1;  // never a tag (tags are even, >= 0)
  // KP_RCCL_SOLO=1 (tests): a one-rank context given an RCCL id builds a
  // one-rank communicator and runs the multi-rank solve (pack -> ncclAllGather
  // -> unpack every round, the preemption all-gather), so that the RCCL path
  // executes on a one-GPU box exactly as each rank of an N-GPU job runs it
  const char *solo_env = knob("KP_RCCL_SOLO");
  const bool solo = solo_env && std::atoi(solo_env) != 0;
  if (nccl_comm) {
    c->nccl_comm = nccl_comm;
  } else if ((world > 1 || solo) && nccl_id) {  // else: host-staged exchange (kp_set_allgather)
    ncclUniqueId id;
    std::memcpy(&id, nccl_id, sizeof id);
    ncclComm_t comm;
    if (ncclCommInitRank(&comm, world, id, rank) != ncclSuccess) {
      kp_destroy(c);
      return KP_ERCCL;
    }
    c->nccl_comm = comm;
  }
  c->xchg = world > 1 || c->nccl_comm != nullptr;
  *out = c;
  return KP_OK;
}

// ---------------------------------------------------------------------------
// loads (caller holds the lock)
// ---------------------------------------------------------------------------
static int load_nodes_impl(kp_ctx *c, int32_t N, int32_t D, const int64_t *cap,
                           const int64_t *used, const int32_t *topo) {
  // any failure below leaves no node table (nor the jobs / solve that depend
  // on it) loaded; sizes are committed only after every copy
  c->nodes_loaded = false;
  c->solved = false;
  if (N < 0 || D < 1 || D > KP_MAX_DIMS || (N > 0 && !cap))
    return fail(KP_EINVAL, "kp_load_nodes: N=%d D=%d cap=%p", N, D, (const void *)cap);
  for (int64_t i = 0; i < (int64_t)D * N; ++i) {
    const int64_t cc = cap[i], u = used ? used[i] : 0;
    if (cc < 0 || cc > KP_MAX_VALUE || u < 0 || u > cc)
      return fail(KP_EINVAL, "kp_load_nodes: dim %lld node %lld: cap %lld used %lld",
                  (long long)(i / std::max(N, 1)), (long long)(i % std::max(N, 1)),
                  (long long)cc, (long long)u);
  }
  if (topo)
    for (int32_t n = 0; n < N; ++n)
      if (topo[n] < 0) return fail(KP_EINVAL, "kp_load_nodes: topo_domain[%d] < 0", n);
  if (D != c->D) c->jobs_loaded = false;  // request layout depends on D
  KP_HIP(hipSetDevice(c->device));
  try {
    c->h_cap.assign(cap, cap + (size_t)D * N);
    c->h_used.assign((size_t)D * N, 0);
    if (used) std::copy(used, used + (size_t)D * N, c->h_used.begin());
    c->h_topo.resize(N);
    for (int32_t n = 0; n < N; ++n) c->h_topo[n] = topo ? topo[n] : n;
    // canonical order: nodes sorted by capacity vector, then
    // index; the solve's score columns follow it, so that a wave's columns
    // share their capacities and the per-pair division becomes a per-row one
    c->h_perm.resize(N);
    for (int32_t n = 0; n < N; ++n) c->h_perm[n] = n;
    std::stable_sort(c->h_perm.begin(), c->h_perm.end(), [&](int32_t a, int32_t b) {
      for (int d = 0; d < D; ++d) {
        const int64_t ca = cap[(int64_t)d * N + a], cb = cap[(int64_t)d * N + b];
        if (ca != cb) return ca < cb;
      }
      return false;
    });
  } catch (const std::bad_alloc &) {
    return fail(KP_ENOMEM, "kp_load_nodes: host copy");
  }
  // class-aligned layout of the fused solve (kp_topk.hip): each run of equal
  // capacity vectors in canonical order starts on a 128-column wave tile
  std::vector<int32_t> colnode, wshift;
  int64_t fz_cols = 0;
  try {
    auto same = [&](int32_t a, int32_t b) {
      for (int d = 0; d < D; ++d)
        if (cap[(int64_t)d * N + a] != cap[(int64_t)d * N + b]) return false;
      return true;
    };
    std::vector<std::pair<int32_t, int32_t>> cls;  // (first position, length)
    for (int32_t i = 0; i < N;) {
      int32_t e = i + 1;
      while (e < N && same(c->h_perm[e], c->h_perm[i])) ++e;
      cls.emplace_back(i, e - i);
      fz_cols = ((fz_cols + 127) & ~(int64_t)127) + (e - i);
      i = e;
    }
    const int64_t P = (std::max<int64_t>(fz_cols, 1) + kFzTileMax - 1) & ~(int64_t)(kFzTileMax - 1);
    if (N > 0 && P <= ((int64_t)1 << 24)) {
      colnode.assign((size_t)P, -1);
      wshift.assign((size_t)(P / 128), 0);
      int64_t col = 0;
      for (const auto &cl : cls) {
        col = (col + 127) & ~(int64_t)127;
        for (int64_t t = col; t < col + cl.second; t += 128)
          wshift[(size_t)(t / 128)] = (int32_t)(col - cl.first);
        for (int32_t k = 0; k < cl.second; ++k) colnode[(size_t)(col + k)] = c->h_perm[cl.first + k];
        col += cl.second;
      }
    }
  } catch (const std::bad_alloc &) {
    return fail(KP_ENOMEM, "kp_load_nodes: host copy");
  }
  const int32_t fz_P = (int32_t)colnode.size();
  // the fused layout's classes: per wave tile its class, per class its
  // capacity vector (32-bit: the fused path needs every cap < 2^30)
  std::vector<int32_t> tcls;
  std::vector<uint32_t> fccap;
  try {
    if (fz_P > 0) {
      tcls.assign((size_t)fz_P / 128, 0);
      int32_t k = 0;
      int64_t col = 0;
      for (int32_t i = 0; i < N; ++k) {
        int32_t e = i + 1;
        while (e < N && [&] {
          for (int d = 0; d < D; ++d)
            if (cap[(int64_t)d * N + c->h_perm[e]] != cap[(int64_t)d * N + c->h_perm[i]]) return false;
          return true;
        }()) ++e;
        col = (col + 127) & ~(int64_t)127;
        for (int64_t t = col; t < col + (e - i); t += 128) tcls[(size_t)(t / 128)] = k;
        col += e - i;
        for (int d = 0; d < D; ++d)
          fccap.push_back((uint32_t)std::min<int64_t>(cap[(int64_t)d * N + c->h_perm[i]], 0xFFFFFFFFll));
        i = e;
      }
    }
  } catch (const std::bad_alloc &) {
    return fail(KP_ENOMEM, "kp_load_nodes: host copy");
  }
  const int32_t nfc = (int32_t)(fccap.size() / std::max(D, 1));
  // capacity classes for k_score32's class form: the runs of equal capacity
  // vectors in canonical order (at most kScoreClasses of them)
  std::vector<uint32_t> ncls, ccap;
  int32_t n_classes = 0;
  try {
    int32_t k = 0;
    for (int32_t i = 0; i < N && k <= kScoreClasses; ++k) {
      int32_t e = i + 1;
      while (e < N && [&] {
        for (int d = 0; d < D; ++d)
          if (cap[(int64_t)d * N + c->h_perm[e]] != cap[(int64_t)d * N + c->h_perm[i]]) return false;
        return true;
      }()) ++e;
      if (k < kScoreClasses) {
        if (ncls.empty()) {
          ncls.assign((size_t)N, 0u);
          ccap.assign((size_t)kScoreClasses * D, 0u);
        }
        for (int32_t j = i; j < e; ++j) ncls[(size_t)c->h_perm[j]] = (uint32_t)k;
        for (int d = 0; d < D; ++d) ccap[(size_t)k * D + d] = (uint32_t)cap[(int64_t)d * N + c->h_perm[i]];
      }
      i = e;
      if (i >= N) n_classes = k + 1;
    }
    if (n_classes > kScoreClasses) n_classes = 0;
  } catch (const std::bad_alloc &) {
    return fail(KP_ENOMEM, "kp_load_nodes: host copy");
  }
  KP_TRY(ensure_nodes(c, N, D));
  KP_TRY(ensure_np32(c, std::max<int64_t>(fz_P, ((int64_t)N + 1023) & ~(int64_t)1023), D));
  if (fz_P > 0) {
    if ((int64_t)fz_P > c->cap_fz) {
      c->cap_fz = 0;
      KP_TRY(dalloc(&c->d.colnode, (size_t)fz_P));
      KP_TRY(dalloc(&c->d.wshift, (size_t)fz_P / 128));
      c->cap_fz = fz_P;
    }
    KP_HIP(hipMemcpyAsync(c->d.colnode, colnode.data(), sizeof(int32_t) * fz_P,
                          hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(c->d.wshift, wshift.data(), sizeof(int32_t) * (fz_P / 128),
                          hipMemcpyHostToDevice, c->stream));
    // grow-only, like colnode: a reload of the same table shape allocates
    // nothing (hipFree synchronises the device)
    if ((int64_t)fz_P / 128 > c->cap_tcls) {
      c->cap_tcls = 0;
      KP_TRY(dalloc(&c->d.tcls, (size_t)fz_P / 128));
      c->cap_tcls = fz_P / 128;
    }
    if ((int64_t)std::max<size_t>(fccap.size(), 1) > c->cap_fccap) {
      c->cap_fccap = 0;
      KP_TRY(dalloc(&c->d.fccap, std::max<size_t>(fccap.size(), 1)));
      c->cap_fccap = (int64_t)std::max<size_t>(fccap.size(), 1);
    }
    KP_HIP(hipMemcpyAsync(c->d.tcls, tcls.data(), sizeof(int32_t) * (fz_P / 128),
                          hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(c->d.fccap, fccap.data(), sizeof(uint32_t) * fccap.size(),
                          hipMemcpyHostToDevice, c->stream));
  }
  c->nfc = fz_P > 0 ? nfc : 0;
  if (N > 0) {
    KP_HIP(hipMemcpyAsync(c->d.cap, c->h_cap.data(), sizeof(int64_t) * D * N,
                          hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(c->d.used, c->h_used.data(), sizeof(int64_t) * D * N,
                          hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(c->d.used0, c->d.used, sizeof(int64_t) * D * N,
                          hipMemcpyDeviceToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(c->d.topo, c->h_topo.data(), sizeof(int32_t) * N,
                          hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(c->d.perm, c->h_perm.data(), sizeof(int32_t) * N,
                          hipMemcpyHostToDevice, c->stream));
    if (n_classes > 0) {
      KP_HIP(hipMemcpyAsync(c->d.ncls, ncls.data(), sizeof(uint32_t) * N, hipMemcpyHostToDevice,
                            c->stream));
      KP_HIP(hipMemcpyAsync(c->d.ccap, ccap.data(), sizeof(uint32_t) * (size_t)n_classes * D,
                            hipMemcpyHostToDevice, c->stream));
    }
  }
  // the victim pool belongs to the previous node table
  KP_HIP(hipMemsetAsync(c->d.roff, 0, sizeof(int32_t) * ((size_t)N + 1), c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  c->R = 0;
  c->pre_key_ok = false;  // described the previous table's victim pool
  c->N = N;
  c->D = D;
  c->max_cap = 0;
  for (int64_t i = 0; i < (int64_t)D * N; ++i) c->max_cap = std::max(c->max_cap, cap[i]);
  // per-dim totals for the automatic bid-minima dims (a heuristic: every
  // 4th node, so the load stays one pass over the table)
  for (int d = 0; d < KP_MAX_DIMS; ++d) {
    double cs = 0, us = 0;
    if (d < D)
      for (int32_t n = 0; n < N; n += 4) {
        cs += (double)cap[(int64_t)d * N + n];
        us += used ? (double)used[(int64_t)d * N + n] : 0.0;
      }
    c->cap_sum[d] = cs;
    c->used_sum[d] = us;
  }
  c->caps32 = c->max_cap < ((int64_t)1 << 32);
  // the fused layout pays off while the padding stays small (few capacity
  // classes); the merge holds at most 2,048 keys per row (tiles x K)
  c->fz_P = fz_P;
  c->n_classes = (c->max_cap < ((int64_t)1 << 32)) ? n_classes : 0;
  c->fz_layout_ok = fz_P > 0 && fz_cols - N <= N / 8 + 1024;
  c->fits32 = c->caps32 && c->reqs32 && c->jobs_loaded;
  c->util_scale_loaded = 0;  // force a division-table rebuild at the next solve
  c->pack_full = true;
  c->nodes_loaded = true;
  return KP_OK;
}

static int load_jobs_impl(kp_ctx *c, int32_t J, const int64_t *req, const int32_t *prio,
                          const int32_t *gang_id, const int32_t *gang_size,
                          const int32_t *aff) {
  c->jobs_loaded = false;  // any failure below leaves no queue loaded
  c->solved = false;
  if (!c->nodes_loaded) return fail(KP_ESTATE, "kp_load_jobs: no node table loaded");
  const int32_t D = c->D;
  if (J < 0 || (J > 0 && !req)) return fail(KP_EINVAL, "kp_load_jobs: J=%d req=%p", J, (const void *)req);
  for (int64_t i = 0; i < (int64_t)D * J; ++i)
    if (req[i] < 0 || req[i] > KP_MAX_VALUE)
      return fail(KP_EINVAL, "kp_load_jobs: req of job %lld dim %lld out of [0, 2^56]",
                  (long long)(i % std::max(J, 1)), (long long)(i / std::max(J, 1)));
  // units: maximal runs of equal gang_id >= 0 (one CR's replicas); rank order
  std::vector<int32_t> leader, size, uprio, uaff;
  try {
    leader.reserve(J);
    size.reserve(J);
    uprio.reserve(J);
    uaff.reserve(J);
    for (int32_t j = 0; j < J;) {
      const int32_t gid = gang_id ? gang_id[j] : -1;
      int32_t e = j + 1;
      if (gid >= 0)
        while (e < J && gang_id[e] == gid) ++e;
      const int32_t len = e - j;
      if (len > KP_MAX_GANG) return fail(KP_EINVAL, "kp_load_jobs: gang %d has %d > 64 members", gid, len);
      for (int32_t k = j; k < e; ++k) {
        if (gang_size && gang_size[k] != len)
          return fail(KP_EINVAL, "kp_load_jobs: job %d gang_size %d != run length %d", k, gang_size[k], len);
        if (prio && prio[k] != prio[j])
          return fail(KP_EINVAL, "kp_load_jobs: gang %d mixes priorities", gid);
        if (aff && (aff[k] != aff[j] || aff[k] < -1))
          return fail(KP_EINVAL, "kp_load_jobs: job %d affinity %d", k, aff[k]);
        for (int d = 0; d < D; ++d)
          if (req[(int64_t)d * J + k] != req[(int64_t)d * J + j])
            return fail(KP_EINVAL, "kp_load_jobs: gang %d mixes requests", gid);
      }
      leader.push_back(j);
      size.push_back(len);
      uprio.push_back(prio ? prio[j] : 0);
      uaff.push_back(aff ? aff[j] : -1);
      j = e;
    }
    if (gang_id) {  // a gang id may not reappear in a later run
      int32_t idmax = -1;
      for (size_t u = 0; u < leader.size(); ++u) idmax = std::max(idmax, gang_id[leader[u]]);
      if (idmax >= 0 && (int64_t)idmax < 8 * (int64_t)leader.size() + 4096) {
        std::vector<uint8_t> seen((size_t)idmax + 1, 0);  // ids are usually CR indices
        for (size_t u = 0; u < leader.size(); ++u) {
          const int32_t g = gang_id[leader[u]];
          if (g < 0) continue;
          if (seen[(size_t)g]) return fail(KP_EINVAL, "kp_load_jobs: gang id %d reappears", g);
          seen[(size_t)g] = 1;
        }
      } else if (idmax >= 0) {
        std::vector<int32_t> ids;
        for (size_t u = 0; u < leader.size(); ++u)
          if (gang_id[leader[u]] >= 0) ids.push_back(gang_id[leader[u]]);
        std::sort(ids.begin(), ids.end());
        auto it = std::adjacent_find(ids.begin(), ids.end());
        if (it != ids.end()) return fail(KP_EINVAL, "kp_load_jobs: gang id %d reappears", *it);
      }
    }
    const int32_t U = (int32_t)leader.size();
    std::vector<int32_t> ord(U);
    // rank order (prio desc, leader asc): leaders ascend with u, so a stable
    // order by priority; a counting sort when the priorities span a small
    // range (priority tiers), else a stable comparison sort
    int32_t pmin = INT32_MAX, pmax = INT32_MIN;
    for (int32_t u = 0; u < U; ++u) {
      pmin = std::min(pmin, uprio[u]);
      pmax = std::max(pmax, uprio[u]);
    }
    if (U > 0 && (int64_t)pmax - pmin < 65536) {
      const int32_t R = pmax - pmin + 1;
      std::vector<int32_t> at((size_t)R + 1, 0);
      for (int32_t u = 0; u < U; ++u) ++at[(size_t)(pmax - uprio[u]) + 1];
      for (int32_t r = 0; r < R; ++r) at[(size_t)r + 1] += at[(size_t)r];
      for (int32_t u = 0; u < U; ++u) ord[(size_t)at[(size_t)(pmax - uprio[u])]++] = u;
    } else {
      for (int32_t u = 0; u < U; ++u) ord[u] = u;
      std::stable_sort(ord.begin(), ord.end(),
                       [&](int32_t a, int32_t b) { return uprio[a] > uprio[b]; });
    }
    c->h_leader.resize(U);
    c->h_size.resize(U);
    c->h_prio.resize(U);
    c->h_aff.resize(U);
    c->h_q.resize((size_t)D * U);
    for (int32_t r = 0; r < U; ++r) {
      c->h_leader[r] = leader[ord[r]];
      c->h_size[r] = size[ord[r]];
      c->h_prio[r] = uprio[ord[r]];
      c->h_aff[r] = uaff[ord[r]];
      for (int d = 0; d < D; ++d)
        c->h_q[(size_t)d * U + r] = req[(int64_t)d * J + leader[ord[r]]];
    }
  } catch (const std::bad_alloc &) {
    return fail(KP_ENOMEM, "kp_load_jobs: host copy");
  }
  const int32_t U = (int32_t)c->h_leader.size();
  KP_HIP(hipSetDevice(c->device));
  KP_TRY(ensure_units(c, U, J));
  KP_TRY(ensure_q(c, U, D));
  if (U > 0) {
    // one pinned staging block (DMA straight from it; pageable copies go
    // through the runtime's staging buffers one call at a time)
    const size_t need = sizeof(int64_t) * D * U + 4 * sizeof(int32_t) * U;
    if (need > c->stage_bytes) {
      if (c->stage) (void)hipHostFree(c->stage);
      c->stage = nullptr;
      c->stage_bytes = 0;
      if (hipHostMalloc(&c->stage, need, hipHostMallocDefault) != hipSuccess) {
        c->stage = nullptr;
        return fail(KP_ENOMEM, "kp_load_jobs: pinned staging of %zu bytes", need);
      }
      c->stage_bytes = need;
    }
    int64_t *sq = static_cast<int64_t *>(c->stage);
    int32_t *s32 = reinterpret_cast<int32_t *>(sq + (size_t)D * U);
    std::memcpy(sq, c->h_q.data(), sizeof(int64_t) * D * U);
    std::memcpy(s32, c->h_leader.data(), sizeof(int32_t) * U);
    std::memcpy(s32 + U, c->h_size.data(), sizeof(int32_t) * U);
    std::memcpy(s32 + 2 * (size_t)U, c->h_prio.data(), sizeof(int32_t) * U);
    std::memcpy(s32 + 3 * (size_t)U, c->h_aff.data(), sizeof(int32_t) * U);
    KP_HIP(hipMemcpyAsync(c->d.q, sq, sizeof(int64_t) * D * U, hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(c->d.leader, s32, sizeof(int32_t) * U, hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(c->d.size, s32 + U, sizeof(int32_t) * U, hipMemcpyHostToDevice,
                          c->stream));
    KP_HIP(hipMemcpyAsync(c->d.uprio, s32 + 2 * (size_t)U, sizeof(int32_t) * U,
                          hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(c->d.aff, s32 + 3 * (size_t)U, sizeof(int32_t) * U,
                          hipMemcpyHostToDevice, c->stream));
  }
  KP_HIP(hipStreamSynchronize(c->stream));
  c->J = J;
  c->U = U;
  // this rank's shard: a contiguous block of rank positions
  c->u_lo = (int32_t)((int64_t)U * c->rank / c->world);
  c->u_hi = (int32_t)((int64_t)U * (c->rank + 1) / c->world);
  c->max_req = 0;
  for (int64_t i = 0; i < (int64_t)D * J; ++i) c->max_req = std::max(c->max_req, req[i]);
  // pending requests per dim, on the node totals' scale: every 16th job x 16
  // against every 4th node x 4 (the automatic bid-minima dims only)
  for (int d = 0; d < KP_MAX_DIMS; ++d) {
    double rs = 0;
    if (d < D)
      for (int32_t j = 0; j < J; j += 16) rs += (double)req[(int64_t)d * J + j];
    c->req_sum[d] = rs * 16.0 / 4.0;
  }
  c->reqs32 = c->max_req < ((int64_t)1 << 32);
  c->fits32 = c->caps32 && c->reqs32;
  c->jobs_loaded = true;
  return KP_OK;
}

// Waits of a multi-rank solve. A shard of kp_create_multi polls instead of
// blocking, so that a peer shard that failed (and so never joins the next
// collective, whose kernels would then wait for it forever) releases it: the
// multi context aborts the communicators once every shard has returned.
static int wait_event(kp_ctx *c, hipEvent_t ev) {
  if (!c->peer_failed) {
    KP_HIP(hipEventSynchronize(ev));
    return KP_OK;
  }
  for (uint32_t spin = 0;; ++spin) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return KP_OK;
    if (e != hipErrorNotReady) {
      kp_set_error("hipEventQuery", e);
      return KP_EHIP;
    }
    if (c->peer_failed->load(std::memory_order_acquire))
      return fail(KP_ERCCL, "kp_solve: a peer shard failed; the exchange cannot complete");
    if (spin < 256)
      std::this_thread::yield();
    else
      std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

static int wait_stream(kp_ctx *c, hipEvent_t ev) {
  KP_HIP(hipEventRecord(ev, c->stream));
  return wait_event(c, ev);
}

// ---------------------------------------------------------------------------
// One all-gather of `per` int32 per rank (device send [per] -> device recv
// [world][per]) over the context's transport: RCCL over xGMI, or the
// host-staged callback (kp_set_allgather, or the in-process exchange of
// kp_create_multi with a repeated GPU id) through host memory.
static int allgather_i32(kp_ctx *c, const int32_t *send, int32_t *recv, size_t per) {
  if (c->nccl_comm) {
    if (c->peer_failed && c->peer_failed->load(std::memory_order_acquire))
      return fail(KP_ERCCL, "a peer shard failed before the exchange");
    c->in_collective = true;
    c->rccl_calls++;
    if (ncclAllGather(send, recv, per, ncclInt32, static_cast<ncclComm_t>(c->nccl_comm),
                      c->stream) != ncclSuccess)
      return fail(KP_ERCCL, "ncclAllGather of %zu ints", per);
    return KP_OK;
  }
  try {
    c->h_xg_send.resize(per);
    c->h_xg_recv.resize(per * c->world);
  } catch (const std::bad_alloc &) {
    return fail(KP_ENOMEM, "exchange staging");
  }
  KP_HIP(hipMemcpyAsync(c->h_xg_send.data(), send, sizeof(int32_t) * per, hipMemcpyDeviceToHost,
                        c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  if (c->allgather(c->allgather_user, c->h_xg_send.data(), sizeof(int32_t) * per,
                   c->h_xg_recv.data()) != 0)
    return fail(KP_ERCCL, "host-staged all-gather failed");
  KP_HIP(hipMemcpyAsync(recv, c->h_xg_recv.data(), sizeof(int32_t) * per * c->world,
                        hipMemcpyHostToDevice, c->stream));
  return KP_OK;
}

// This rank's candidates -> every rank's, as fixed-size blocks
// [count, (unit, K candidates) x B] (B: the same slot bound on every rank), so
// the all-gather needs no host-known count: one collective per round and, over
// RCCL, no host synchronisation.
static int exchange_round(kp_ctx *c, int32_t B, int32_t K) {
  const size_t per = 1 + (size_t)B * (K + 1);
  KP_TRY(launch_pack_exchange(c, B, K));
  KP_TRY(allgather_i32(c, c->d.xg_send, c->d.xg_recv, per));
  return launch_unpack_exchange(c, c->world, B, K);
}

static double ev_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.0;
  return ms;
}

static int solve_impl(kp_ctx *c, const kp_params *p, kp_result *stats) {
  if (!c->nodes_loaded || !c->jobs_loaded) return fail(KP_ESTATE, "kp_solve: load nodes and jobs first");
  if (c->xchg && !c->nccl_comm && !c->allgather)
    return fail(KP_ESTATE, "kp_solve: multi-rank context without an exchange");
  KP_TRY(check_params(p, c->D));
  c->solved = false;
  // per-solve state that an earlier failed solve may have left set
  c->keys_in_merge = false;
  c->in_collective = false;
  c->rccl_calls = 0;
  KP_HIP(hipSetDevice(c->device));
  const ScoreParams sp = make_sp(c, p);
  const int32_t K = p->n_cand, U = c->U, N = c->N;
  const int64_t Ns = (N + 63) & ~63;
  KP_TRY(prep_for(c, p));
  KP_TRY(launch_node_rec(c));
  {  // every buffer the solve's kernels touch exists (never launch on a null)
    const DevState &d = c->d;
    const void *need[] = {d.cap, d.used, d.R32, d.K32, d.base, d.topo, d.perm, d.np32, d.q, d.leader,
                          d.size, d.status, d.salt, d.aff, d.job_node, d.job_score, d.job_status,
                          d.act, d.act_local, d.cand, d.cand_local, d.open, d.flag, d.s0, d.bid,
                          d.win, d.winmin, d.bmin, d.gpart, d.nparts, d.arrive, d.inv, d.ent_unit,
                          d.ent_slot, d.ent_size, d.ent_lead, d.ent_q, d.csr_kin, d.csr_vin,
                          d.csr_keys, d.csr_vals, d.seg_start, d.seg_end, d.node_flag, d.node_list, d.nrec, d.nst,
                          d.pass_flag, d.counters, d.stats, d.temp};
    for (const void *ptr : need)
      if (!ptr) return fail(KP_ENOMEM, "kp_solve: a device buffer is missing");
  }
  KP_TRY(launch_reset_units(c, p->tie_seed));  // also the salts of the rotated tie-break
  c->pack_sp = sp;
  c->pack_canonical = true;  // the solve scores in canonical column order
  const int32_t shard = c->u_hi - c->u_lo;
  // Fused filter + score + top-K (kp_topk.hip) when the class-aligned layout
  // is compact, every cap and request < 2^30 (exact signed differences in its
  // fit test) and every score fits the 32-bit key's score field; else the
  // materialised score matrix + top-K select.
  int32_t ksh = 0;
  {
    int64_t bound = (int64_t)p->w_gpu_fit + p->w_affinity + 1;
    for (int d = 0; d < c->D; ++d) bound += (int64_t)p->w_dim[d] * p->util_scale;
    int bits = 0;
    while (bits < 63 && (bound >> bits) != 0) ++bits;
    ksh = 32 - bits;  // (score + 1) << ksh keeps the score; >= 8 tie-key bits below it
  }
  const bool fused = c->fused_enabled && c->fz_layout_ok && c->fits32 &&
                     c->max_cap < ((int64_t)1 << 30) && c->max_req < ((int64_t)1 << 30) &&
                     ksh >= 8 && (int64_t)(c->fz_P / fz_tile(c)) * K <= 2048;
  c->pack_fused = fused;
  c->pack_full = true;
  c->last_fused = fused;
  int64_t rpc = rows_per_chunk(c);
  c->crec_ok = false;
  if (fused) {
    // the row records of every unit and class, once for the whole solve
    // (they depend on the requests and the class capacities, not on usage)
    const int RWr = (2 * c->D + 4 + 3) & ~3;
    const int64_t words = (int64_t)std::max(U, 1) * std::max(c->nfc, 1) * RWr;
    if (c->nfc > 0 && c->crec_enabled && words * 4 <= c->crec_max_bytes) {
      if (words > c->cap_crec) {
        c->cap_crec = 0;
        if (dalloc(&c->d.crec, (size_t)words) == KP_OK) {
          c->cap_crec = words;
        } else {
          // the table is an optimisation: k_score_topk computes the records
          // itself without it, so a short device does not fail the solve
          (void)hipGetLastError();
          c->last_error.clear();
        }
      }
      if (c->cap_crec >= words) {
        KP_TRY(launch_unit_rec(c, sp));
        c->crec_ok = true;
      }
    }
    rpc = INT64_MAX;  // no matrix, no chunks: per row only tiles x K keys
    KP_TRY(ensure_part(c, (int64_t)std::max(shard, 1) * (c->fz_P / fz_tile(c)) * K));
    if (!c->d.part || !c->d.colnode || !c->d.wshift)
      return fail(KP_ENOMEM, "kp_solve: a fused-path buffer is missing");
  } else {
    KP_TRY(ensure_matrix(c, (int32_t)std::min<int64_t>(std::max(shard, 1), rpc)));
  }

  Events E;  // every event of this solve, destroyed on every exit path
  // timing-only events: no system-scope fence (cache writeback/invalidate)
  // at each record, so the bracket measures the kernel, not the fence
  struct KEv {
    hipEvent_t a, b;
    int32_t round;
    int64_t rows_bound;
  };
  std::vector<KEv> kev;
  hipEvent_t t0, t1;
  KP_TRY(E.make(&t0, hipEventDefault));
  KP_TRY(E.make(&t1, hipEventDefault));
  KP_HIP(hipMemsetAsync(c->d.stats, 0, sizeof(SolveStats), c->stream));
  KP_HIP(hipMemsetAsync(c->d.pass_flag, 0, sizeof(int32_t) * kPassFlagWords, c->stream));
  KP_HIP(hipEventRecord(t0, c->stream));
  std::vector<int32_t> round_active;  // exact active units per round (when known)
  kp_timing tm{};
  // profiling level 2: per round, events at the round start, after the
  // candidate phase, after the exchange (multi-rank) and after the passes
  std::vector<std::array<hipEvent_t, 4>> pev;
  auto mark = [&](int i) -> int {
    if (c->profiling < 2) return KP_OK;
    if (i == 0) pev.push_back({nullptr, nullptr, nullptr, nullptr});
    if (pev.empty()) return KP_OK;
    KP_TRY(E.make(&pev.back()[i], hipEventDisableSystemFence));
    KP_HIP(hipEventRecord(pev.back()[i], c->stream));
    return KP_OK;
  };
  // filter+score and top-K select of `rows` rows starting at act_local[r0];
  // rows_dev (nullable) clamps them to the device count
  auto score_select = [&](int64_t r0, int32_t rows, const int32_t *rows_dev,
                          int32_t round) -> int {
    // profiling brackets the filter+score launch only (each event record is
    // a GPU packet of a few us: the select is timed by rocprofv3 instead)
    KEv ke{nullptr, nullptr, round, rows};
    if (c->profiling) {
      KP_TRY(E.make(&ke.a, hipEventDisableSystemFence));
      KP_TRY(E.make(&ke.b, hipEventDisableSystemFence));
      KP_HIP(hipEventRecord(ke.a, c->stream));
    }
    // the solve needs only the score matrix: its -1 sentinel is the
    // feasibility filter, so the bit mask (kp_score's second output) is not
    // materialised here
    if (fused) {
      // one GPU, counting mode: the merge also does k_csr_keys' work
      c->keys_in_merge = false;
      if (!c->xchg && c->keys_merge_enabled && r0 == 0 && rows > 0) {
        KP_TRY(csr_prepare(c, rows, K));
        c->keys_in_merge = c->csr_mode == 1;
      }
      // the profiling bracket ends right after k_score_topk (before the merge)
      c->fz_end_event = c->profiling ? ke.b : nullptr;
      const int rc = launch_score_topk(c, sp, c->d.act_local + r0, rows, ksh,
                                       c->d.cand_local + r0 * K, rows_dev, true);
      c->fz_end_event = nullptr;
      KP_TRY(rc);
    } else {
      KP_TRY(launch_score(c, sp, c->d.act_local + r0, rows, c->d.score, nullptr, c->d.q, U,
                          rows_dev));
    }
    if (c->profiling) {
      if (!fused) KP_HIP(hipEventRecord(ke.b, c->stream));
      kev.push_back(ke);
    }
    if (!fused)
      KP_TRY(launch_select(c, sp, c->d.act_local + r0, rows, c->d.score,
                           c->d.cand_local + r0 * K, rows_dev));
    tm.score_launches++;
    return KP_OK;
  };
  double pass_wait_us = 0;
  hipEvent_t evP;  // host-followed passes: the fallback wait on the stream
  KP_TRY(E.make(&evP, hipEventDisableTiming));
  // this round's serial: the host-followed pass tags (hpass) keep 30 bits of
  // it, so before it reaches 2^30 the slots are reset (once the stream has
  // drained, no k_accept still writes them) and the serial restarts: a stale
  // slot can never match
  auto next_serial = [&]() -> int {
    if (c->round_serial >= (1 << 30) - 1) {
      KP_TRY(wait_stream(c, evP));
      for (int i = 0; i < 64; ++i) c->hpass[i] = -1;
      c->round_serial = 0;
    }
    c->cur_serial = c->round_serial++;
    return KP_OK;
  };
  auto passes_of_round = [&](int32_t A, const int32_t *A_dev, bool follow) -> int {
    // also opens the slots, banks + clears the pass flags
    KP_TRY(launch_csr_build(c, A, K, A_dev));
    // passes run back to back on the device: no host round trip inside a round
    const int32_t M = follow && A > 0 && c->N > 0 ? c->pass_follow : 0;
    if (M == 0 || M >= p->max_passes) {
      for (int32_t pass = 0; pass < p->max_passes; ++pass) {
        KP_TRY(launch_plan(c, sp, A, pass, A_dev));
        KP_TRY(launch_accept(c, sp, pass, A));
      }
      return KP_OK;
    }
    // host-followed: pass p is enqueued once pass p - M's flag (stored by its
    // k_accept into coherent host memory, tagged with the round serial) says
    // that pass had proposals; the first pass without any ends the round, so a
    // round that converges early leaves at most M - 1 no-op passes behind
    // instead of max_passes - passes
    const int32_t tag = (int32_t)(((uint32_t)c->cur_serial & 0x3FFFFFFFu) << 1);
    struct HpassOff {
      kp_ctx *c;
      ~HpassOff() { c->hpass_on = false; }
    } hoff{c};
    c->hpass_on = true;
    for (int32_t pass = 0; pass < p->max_passes; ++pass) {
      if (pass >= M) {
        const auto w0 = std::chrono::steady_clock::now();
        const int32_t *f = c->hpass + (pass - M);
        int32_t v;
        for (uint32_t spin = 0; ((v = __atomic_load_n(f, __ATOMIC_ACQUIRE)) & ~1) != tag; ++spin) {
          // a kp_create_multi shard whose peer failed before its exchange:
          // this round's collective never completes, so its pass flags never
          // arrive (the multi context aborts the communicators afterwards)
          if ((spin & 255u) == 255u && c->peer_failed &&
              c->peer_failed->load(std::memory_order_acquire))
            return fail(KP_ERCCL, "kp_solve: a peer shard failed; the exchange cannot complete");
          if ((spin & 1023u) == 1023u &&
              std::chrono::steady_clock::now() - w0 > std::chrono::milliseconds(200)) {
            // the stream has stored it for sure once it drains (polled, so a
            // failed peer still releases a multi shard)
            KP_TRY(wait_stream(c, evP));
            v = __atomic_load_n(f, __ATOMIC_ACQUIRE);
            if ((v & ~1) != tag) return fail(KP_EHIP, "kp_solve: pass flag not delivered");
            break;
          }
        }
        pass_wait_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - w0).count();
        if ((v & 1) == 0) break;  // pass - M had no proposals: the round is over
      }
      KP_TRY(launch_plan(c, sp, A, pass, A_dev));
      KP_TRY(launch_accept(c, sp, pass, A));
    }
    return KP_OK;
  };
  if (!c->xchg) {
    // Device-driven rounds: a round is enqueued with its grids sized by the
    // previous round's active count (active units only shrink) and every
    // kernel clamps to the device count. The host learns a round's count
    // from an async copy that lands early in the round, while the GPU is
    // still busy with it, so there is no idle gap between rounds. A round
    // that turns out empty is a string of no-op launches and ends the solve.
    hipEvent_t evA;
    KP_TRY(E.make(&evA, hipEventDisableTiming));
    int32_t *A_h = c->pinned + 256;
    int64_t A_bound = shard;
    // the round's count: stored by the compaction kernel into coherent pinned
    // memory (spin on the -1 sentinel), or copied + event
    double wait_us = 0;
    const auto h_start = std::chrono::steady_clock::now();
    auto round_count = [&](bool direct) -> int {
      const auto w0 = std::chrono::steady_clock::now();
      struct WaitAcc {
        double &acc;
        std::chrono::steady_clock::time_point t;
        ~WaitAcc() {
          acc += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count();
        }
      } wacc{wait_us, w0};
      if (!direct) {
        KP_HIP(hipEventSynchronize(evA));
        return KP_OK;
      }
      const auto t0 = std::chrono::steady_clock::now();
      int32_t v;
      for (uint32_t spin = 0; (v = __atomic_load_n(c->pinned_coh, __ATOMIC_ACQUIRE)) < 0; ++spin) {
        if ((spin & 1023u) == 1023u &&
            std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
          // not seen yet (e.g. a busy host): the stream has it for sure
          KP_HIP(hipStreamSynchronize(c->stream));
          v = __atomic_load_n(c->pinned_coh, __ATOMIC_ACQUIRE);
          if (v < 0) return fail(KP_EHIP, "kp_solve: round count not delivered");
          break;
        }
      }
      *A_h = v;
      return KP_OK;
    };
    for (int32_t r = 0; A_bound > 0; ++r) {
      if (p->max_rounds > 0 && r >= p->max_rounds) break;
      KP_TRY(next_serial());
      KP_TRY(mark(0));
      bool direct = true;
      KP_TRY(launch_active_async(c, c->u_lo, c->u_hi, A_h, &direct));
      if (!direct) KP_HIP(hipEventRecord(evA, c->stream));
      if (A_bound > rpc) {  // chunked score matrix: needs the exact count first
        KP_TRY(round_count(direct));
        const int32_t A = *A_h;
        if (A == 0) break;
        for (int64_t r0 = 0; r0 < A; r0 += rpc)
          KP_TRY(score_select(r0, (int32_t)std::min<int64_t>(rpc, A - r0), nullptr, r));
        KP_TRY(mark(1));
        round_active.push_back(A);
        KP_TRY(passes_of_round(A, nullptr, true));
        KP_TRY(mark(3));
        A_bound = A;
        continue;
      }
      const int32_t *A_dev = c->d.counters;
      KP_TRY(score_select(0, (int32_t)A_bound, A_dev, r));
      KP_TRY(mark(1));
      KP_TRY(passes_of_round((int32_t)A_bound, A_dev, true));
      KP_TRY(mark(3));
      KP_TRY(round_count(direct));  // landed long ago on a busy round
      round_active.push_back(*A_h);
      A_bound = *A_h;
      if (c->host_prof) {
        const double now = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h_start).count();
        std::fprintf(stderr, "kp_host_round %d A %d t_us %.1f wait_us %.1f\n", r, *A_h, now, wait_us);
      }
    }
    if (c->host_prof) {
      const double tot = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h_start).count();
      std::fprintf(stderr, "kp_host_prof pass_wait_us %.1f\n", pass_wait_us);
      std::fprintf(stderr, "kp_host_prof rounds %zu host_loop_us %.1f wait_us %.1f enqueue_us %.1f\n",
                   round_active.size(), tot, wait_us, tot - wait_us);
    }
  } else {
    // Multi-GPU, device-driven like the single-GPU loop: the local and the
    // global active counts stay on the device (counters[0] / counters[1]);
    // grids and exchange blocks are sized by the previous round's global
    // count, which every rank reads asynchronously (the same value on all
    // ranks, so every rank calls the all-gather with the same size).
    hipEvent_t evG;
    KP_TRY(E.make(&evG, hipEventDisableTiming));
    hipEvent_t evS;
    KP_TRY(E.make(&evS, hipEventDisableTiming));
    int32_t *Al_h = c->pinned + 256, *G_h = c->pinned + 320;
    int64_t Smax = 0;  // largest shard
    for (int r = 0; r < c->world; ++r)
      Smax = std::max<int64_t>(Smax, (int64_t)U * (r + 1) / c->world - (int64_t)U * r / c->world);
    const bool chunked = std::min<int64_t>(shard, Smax) > rpc;
    KP_TRY(csr_reserve(c, U));  // no reallocation between the round's collectives
    int64_t G_bound = U;
    for (int32_t r = 0; G_bound > 0; ++r) {
      if (p->max_rounds > 0 && r >= p->max_rounds) break;
      KP_TRY(next_serial());
      KP_TRY(mark(0));
      const int32_t B = (int32_t)std::min<int64_t>(Smax, G_bound);  // per-rank slot bound
      if (shard > 0) {
        KP_TRY(launch_active_async(c, c->u_lo, c->u_hi, Al_h));
      } else {  // an empty shard (fewer units than ranks) still joins the exchange
        KP_HIP(hipMemsetAsync(c->d.counters, 0, sizeof(int32_t), c->stream));
        *Al_h = 0;
      }
      const int32_t rows = (int32_t)std::min<int64_t>(shard, B);
      if (chunked) {  // the score matrix is chunked: needs the exact local count
        KP_TRY(wait_stream(c, evS));
        for (int64_t r0 = 0; r0 < *Al_h; r0 += rpc)
          KP_TRY(score_select(r0, (int32_t)std::min<int64_t>(rpc, *Al_h - r0), nullptr, r));
      } else if (rows > 0) {
        KP_TRY(score_select(0, rows, c->d.counters, r));
      }
      if (c->test_fail_solve) {  // test knob: this rank never reaches the exchange
        c->test_fail_solve = 0;
        return fail(KP_ENOMEM, "KP_TEST_FAIL_SOLVE: injected failure of rank %d before its exchange", c->rank);
      }
      KP_TRY(mark(1));
      KP_TRY(exchange_round(c, B, K));
      KP_TRY(mark(2));
      KP_HIP(hipMemcpyAsync(G_h, c->d.counters + 1, sizeof(int32_t), hipMemcpyDeviceToHost,
                            c->stream));
      KP_HIP(hipEventRecord(evG, c->stream));
      KP_TRY(passes_of_round((int32_t)std::min<int64_t>(U, (int64_t)B * c->world),
                             c->d.counters + 1, true));
      KP_TRY(mark(3));
      KP_TRY(wait_event(c, evG));  // lands before this round's passes run
      round_active.push_back(*Al_h);
      G_bound = *G_h;
    }
  }
  KP_TRY(launch_finalize(c));
  KP_HIP(hipEventRecord(t1, c->stream));
  if (c->host_prof && !c->xchg) {
    launch_probe(c, sp, std::min<int32_t>(shard, 26000));
    launch_probe(c, sp, std::min<int32_t>(shard, 1000));
  }
  // per-unit status and the device-side statistics
  std::vector<int32_t> status(U);
  if (U > 0)
    KP_HIP(hipMemcpyAsync(status.data(), c->d.status, sizeof(int32_t) * U, hipMemcpyDeviceToHost,
                          c->stream));
  SolveStats dst{};
  KP_HIP(hipMemcpyAsync(&dst, c->d.stats, sizeof dst, hipMemcpyDeviceToHost, c->stream));
  if (c->xchg) {
    hipEvent_t evF;
    KP_TRY(E.make(&evF, hipEventDisableTiming));
    KP_TRY(wait_stream(c, evF));
  } else {
    KP_HIP(hipStreamSynchronize(c->stream));
  }
  c->in_collective = false;  // every collective of this solve completed
  const int32_t rounds = (int32_t)dst.rounds, passes = (int32_t)dst.passes;
  const int64_t pairs = dst.active_sum * N;
  tm.solve_ms = ev_ms(t0, t1);
  for (auto &ke : kev) {
    tm.score_ms += ev_ms(ke.a, ke.b);
    // algorithmic bytes of the rows the launch actually had (device count)
    int64_t rows = ke.rows_bound;
    if (ke.round < (int32_t)round_active.size())
      rows = std::min<int64_t>(rows, round_active[ke.round]);
    if (fused) {  // compulsory bytes: requests in, per-tile lists out, node planes once
      const int64_t lists = (int64_t)(c->fz_P / fz_tile(c)) * K * 8;
      tm.score_bytes += rows * ((int64_t)8 * c->D + 12 + lists) +
                        (int64_t)(2 * c->D + 3) * 4 * c->fz_P;
      tm.select_bytes += rows * (lists + K * 4);  // k_merge_tour
    } else {
      tm.score_bytes += rows * Ns * 4 + (int64_t)8 * c->D * rows + (int64_t)3 * 8 * c->D * N +
                        8 * (int64_t)N;
      tm.select_bytes += rows * Ns * 4 + rows * K * 4;
    }
  }
  tm.accept_ms = tm.solve_ms - tm.score_ms - tm.select_ms;
  for (const auto &e : pev) {  // phase split (profiling level 2)
    if (e[0] && e[1]) tm.cand_ms += ev_ms(e[0], e[1]);
    if (e[1] && e[2]) tm.xchg_ms += ev_ms(e[1], e[2]);
    const hipEvent_t from = e[2] ? e[2] : e[1];
    if (from && e[3]) tm.pass_ms += ev_ms(from, e[3]);
  }
  tm.fused = fused ? 1 : 0;
  tm.score_classes = c->n_classes;
  tm.score_form = !fused && c->fits32 && c->n_classes > 0 && c->score_classes ? 1 : 0;
  c->timing = tm;
  int32_t placed = 0;
  for (int32_t u = 0; u < U; ++u)
    if (status[u] == kPlaced) placed += c->h_size[u];
  c->last.rounds = rounds;
  c->last.passes = passes;
  c->last.placed_jobs = placed;
  c->last.unplaced_jobs = c->J - placed;
  c->last.units = U;
  c->last.pairs_scored = pairs;
  if (stats) {
    stats->rounds = rounds;
    stats->passes = passes;
    stats->placed_jobs = placed;
    stats->unplaced_jobs = c->J - placed;
    stats->units = U;
    stats->pairs_scored = pairs;
  }
  c->solved = true;
  return KP_OK;
}

static int fetch_impl(kp_ctx *c, kp_result *r) {
  if (!c->solved) return fail(KP_ESTATE, "kp_fetch: no solve since the last load");
  KP_HIP(hipSetDevice(c->device));
  const int32_t J = c->J;
  if (J > 0) {
    if (r->node_of_job)
      KP_HIP(hipMemcpyAsync(r->node_of_job, c->d.job_node, sizeof(int32_t) * J,
                            hipMemcpyDeviceToHost, c->stream));
    if (r->score_of_job)
      KP_HIP(hipMemcpyAsync(r->score_of_job, c->d.job_score, sizeof(int32_t) * J,
                            hipMemcpyDeviceToHost, c->stream));
    if (r->status_of_job)
      KP_HIP(hipMemcpyAsync(r->status_of_job, c->d.job_status, sizeof(int32_t) * J,
                            hipMemcpyDeviceToHost, c->stream));
  }
  if (r->used_out && c->N > 0)
    KP_HIP(hipMemcpyAsync(r->used_out, c->d.used, sizeof(int64_t) * c->D * c->N,
                          hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  r->rounds = c->last.rounds;
  r->passes = c->last.passes;
  r->placed_jobs = c->last.placed_jobs;
  r->unplaced_jobs = c->last.unplaced_jobs;
  r->units = c->last.units;
  r->pairs_scored = c->last.pairs_scored;
  return KP_OK;
}

}  // namespace kp

using namespace kp;

extern "C" {

void kp_params_default(kp_params *p) {
  if (!p) return;
  static const int32_t w[KP_MAX_DIMS] = {1, 1, 4, 2, 1, 1, 1, 1};
  std::memset(p, 0, sizeof *p);
  for (int d = 0; d < KP_MAX_DIMS; ++d) p->w_dim[d] = w[d];
  p->score_mode = KP_SCORE_MOST_ALLOCATED;
  p->gpu_dim = 2;
  p->w_gpu_fit = 1024;
  p->w_spread = 256;
  p->tie_mode = KP_TIE_ROTATED;
  p->tie_seed = 0x6B706C61u;
  p->max_rounds = 0;
  p->n_cand = 16;
  p->util_scale = 100;
  p->max_passes = 16;
  p->w_affinity = 512;
}

int kp_abi_version(void) { return KP_ABI_VERSION; }

const char *kp_strerror(int code) {
  switch (code) {
    case KP_OK: return "ok";
    case KP_EINVAL: return "invalid argument";
    case KP_EHIP: return "HIP runtime error";
    case KP_ERCCL: return "RCCL error";
    case KP_ENOMEM: return "out of memory";
    case KP_ESTATE: return "call order violated";
    case KP_ENODEV: return "no usable gfx950 device";
  }
  return "unknown error";
}

const char *kp_last_error(kp_ctx *c) {
  if (!c) return "";
  std::lock_guard<std::mutex> g(c->mu);
  // a copy in storage owned by the context: never freed by a later call
  const size_t n = std::min(c->last_error.size(), sizeof c->last_error_buf - 1);
  std::memcpy(c->last_error_buf, c->last_error.data(), n);
  c->last_error_buf[n] = '\0';
  return c->last_error_buf;
}

int kp_last_error_r(kp_ctx *c, char *buf, size_t len) {
  if (!c) {
    if (buf && len) buf[0] = '\0';
    return 0;
  }
  std::lock_guard<std::mutex> g(c->mu);
  if (buf && len) {
    const size_t n = std::min(c->last_error.size(), len - 1);
    std::memcpy(buf, c->last_error.data(), n);
    buf[n] = '\0';
  }
  return (int)std::min<size_t>(c->last_error.size(), INT32_MAX);
}

int kp_dist_unique_id(void *out128) {
  if (!out128) return KP_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return KP_ERCCL;
  static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
  std::memcpy(out128, &id, sizeof id);
  return KP_OK;
}

int kp_create(kp_ctx **out, const kp_config *cfg) {
  if (!out) return KP_EINVAL;
  *out = nullptr;
  kp_config def{};
  def.device = -1;
  def.world_size = 1;
  if (!cfg) cfg = &def;
  if (cfg->world_size < 1 || cfg->rank < 0 || cfg->rank >= cfg->world_size) return KP_EINVAL;
  return create_one(out, cfg->device, cfg->world_size, cfg->rank, cfg->nccl_id, nullptr,
                    cfg->max_pairs_matrix);
}

int kp_create_multi(kp_ctx **out, const int32_t *gpu_ids, int32_t n, const kp_config *cfg) {
  if (!out) return KP_EINVAL;
  *out = nullptr;
  if (!gpu_ids || n < 1) return KP_EINVAL;
  return multi_create(out, gpu_ids, n, cfg ? cfg->max_pairs_matrix : 0);
}

void kp_destroy(kp_ctx *c) {
  if (!c) return;
  if (c->multi) {
    multi_destroy(c);
    return;
  }
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->nccl_comm) ncclCommDestroy(static_cast<ncclComm_t>(c->nccl_comm));
  DevState &d = c->d;
  if (d.fz_prof) {  // KP_FZ_PROF: the accumulated phase clocks
    std::vector<uint64_t> h(kProfWords, 0);
    if (hipMemcpy(h.data(), d.fz_prof, kProfWords * 8, hipMemcpyDeviceToHost) == hipSuccess) {
      if (knob("KP_PASS_SPANS"))
        for (int L = 0; L < 1024; ++L) {
          const uint64_t *x = h.data() + 16 + 64 + 4 * L;
          if (x[0] == ~0ull || x[2] == ~0ull) continue;
          std::fprintf(stderr, "kp_pass_span %d %d plan %.2f acc %.2f gap %.2f\n", L / 16, L % 16,
                       (double)(x[1] - x[0]) * 0.01, (double)(x[3] - x[2]) * 0.01,
                       ((double)x[2] - (double)x[1]) * 0.01);
        }
      std::fprintf(stderr, "kp_fz_prof");
      for (int i = 0; i < 9; ++i) std::fprintf(stderr, " %llu", (unsigned long long)h[i]);
      std::fprintf(stderr, "\n");
      const uint64_t *pp = h.data() + 16;  // KP_PASS_PROFILE (kp_pass.hip)
      for (int k = 0; k < 2; ++k) {
        const uint64_t *b = pp + 16 * k;
        std::fprintf(stderr, "kp_pass_prof %s waves %llu working %llu phase_clk", k ? "accept" : "plan",
                     (unsigned long long)b[8], (unsigned long long)b[9]);
        for (int i = 0; i < 8; ++i) std::fprintf(stderr, " %llu", (unsigned long long)b[i]);
        double span = 0;
        int n = 0;
        for (int L = 0; L < 1024; ++L) {
          const uint64_t lo = pp[64 + 4 * L + 2 * k], hi = pp[64 + 4 * L + 2 * k + 1];
          if (lo != ~0ull && hi >= lo) { span += (double)(hi - lo) * 0.01; ++n; }
        }
        std::fprintf(stderr, " launches %d span_us %.1f wave_clk %llu wave_rt %llu\n", n, span,
                     (unsigned long long)b[10], (unsigned long long)b[11]);
      }
    }
  }
  void *ptrs[] = {d.cap, d.used, d.used0, d.R32, d.K32, d.base, d.topo, d.q, d.leader, d.size,
                  d.status, d.salt, d.aff,
                  d.job_node, d.job_score, d.job_status, d.act_local, d.cand_local, d.score,
                  d.mask, d.open, d.flag, d.s0, d.bid, d.gpart, d.nparts, d.arrive, d.win, d.winmin, d.bmin,
                  d.inv, d.ent_unit,
                  d.ent_slot, d.ent_size, d.ent_lead, d.ent_q, d.perm,
                  d.csr_kin, d.csr_vin,
                  d.csr_keys, d.csr_vals, d.seg_start, d.seg_end, d.pass_flag, d.counters,
                  d.temp, d.xg_counts, d.xg_send, d.xg_recv, d.uprio, d.plist, d.pre_send, d.pre_recv, d.roff,
                  d.rreq, d.rsuf, d.rprio, d.pre_node, d.pre_vict, d.pre_cost,
                  d.dl_node, d.dl_delta, d.dl_bad, d.node_flag, d.node_list, d.nrec, d.nst, d.stats, d.np32, d.ncls, d.ccap, d.colnode, d.wshift, d.part, d.fz_prof,
                  d.bm, d.bms, d.rowinfo, d.cnt, d.rowmap, d.tcls, d.fccap, d.crec};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  if (d.act && d.act != d.act_local) (void)hipFree(d.act);  // multi-rank: separate buffers
  if (d.cand && d.cand != d.cand_local) (void)hipFree(d.cand);
  if (c->pinned) (void)hipHostFree(c->pinned);
  if (c->pinned_coh) (void)hipHostFree(c->pinned_coh);
  if (c->stage) (void)hipHostFree(c->stage);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int kp_set_allgather(kp_ctx *c, kp_allgather_fn fn, void *user) {
  if (!c || !fn) return KP_EINVAL;
  if (c->multi) return KP_ESTATE;  // shards exchange inside the library
  Entry en(c);
  if (c->world < 2 || c->nccl_comm) return fail(KP_ESTATE, "kp_set_allgather: not a host-staged multi-rank context");
  c->allgather = fn;
  c->allgather_user = user;
  return KP_OK;
}

int kp_set_profiling(kp_ctx *c, int level) {
  if (!c) return KP_EINVAL;
  if (c->multi) return multi_run(c, [&](kp_ctx *sh, int) { return kp_set_profiling(sh, level); }, true);
  Entry en(c);
  c->profiling = level <= 0 ? 0 : std::min(level, 2);
  return KP_OK;
}

// every shard's kp_timing of a kp_create_multi context (shard order)
static int shard_timings(kp_ctx *c, std::vector<kp_timing> &all) {
  all.assign((size_t)c->world, kp_timing{});
  return multi_run(c, [&](kp_ctx *sh, int i) { return kp_last_timing(sh, &all[(size_t)i]); }, true);
}

int kp_last_timing(kp_ctx *c, kp_timing *t) {
  if (!c || !t) return KP_EINVAL;
  if (c->multi) {
    // the shards run concurrently: times are the slowest shard's (max per
    // field, like the one-process-per-GPU bench's max over ranks), counts and
    // bytes the sum over shards, the form fields shard 0's
    std::vector<kp_timing> all;
    KP_TRY(shard_timings(c, all));
    kp_timing m = all[0];
    for (size_t i = 1; i < all.size(); ++i) {
      const kp_timing &s = all[i];
      m.solve_ms = std::max(m.solve_ms, s.solve_ms);
      m.score_ms = std::max(m.score_ms, s.score_ms);
      m.select_ms = std::max(m.select_ms, s.select_ms);
      m.accept_ms = std::max(m.accept_ms, s.accept_ms);
      m.cand_ms = std::max(m.cand_ms, s.cand_ms);
      m.xchg_ms = std::max(m.xchg_ms, s.xchg_ms);
      m.pass_ms = std::max(m.pass_ms, s.pass_ms);
      m.score_launches += s.score_launches;
      m.score_bytes += s.score_bytes;
      m.select_bytes += s.select_bytes;
    }
    *t = m;
    return KP_OK;
  }
  Entry en(c);
  *t = c->timing;
  t->rccl_calls = c->rccl_calls;  // the solve's, plus any kp_preempt since
  return KP_OK;
}

int kp_last_timing_shards(kp_ctx *c, kp_timing *t, int32_t n) {
  if (!c || n < 0 || (n > 0 && !t)) return KP_EINVAL;
  if (!c->multi) {
    if (n > 0) KP_TRY(kp_last_timing(c, t));
    return 1;
  }
  std::vector<kp_timing> all;
  KP_TRY(shard_timings(c, all));
  for (int32_t i = 0; i < n && i < (int32_t)all.size(); ++i) t[i] = all[(size_t)i];
  return (int)all.size();
}

// ---------------------------------------------------------------------------
int kp_load_nodes(kp_ctx *c, int32_t N, int32_t D, const int64_t *cap, const int64_t *used,
                  const int32_t *topo) {
  if (!c) return KP_EINVAL;
  if (c->multi)
    return multi_run(c, [&](kp_ctx *sh, int) { return kp_load_nodes(sh, N, D, cap, used, topo); },
                     true);
  Entry en(c);
  return load_nodes_impl(c, N, D, cap, used, topo);
}

int kp_load_jobs(kp_ctx *c, int32_t J, const int64_t *req, const int32_t *prio,
                 const int32_t *gang_id, const int32_t *gang_size, const int32_t *aff) {
  if (!c) return KP_EINVAL;
  if (c->multi)
    return multi_run(
        c, [&](kp_ctx *sh, int) { return kp_load_jobs(sh, J, req, prio, gang_id, gang_size, aff); },
        true);
  Entry en(c);
  return load_jobs_impl(c, J, req, prio, gang_id, gang_size, aff);
}

int kp_solve(kp_ctx *c, const kp_params *p, kp_result *stats) {
  if (!c) return KP_EINVAL;
  if (c->multi)
    return multi_run(c, [&](kp_ctx *sh, int r) { return kp_solve(sh, p, r == 0 ? stats : nullptr); },
                     true);
  Entry en(c);
  try {
    return solve_impl(c, p, stats);
  } catch (const std::bad_alloc &) {
    return fail(KP_ENOMEM, "kp_solve: host allocation");
  }
}

int kp_fetch(kp_ctx *c, kp_result *r) {
  if (!c || !r) return KP_EINVAL;
  if (c->multi) return multi_run(c, [&](kp_ctx *sh, int) { return kp_fetch(sh, r); }, false);
  Entry en(c);
  return fetch_impl(c, r);
}

int kp_place(kp_ctx *c, const kp_snapshot *s, const kp_params *p, kp_result *r) {
  if (!c || !s || !p || !r) return KP_EINVAL;
  if (c->multi)
    return multi_run(c,
                     [&](kp_ctx *sh, int k) {
                       kp_result none{};  // shard k > 0: same solve, no outputs
                       return kp_place(sh, s, p, k == 0 ? r : &none);
                     },
                     true);
  Entry en(c);  // one acquisition: load + solve + fetch never interleave
  KP_TRY(check_params(p, s->D));
  KP_TRY(load_nodes_impl(c, s->N, s->D, s->cap, s->used, s->topo_domain));
  KP_TRY(load_jobs_impl(c, s->J, s->req, s->prio, s->gang_id, s->gang_size, s->affinity));
  try {
    KP_TRY(solve_impl(c, p, nullptr));
  } catch (const std::bad_alloc &) {
    return fail(KP_ENOMEM, "kp_place: host allocation");
  }
  return fetch_impl(c, r);
}

int kp_apply_delta(kp_ctx *c, const int32_t *node_idx, const int64_t *delta, int32_t K) {
  if (!c || K < 0 || (K > 0 && (!node_idx || !delta))) return KP_EINVAL;
  if (c->multi)
    return multi_run(c, [&](kp_ctx *sh, int) { return kp_apply_delta(sh, node_idx, delta, K); },
                     true);
  Entry en(c);
  if (!c->nodes_loaded) return fail(KP_ESTATE, "kp_apply_delta: no node table loaded");
  const int32_t N = c->N, D = c->D;
  for (int32_t k = 0; k < K; ++k)
    if (node_idx[k] < 0 || node_idx[k] >= N)
      return fail(KP_EINVAL, "kp_apply_delta: node_idx[%d] = %d", k, node_idx[k]);
  for (int64_t i = 0; i < (int64_t)D * K; ++i)
    if (delta[i] > KP_MAX_VALUE || delta[i] < -KP_MAX_VALUE)
      return fail(KP_EINVAL, "kp_apply_delta: |delta| > 2^56");
  if (K == 0) return KP_OK;
  KP_HIP(hipSetDevice(c->device));
  // device-side: atomic apply, check the touched entries against [0, cap],
  // undo on violation (the call is all-or-nothing); one host round trip
  if (K > c->cap_delta) {
    c->cap_delta = 0;
    KP_TRY(dalloc(&c->d.dl_node, (size_t)K));
    KP_TRY(dalloc(&c->d.dl_delta, (size_t)D * K));
    c->cap_delta = K;
  }
  KP_HIP(hipMemcpyAsync(c->d.dl_node, node_idx, sizeof(int32_t) * K, hipMemcpyHostToDevice,
                        c->stream));
  KP_HIP(hipMemcpyAsync(c->d.dl_delta, delta, sizeof(int64_t) * D * K, hipMemcpyHostToDevice,
                        c->stream));
  int32_t bad = 0;
  KP_TRY(launch_delta(c, K, &bad));
  if (bad) return fail(KP_EINVAL, "kp_apply_delta: a node would leave [0, cap]; nothing applied");
  return KP_OK;
}

int kp_reset_nodes(kp_ctx *c) {
  if (!c) return KP_EINVAL;
  if (c->multi) return multi_run(c, [&](kp_ctx *sh, int) { return kp_reset_nodes(sh); }, true);
  Entry en(c);
  if (!c->nodes_loaded) return fail(KP_ESTATE, "kp_reset_nodes: no node table loaded");
  KP_HIP(hipSetDevice(c->device));
  if (c->N > 0)
    KP_HIP(hipMemcpyAsync(c->d.used, c->d.used0, sizeof(int64_t) * c->D * c->N,
                          hipMemcpyDeviceToDevice, c->stream));
  return KP_OK;
}

int kp_score(kp_ctx *c, const kp_params *p, int32_t job_lo, int32_t job_hi, int32_t *score,
             uint64_t *mask) {
  if (!c) return KP_EINVAL;
  if (c->multi)
    return multi_run(c, [&](kp_ctx *sh, int) { return kp_score(sh, p, job_lo, job_hi, score, mask); },
                     false);
  Entry en(c);
  if (!c->nodes_loaded || !c->jobs_loaded) return fail(KP_ESTATE, "kp_score: load nodes and jobs first");
  KP_TRY(check_params(p, c->D));
  if (job_lo < 0 || job_hi > c->J || job_lo > job_hi)
    return fail(KP_EINVAL, "kp_score: job range [%d, %d) of %d", job_lo, job_hi, c->J);
  KP_HIP(hipSetDevice(c->device));
  const int32_t rows = job_hi - job_lo, N = c->N;
  if (rows == 0 || N == 0) return KP_OK;
  KP_TRY(prep_for(c, p));
  const ScoreParams sp = make_sp(c, p);
  const int64_t Ns = (N + 63) & ~63, words = Ns / 64, uw = (N + 63) / 64;
  // job -> unit (rank position) map for the requested rows
  std::vector<int32_t> unit_of(rows);
  {
    std::vector<int32_t> u_of_job(c->J);
    for (int32_t u = 0; u < c->U; ++u)
      for (int32_t m = 0; m < c->h_size[u]; ++m) u_of_job[c->h_leader[u] + m] = u;
    for (int32_t r = 0; r < rows; ++r) unit_of[r] = u_of_job[job_lo + r];
  }
  const int64_t rpc = std::min<int64_t>(rows_per_chunk(c), std::max(c->cap_U, 1));
  const int32_t chunk = (int32_t)std::min<int64_t>(rows, rpc);
  KP_TRY(ensure_matrix(c, chunk));
  KP_TRY(ensure_mask(c, chunk));
  std::vector<int32_t> hs;
  std::vector<uint64_t> hm;
  c->pack_sp = sp;
  c->pack_canonical = false;  // kp_score returns columns in node order
  c->pack_fused = false;
  c->pack_full = true;
  KP_TRY(launch_pack(c));  // 32-bit node planes of the current usage
  for (int64_t r0 = 0; r0 < rows; r0 += rpc) {
    const int32_t nr = (int32_t)std::min<int64_t>(rpc, rows - r0);
    KP_HIP(hipMemcpyAsync(c->d.act_local, unit_of.data() + r0, sizeof(int32_t) * nr,
                          hipMemcpyHostToDevice, c->stream));
    KP_TRY(launch_score(c, sp, c->d.act_local, nr, c->d.score, c->d.mask, c->d.q, c->U));
    hs.resize((size_t)nr * Ns);
    hm.resize((size_t)nr * words);
    KP_HIP(hipMemcpyAsync(hs.data(), c->d.score, sizeof(int32_t) * nr * Ns, hipMemcpyDeviceToHost,
                          c->stream));
    KP_HIP(hipMemcpyAsync(hm.data(), c->d.mask, sizeof(uint64_t) * nr * words,
                          hipMemcpyDeviceToHost, c->stream));
    KP_HIP(hipStreamSynchronize(c->stream));
    for (int32_t r = 0; r < nr; ++r) {
      if (score) std::memcpy(score + (r0 + r) * N, hs.data() + (size_t)r * Ns, sizeof(int32_t) * N);
      if (mask) std::memcpy(mask + (r0 + r) * uw, hm.data() + (size_t)r * words, sizeof(uint64_t) * uw);
    }
  }
  return KP_OK;
}

int kp_score_dev(kp_ctx *c, const kp_params *p, int32_t job_lo, int32_t job_hi,
                 int32_t *score_dev, uint64_t *mask_dev) {
  if (!c) return KP_EINVAL;
  if (c->multi) {
    std::lock_guard<std::mutex> g(c->mu);
    c->last_error = "kp_score_dev: not available on a kp_create_multi context";
    return KP_EINVAL;
  }
  Entry en(c);
  if (!c->nodes_loaded || !c->jobs_loaded)
    return fail(KP_ESTATE, "kp_score_dev: load nodes and jobs first");
  KP_TRY(check_params(p, c->D));
  if (job_lo < 0 || job_hi > c->J || job_lo > job_hi)
    return fail(KP_EINVAL, "kp_score_dev: job range [%d, %d) of %d", job_lo, job_hi, c->J);
  KP_HIP(hipSetDevice(c->device));
  const int32_t rows = job_hi - job_lo, N = c->N, D = c->D;
  kp_timing tm{};
  tm.score_classes = c->n_classes;
  tm.score_form = c->fits32 && c->n_classes > 0 && c->score_classes ? 1 : 0;
  c->timing = tm;
  // nothing to write: no launch (and no profiling events left unrecorded)
  if (rows == 0 || N == 0 || (!score_dev && !mask_dev)) return KP_OK;
  KP_TRY(prep_for(c, p));
  const ScoreParams sp = make_sp(c, p);
  const int64_t Ns = (N + 63) & ~63, words = Ns / 64;
  // job -> unit (rank position) of every requested row, staged in chunks of
  // at most cap_U rows through act_local
  std::vector<int32_t> unit_of(rows);
  {
    std::vector<int32_t> u_of_job(c->J);
    for (int32_t u = 0; u < c->U; ++u)
      for (int32_t m = 0; m < c->h_size[u]; ++m) u_of_job[c->h_leader[u] + m] = u;
    for (int32_t r = 0; r < rows; ++r) unit_of[r] = u_of_job[job_lo + r];
  }
  c->pack_sp = sp;
  c->pack_canonical = false;  // node order
  c->pack_fused = false;
  c->pack_full = true;
  KP_TRY(launch_pack(c));
  // one launch over every requested row (a row -> unit map of `rows` entries
  // on the device): the grid's last partial wave of workgroups is paid once,
  // not once per cap_U-row chunk (tools/score_roof.hip: 4 chunks cost 0.74 ->
  // 0.78 ms of stores alone and more with the score arithmetic). Chunks only
  // past the grid's y limit of 65,535 row blocks: the 32-bit forms take 64
  // (k_score32c) or 128 (k_score32) rows per block at that size, the 64-bit
  // k_score always 32.
  const int64_t chunk = (int64_t)65535 * (c->fits32 ? 64 : 32);
  if (c->cap_rowmap < rows) {
    c->cap_rowmap = 0;
    KP_TRY(dalloc(&c->d.rowmap, (size_t)rows));
    c->cap_rowmap = rows;
  }
  KP_HIP(hipMemcpyAsync(c->d.rowmap, unit_of.data(), sizeof(int32_t) * rows, hipMemcpyHostToDevice,
                        c->stream));
  Events E;
  for (int64_t r0 = 0; r0 < rows; r0 += chunk) {
    const int32_t nr = (int32_t)std::min<int64_t>(chunk, rows - r0);
    // profiling: the kernel's own start / end stamps (hipExtLaunchKernel),
    // not events recorded around the launch call, which also caught the
    // device idling while the host submitted the kernel (~80 us per call)
    // (the class form; the other forms keep events around the launch)
    const bool ext = tm.score_form == 1;
    hipEvent_t a = nullptr, b = nullptr;
    if (c->profiling) {
      KP_TRY(E.make(&a, 0));
      KP_TRY(E.make(&b, 0));
      if (!ext) KP_HIP(hipEventRecord(a, c->stream));
    }
    c->score_ev0 = ext ? a : nullptr;
    c->score_ev1 = ext ? b : nullptr;
    const int rc = launch_score(c, sp, c->d.rowmap + r0, nr, score_dev ? score_dev + r0 * Ns : nullptr,
                                mask_dev ? mask_dev + r0 * words : nullptr, c->d.q, c->U);
    c->score_ev0 = c->score_ev1 = nullptr;
    KP_TRY(rc);
    if (c->profiling) {
      if (!ext) KP_HIP(hipEventRecord(b, c->stream));
      KP_HIP(hipEventSynchronize(b));
      c->timing.score_ms += ev_ms(a, b);
    }
    // algorithmic bytes: the outputs written once, each row's request and the
    // node planes (free, a per dim; base, topo, WA, class) read once
    c->timing.score_bytes += (score_dev ? (int64_t)nr * Ns * 4 : 0) + (mask_dev ? (int64_t)nr * words * 8 : 0) +
                             (int64_t)nr * (8 * D + 4) + (int64_t)(2 * D + 4) * 4 * Ns;
    c->timing.score_launches++;
  }
  KP_HIP(hipStreamSynchronize(c->stream));
  return KP_OK;
}

int kp_load_running(kp_ctx *c, int32_t R, const int32_t *node, const int64_t *req,
                    const int32_t *prio) {
  if (!c) return KP_EINVAL;
  if (c->multi)  // every shard scores its share of the preemptors (kp_preempt)
    return multi_run(c, [&](kp_ctx *sh, int) { return kp_load_running(sh, R, node, req, prio); },
                     true);
  Entry en(c);
  if (!c->nodes_loaded) return fail(KP_ESTATE, "kp_load_running: no node table loaded");
  if (R < 0 || (R > 0 && (!node || !req || !prio)))
    return fail(KP_EINVAL, "kp_load_running: R=%d", R);
  const int32_t N = c->N, D = c->D;
  std::vector<int32_t> ord, off;
  std::vector<int64_t> sum, rreq, rsuf, cur;
  std::vector<int32_t> rprio;
  KP_HIP(hipSetDevice(c->device));
  try {
    cur.resize((size_t)D * N + 1);
  } catch (const std::bad_alloc &) {
    return fail(KP_ENOMEM, "kp_load_running: host copy");
  }
  if (N > 0)
    KP_HIP(hipMemcpyAsync(cur.data(), c->d.used, sizeof(int64_t) * D * N, hipMemcpyDeviceToHost,
                          c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  try {
    // validation identical to oracle kpo_check_running: running usage is part
    // of the loaded `used`
    sum.assign((size_t)D * N + 1, 0);
    for (int32_t r = 0; r < R; ++r) {
      const int32_t n = node[r];
      if (n < 0 || n >= N) return fail(KP_EINVAL, "kp_load_running: node[%d] = %d", r, n);
      for (int d = 0; d < D; ++d) {
        const int64_t q = req[(int64_t)d * R + r];
        if (q < 0 || q > KP_MAX_VALUE) return fail(KP_EINVAL, "kp_load_running: req of %d", r);
        if ((sum[(size_t)d * N + n] += q) > cur[(size_t)d * N + n])
          return fail(KP_EINVAL, "kp_load_running: running jobs on node %d exceed its usage", n);
      }
    }
    // node-major CSR in reprieve order: (node, prio desc, running index asc)
    ord.resize(R);
    for (int32_t r = 0; r < R; ++r) ord[r] = r;
    std::sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) {
      if (node[a] != node[b]) return node[a] < node[b];
      if (prio[a] != prio[b]) return prio[a] > prio[b];
      return a < b;
    });
    off.assign((size_t)N + 1, 0);
    for (int32_t r = 0; r < R; ++r) off[node[r] + 1]++;
    for (int32_t n = 0; n < N; ++n) off[n + 1] += off[n];
    rreq.resize((size_t)D * R);
    rsuf.resize((size_t)D * R);
    rprio.resize(R);
    for (int32_t e = 0; e < R; ++e) {
      rprio[e] = prio[ord[e]];
      for (int d = 0; d < D; ++d) rreq[(size_t)d * R + e] = req[(int64_t)d * R + ord[e]];
    }
    // suffix sums of the requests within each node's segment
    for (int32_t n = 0; n < N; ++n)
      for (int d = 0; d < D; ++d) {
        int64_t acc = 0;
        for (int32_t e = off[n + 1] - 1; e >= off[n]; --e) {
          acc += rreq[(size_t)d * R + e];
          rsuf[(size_t)d * R + e] = acc;
        }
      }
  } catch (const std::bad_alloc &) {
    return fail(KP_ENOMEM, "kp_load_running: host arrays");
  }
  c->R = 0;  // no pool until every copy succeeded
  if (R > c->cap_R) {
    c->cap_R = 0;
    KP_TRY(dalloc(&c->d.rreq, (size_t)D * R));
    KP_TRY(dalloc(&c->d.rsuf, (size_t)D * R));
    KP_TRY(dalloc(&c->d.rprio, (size_t)R));
    c->cap_R = R;
  }
  if (R > 0) {
    KP_HIP(hipMemcpyAsync(c->d.rreq, rreq.data(), sizeof(int64_t) * D * R, hipMemcpyHostToDevice,
                          c->stream));
    KP_HIP(hipMemcpyAsync(c->d.rsuf, rsuf.data(), sizeof(int64_t) * D * R, hipMemcpyHostToDevice,
                          c->stream));
    KP_HIP(hipMemcpyAsync(c->d.rprio, rprio.data(), sizeof(int32_t) * R, hipMemcpyHostToDevice,
                          c->stream));
  }
  KP_HIP(hipMemcpyAsync(c->d.roff, off.data(), sizeof(int32_t) * ((size_t)N + 1),
                        hipMemcpyHostToDevice, c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  c->R = R;
  {  // k_preempt_t's packed key bounds
    int64_t worst = 0, maxrun = 0;
    for (int32_t n = 0; n < N; ++n) {
      int64_t sp = 0, sn = 0;
      for (int32_t e = off[n]; e < off[n + 1]; ++e) (rprio[e] > 0 ? sp : sn) += rprio[e];
      worst = std::max(worst, std::max(sp, -sn));
      maxrun = std::max<int64_t>(maxrun, off[n + 1] - off[n]);
    }
    c->pre_key_ok = N < (1 << 20) && maxrun < (1 << 11) && worst < ((int64_t)1 << 31);
  }
  return KP_OK;
}

int kp_preempt(kp_ctx *c, kp_preemption *out) {
  if (!c || !out) return KP_EINVAL;
  if (c->multi) {
    // every shard scores its rows and all-gathers them (identical outputs on
    // every shard); shard 0 writes the caller's arrays
    std::vector<kp_preemption> outs(c->world, kp_preemption{});
    const int rc = multi_run(c, [&](kp_ctx *sh, int i) {
      if (i == 0) return kp_preempt(sh, out);
      return kp_preempt(sh, &outs[i]);  // counts only, no arrays
    }, true);
    return rc;
  }
  Entry en(c);
  if (!c->solved) return fail(KP_ESTATE, "kp_preempt: no solve since the last load");
  KP_HIP(hipSetDevice(c->device));
  int32_t P = 0, lo = 0, hi = 0;
  KP_TRY(launch_preempt(c, &P, &lo, &hi));
  if (c->xchg && P > 0) {
    // rank r scored rows [lo, hi): one all-gather of B = ceil(P / world) rows
    // per rank gives every rank every nomination
    if (!c->nccl_comm && !c->allgather)
      return fail(KP_ESTATE, "kp_preempt: multi-rank context without an exchange");
    const int32_t B = (int32_t)(((int64_t)P + c->world - 1) / c->world);
    const int64_t per = (int64_t)B * 4;
    if (per > c->cap_pre_xg || !c->d.pre_send || !c->d.pre_recv) {
      c->cap_pre_xg = 0;
      KP_TRY(dalloc(&c->d.pre_send, (size_t)per));
      KP_TRY(dalloc(&c->d.pre_recv, (size_t)per * c->world));
      c->cap_pre_xg = per;
    }
    KP_TRY(launch_preempt_pack(c, lo, hi, c->d.pre_send));
    KP_TRY(allgather_i32(c, c->d.pre_send, c->d.pre_recv, (size_t)per));
    KP_TRY(launch_preempt_unpack(c, P, B, c->d.pre_recv));
  }
  const int32_t J = c->J;
  if (J > 0) {
    if (out->node_of_job)
      KP_HIP(hipMemcpyAsync(out->node_of_job, c->d.pre_node, sizeof(int32_t) * J,
                            hipMemcpyDeviceToHost, c->stream));
    if (out->victims_of_job)
      KP_HIP(hipMemcpyAsync(out->victims_of_job, c->d.pre_vict, sizeof(int32_t) * J,
                            hipMemcpyDeviceToHost, c->stream));
    if (out->cost_of_job)
      KP_HIP(hipMemcpyAsync(out->cost_of_job, c->d.pre_cost, sizeof(int64_t) * J,
                            hipMemcpyDeviceToHost, c->stream));
  }
  std::vector<int32_t> nom(J > 0 ? J : 1);
  if (J > 0)
    KP_HIP(hipMemcpyAsync(nom.data(), c->d.pre_node, sizeof(int32_t) * J, hipMemcpyDeviceToHost,
                          c->stream));
  if (c->xchg) {
    hipEvent_t ev;
    Events E;
    KP_TRY(E.make(&ev, hipEventDisableTiming));
    KP_TRY(wait_stream(c, ev));  // a shard polls: a failed peer releases it
  } else {
    KP_HIP(hipStreamSynchronize(c->stream));
  }
  c->in_collective = false;
  int32_t n_nom = 0;
  for (int32_t j = 0; j < J; ++j) n_nom += nom[j] >= 0;
  out->preemptors = P;
  out->nominated = n_nom;
  out->pairs_scored = (int64_t)P * c->N;
  return KP_OK;
}

int kp_parse_gpu_memory(const char *s, int64_t *mib) {
  // CRD pattern ^\d+(Gi|Mi)$ (config/crd/bases/ai.ruijie.io_llmservices.yaml:48-51);
  // the field is optional (omitempty, api/v1/llmservice_types.go:49-51): "" -> 0.
  if (!s || !mib) return KP_EINVAL;
  const size_t n = std::strlen(s);
  if (n == 0) {
    *mib = 0;
    return KP_OK;
  }
  if (n < 3) return KP_EINVAL;
  const char *suf = s + n - 2;
  int64_t mul;
  if (suf[0] == 'G' && suf[1] == 'i')
    mul = 1024;
  else if (suf[0] == 'M' && suf[1] == 'i')
    mul = 1;
  else
    return KP_EINVAL;
  int64_t v = 0;
  for (const char *q = s; q < suf; ++q) {
    if (*q < '0' || *q > '9') return KP_EINVAL;
    if (v > (INT64_MAX - (*q - '0')) / 10) return KP_EINVAL;
    v = v * 10 + (*q - '0');
  }
  if (v > INT64_MAX / mul) return KP_EINVAL;
  *mib = v * mul;
  return KP_OK;
}

}  // extern "C"
