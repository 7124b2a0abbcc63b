/*
 * kp_oracle.c — CPU restatement of the kplace placement spec.
 *
 * TEST INFRASTRUCTURE ONLY (see kp_oracle.h). Written for clarity, not speed:
 * every step is a direct transcription of the spec section cited beside it.
 * Parity of the placement is "unpinned" against the reference (it has no
 * placement code); the input model follows
 * api/v1/llmservice_types.go:25-52 (Replicas, GpuPerReplica, GPUMemory) and
 * internal/controller/llmservice_controller.go:182-203 (one CR -> Replicas
 * identical pods = one all-or-nothing gang here).
 */
#include "kp_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ACTIVE 0
#define PLACED 1
#define NO_FIT 2

struct kpo_state {
  int32_t J, N, D;
  kp_params p;
  const int64_t *req; /* borrowed from the snapshot for the state's lifetime */
  const int64_t *cap;
  int64_t *used;      /* [D*N] committed usage                               */
  int32_t *topo;      /* [N]                                                 */
  int32_t *pos;       /* [N] canonical position: rank of the node in the
                         order (cap vector lexicographic, node index) (§2.3) */
  /* units in rank order (§2.2) */
  int32_t U;
  int32_t *leader;    /* [U] first job index                                 */
  int32_t *size;      /* [U] members                                         */
  uint32_t *salt;     /* [U] rotated tie-break salt (§2.3)                   */
  int32_t *status;    /* [U] ACTIVE / PLACED / NO_FIT                        */
  int32_t *prio;      /* [U] unit priority                                   */
  int32_t *aff;       /* [U] affinity topo domain, -1 = none (§2.3)          */
  int32_t *job_node;  /* [J]                                                 */
  int32_t *job_score; /* [J]                                                 */
  int32_t rounds;
  int32_t passes;
  int64_t pairs;
};

/* ---- §2.1 validation ----------------------------------------------------- */
static int check_params(const kp_params *p, int32_t D) {
  if (!p) return KP_EINVAL;
  for (int d = 0; d < KP_MAX_DIMS; ++d)
    if (p->w_dim[d] < 0 || p->w_dim[d] > 65535) return KP_EINVAL;
  if (p->score_mode != KP_SCORE_MOST_ALLOCATED &&
      p->score_mode != KP_SCORE_LEAST_ALLOCATED)
    return KP_EINVAL;
  if (p->gpu_dim < -1 || p->gpu_dim >= D) return KP_EINVAL;
  if (p->w_gpu_fit < 0 || p->w_gpu_fit > (1 << 20)) return KP_EINVAL;
  if (p->w_spread < 0 || p->w_spread > (1 << 20)) return KP_EINVAL;
  if (p->tie_mode != KP_TIE_NODE_INDEX && p->tie_mode != KP_TIE_ROTATED)
    return KP_EINVAL;
  if (p->max_rounds < 0) return KP_EINVAL;
  if (p->n_cand < 1 || p->n_cand > KP_MAX_CAND) return KP_EINVAL;
  if (p->util_scale < 1 || p->util_scale > 1024) return KP_EINVAL;
  if (p->max_passes < 1 || p->max_passes > 64) return KP_EINVAL;
  if (p->w_affinity < 0 || p->w_affinity > (1 << 20)) return KP_EINVAL;
  return KP_OK;
}

static int check_nodes(const kp_snapshot *s) {
  if (s->N < 0 || s->D < 1 || s->D > KP_MAX_DIMS) return KP_EINVAL;
  if (s->N > 0 && !s->cap) return KP_EINVAL;
  for (int64_t i = 0; i < (int64_t)s->D * s->N; ++i) {
    int64_t c = s->cap[i], u = s->used ? s->used[i] : 0;
    if (c < 0 || c > KP_MAX_VALUE || u < 0 || u > c) return KP_EINVAL;
  }
  if (s->topo_domain)
    for (int32_t n = 0; n < s->N; ++n)
      if (s->topo_domain[n] < 0) return KP_EINVAL;
  return KP_OK;
}

/* ---- §2.3 tie-break ------------------------------------------------------ */
static uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
/* The tie key is a function of the node's canonical position pos(n): the
   rank of n when the nodes are sorted by (cap[0], ..., cap[D-1], n). Nodes
   with the same capacities keep index order, so "lowest index" still holds
   among identical nodes. */
static uint32_t tie_key(const kpo_state *st, int32_t u, int32_t n) {
  if (st->p.tie_mode == KP_TIE_NODE_INDEX) return (uint32_t)st->pos[n];
  return (uint32_t)st->pos[n] * 0x9E3779B1u + st->salt[u];
}

/* ---- §2.3 filter + score ---------------------------------------------------
 * Per dim with cap c > 0 and x = used + q <= c, exactly as kube-scheduler's
 * NodeResourcesFit scorers compute one resource (k8s.io/kubernetes
 * pkg/scheduler/framework/plugins/noderesources, not vendored by the
 * reference):
 *   MostAllocated  (mostRequestedScore):  util = floor(x * S / c)
 *   LeastAllocated (leastRequestedScore): util = floor((c - x) * S / c)
 * with S = util_scale (MaxNodeScore = 100 by default); cap-0 dims are
 * skipped as kube-scheduler skips zero allocatable. The node score is the
 * weighted SUM over dims (kube-scheduler divides it by the weight sum; see
 * DESIGN.md §2.3 for why the numerator is kept). x * S needs up to 67 bits:
 * 128-bit integer arithmetic, no reciprocal. */
static int64_t util_of(int64_t x, int64_t c, int64_t S, int most) {
  const unsigned __int128 n = (unsigned __int128)(uint64_t)x * (uint64_t)S;
  if (most) return (int64_t)(n / (uint64_t)c);
  const unsigned __int128 m = (unsigned __int128)(uint64_t)(c - x) * (uint64_t)S;
  return (int64_t)(m / (uint64_t)c);
}

/* S(q | n, base_used): the score of one more copy of unit u's request q on
 * node n when the node's usage is base_used (a D-vector); -1 if it does not
 * fit. */
static int64_t score_at(const kpo_state *st, int32_t u, const int64_t *q, int32_t n,
                        const int64_t *base_used) {
  const int32_t D = st->D, N = st->N;
  const int most = st->p.score_mode == KP_SCORE_MOST_ALLOCATED;
  int64_t s = 0;
  for (int d = 0; d < D; ++d) {
    int64_t cap = st->cap[(int64_t)d * N + n];
    int64_t used = base_used[d];
    if (q[d] > cap - used) return -1; /* filter: used + q <= cap */
    if (cap > 0) s += (int64_t)st->p.w_dim[d] * util_of(used + q[d], cap, st->p.util_scale, most);
  }
  int g = st->p.gpu_dim;
  if (g >= 0 && q[g] > 0 && st->cap[(int64_t)g * N + n] - base_used[g] - q[g] == 0)
    s += st->p.w_gpu_fit; /* exact fill of the node's free GPUs */
  if (st->aff[u] >= 0 && st->topo[n] == st->aff[u])
    s += st->p.w_affinity; /* CacheStrategy shared: the coordinator's domain */
  return s;
}

static void node_used(const kpo_state *st, const int64_t *usedv, int32_t n,
                      int64_t *out) {
  for (int d = 0; d < st->D; ++d) out[d] = usedv[(int64_t)d * st->N + n];
}

/* ---- §2.2 state construction -------------------------------------------- */
static const int32_t *g_prio_sort; /* qsort context (single-threaded use) */
static const int32_t *g_lead_sort;
static int cmp_rank(const void *a, const void *b) {
  int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
  if (g_prio_sort[x] != g_prio_sort[y])
    return g_prio_sort[x] > g_prio_sort[y] ? -1 : 1; /* prio desc */
  return g_lead_sort[x] < g_lead_sort[y] ? -1 : (g_lead_sort[x] > g_lead_sort[y]);
}
static const int64_t *g_cap_sort; /* qsort context: cap [D*N] */
static int32_t g_cap_D, g_cap_N;
static int cmp_canon(const void *a, const void *b) {
  int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
  for (int d = 0; d < g_cap_D; ++d) {
    int64_t cx = g_cap_sort[(int64_t)d * g_cap_N + x], cy = g_cap_sort[(int64_t)d * g_cap_N + y];
    if (cx != cy) return cx < cy ? -1 : 1;
  }
  return x < y ? -1 : (x > y);
}
static int cmp_i32(const void *a, const void *b) {
  int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
  return x < y ? -1 : (x > y);
}

void kpo_state_free(kpo_state *st) {
  if (!st) return;
  free(st->used); free(st->topo); free(st->aff); free(st->pos);
  free(st->leader); free(st->size); free(st->salt);
  free(st->status); free(st->prio); free(st->job_node); free(st->job_score);
  free(st);
}

#define XALLOC(ptr, n, T) ((ptr) = (T *)malloc(((size_t)(n) + 1) * sizeof(T)))

int kpo_state_new(const kp_snapshot *s, const kp_params *p, kpo_state **out) {
  *out = NULL;
  if (!s || s->J < 0) return KP_EINVAL;
  int rc = check_nodes(s);
  if (rc) return rc;
  if ((rc = check_params(p, s->D))) return rc;
  const int32_t J = s->J, N = s->N, D = s->D;
  if (J > 0 && !s->req) return KP_EINVAL;
  for (int64_t i = 0; i < (int64_t)D * J; ++i)
    if (s->req[i] < 0 || s->req[i] > KP_MAX_VALUE) return KP_EINVAL;

  kpo_state *st = (kpo_state *)calloc(1, sizeof *st);
  if (!st) return KP_ENOMEM;
  st->J = J; st->N = N; st->D = D; st->p = *p;
  st->req = s->req; st->cap = s->cap;
  int32_t *uleader, *usize, *uprio, *uaff;
  XALLOC(st->used, (size_t)D * N, int64_t); XALLOC(st->topo, N, int32_t);

  XALLOC(st->job_node, J, int32_t); XALLOC(st->job_score, J, int32_t);
  XALLOC(uleader, J, int32_t); XALLOC(usize, J, int32_t); XALLOC(uprio, J, int32_t);
  XALLOC(uaff, J, int32_t);
  if (!st->used || !st->topo || !st->job_node ||
      !st->job_score || !uleader || !usize || !uprio || !uaff) {
    free(uleader); free(usize); free(uprio); free(uaff); kpo_state_free(st);
    return KP_ENOMEM;
  }
  for (int64_t i = 0; i < (int64_t)D * N; ++i) st->used[i] = s->used ? s->used[i] : 0;
  for (int32_t n = 0; n < N; ++n) st->topo[n] = s->topo_domain ? s->topo_domain[n] : n;
  { /* canonical positions (§2.3 tie keys) */
    int32_t *ord;
    XALLOC(ord, N, int32_t);
    XALLOC(st->pos, N, int32_t);
    if (!ord || !st->pos) { free(ord); free(uleader); free(usize); free(uprio); free(uaff); kpo_state_free(st); return KP_ENOMEM; }
    for (int32_t n = 0; n < N; ++n) ord[n] = n;
    g_cap_sort = s->cap; g_cap_D = D; g_cap_N = N;
    qsort(ord, N, sizeof(int32_t), cmp_canon);
    for (int32_t i = 0; i < N; ++i) st->pos[ord[i]] = i;
    free(ord);
  }
  for (int32_t j = 0; j < J; ++j) { st->job_node[j] = -1; st->job_score[j] = KP_SCORE_NONE; }

  /* units: maximal runs of equal gang_id >= 0; gang_id < 0 stands alone */
  int32_t U = 0;
  for (int32_t j = 0; j < J;) {
    int32_t g = s->gang_id ? s->gang_id[j] : -1;
    int32_t e = j + 1;
    if (g >= 0)
      while (e < J && s->gang_id[e] == g) ++e;
    int32_t len = e - j;
    if (len > KP_MAX_GANG) rc = KP_EINVAL;
    for (int32_t k = j; k < e && !rc; ++k) {
      if (s->gang_size && s->gang_size[k] != len) rc = KP_EINVAL;
      if (s->prio && s->prio[k] != s->prio[j]) rc = KP_EINVAL;
      if (s->affinity && s->affinity[k] != s->affinity[j]) rc = KP_EINVAL;
      if (s->affinity && s->affinity[k] < -1) rc = KP_EINVAL;
      for (int d = 0; d < D && !rc; ++d)
        if (s->req[(int64_t)d * J + k] != s->req[(int64_t)d * J + j]) rc = KP_EINVAL;
    }
    uleader[U] = j; usize[U] = len; uprio[U] = s->prio ? s->prio[j] : 0;
    uaff[U] = s->affinity ? s->affinity[j] : -1;
    ++U;
    j = e;
  }
  if (!rc && s->gang_id) { /* a gang id may not reappear in a later run */
    int32_t *ids, m = 0;
    XALLOC(ids, U, int32_t);
    for (int32_t u = 0; u < U; ++u)
      if (s->gang_id[uleader[u]] >= 0) ids[m++] = s->gang_id[uleader[u]];
    qsort(ids, m, sizeof(int32_t), cmp_i32);
    for (int32_t i = 1; i < m; ++i)
      if (ids[i] == ids[i - 1]) rc = KP_EINVAL;
    free(ids);
  }
  if (rc) { free(uleader); free(usize); free(uprio); free(uaff); kpo_state_free(st); return rc; }

  /* rank order: prio desc, leader (job index) asc */
  int32_t *ord;
  XALLOC(ord, U, int32_t);
  for (int32_t u = 0; u < U; ++u) ord[u] = u;
  g_prio_sort = uprio; g_lead_sort = uleader;
  qsort(ord, U, sizeof(int32_t), cmp_rank);
  st->U = U;
  XALLOC(st->leader, U, int32_t); XALLOC(st->size, U, int32_t);
  XALLOC(st->salt, U, uint32_t); XALLOC(st->status, U, int32_t);
  XALLOC(st->prio, U, int32_t); XALLOC(st->aff, U, int32_t);
  for (int32_t r = 0; r < U; ++r) {
    int32_t u = ord[r];
    st->leader[r] = uleader[u]; st->size[r] = usize[u]; st->prio[r] = uprio[u];
    st->aff[r] = uaff[u];
    st->salt[r] = fmix32((uint32_t)uleader[u] ^ p->tie_seed);
    st->status[r] = ACTIVE;
  }
  free(ord); free(uleader); free(usize); free(uprio); free(uaff);
  *out = st;
  return KP_OK;
}

int32_t kpo_state_units(const kpo_state *st) { return st->U; }
int32_t kpo_state_unit_leader(const kpo_state *st, int32_t u) { return st->leader[u]; }
int32_t kpo_state_unit_size(const kpo_state *st, int32_t u) { return st->size[u]; }
int32_t kpo_state_active(const kpo_state *st) {
  int32_t a = 0;
  for (int32_t u = 0; u < st->U; ++u) a += st->status[u] == ACTIVE;
  return a;
}

static void unit_req(const kpo_state *st, int32_t u, int64_t *q) {
  for (int d = 0; d < st->D; ++d) q[d] = st->req[(int64_t)d * st->J + st->leader[u]];
}

/* ---- §2.4 candidate phase -------------------------------------------------
 * top-n_cand nodes by (score desc, tie key asc) over the nodes where one
 * member fits, scored against the round-start usage. */
int kpo_round_candidates(const kpo_state *st, int32_t unit_lo, int32_t unit_hi,
                         int32_t *cand, int nthreads) {
  const int32_t N = st->N, K = st->p.n_cand;
  if (unit_lo < 0 || unit_hi > st->U || unit_lo > unit_hi) return KP_EINVAL;
  (void)nthreads;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1)
#endif
  for (int32_t u = unit_lo; u < unit_hi; ++u) {
    int32_t *cn = cand + (size_t)(u - unit_lo) * K;
    for (int k = 0; k < K; ++k) cn[k] = -1;
    if (st->status[u] != ACTIVE) continue;
    int64_t q[KP_MAX_DIMS], bu[KP_MAX_DIMS];
    unit_req(st, u, q);
    int64_t cs[KP_MAX_CAND];
    uint32_t ck[KP_MAX_CAND];
    int nc = 0;
    for (int32_t n = 0; n < N; ++n) {
      node_used(st, st->used, n, bu);
      int64_t s = score_at(st, u, q, n, bu);
      if (s < 0) continue;
      uint32_t k = tie_key(st, u, n);
      int pos = nc;
      while (pos > 0 && (cs[pos - 1] < s || (cs[pos - 1] == s && ck[pos - 1] > k))) --pos;
      if (pos >= K) continue;
      for (int i = (nc < K ? nc : K - 1); i > pos; --i) {
        cn[i] = cn[i - 1]; cs[i] = cs[i - 1]; ck[i] = ck[i - 1];
      }
      cn[pos] = n; cs[pos] = s; ck[pos] = k;
      if (nc < K) ++nc;
    }
  }
  return KP_OK;
}

/* ---- §2.5 passes ---------------------------------------------------------- */
typedef struct {
  int32_t unit, node, count, member_off;
  int32_t score; /* S(q | node, pass-start usage) */
} prop_t;

static int cmp_prop(const void *a, const void *b) {
  const prop_t *x = (const prop_t *)a, *y = (const prop_t *)b;
  if (x->node != y->node) return x->node < y->node ? -1 : 1;
  if (x->unit != y->unit) return x->unit < y->unit ? -1 : 1;
  return x->member_off < y->member_off ? -1 : (x->member_off > y->member_off);
}

/* Plan unit u against usage `cur` (= cap - remaining): its members one at a
   time onto the candidate maximising S(q | c, cur_c + planned_c*q) minus
   w_spread x (members already planned into c's topo domain); ties -> earlier
   candidate. Returns #proposals (in candidate order, members consecutive),
   0 if some member fits no candidate. */
static int plan_unit(const kpo_state *st, int32_t u, const int32_t *cn,
                     const int64_t *cur, prop_t *out) {
  const int K = st->p.n_cand, D = st->D;
  int64_t q[KP_MAX_DIMS], bu[KP_MAX_DIMS];
  unit_req(st, u, q);
  int64_t planned[KP_MAX_CAND] = {0};
  for (int m = 0; m < st->size[u]; ++m) {
    int best = -1;
    int64_t best_s = 0;
    for (int c = 0; c < K && cn[c] >= 0; ++c) {
      node_used(st, cur, cn[c], bu);
      for (int d = 0; d < D; ++d) bu[d] += planned[c] * q[d];
      int64_t s = score_at(st, u, q, cn[c], bu);
      if (s < 0) continue;
      int64_t dom = 0;
      for (int c2 = 0; c2 < K && cn[c2] >= 0; ++c2)
        if (st->topo[cn[c2]] == st->topo[cn[c]]) dom += planned[c2];
      s -= (int64_t)st->p.w_spread * dom;
      if (best < 0 || s > best_s) { best = c; best_s = s; }
    }
    if (best < 0) return 0;
    planned[best]++;
  }
  int np = 0, off = 0;
  for (int c = 0; c < K && cn[c] >= 0; ++c) {
    if (!planned[c]) continue;
    node_used(st, cur, cn[c], bu);
    out[np].unit = u; out[np].node = cn[c]; out[np].count = (int32_t)planned[c];
    out[np].member_off = off; out[np].score = (int32_t)score_at(st, u, q, cn[c], bu);
    off += (int32_t)planned[c];
    ++np;
  }
  return np;
}

int32_t kpo_round_run(kpo_state *st, const int32_t *cand) {
  const int32_t N = st->N, D = st->D, U = st->U, K = st->p.n_cand;
  uint8_t *open, *ok, *gang_bad;
  prop_t *props;
  XALLOC(open, U, uint8_t); XALLOC(props, (size_t)U * K, prop_t);
  XALLOC(ok, (size_t)U * K, uint8_t); XALLOC(gang_bad, U, uint8_t);
  int32_t active0 = 0;
  for (int32_t u = 0; u < U; ++u) {
    open[u] = 0;
    if (st->status[u] != ACTIVE) continue;
    ++active0;
    if (cand[(size_t)u * K] < 0) st->status[u] = NO_FIT; /* no node fits one member */
    else open[u] = 1;
  }
  st->pairs += (int64_t)active0 * N;

  const char *trace_env = getenv("KPO_TRACE"); /* KPO_TRACE=1: per-round counts on stderr */
  int32_t passes0 = st->passes;
#ifdef KPO_ANALYSIS
  /* analysis build only (make -C oracle analysis, tools/): KPO_TRACE=2/3
     per-pass and accept-row statistics; KPO_DUMP=path (tools/accept_sim.py):
     per round the candidates, per pass the proposals with their first-fit
     outcome, appended as int32 */
  const int trace = trace_env ? (atoi(trace_env) > 2 ? 3 : atoi(trace_env) > 1 ? 2 : 1) : 0;
  FILE *dump = getenv("KPO_DUMP") ? fopen(getenv("KPO_DUMP"), "ab") : NULL;
  if (dump) {
    int32_t h[4] = {-1, st->rounds, U, K};
    fwrite(h, sizeof h, 1, dump);
    fwrite(cand, sizeof(int32_t), (size_t)U * K, dump);
  }
  int32_t *chg_pass = NULL; /* last pass that changed each node's usage */
  if (trace >= 2) {
    chg_pass = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
    for (int32_t n = 0; chg_pass && n < N; ++n) chg_pass[n] = -2;
  }
#else
  const int trace = trace_env && atoi(trace_env) > 0 ? 1 : 0;
#endif
  for (int pass = 0; pass < st->p.max_passes; ++pass) {
    /* proposals of every open unit, planned against the current usage */
    int32_t np = 0;
    for (int32_t u = 0; u < U; ++u) {
      if (!open[u]) continue;
      int k = plan_unit(st, u, cand + (size_t)u * K, st->used, props + np);
      if (k == 0) {
        open[u] = 0; /* closed for this round */
        if (pass == 0) st->status[u] = NO_FIT; /* gang does not fit its top-K */
      }
      np += k;
    }
    if (np == 0) break;
    st->passes++;
    qsort(props, np, sizeof *props, cmp_prop);
#ifdef KPO_ANALYSIS
    if (trace > 1) { /* KPO_TRACE=2: per-pass open units, proposals, bid nodes */
      int32_t nopen = 0, nodes = 0, dirty = 0, nchg = 0;
      for (int32_t u = 0; u < U; ++u) nopen += open[u];
      for (int32_t k = 0; k < np; ++k) nodes += k == 0 || props[k].node != props[k - 1].node;
      if (chg_pass) { /* open units with a candidate whose usage the previous pass changed */
        for (int32_t n = 0; n < N; ++n) nchg += chg_pass[n] == pass - 1;
        for (int32_t u = 0; u < U; ++u) {
          if (!open[u]) continue;
          int d = pass == 0;
          for (int k = 0; k < K && !d && cand[(size_t)u * K + k] >= 0; ++k)
            d = chg_pass[cand[(size_t)u * K + k]] == pass - 1;
          dirty += d;
        }
      }
      fprintf(stderr, "kpo pass %d.%d open %d props %d nodes %d changed %d dirty %d\n", st->rounds, pass,
              nopen, np, nodes, nchg, dirty);
    }
#endif
    /* per node, in unit rank order: first-fit against the remaining capacity */
    int64_t rem[KP_MAX_DIMS];
#ifdef KPO_ANALYSIS
    int32_t tr_maxrow = 0, tr_maxlast = 0, tr_maxsuf = 0; /* KPO_TRACE=3 */
#endif
    for (int32_t i = 0; i < np;) {
      int32_t node = props[i].node, e = i;
      while (e < np && props[e].node == node) ++e;
      for (int d = 0; d < D; ++d)
        rem[d] = st->cap[(int64_t)d * N + node] - st->used[(int64_t)d * N + node];
      for (int32_t k = i; k < e; ++k) {
        int64_t q[KP_MAX_DIMS];
        unit_req(st, props[k].unit, q);
        int fits = 1;
        for (int d = 0; d < D; ++d)
          if ((int64_t)props[k].count * q[d] > rem[d]) fits = 0;
        ok[k] = (uint8_t)fits;
        if (fits)
          for (int d = 0; d < D; ++d) rem[d] -= (int64_t)props[k].count * q[d];
      }
#ifdef KPO_ANALYSIS
      if (trace > 2) {
        /* bids of the row; index of its last accepted bid; bids walked until the
           remaining capacity is below the smallest later request in some dim */
        int32_t last = -1, suf = e - i;
        for (int32_t k = i; k < e; ++k) if (ok[k]) last = k - i;
        int64_t r2[KP_MAX_DIMS];
        for (int d = 0; d < D; ++d) r2[d] = st->cap[(int64_t)d * N + node] - st->used[(int64_t)d * N + node];
        for (int32_t k = i; k < e; ++k) {
          int64_t q[KP_MAX_DIMS];
          unit_req(st, props[k].unit, q);
          if (ok[k]) for (int d = 0; d < D; ++d) r2[d] -= (int64_t)props[k].count * q[d];
          int stop = 0;
          for (int d = 0; d < D && !stop; ++d) {
            int64_t mn = INT64_MAX;
            for (int32_t k2 = k + 1; k2 < e; ++k2) {
              int64_t q2[KP_MAX_DIMS];
              unit_req(st, props[k2].unit, q2);
              if (q2[d] < mn) mn = q2[d];
            }
            if (k + 1 < e && r2[d] < mn) stop = 1;
          }
          if (stop) { suf = k + 1 - i; break; }
        }
        if (e - i > tr_maxrow) tr_maxrow = e - i;
        if (last + 1 > tr_maxlast) tr_maxlast = last + 1;
        if (suf > tr_maxsuf) tr_maxsuf = suf;
      }
#endif
      i = e;
    }
#ifdef KPO_ANALYSIS
    if (trace > 2)
      fprintf(stderr, "kpo accept %d.%d maxrow %d maxlast %d maxsuf %d\n", st->rounds, pass, tr_maxrow,
              tr_maxlast, tr_maxsuf);
    if (dump) {
      int32_t h[4] = {-2, pass, np, 0};
      fwrite(h, sizeof h, 1, dump);
      for (int32_t k = 0; k < np; ++k) {
        int32_t r[4] = {props[k].unit, props[k].node, props[k].count, ok[k]};
        fwrite(r, sizeof r, 1, dump);
      }
    }
#endif
    /* all-or-nothing: a unit is placed iff every proposal was accepted */
    for (int32_t k = 0; k < np; ++k) gang_bad[props[k].unit] = 0;
    for (int32_t k = 0; k < np; ++k)
      if (!ok[k]) gang_bad[props[k].unit] = 1;
    for (int32_t k = 0; k < np; ++k) {
      const int32_t u = props[k].unit;
      if (gang_bad[u]) continue;
      int64_t q[KP_MAX_DIMS];
      unit_req(st, u, q);
      for (int d = 0; d < D; ++d)
        st->used[(int64_t)d * N + props[k].node] += (int64_t)props[k].count * q[d];
#ifdef KPO_ANALYSIS
      if (chg_pass) chg_pass[props[k].node] = pass;
#endif
      for (int32_t m = 0; m < props[k].count; ++m) {
        st->job_node[st->leader[u] + props[k].member_off + m] = props[k].node;
        st->job_score[st->leader[u] + props[k].member_off + m] = props[k].score;
      }
      st->status[u] = PLACED;
      open[u] = 0;
    }
  }
  if (trace)
    fprintf(stderr, "kpo round %d active %d passes %d\n", st->rounds, active0, st->passes - passes0);
  st->rounds++;
#ifdef KPO_ANALYSIS
  if (dump) fclose(dump);
  free(chg_pass);
#endif
  free(open); free(props); free(ok); free(gang_bad);
  return kpo_state_active(st);
}

int kpo_state_result(const kpo_state *st, kp_result *r) {
  const int32_t N = st->N, D = st->D;
  int32_t placed = 0;
  for (int32_t u = 0; u < st->U; ++u) {
    int32_t code = st->status[u] == PLACED ? KP_JOB_PLACED
                 : st->status[u] == NO_FIT ? KP_JOB_NO_FIT : KP_JOB_ROUND_LIMIT;
    if (code == KP_JOB_PLACED) placed += st->size[u];
    for (int32_t m = 0; m < st->size[u]; ++m) {
      int32_t j = st->leader[u] + m;
      if (r->node_of_job) r->node_of_job[j] = code == KP_JOB_PLACED ? st->job_node[j] : -1;
      if (r->score_of_job) r->score_of_job[j] = code == KP_JOB_PLACED ? st->job_score[j] : KP_SCORE_NONE;
      if (r->status_of_job) r->status_of_job[j] = code;
    }
  }
  if (r->used_out) memcpy(r->used_out, st->used, (size_t)D * N * sizeof(int64_t));
  r->rounds = st->rounds;
  r->passes = st->passes;
  r->placed_jobs = placed;
  r->unplaced_jobs = st->J - placed;
  r->units = st->U;
  r->pairs_scored = st->pairs;
  return KP_OK;
}

/* ---- §2.6 driver ---------------------------------------------------------- */
int kpo_place(const kp_snapshot *s, const kp_params *p, kp_result *r, int nthreads) {
  kpo_state *st;
  int rc = kpo_state_new(s, p, &st);
  if (rc) return rc;
  int32_t *cand;
  XALLOC(cand, (size_t)st->U * p->n_cand, int32_t);
  if (!cand) { kpo_state_free(st); return KP_ENOMEM; }
  while (kpo_state_active(st) > 0) {
    if (p->max_rounds > 0 && st->rounds >= p->max_rounds) break;
    kpo_round_candidates(st, 0, st->U, cand, nthreads);
    kpo_round_run(st, cand);
  }
  rc = kpo_state_result(st, r);
  free(cand);
  kpo_state_free(st);
  return rc;
}

/* ---- §2.3 filter + score matrix (per job row, round-start usage) ---------- */
int kpo_score(const kp_snapshot *s, const kp_params *p, int32_t job_lo,
              int32_t job_hi, int32_t *score, uint64_t *mask) {
  kpo_state *st;
  kp_snapshot s2 = *s;
  s2.gang_id = NULL; s2.gang_size = NULL; s2.prio = NULL; /* per-job rows */
  if (job_lo < 0 || job_hi > s->J || job_lo > job_hi) return KP_EINVAL;
  int rc = kpo_state_new(&s2, p, &st);
  if (rc) return rc;
  const int32_t N = st->N, D = st->D, words = (N + 63) / 64;
  for (int32_t j = job_lo; j < job_hi; ++j) {
    int64_t q[KP_MAX_DIMS], bu[KP_MAX_DIMS];
    for (int d = 0; d < D; ++d) q[d] = s->req[(int64_t)d * s->J + j];
    int64_t row = j - job_lo;
    if (mask) memset(mask + row * words, 0, (size_t)words * sizeof(uint64_t));
    for (int32_t n = 0; n < N; ++n) {
      node_used(st, st->used, n, bu);
      int64_t sc = score_at(st, j, q, n, bu); /* unit j = job j: no gangs/prio */
      if (score) score[row * N + n] = sc < 0 ? KP_SCORE_INFEASIBLE : (int32_t)sc;
      if (mask && sc >= 0) mask[row * words + n / 64] |= (uint64_t)1 << (n % 64);
    }
  }
  kpo_state_free(st);
  return KP_OK;
}

/* ---- §2.9 preemption candidates (BASELINE config #4) ----------------------
 * The victim pool is the running jobs of the snapshot. For a NO_FIT singleton
 * unit of priority p and request q, on node n: V = running jobs on n with
 * priority < p in (priority desc, running index asc) order — the order in which
 * kube-scheduler's selectVictimsOnNode tries to reprieve them; n qualifies iff
 * q <= free + sum(V) in every dim (free = cap - post-solve used); walking V,
 * a job is spared if q still fits without its resources, else it is a victim.
 * Best node: fewest victims, then lowest sum of victim priorities, then
 * lowest node index. */
typedef struct {
  int32_t node, idx, prio;
} run_ref;

static int cmp_run(const void *a, const void *b) {
  const run_ref *x = (const run_ref *)a, *y = (const run_ref *)b;
  if (x->node != y->node) return x->node < y->node ? -1 : 1;
  if (x->prio != y->prio) return x->prio > y->prio ? -1 : 1; /* prio desc */
  return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

int kpo_check_running(const kp_snapshot *s, int32_t R, const int32_t *node,
                      const int64_t *req, const int32_t *prio) {
  if (R < 0 || (R > 0 && (!node || !req || !prio))) return KP_EINVAL;
  const int32_t N = s->N, D = s->D;
  int64_t *sum = (int64_t *)calloc((size_t)D * N + 1, sizeof(int64_t));
  if (!sum) return KP_ENOMEM;
  int rc = KP_OK;
  for (int32_t r = 0; r < R && !rc; ++r) {
    const int32_t n = node[r];
    if (n < 0 || n >= N) { rc = KP_EINVAL; break; }
    for (int d = 0; d < D && !rc; ++d) {
      const int64_t q = req[(int64_t)d * R + r];
      const int64_t u = s->used ? s->used[(int64_t)d * N + n] : 0;
      if (q < 0 || q > KP_MAX_VALUE) rc = KP_EINVAL;
      else if ((sum[(int64_t)d * N + n] += q) > u) rc = KP_EINVAL; /* stays <= 2^57 */
    }
  }
  free(sum);
  return rc;
}

int kpo_preempt(const kp_snapshot *s, const kp_params *p, int32_t R, const int32_t *node,
                const int64_t *req, const int32_t *prio, kp_result *res,
                kp_preemption *pr, int nthreads) {
  kpo_state *st;
  int rc = kpo_state_new(s, p, &st);
  if (rc) return rc;
  if ((rc = kpo_check_running(s, R, node, req, prio))) { kpo_state_free(st); return rc; }
  int32_t *cand;
  XALLOC(cand, (size_t)st->U * p->n_cand, int32_t);
  run_ref *rr;
  int32_t *off;
  XALLOC(rr, R, run_ref);
  off = (int32_t *)calloc((size_t)s->N + 2, sizeof(int32_t));
  if (!cand || !rr || !off) { free(cand); free(rr); free(off); kpo_state_free(st); return KP_ENOMEM; }
  while (kpo_state_active(st) > 0) { /* the placement itself, as kpo_place */
    if (p->max_rounds > 0 && st->rounds >= p->max_rounds) break;
    kpo_round_candidates(st, 0, st->U, cand, nthreads);
    kpo_round_run(st, cand);
  }
  if (res) kpo_state_result(st, res);
  const int32_t N = st->N, D = st->D, J = st->J;
  for (int32_t r = 0; r < R; ++r) { rr[r].node = node[r]; rr[r].idx = r; rr[r].prio = prio[r]; }
  qsort(rr, R, sizeof *rr, cmp_run);
  for (int32_t r = 0; r < R; ++r) off[rr[r].node + 1]++;
  for (int32_t n = 0; n < N; ++n) off[n + 1] += off[n];
  for (int32_t j = 0; j < J; ++j) {
    if (pr->node_of_job) pr->node_of_job[j] = -1;
    if (pr->victims_of_job) pr->victims_of_job[j] = 0;
    if (pr->cost_of_job) pr->cost_of_job[j] = 0;
  }
  int32_t npre = 0, nnom = 0;
  (void)nthreads;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 8) reduction(+ : npre, nnom) \
    num_threads(nthreads > 0 ? nthreads : 1)
#endif
  for (int32_t u = 0; u < st->U; ++u) {
    if (st->status[u] != NO_FIT || st->size[u] != 1) continue;
    ++npre;
    int64_t q[KP_MAX_DIMS], avail[KP_MAX_DIMS];
    unit_req(st, u, q);
    const int32_t pu = st->prio[u];
    int32_t best_n = -1, best_c = 0;
    int64_t best_cost = 0;
    for (int32_t n = 0; n < N; ++n) {
      int32_t f = off[n];
      const int32_t e1 = off[n + 1];
      while (f < e1 && rr[f].prio >= pu) ++f; /* V = [f, e1) */
      int ok = 1;
      for (int d = 0; d < D; ++d) {
        avail[d] = st->cap[(int64_t)d * N + n] - st->used[(int64_t)d * N + n];
        for (int32_t e = f; e < e1; ++e) avail[d] += req[(int64_t)d * R + rr[e].idx];
        if (q[d] > avail[d]) ok = 0;
      }
      if (!ok) continue;
      int32_t cnt = 0;
      int64_t cost = 0;
      for (int32_t e = f; e < e1; ++e) {
        int spare = 1;
        for (int d = 0; d < D; ++d)
          if (q[d] > avail[d] - req[(int64_t)d * R + rr[e].idx]) spare = 0;
        if (spare) {
          for (int d = 0; d < D; ++d) avail[d] -= req[(int64_t)d * R + rr[e].idx];
        } else {
          ++cnt;
          cost += rr[e].prio;
        }
      }
      if (best_n < 0 || cnt < best_c || (cnt == best_c && cost < best_cost)) {
        best_n = n; best_c = cnt; best_cost = cost;
      }
    }
    if (best_n >= 0) ++nnom;
    const int32_t j = st->leader[u];
    if (pr->node_of_job) pr->node_of_job[j] = best_n;
    if (pr->victims_of_job) pr->victims_of_job[j] = best_n >= 0 ? best_c : 0;
    if (pr->cost_of_job) pr->cost_of_job[j] = best_n >= 0 ? best_cost : 0;
  }
  pr->preemptors = npre;
  pr->nominated = nnom;
  pr->pairs_scored = (int64_t)npre * N;
  free(cand); free(rr); free(off);
  kpo_state_free(st);
  return KP_OK;
}
