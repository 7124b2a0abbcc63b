// kp_kernels.hip — gfx950 (CDNA4) kernels of the kplace placement engine.
//
// Every kernel implements one step of DESIGN.md §2 bit-exactly (integer
// arithmetic only; the CPU restatement is oracle/kp_oracle.c). The path is
// integer compare/select/reduce, so no MFMA: what matters is coalesced HBM
// streaming (score matrix stores, row re-reads), keeping the node tile in
// VGPRs across job rows, and 64-lane wave ballots / shuffles for the masks,
// argmax and prefix sums.
#include <hip/hip_runtime.h>

#include <cstring>

#include <rocprim/rocprim.hpp>

#include "kp_internal.hpp"

namespace kp {
namespace {

constexpr int kWave = 64;

// ---------------------------------------------------------------------------
// wave helpers (64-lane)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  uint32_t lo = __shfl_xor((uint32_t)v, m, kWave);
  uint32_t hi = __shfl_xor((uint32_t)(v >> 32), m, kWave);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int64_t shfl_up_i64(int64_t v, int d) {
  uint32_t lo = __shfl_up((uint32_t)(uint64_t)v, d, kWave);
  uint32_t hi = __shfl_up((uint32_t)((uint64_t)v >> 32), d, kWave);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t shfl_i64(int64_t v, int src) {
  uint32_t lo = __shfl((uint32_t)(uint64_t)v, src, kWave);
  uint32_t hi = __shfl((uint32_t)((uint64_t)v >> 32), src, kWave);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    uint64_t o = shfl_xor_u64(v, m);
    v = o > v ? o : v;
  }
  return v;
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    int64_t o = (int64_t)shfl_xor_u64((uint64_t)v, m);
    v = o > v ? o : v;
  }
  return v;
}
// inclusive prefix sum over the 64 lanes (Hillis-Steele, 6 steps)
__device__ __forceinline__ int64_t wave_incl_scan_i64(int64_t v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    int64_t o = shfl_up_i64(v, d);
    if (l >= d) v += o;
  }
  return v;
}

// ---------------------------------------------------------------------------
// §2.3 score of one more copy of q on a node with usage `used`, 64-bit exact.
// Returns -1 when it does not fit.
// ---------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ int64_t score_at(const ScoreParams &sp,
                                            const int64_t (&q)[D],
                                            const int64_t (&cap)[D],
                                            const int64_t (&used)[D],
                                            const uint64_t (&R)[D], int64_t base) {
  int64_t acc = 0;
  bool fits = true;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    fits &= q[d] <= cap[d] - used[d];
    uint64_t u = (uint64_t)(used[d] + q[d]);
    uint64_t util = (u * R[d]) >> 32;
    acc += (int64_t)sp.w[d] * (int64_t)util;
  }
  int64_t s = sp.most_allocated ? acc : base - acc;
  if (sp.gpu_dim >= 0) {
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (d == sp.gpu_dim && q[d] > 0 && cap[d] - used[d] - q[d] == 0) s += sp.w_gpu_fit;
  }
  return fits ? s : -1;
}

// ---------------------------------------------------------------------------
// node prep: R = floor(S*2^32/cap), LeastAllocated base
// ---------------------------------------------------------------------------
__global__ void k_prep_nodes(const int64_t *__restrict__ cap, uint64_t *__restrict__ R,
                             int64_t *__restrict__ base, int32_t N, int32_t D, int32_t S,
                             int32_t least, ScoreParams sp) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  int64_t b = 0;
  for (int d = 0; d < D; ++d) {
    int64_t c = cap[(int64_t)d * N + n];
    R[(int64_t)d * N + n] = c > 0 ? (((uint64_t)S) << 32) / (uint64_t)c : 0;
    if (c > 0) b += (int64_t)sp.w[d] * S;
  }
  base[n] = least ? b : 0;
}

// ---------------------------------------------------------------------------
// filter + score (materialised). One 256-thread workgroup owns a tile of
// 4 waves x 64 lanes x NPL nodes; the tile's cap/used/R stay in VGPRs while
// the workgroup streams `rows_per_block` job rows past it: per row the
// request is wave-uniform (scalar loads), each lane stores NPL int32 scores
// (coalesced 256-B wave stores) and the wave ballots the feasibility bits
// straight into the row's mask words.
// Row stride of score/mask = Ns = round_up(N, 64); padding is infeasible.
// ---------------------------------------------------------------------------
template <int D, int NPL>
__global__ __launch_bounds__(256) void k_score(ScoreParams sp,
                                               const int64_t *__restrict__ cap,
                                               const int64_t *__restrict__ used,
                                               const uint64_t *__restrict__ R,
                                               const int64_t *__restrict__ base,
                                               const int64_t *__restrict__ q, int32_t qstride,
                                               const int32_t *__restrict__ rows_unit,
                                               int32_t rows, int32_t rows_per_block,
                                               int32_t *__restrict__ score,
                                               uint64_t *__restrict__ mask, int32_t Ns) {
  const int N = sp.N;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile0 = blockIdx.x * (256 * NPL) + wave * (64 * NPL);
  int64_t c_[NPL][D], u_[NPL][D], b_[NPL];
  uint64_t r_[NPL][D];
  bool v_[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int n = tile0 + k * 64 + lane;
    v_[k] = n < N;
    const int nn = v_[k] ? n : 0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      c_[k][d] = cap[(int64_t)d * N + nn];
      u_[k][d] = used[(int64_t)d * N + nn];
      r_[k][d] = R[(int64_t)d * N + nn];
    }
    b_[k] = base[nn];
  }
  const int words = Ns >> 6;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  if (tile0 >= Ns) return;
  for (int r = r0; r < r1; ++r) {
    const int32_t unit = rows_unit[r];
    int64_t qq[D];
#pragma unroll
    for (int d = 0; d < D; ++d) qq[d] = q[(int64_t)d * qstride + unit];
    int32_t *srow = score + (int64_t)r * Ns;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int n = tile0 + k * 64 + lane;
      int64_t s = score_at<D>(sp, qq, c_[k], u_[k], r_[k], b_[k]);
      if (!v_[k]) s = -1;
      const bool feas = s >= 0;
      if (score && n < Ns) srow[n] = feas ? (int32_t)s : KP_SCORE_INFEASIBLE;
      const uint64_t bits = __ballot(feas);
      if (mask && lane == 0 && (tile0 + k * 64) < Ns)
        mask[(int64_t)r * words + ((tile0 + k * 64) >> 6)] = bits;
    }
  }
}

// ---------------------------------------------------------------------------
// top-K select: one wave per score-matrix row. Each lane keeps its own
// descending top-KC list of packed keys (valid bit | score | ~tie key) over a
// strided slice of the row (16-B loads: 4 nodes per lane per step), then the
// wave merges the 64 lists KC times with a butterfly max. Exact: every global
// top-K entry is in its lane's top-K.
// ---------------------------------------------------------------------------
template <int KC>
__device__ __forceinline__ void topk_insert(uint64_t (&k)[KC], uint64_t x) {
  if (x <= k[KC - 1]) return;
  k[KC - 1] = x;
#pragma unroll
  for (int i = KC - 1; i > 0; --i) {
    uint64_t a = k[i - 1], b = k[i];
    bool sw = b > a;
    k[i - 1] = sw ? b : a;
    k[i] = sw ? a : b;
  }
}

__device__ __forceinline__ uint64_t pack_key(int32_t s, uint32_t tk) {
  return (1ull << 63) | ((uint64_t)(uint32_t)s << 32) | (uint64_t)(~tk);
}

template <int KC>
__global__ __launch_bounds__(256) void k_select(ScoreParams sp,
                                                const int32_t *__restrict__ score, int32_t Ns,
                                                const int32_t *__restrict__ rows_unit,
                                                const uint32_t *__restrict__ salt,
                                                int32_t rows, int32_t *__restrict__ cand) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int K = sp.n_cand;
  const int32_t unit = rows_unit[row];
  const uint32_t sl = sp.tie_rotated ? salt[unit] : 0u;
  const uint32_t mul = sp.tie_rotated ? kTieMul : 1u;
  uint64_t k[KC];
#pragma unroll
  for (int i = 0; i < KC; ++i) k[i] = 0;
  const int4 *row4 = reinterpret_cast<const int4 *>(score + (int64_t)row * Ns);
  const int n4 = Ns >> 2;
  for (int i = lane; i < n4; i += 64) {
    const int4 v = row4[i];
    const int n = i * 4;
    if (v.x >= 0) topk_insert<KC>(k, pack_key(v.x, (uint32_t)(n + 0) * mul + sl));
    if (v.y >= 0) topk_insert<KC>(k, pack_key(v.y, (uint32_t)(n + 1) * mul + sl));
    if (v.z >= 0) topk_insert<KC>(k, pack_key(v.z, (uint32_t)(n + 2) * mul + sl));
    if (v.w >= 0) topk_insert<KC>(k, pack_key(v.w, (uint32_t)(n + 3) * mul + sl));
  }
  const uint32_t inv = sp.tie_rotated ? kTieMulInv : 1u;
  for (int it = 0; it < K; ++it) {
    const uint64_t m = wave_max_u64(k[0]);
    if (lane == 0) {
      int32_t node = -1;
      if (m != 0) {
        const uint32_t tk = ~(uint32_t)m;
        node = (int32_t)((tk - sl) * inv);
      }
      cand[(int64_t)row * K + it] = node;
    }
    if (m != 0 && k[0] == m) {  // unique keys: exactly one lane pops
#pragma unroll
      for (int i = 0; i < KC - 1; ++i) k[i] = k[i + 1];
      k[KC - 1] = 0;
    }
  }
}

// ---------------------------------------------------------------------------
// round bookkeeping
// ---------------------------------------------------------------------------
__global__ void k_open_init(const int32_t *__restrict__ act, const int32_t *__restrict__ cand,
                            int32_t A, int32_t K, uint8_t *__restrict__ open,
                            int32_t *__restrict__ status) {
  int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= A) return;
  const bool has = cand[(int64_t)a * K] >= 0;
  open[a] = has ? 1 : 0;
  if (!has) status[act[a]] = kNoFit;
}

__global__ void k_reset_units(int32_t *__restrict__ status, int32_t U,
                              int32_t *__restrict__ job_node, int32_t *__restrict__ job_score,
                              int32_t J) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < U) status[i] = kActive;
  if (i < J) {
    job_node[i] = -1;
    job_score[i] = KP_SCORE_NONE;
  }
}

__global__ void k_flag_active(const int32_t *__restrict__ status, int32_t lo, int32_t hi,
                              int32_t *__restrict__ flag) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < hi - lo) flag[i] = status[lo + i] == kActive ? 1 : 0;
}

__global__ void k_finalize(const int32_t *__restrict__ status, const int32_t *__restrict__ leader,
                           const int32_t *__restrict__ size, int32_t U,
                           int32_t *__restrict__ job_node, int32_t *__restrict__ job_score,
                           int32_t *__restrict__ job_status) {
  int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  const int32_t st = status[u];
  const int32_t code = st == kPlaced ? KP_JOB_PLACED : st == kNoFit ? KP_JOB_NO_FIT
                                                                     : KP_JOB_ROUND_LIMIT;
  for (int m = 0; m < size[u]; ++m) {
    const int j = leader[u] + m;
    job_status[j] = code;
    if (code != KP_JOB_PLACED) {
      job_node[j] = -1;
      job_score[j] = KP_SCORE_NONE;
    }
  }
}

// ---------------------------------------------------------------------------
// §2.5 plan: one wave per active slot, lane c = candidate c. Members are
// planned one at a time: every lane scores its candidate with the members it
// already holds, subtracts the spread penalty of its topo domain, and the
// wave picks (max value, lowest lane).
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void k_plan(ScoreParams sp, int32_t A, int32_t U, int32_t pass,
                                              const int32_t *__restrict__ act,
                                              const int32_t *__restrict__ cand,
                                              uint8_t *__restrict__ open,
                                              int32_t *__restrict__ status,
                                              uint8_t *__restrict__ unit_bad,
                                              const int64_t *__restrict__ cap,
                                              const int64_t *__restrict__ used,
                                              const uint64_t *__restrict__ R,
                                              const int64_t *__restrict__ base,
                                              const int32_t *__restrict__ topo,
                                              const int64_t *__restrict__ q,
                                              const int32_t *__restrict__ size,
                                              int32_t *__restrict__ st_node,
                                              int32_t *__restrict__ st_count,
                                              int32_t *__restrict__ st_off,
                                              int32_t *__restrict__ st_score,
                                              int32_t *__restrict__ st_n) {
  const int lane = threadIdx.x & 63;
  const int a = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (a >= A) return;
  if (!open[a]) {
    if (lane == 0) st_n[a] = 0;
    return;
  }
  const int K = sp.n_cand, N = sp.N;
  const int32_t u = act[a];
  const int32_t sz = size[u];
  int64_t qq[D];
#pragma unroll
  for (int d = 0; d < D; ++d) qq[d] = q[(int64_t)d * U + u];
  const int32_t node = lane < K ? cand[(int64_t)a * K + lane] : -1;
  const bool valid = node >= 0;
  const int nn = valid ? node : 0;
  int64_t c_[D], u0[D];
  uint64_t r_[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    c_[d] = cap[(int64_t)d * N + nn];
    u0[d] = used[(int64_t)d * N + nn];
    r_[d] = R[(int64_t)d * N + nn];
  }
  const int64_t b = base[nn];
  const int32_t tp = topo[nn];
  int32_t planned = 0, dom = 0, s0 = -1;
  bool fail = false;
  for (int m = 0; m < sz; ++m) {
    int64_t uu[D];
#pragma unroll
    for (int d = 0; d < D; ++d) uu[d] = u0[d] + (int64_t)planned * qq[d];
    int64_t s = valid ? score_at<D>(sp, qq, c_, uu, r_, b) : -1;
    if (m == 0) s0 = (int32_t)s;
    const bool feas = s >= 0;
    const int64_t val = feas ? s - (int64_t)sp.w_spread * dom : INT64_MIN;
    const uint64_t fm = __ballot(feas);
    if (fm == 0) {
      fail = true;
      break;
    }
    const int64_t best = wave_max_i64(val);
    const uint64_t wm = __ballot(feas && val == best);
    const int win = __ffsll((unsigned long long)wm) - 1;
    const int32_t wtp = __shfl(tp, win, kWave);
    planned += lane == win ? 1 : 0;
    dom += (valid && tp == wtp) ? 1 : 0;
  }
  if (fail) {
    if (lane == 0) {
      st_n[a] = 0;
      open[a] = 0;
      if (pass == 0) status[u] = kNoFit;
    }
    return;
  }
  const bool has = planned > 0;
  const uint64_t hb = __ballot(has);
  const uint64_t lt = (1ull << lane) - 1ull;
  const int pos = __popcll(hb & lt);
  const int64_t incl = wave_incl_scan_i64((int64_t)planned);
  const int32_t off = (int32_t)(incl - planned);
  if (has) {
    const int64_t i = (int64_t)a * K + pos;
    st_node[i] = node;
    st_count[i] = planned;
    st_off[i] = off;
    st_score[i] = s0;
  }
  if (lane == 0) {
    st_n[a] = __popcll(hb);
    unit_bad[u] = 0;
  }
}

// compact the per-slot staging slabs into rank-ordered proposal arrays
__global__ void k_scatter_props(int32_t A, int32_t K, const int32_t *__restrict__ st_n,
                                const int32_t *__restrict__ st_pos,
                                const int32_t *__restrict__ st_node,
                                const int32_t *__restrict__ st_count,
                                const int32_t *__restrict__ st_off,
                                const int32_t *__restrict__ st_score,
                                int32_t *__restrict__ p_slot, int32_t *__restrict__ p_node,
                                int32_t *__restrict__ p_count, int32_t *__restrict__ p_off,
                                int32_t *__restrict__ p_score, uint32_t *__restrict__ k_in,
                                uint32_t *__restrict__ v_in) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int a = (int)(t / K), k = (int)(t % K);
  if (a >= A || k >= st_n[a]) return;
  const int64_t src = (int64_t)a * K + k;
  const int32_t i = st_pos[a] + k;
  p_slot[i] = a;
  p_node[i] = st_node[src];
  p_count[i] = st_count[src];
  p_off[i] = st_off[src];
  p_score[i] = st_score[src];
  k_in[i] = (uint32_t)st_node[src];
  v_in[i] = (uint32_t)i;
}

__global__ void k_seg_bounds(int32_t P, const uint32_t *__restrict__ keys,
                             int32_t *__restrict__ seg_start, int32_t *__restrict__ seg_end) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const uint32_t k = keys[i];
  if (i == 0 || keys[i - 1] != k) seg_start[k] = i;
  if (i == P - 1 || keys[i + 1] != k) seg_end[k] = i + 1;
}

// ---------------------------------------------------------------------------
// §2.5 first-fit acceptance: one wave per node with proposals. Bidders are in
// unit rank order (stable sort by node of a rank-ordered array). Exact
// parallel first-fit on a 64-bidder window: lanes whose request no longer
// fits alone are rejected; among the rest the wave takes the longest prefix
// whose running sum fits and rejects the first lane that breaks it, then
// repeats on the remainder with the reduced capacity. Each iteration decides
// at least one lane, and every decision equals the sequential one.
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void k_accept(ScoreParams sp, int32_t U,
                                                const int32_t *__restrict__ seg_start,
                                                const int32_t *__restrict__ seg_end,
                                                const uint32_t *__restrict__ v_sorted,
                                                const int32_t *__restrict__ p_slot,
                                                const int32_t *__restrict__ p_count,
                                                const int32_t *__restrict__ act,
                                                const int64_t *__restrict__ q,
                                                const int64_t *__restrict__ cap,
                                                const int64_t *__restrict__ used,
                                                uint8_t *__restrict__ p_ok) {
  const int lane = threadIdx.x & 63;
  const int node = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int N = sp.N;
  if (node >= N) return;
  const int32_t s0 = seg_start[node];
  if (s0 < 0) return;
  const int32_t s1 = seg_end[node];
  int64_t rem[D];
#pragma unroll
  for (int d = 0; d < D; ++d) rem[d] = cap[(int64_t)d * N + node] - used[(int64_t)d * N + node];
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int base = s0; base < s1; base += 64) {
    const int i = base + lane;
    const bool valid = i < s1;
    uint32_t pi = 0;
    int64_t need[D];
    if (valid) {
      pi = v_sorted[i];
      const int32_t u = act[p_slot[pi]];
      const int64_t cnt = p_count[pi];
#pragma unroll
      for (int d = 0; d < D; ++d) need[d] = cnt * q[(int64_t)d * U + u];
    } else {
#pragma unroll
      for (int d = 0; d < D; ++d) need[d] = 0;
    }
    bool undecided = valid, accepted = false;
    while (__ballot(undecided) != 0) {
      bool fa = undecided;
#pragma unroll
      for (int d = 0; d < D; ++d) fa &= need[d] <= rem[d];
      undecided = fa;  // lanes that do not fit alone are rejected for good
      bool ok = fa;
      int64_t pre[D];
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int64_t x = fa ? need[d] : 0;
        pre[d] = wave_incl_scan_i64(x) - x;  // exclusive
        ok &= pre[d] + need[d] <= rem[d];
      }
      const uint64_t fail = __ballot(fa && !ok);
      if (fail == 0) {
        accepted |= fa;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          const int64_t tot = wave_incl_scan_i64(fa ? need[d] : 0);
          rem[d] -= shfl_i64(tot, 63);
        }
        undecided = false;
      } else {
        const int f = __ffsll((unsigned long long)fail) - 1;
        const bool take = fa && lane < f;
        accepted |= take;
#pragma unroll
        for (int d = 0; d < D; ++d) rem[d] -= shfl_i64(pre[d], f);
        undecided = fa && lane >= f;  // lane f is rejected on the next check
      }
    }
    if (valid) p_ok[pi] = accepted ? 1 : 0;
    (void)lt;
  }
}

__global__ void k_mark_bad(int32_t P, const uint8_t *__restrict__ p_ok,
                           const int32_t *__restrict__ p_slot, const int32_t *__restrict__ act,
                           uint8_t *__restrict__ unit_bad) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  if (!p_ok[i]) unit_bad[act[p_slot[i]]] = 1;
}

__global__ void k_commit(int32_t P, int32_t D, int32_t N, int32_t U,
                         const int32_t *__restrict__ p_slot, const int32_t *__restrict__ p_node,
                         const int32_t *__restrict__ p_count, const int32_t *__restrict__ p_off,
                         const int32_t *__restrict__ p_score, const int32_t *__restrict__ act,
                         const uint8_t *__restrict__ unit_bad, const int64_t *__restrict__ q,
                         const int32_t *__restrict__ leader, int64_t *__restrict__ used,
                         int32_t *__restrict__ status, uint8_t *__restrict__ open,
                         int32_t *__restrict__ job_node, int32_t *__restrict__ job_score) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const int32_t a = p_slot[i];
  const int32_t u = act[a];
  if (unit_bad[u]) return;
  const int32_t node = p_node[i], cnt = p_count[i];
  for (int d = 0; d < D; ++d)
    atomicAdd(reinterpret_cast<unsigned long long *>(&used[(int64_t)d * N + node]),
              (unsigned long long)((int64_t)cnt * q[(int64_t)d * U + u]));
  const int32_t j0 = leader[u] + p_off[i];
  for (int m = 0; m < cnt; ++m) {
    job_node[j0 + m] = node;
    job_score[j0 + m] = p_score[i];
  }
  status[u] = kPlaced;
  open[a] = 0;
}

__global__ void k_unpack(int32_t world, int32_t Umax, int32_t K,
                         const int32_t *__restrict__ counts, const int32_t *__restrict__ recv,
                         int32_t *__restrict__ act, int32_t *__restrict__ cand) {
  // one thread per (rank, local slot); destination = prefix of counts
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int r = (int)(t / Umax), i = (int)(t % Umax);
  if (r >= world || i >= counts[r]) return;
  int32_t dst = i;
  for (int k = 0; k < r; ++k) dst += counts[k];
  const int32_t *src = recv + ((int64_t)r * Umax + i) * (K + 1);
  act[dst] = src[0];
  for (int k = 0; k < K; ++k) cand[(int64_t)dst * K + k] = src[1 + k];
}

__global__ void k_pack(int32_t A, int32_t K, const int32_t *__restrict__ act,
                       const int32_t *__restrict__ cand, int32_t *__restrict__ send) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= A) return;
  int32_t *dst = send + t * (K + 1);
  dst[0] = act[t];
  for (int k = 0; k < K; ++k) dst[1 + k] = cand[t * K + k];
}

inline int blocks(int64_t n, int b) { return (int)((n + b - 1) / b); }

template <template <int> class F, typename... Args>
int dispatch_D(int D, Args &&...args) {
  switch (D) {
    case 1: return F<1>::run(args...);
    case 2: return F<2>::run(args...);
    case 3: return F<3>::run(args...);
    case 4: return F<4>::run(args...);
    case 5: return F<5>::run(args...);
    case 6: return F<6>::run(args...);
    case 7: return F<7>::run(args...);
    case 8: return F<8>::run(args...);
  }
  return KP_EINVAL;
}

}  // namespace

// ===========================================================================
// launchers
// ===========================================================================
int launch_prep_nodes(kp_ctx *c, int32_t S, int most_allocated, const int32_t *w) {
  ScoreParams sp{};
  for (int d = 0; d < KP_MAX_DIMS; ++d) sp.w[d] = w[d];
  if (c->N == 0) return KP_OK;
  hipLaunchKernelGGL(k_prep_nodes, dim3(blocks(c->N, 256)), dim3(256), 0, c->stream, c->d.cap,
                     c->d.R, c->d.base, c->N, c->D, S, most_allocated ? 0 : 1, sp);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

namespace {
template <int D>
struct ScoreL {
  static int run(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit, int32_t rows,
                 int32_t *score, uint64_t *mask, const int64_t *q, int32_t qstride) {
    constexpr int NPL = D <= 4 ? 2 : 1;
    const int Ns = (c->N + 63) & ~63;
    const int rpb = 32;
    dim3 grid(blocks(Ns, 256 * NPL), blocks(rows, rpb));
    hipLaunchKernelGGL((k_score<D, NPL>), grid, dim3(256), 0, c->stream, sp, c->d.cap,
                       c->d.used, c->d.R, c->d.base, q, qstride, rows_unit, rows, rpb, score,
                       mask, Ns);
    KP_HIP(hipGetLastError());
    return KP_OK;
  }
};
template <int D>
struct PlanL {
  static int run(kp_ctx *c, const ScoreParams &sp, int32_t A, int32_t pass) {
    hipLaunchKernelGGL((k_plan<D>), dim3(blocks(A, 4)), dim3(256), 0, c->stream, sp, A, c->U,
                       pass, c->d.act, c->d.cand, c->d.open, c->d.status, c->d.unit_bad,
                       c->d.cap, c->d.used, c->d.R, c->d.base, c->d.topo, c->d.q, c->d.size,
                       c->d.st_node, c->d.st_count, c->d.st_off, c->d.st_score, c->d.st_n);
    KP_HIP(hipGetLastError());
    return KP_OK;
  }
};
template <int D>
struct AcceptL {
  static int run(kp_ctx *c, const ScoreParams &sp, int32_t P) {
    (void)P;
    int32_t *seg_start = c->d.heads, *seg_end = c->d.heads + c->cap_N;
    hipLaunchKernelGGL((k_accept<D>), dim3(blocks(c->N, 4)), dim3(256), 0, c->stream, sp, c->U,
                       seg_start, seg_end, c->d.v_out, c->d.p_slot, c->d.p_count, c->d.act,
                       c->d.q, c->d.cap, c->d.used, c->d.p_ok);
    KP_HIP(hipGetLastError());
    return KP_OK;
  }
};
}  // namespace

int launch_score(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit, int32_t rows,
                 int32_t *score, uint64_t *mask, const int64_t *q, int32_t qstride) {
  if (rows <= 0 || c->N == 0) return KP_OK;
  return dispatch_D<ScoreL>(c->D, c, sp, rows_unit, rows, score, mask, q, qstride);
}

int launch_select(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit, int32_t rows,
                  const int32_t *score, int32_t *cand) {
  if (rows <= 0) return KP_OK;
  const int Ns = (c->N + 63) & ~63;
  dim3 grid(blocks(rows, 4)), blk(256);
  const int K = sp.n_cand;
  if (K <= 4)
    hipLaunchKernelGGL(k_select<4>, grid, blk, 0, c->stream, sp, score, Ns, rows_unit, c->d.salt, rows, cand);
  else if (K <= 8)
    hipLaunchKernelGGL(k_select<8>, grid, blk, 0, c->stream, sp, score, Ns, rows_unit, c->d.salt, rows, cand);
  else if (K <= 16)
    hipLaunchKernelGGL(k_select<16>, grid, blk, 0, c->stream, sp, score, Ns, rows_unit, c->d.salt, rows, cand);
  else
    hipLaunchKernelGGL(k_select<32>, grid, blk, 0, c->stream, sp, score, Ns, rows_unit, c->d.salt, rows, cand);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

int launch_open_init(kp_ctx *c, int32_t A, int32_t K) {
  if (A <= 0) return KP_OK;
  hipLaunchKernelGGL(k_open_init, dim3(blocks(A, 256)), dim3(256), 0, c->stream, c->d.act,
                     c->d.cand, A, K, c->d.open, c->d.status);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

int launch_plan(kp_ctx *c, const ScoreParams &sp, int32_t A, int32_t pass) {
  if (A <= 0) return KP_OK;
  return dispatch_D<PlanL>(c->D, c, sp, A, pass);
}

size_t rocprim_temp_bytes(int32_t max_items) {
  size_t a = 0, b = 0, s = 0;
  rocprim::radix_sort_pairs(nullptr, a, (uint32_t *)nullptr,
                                                (uint32_t *)nullptr, (uint32_t *)nullptr,
                                                (uint32_t *)nullptr, (size_t)max_items, 0u, 32u);
  rocprim::exclusive_scan(nullptr, b, (int32_t *)nullptr, (int32_t *)nullptr, 0,
                          (size_t)max_items + 1, rocprim::plus<int32_t>());
  rocprim::select(nullptr, s, rocprim::counting_iterator<int32_t>(0), (int32_t *)nullptr,
                  (int32_t *)nullptr, (int32_t *)nullptr, (size_t)max_items);
  size_t m = a > b ? a : b;
  return (m > s ? m : s) + 256;
}

// proposal compaction: scan of per-slot counts, host read of the total
int launch_compact(kp_ctx *c, int32_t A, int32_t K, int32_t *P_host) {
  *P_host = 0;
  if (A <= 0) return KP_OK;
  KP_HIP(hipMemsetAsync(c->d.st_n + A, 0, sizeof(int32_t), c->stream));
  size_t tb = c->d.temp_bytes;
  KP_HIP(rocprim::exclusive_scan(c->d.temp, tb, c->d.st_n, c->d.st_pos, 0, (size_t)A + 1,
                                 rocprim::plus<int32_t>(), c->stream));
  KP_HIP(hipMemcpyAsync(c->pinned, c->d.st_pos + A, sizeof(int32_t), hipMemcpyDeviceToHost,
                        c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  const int32_t P = c->pinned[0];
  *P_host = P;
  if (P == 0) return KP_OK;
  hipLaunchKernelGGL(k_scatter_props, dim3(blocks((int64_t)A * K, 256)), dim3(256), 0, c->stream,
                     A, K, c->d.st_n, c->d.st_pos, c->d.st_node, c->d.st_count, c->d.st_off,
                     c->d.st_score, c->d.p_slot, c->d.p_node, c->d.p_count, c->d.p_off,
                     c->d.p_score, c->d.k_in, c->d.v_in);
  KP_HIP(hipGetLastError());
  // stable radix sort by node keeps rank order inside each node's segment
  int bits = 1;
  while ((1ll << bits) < c->N) ++bits;
  tb = c->d.temp_bytes;
  KP_HIP(rocprim::radix_sort_pairs(c->d.temp, tb, c->d.k_in, c->d.k_out, c->d.v_in, c->d.v_out,
                                   (size_t)P, 0u, (unsigned)bits, c->stream));
  int32_t *seg_start = c->d.heads, *seg_end = c->d.heads + c->cap_N;
  KP_HIP(hipMemsetAsync(seg_start, 0xFF, sizeof(int32_t) * c->N, c->stream));
  hipLaunchKernelGGL(k_seg_bounds, dim3(blocks(P, 256)), dim3(256), 0, c->stream, P, c->d.k_out,
                     seg_start, seg_end);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

int launch_accept(kp_ctx *c, const ScoreParams &sp, int32_t P) {
  if (P <= 0) return KP_OK;
  return dispatch_D<AcceptL>(c->D, c, sp, P);
}

int launch_commit(kp_ctx *c, const ScoreParams &sp, int32_t P) {
  (void)sp;
  if (P <= 0) return KP_OK;
  hipLaunchKernelGGL(k_mark_bad, dim3(blocks(P, 256)), dim3(256), 0, c->stream, P, c->d.p_ok,
                     c->d.p_slot, c->d.act, c->d.unit_bad);
  KP_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_commit, dim3(blocks(P, 256)), dim3(256), 0, c->stream, P, c->D, c->N,
                     c->U, c->d.p_slot, c->d.p_node, c->d.p_count, c->d.p_off, c->d.p_score,
                     c->d.act, c->d.unit_bad, c->d.q, c->d.leader, c->d.used, c->d.status,
                     c->d.open, c->d.job_node, c->d.job_score);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

// active units of [lo, hi) in rank order -> act_local; count to host
int launch_active(kp_ctx *c, int32_t lo, int32_t hi, int32_t *A_host) {
  *A_host = 0;
  const int32_t n = hi - lo;
  if (n <= 0) return KP_OK;
  int32_t *flag = c->d.st_pos;  // scratch [U+1]
  hipLaunchKernelGGL(k_flag_active, dim3(blocks(n, 256)), dim3(256), 0, c->stream, c->d.status,
                     lo, hi, flag);
  KP_HIP(hipGetLastError());
  size_t tb = c->d.temp_bytes;
  KP_HIP(rocprim::select(c->d.temp, tb, rocprim::counting_iterator<int32_t>(lo), flag,
                         c->d.act_local, c->d.counters, (size_t)n, c->stream));
  KP_HIP(hipMemcpyAsync(c->pinned, c->d.counters, sizeof(int32_t), hipMemcpyDeviceToHost,
                        c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  *A_host = c->pinned[0];
  return KP_OK;
}

int launch_reset_units(kp_ctx *c) {
  const int32_t n = c->U > c->J ? c->U : c->J;
  if (n <= 0) return KP_OK;
  hipLaunchKernelGGL(k_reset_units, dim3(blocks(n, 256)), dim3(256), 0, c->stream, c->d.status,
                     c->U, c->d.job_node, c->d.job_score, c->J);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

int launch_finalize(kp_ctx *c) {
  if (c->U <= 0) return KP_OK;
  hipLaunchKernelGGL(k_finalize, dim3(blocks(c->U, 256)), dim3(256), 0, c->stream, c->d.status,
                     c->d.leader, c->d.size, c->U, c->d.job_node, c->d.job_score,
                     c->d.job_status);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

int launch_unpack_exchange(kp_ctx *c, int32_t world, int32_t Umax, int32_t K,
                           int32_t *A_total) {
  (void)A_total;
  if (Umax <= 0) return KP_OK;
  hipLaunchKernelGGL(k_unpack, dim3(blocks((int64_t)world * Umax, 256)), dim3(256), 0, c->stream,
                     world, Umax, K, c->d.xg_counts, c->d.xg_recv, c->d.act, c->d.cand);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

int launch_pack_exchange(kp_ctx *c, int32_t A, int32_t K) {
  if (A <= 0) return KP_OK;
  hipLaunchKernelGGL(k_pack, dim3(blocks(A, 256)), dim3(256), 0, c->stream, A, K,
                     c->d.act_local, c->d.cand_local, c->d.xg_send);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

}  // namespace kp
