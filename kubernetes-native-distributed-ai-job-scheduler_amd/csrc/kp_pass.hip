// kp_pass.hip — gfx950 kernels of one auction round's acceptance passes
// (DESIGN.md §2.5), bit-exact with oracle/kp_oracle.c kpo_round_run.
//
// After the candidate phase every active slot a has K candidate nodes
// cand[a*K + c]. One radix sort per ROUND builds the node -> (slot,
// candidate) inverse index in slot order (= unit rank order): entry e of the
// sorted order belongs to node key[e]; inv[a*K + c] = e. A pass then needs no
// sort and no host round trip:
//   plan   : a G-lane group per open slot (lane c = candidate c) plans the
//            unit's members against the current usage and writes a
//            pass-tagged bid (pass << 8 | members) straight into bid[inv[..]]
//            plus a per-64-entry window flag;
//   accept : one wave per node visits only its flagged windows, runs an exact
//            parallel first-fit in rank order, commits units whose members
//            all sit on this node (the wave owns the node: plain stores), and
//            records ok[e] for multi-node gangs;
//   gang   : all-or-nothing commit of multi-node gangs (int64 atomics).
#include <hip/hip_runtime.h>

#include <cstring>

#include <rocprim/rocprim.hpp>

#include "kp_device.hpp"
#include "kp_internal.hpp"

namespace kp {
namespace {
using namespace dev;

constexpr uint32_t kNoBid = 0xFFFFFFFFu;  // tag that matches no pass

// ---- inverse index (once per round) --------------------------------------------
__global__ void k_csr_keys(int32_t A, int32_t K, int32_t N, const int32_t *__restrict__ cand,
                           uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)A * K) return;
  const int32_t n = cand[t];
  const int32_t a = (int32_t)(t / K), c = (int32_t)(t % K);
  keys[t] = n >= 0 ? (uint32_t)n : (uint32_t)N;  // invalid entries sort after every node
  vals[t] = ((uint32_t)a << 5) | (uint32_t)c;     // K <= 32
}

__global__ void k_csr_finish(int32_t P, int32_t N, int32_t K, int32_t D, int32_t U,
                             const uint32_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                             const int32_t *__restrict__ act, const int64_t *__restrict__ q,
                             const int32_t *__restrict__ size, const int32_t *__restrict__ leader,
                             int32_t *__restrict__ seg_start, int32_t *__restrict__ seg_end,
                             int32_t *__restrict__ inv, int32_t *__restrict__ ent_unit,
                             int32_t *__restrict__ ent_slot, int32_t *__restrict__ ent_size,
                             int32_t *__restrict__ ent_lead, int64_t *__restrict__ ent_q) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P) return;
  const uint32_t k = keys[e];
  if (k >= (uint32_t)N) return;
  const uint32_t v = vals[e];
  const int32_t a = (int32_t)(v >> 5), c = (int32_t)(v & 31u);
  const int32_t u = act[a];
  inv[(int64_t)a * K + c] = e;
  // operands of entry e, laid out in bidder order so that a window's loads in
  // k_accept are independent and coalesced (no unit -> request gather chain)
  ent_unit[e] = u;
  ent_slot[e] = a;
  ent_size[e] = size[u];
  ent_lead[e] = leader[u];
  for (int d = 0; d < D; ++d) ent_q[(int64_t)d * P + e] = q[(int64_t)d * U + u];
  if (e == 0 || keys[e - 1] != k) seg_start[k] = e;
  if (e == P - 1 || keys[e + 1] != k) seg_end[k] = e + 1;
}

// ---- plan ------------------------------------------------------------------------
// G lanes per slot (G >= K), 64/G slots per wave. Members are planned one at a
// time: each lane scores its candidate with the members it already holds,
// subtracts the spread penalty of its topo domain, and the group takes the
// (max value, lowest lane).
template <int D, int G>
__global__ __launch_bounds__(256) void k_plan(ScoreParams sp, int32_t A, int32_t U, int32_t pass,
                                              const int32_t *__restrict__ act,
                                              const int32_t *__restrict__ cand,
                                              const int32_t *__restrict__ inv,
                                              uint8_t *__restrict__ open,
                                              int32_t *__restrict__ status,
                                              const int64_t *__restrict__ cap,
                                              const int64_t *__restrict__ used,
                                              const uint64_t *__restrict__ R,
                                              const int64_t *__restrict__ base,
                                              const int32_t *__restrict__ topo,
                                              const int64_t *__restrict__ q,
                                              const int32_t *__restrict__ size,
                                              uint32_t *__restrict__ bid,
                                              int32_t *__restrict__ win,
                                              int32_t *__restrict__ s0_out,
                                              int32_t *__restrict__ pass_flag) {
  constexpr int SPW = 64 / G;  // slots per wave
  constexpr uint64_t GMASK = G == 64 ? ~0ull : ((1ull << G) - 1);
  const int lane = threadIdx.x & 63;
  const int gl = lane & (G - 1);      // lane within the group = candidate index
  const int gbase = lane & ~(G - 1);  // first lane of the group
  const int wave_global = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int a = wave_global * SPW + lane / G;
  const int K = sp.n_cand, N = sp.N;
  const bool slot_ok = a < A && open[a];
  if (__ballot(slot_ok) == 0) return;
  int32_t u = 0, sz = 0;
  int64_t qq[D];
  if (slot_ok) {
    u = act[a];
    sz = size[u];
  }
#pragma unroll
  for (int d = 0; d < D; ++d) qq[d] = slot_ok ? q[(int64_t)d * U + u] : 0;
  const int32_t node = (slot_ok && gl < K) ? cand[(int64_t)a * K + gl] : -1;
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
  int32_t szmax = sz;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) szmax = max(szmax, __shfl_xor(szmax, m, kWave));
  int32_t planned = 0, dom = 0, s0 = -1;
  bool fail = !slot_ok;
  for (int m = 0; m < szmax; ++m) {
    const bool live = !fail && m < sz;  // group-uniform
    int64_t uu[D];
#pragma unroll
    for (int d = 0; d < D; ++d) uu[d] = u0[d] + (int64_t)planned * qq[d];
    const int64_t s = (live && valid) ? score_at<D>(sp, qq, c_, uu, r_, b) : -1;
    if (m == 0) s0 = (int32_t)s;
    const bool feas = s >= 0;
    const int64_t val = feas ? s - (int64_t)sp.w_spread * dom : INT64_MIN;
    const uint64_t gm = (__ballot(feas) >> gbase) & GMASK;
    if (live && gm == 0) fail = true;
    const int64_t best = group_max_i64<G>(val);
    const uint64_t wm = (__ballot(feas && val == best) >> gbase) & GMASK;
    const int w = wm ? (__ffsll((unsigned long long)wm) - 1) : 0;
    const int32_t wtp = __shfl(tp, gbase + w, kWave);
    if (live && !fail) {
      planned += gl == w ? 1 : 0;
      dom += (valid && tp == wtp) ? 1 : 0;
    }
  }
  if (!slot_ok) return;
  if (fail) {
    if (gl == 0) {
      open[a] = 0;
      if (pass == 0) status[u] = kNoFit;
    }
    return;
  }
  if (gl < K && planned > 0) {
    const int32_t e = inv[(int64_t)a * K + gl];
    bid[e] = ((uint32_t)pass << 8) | (uint32_t)planned;
    s0_out[e] = s0;
    win[e >> 6] = pass;
  }
  if (gl == 0) pass_flag[pass] = 1;
}

// ---- accept ----------------------------------------------------------------------
// One wave per node over the flagged 64-entry windows of its bidder row (rank
// order). Exact parallel first-fit per window: lanes that no longer fit alone are
// rejected; among the rest the longest prefix whose running sum fits is accepted
// and the first lane that breaks it is rejected (it cannot fit the reduced
// remainder); repeat on what is left. A unit whose members all bid here (count ==
// size) is committed on the spot; for multi-node gangs ok[e] = pass + 1 marks an
// accepted part for k_gang_commit. The operands of the next flagged window are
// loaded before the current one is decided (one HBM latency per window, hidden).
template <int D>
struct Win {
  int32_t e, m, unit, size, lead, slot, s0;
  int64_t need[D];
};

template <int D>
__device__ __forceinline__ void load_win(Win<D> &w, int wi, int lane, int32_t e0, int32_t e1,
                                         int32_t pass, int64_t P,
                                         const uint32_t *__restrict__ bid,
                                         const int64_t *__restrict__ ent_q,
                                         const int32_t *__restrict__ ent_unit,
                                         const int32_t *__restrict__ ent_size,
                                         const int32_t *__restrict__ ent_lead,
                                         const int32_t *__restrict__ ent_slot,
                                         const int32_t *__restrict__ s0) {
  w.e = (wi << 6) + lane;
  w.m = 0;
  const bool in_row = wi >= 0 && w.e >= e0 && w.e < e1;
  const int32_t ee = in_row ? w.e : e0;
  const uint32_t t = bid[ee];
  w.unit = ent_unit[ee];
  w.size = ent_size[ee];
  w.lead = ent_lead[ee];
  w.slot = ent_slot[ee];
  w.s0 = s0[ee];
#pragma unroll
  for (int d = 0; d < D; ++d) w.need[d] = ent_q[(int64_t)d * P + ee];
  if (in_row && (t >> 8) == (uint32_t)pass) w.m = (int32_t)(t & 0xFFu);
#pragma unroll
  for (int d = 0; d < D; ++d) w.need[d] = w.m > 0 ? (int64_t)w.m * w.need[d] : 0;
}

// Exact parallel first-fit of one 64-entry window against the node's
// remaining capacity `rem` (wave-uniform), in lane (= rank) order.
template <int D>
__device__ __forceinline__ void decide_window(const Win<D> &wc, int64_t (&rem)[D],
                                              int64_t (&add)[D], int lane, int node,
                                              int32_t pass, uint8_t *__restrict__ ok,
                                              uint8_t *__restrict__ open,
                                              int32_t *__restrict__ status,
                                              int32_t *__restrict__ job_node,
                                              int32_t *__restrict__ job_score) {
  bool undecided = wc.m > 0, accepted = false;
  while (true) {
    bool fa = undecided;
#pragma unroll
    for (int d = 0; d < D; ++d) fa &= wc.need[d] <= rem[d];
    // lanes that do not fit alone are rejected for good; if none fits, the
    // window is done without any prefix scan
    if (__ballot(fa) == 0) break;
    bool okp = fa;
    int64_t pre[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int64_t x = fa ? wc.need[d] : 0;
      pre[d] = wave_incl_scan_i64(x) - x;  // exclusive
      okp &= pre[d] + wc.need[d] <= rem[d];
    }
    const uint64_t failm = __ballot(fa && !okp);
    if (failm == 0) {
      accepted |= fa;
#pragma unroll
      for (int d = 0; d < D; ++d) rem[d] -= shfl_i64(pre[d], 63) + shfl_i64(fa ? wc.need[d] : 0, 63);
      break;
    }
    const int f = __ffsll((unsigned long long)failm) - 1;
    accepted |= fa && lane < f;
#pragma unroll
    for (int d = 0; d < D; ++d) rem[d] -= shfl_i64(pre[d], f);
    undecided = fa && lane >= f;  // lane f is rejected on the next check
  }
  if (wc.m > 0 && accepted) {
    if (wc.m == wc.size) {  // the whole unit bid on this node: commit now
      for (int i = 0; i < wc.m; ++i) {
        job_node[wc.lead + i] = node;
        job_score[wc.lead + i] = wc.s0;
      }
      status[wc.unit] = kPlaced;
      open[wc.slot] = 0;
#pragma unroll
      for (int d = 0; d < D; ++d) add[d] += wc.need[d];
    } else {
      ok[wc.e] = (uint8_t)(pass + 1);
    }
  }
}

template <int D>
__global__ __launch_bounds__(256) void k_accept(ScoreParams sp, int32_t pass, int64_t P,
                                                const int32_t *__restrict__ seg_start,
                                                const int32_t *__restrict__ seg_end,
                                                const uint32_t *__restrict__ bid,
                                                const int32_t *__restrict__ win,
                                                const int32_t *__restrict__ s0,
                                                const int64_t *__restrict__ ent_q,
                                                const int32_t *__restrict__ ent_unit,
                                                const int32_t *__restrict__ ent_size,
                                                const int32_t *__restrict__ ent_lead,
                                                const int32_t *__restrict__ ent_slot,
                                                const int64_t *__restrict__ cap,
                                                int64_t *__restrict__ used,
                                                uint8_t *__restrict__ ok,
                                                uint8_t *__restrict__ open,
                                                int32_t *__restrict__ status,
                                                int32_t *__restrict__ job_node,
                                                int32_t *__restrict__ job_score) {
  const int lane = threadIdx.x & 63;
  const int node = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int N = sp.N;
  if (node >= N) return;
  const int32_t e0 = seg_start[node];
  if (e0 < 0) return;
  const int32_t e1 = seg_end[node];
  const int32_t w0 = e0 >> 6, w1 = (e1 - 1) >> 6;
  int64_t rem[D], add[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    rem[d] = cap[(int64_t)d * N + node] - used[(int64_t)d * N + node];
    add[d] = 0;
  }
  constexpr int BATCH = 4;  // flagged windows whose operands are loaded together
  for (int wb = w0; wb <= w1; wb += 64) {
    uint64_t flagged = __ballot(wb + lane <= w1 && win[wb + lane] == pass);
    while (flagged) {
      int wl[BATCH];
#pragma unroll
      for (int t = 0; t < BATCH; ++t) {
        wl[t] = flagged ? wb + __ffsll((unsigned long long)flagged) - 1 : -1;
        flagged &= flagged ? flagged - 1 : 0;
      }
      Win<D> wv[BATCH];
#pragma unroll
      for (int t = 0; t < BATCH; ++t)
        load_win<D>(wv[t], wl[t], lane, e0, e1, pass, P, bid, ent_q, ent_unit, ent_size,
                    ent_lead, ent_slot, s0);
#pragma unroll
      for (int t = 0; t < BATCH; ++t) {
        Win<D> &wc = wv[t];
        if (wl[t] < 0) break;
        decide_window<D>(wc, rem, add, lane, node, pass, ok, open, status, job_node, job_score);
      }
    }
  }
  // this wave owns the node: fold the committed single-node units into `used`
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const int64_t tot = wave_incl_scan_i64(add[d]);
    if (lane == 63 && tot != 0) used[(int64_t)d * N + node] += tot;
  }
}

// ---- multi-node gang commit --------------------------------------------------------
// A G-lane group per slot, lane c = candidate c: all-or-nothing over the parts
// accepted this pass; members map to nodes in candidate order.
template <int G>
__global__ __launch_bounds__(256) void k_gang_commit(int32_t A, int32_t K, int32_t D, int32_t N,
                                                     int32_t U, int32_t pass,
                                                     const int32_t *__restrict__ act,
                                                     const int32_t *__restrict__ cand,
                                                     const int32_t *__restrict__ inv,
                                                     const uint32_t *__restrict__ bid,
                                                     const int32_t *__restrict__ s0,
                                                     const uint8_t *__restrict__ ok,
                                                     const int64_t *__restrict__ q,
                                                     const int32_t *__restrict__ size,
                                                     const int32_t *__restrict__ leader,
                                                     uint8_t *__restrict__ open,
                                                     int32_t *__restrict__ status,
                                                     int64_t *__restrict__ used,
                                                     int32_t *__restrict__ job_node,
                                                     int32_t *__restrict__ job_score) {
  constexpr int SPW = 64 / G;
  constexpr uint64_t GMASK = G == 64 ? ~0ull : ((1ull << G) - 1);
  const int lane = threadIdx.x & 63;
  const int gl = lane & (G - 1), gbase = lane & ~(G - 1);
  const int a = (blockIdx.x * 4 + (threadIdx.x >> 6)) * SPW + lane / G;
  bool live = a < A && open[a];
  int32_t u = 0, sz = 1;
  if (live) {
    u = act[a];
    sz = size[u];
    live = sz > 1;  // singletons and single-node gangs are decided in k_accept
  }
  if (__ballot(live) == 0) return;
  int32_t m = 0, e = 0, node = -1;
  bool part_ok = true;
  if (live && gl < K) {
    node = cand[(int64_t)a * K + gl];
    if (node >= 0) {
      e = inv[(int64_t)a * K + gl];
      const uint32_t t = bid[e];
      if ((t >> 8) == (uint32_t)pass) {
        m = (int32_t)(t & 0xFFu);
        part_ok = ok[e] == (uint8_t)(pass + 1);
      }
    }
  }
  const uint64_t has = (__ballot(m > 0) >> gbase) & GMASK;
  const uint64_t bad = (__ballot(m > 0 && !part_ok) >> gbase) & GMASK;
  const uint64_t whole = (__ballot(m > 0 && m == sz) >> gbase) & GMASK;
  if (!live || has == 0 || bad != 0 || whole != 0) return;
  // member offset = members of the earlier candidates of this slot
  int32_t off = 0;
  for (int c = 0; c < G; ++c) {
    const int32_t mc = __shfl(m, gbase + c, 64);
    if (c < gl) off += mc;
  }
  if (m > 0) {
    for (int d = 0; d < D; ++d)
      atomicAdd(reinterpret_cast<unsigned long long *>(&used[(int64_t)d * N + node]),
                (unsigned long long)((int64_t)m * q[(int64_t)d * U + u]));
    const int32_t j0 = leader[u] + off, sc = s0[e];
    for (int i = 0; i < m; ++i) {
      job_node[j0 + i] = node;
      job_score[j0 + i] = sc;
    }
  }
  if (gl == 0) {
    status[u] = kPlaced;
    open[a] = 0;
  }
}

template <int D>
struct PlanL {
  static int run(kp_ctx *c, const ScoreParams &sp, int32_t A, int32_t pass) {
    if (sp.n_cand <= 16) {
      constexpr int G = 16;
      hipLaunchKernelGGL((k_plan<D, G>), dim3(blocks(A, 4 * (64 / G))), dim3(256), 0, c->stream,
                         sp, A, c->U, pass, c->d.act, c->d.cand, c->d.inv, c->d.open,
                         c->d.status, c->d.cap, c->d.used, c->d.R, c->d.base, c->d.topo, c->d.q,
                         c->d.size, c->d.bid, c->d.win, c->d.s0, c->d.pass_flag);
    } else {
      constexpr int G = 32;
      hipLaunchKernelGGL((k_plan<D, G>), dim3(blocks(A, 4 * (64 / G))), dim3(256), 0, c->stream,
                         sp, A, c->U, pass, c->d.act, c->d.cand, c->d.inv, c->d.open,
                         c->d.status, c->d.cap, c->d.used, c->d.R, c->d.base, c->d.topo, c->d.q,
                         c->d.size, c->d.bid, c->d.win, c->d.s0, c->d.pass_flag);
    }
    KP_HIP(hipGetLastError());
    return KP_OK;
  }
};

template <int D>
struct AcceptL {
  static int run(kp_ctx *c, const ScoreParams &sp, int32_t pass, int64_t P) {
    hipLaunchKernelGGL((k_accept<D>), dim3(blocks(c->N, 4)), dim3(256), 0, c->stream, sp, pass,
                       P, c->d.seg_start, c->d.seg_end, c->d.bid, c->d.win, c->d.s0, c->d.ent_q,
                       c->d.ent_unit, c->d.ent_size, c->d.ent_lead, c->d.ent_slot, c->d.cap,
                       c->d.used, c->d.ok, c->d.open, c->d.status, c->d.job_node,
                       c->d.job_score);
    KP_HIP(hipGetLastError());
    return KP_OK;
  }
};

}  // namespace

size_t rocprim_temp_bytes(int32_t max_items) {
  size_t a = 0, s = 0;
  (void)rocprim::radix_sort_pairs(nullptr, a, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                  (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)max_items,
                                  0u, 32u);
  (void)rocprim::select(nullptr, s, rocprim::counting_iterator<int32_t>(0), (int32_t *)nullptr,
                        (int32_t *)nullptr, (int32_t *)nullptr, (size_t)max_items);
  return (a > s ? a : s) + 256;
}

// node -> bidder inverse index of this round's candidates (one sort per round)
int launch_csr_build(kp_ctx *c, int32_t A, int32_t K) {
  const int64_t P = (int64_t)A * K;
  KP_HIP(hipMemsetAsync(c->d.seg_start, 0xFF, sizeof(int32_t) * c->N, c->stream));
  if (P == 0) return KP_OK;
  KP_HIP(hipMemsetAsync(c->d.bid, 0xFF, sizeof(uint32_t) * P, c->stream));
  KP_HIP(hipMemsetAsync(c->d.win, 0xFF, sizeof(int32_t) * ((P + 63) / 64 + 64), c->stream));
  hipLaunchKernelGGL(k_csr_keys, dim3(blocks(P, 256)), dim3(256), 0, c->stream, A, K, c->N,
                     c->d.cand, c->d.csr_kin, c->d.csr_vin);
  KP_HIP(hipGetLastError());
  unsigned bits = 1;
  while ((1ll << bits) <= c->N) ++bits;  // key N (invalid) must fit too
  size_t tb = c->d.temp_bytes;
  KP_HIP(rocprim::radix_sort_pairs(c->d.temp, tb, c->d.csr_kin, c->d.csr_keys, c->d.csr_vin,
                                   c->d.csr_vals, (size_t)P, 0u, bits, c->stream));
  KP_HIP(hipMemsetAsync(c->d.ok, 0, P, c->stream));
  hipLaunchKernelGGL(k_csr_finish, dim3(blocks(P, 256)), dim3(256), 0, c->stream, (int32_t)P,
                     c->N, K, c->D, c->U, c->d.csr_keys, c->d.csr_vals, c->d.act, c->d.q,
                     c->d.size, c->d.leader, c->d.seg_start, c->d.seg_end, c->d.inv,
                     c->d.ent_unit, c->d.ent_slot, c->d.ent_size, c->d.ent_lead, c->d.ent_q);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

int launch_plan(kp_ctx *c, const ScoreParams &sp, int32_t A, int32_t pass) {
  if (A <= 0) return KP_OK;
  return dispatch_D<PlanL>(c->D, c, sp, A, pass);
}

int launch_accept(kp_ctx *c, const ScoreParams &sp, int32_t pass, int32_t A) {
  if (c->N <= 0 || A <= 0) return KP_OK;
  return dispatch_D<AcceptL>(c->D, c, sp, pass, (int64_t)A * sp.n_cand);
}

int launch_gang_commit(kp_ctx *c, const ScoreParams &sp, int32_t A, int32_t pass) {
  if (A <= 0) return KP_OK;
  if (sp.n_cand <= 16) {
    constexpr int G = 16;
    hipLaunchKernelGGL(k_gang_commit<G>, dim3(blocks(A, 4 * (64 / G))), dim3(256), 0, c->stream,
                       A, sp.n_cand, c->D, c->N, c->U, pass, c->d.act, c->d.cand, c->d.inv,
                       c->d.bid, c->d.s0, c->d.ok, c->d.q, c->d.size, c->d.leader, c->d.open,
                       c->d.status, c->d.used, c->d.job_node, c->d.job_score);
  } else {
    constexpr int G = 32;
    hipLaunchKernelGGL(k_gang_commit<G>, dim3(blocks(A, 4 * (64 / G))), dim3(256), 0, c->stream,
                       A, sp.n_cand, c->D, c->N, c->U, pass, c->d.act, c->d.cand, c->d.inv,
                       c->d.bid, c->d.s0, c->d.ok, c->d.q, c->d.size, c->d.leader, c->d.open,
                       c->d.status, c->d.used, c->d.job_node, c->d.job_score);
  }
  KP_HIP(hipGetLastError());
  return KP_OK;
}

}  // namespace kp
