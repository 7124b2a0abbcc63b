// kp_pass.hip — gfx950 kernels of one auction round's acceptance passes
// (DESIGN.md §2.5), bit-exact with oracle/kp_oracle.c kpo_round_run.
//
// Layout of a round: after the candidate phase every active slot a has K
// candidate nodes cand[a*K + c]. One radix sort per ROUND builds the inverse
// index node -> (slot, candidate) in slot order (= unit rank order), so a
// pass needs no sort and no host round-trip: three kernels
//   plan   : one G-lane lane-group per slot (lane c = candidate c) plans the
//            unit's members against the current usage -> planned[a*K+c]
//   accept : one wave per node walks its bidder list in rank order and runs
//            an exact parallel first-fit over 64-bidder windows -> ok[a*K+c]
//   commit : one thread per slot: all-or-nothing; int64 atomics into `used`
#include <hip/hip_runtime.h>

#include <cstring>

#include <rocprim/rocprim.hpp>

#include "kp_device.hpp"
#include "kp_internal.hpp"

namespace kp {
namespace {
using namespace dev;

// ---- inverse index -----------------------------------------------------------
__global__ void k_csr_keys(int32_t A, int32_t K, int32_t N, const int32_t *__restrict__ cand,
                           uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)A * K) return;
  const int32_t n = cand[t];
  const int32_t a = (int32_t)(t / K), c = (int32_t)(t % K);
  keys[t] = n >= 0 ? (uint32_t)n : (uint32_t)N;  // invalid entries sort after every node
  vals[t] = ((uint32_t)a << 5) | (uint32_t)c;     // K <= 32
}

__global__ void k_seg_bounds(int32_t P, int32_t N, const uint32_t *__restrict__ keys,
                             int32_t *__restrict__ seg_start, int32_t *__restrict__ seg_end) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const uint32_t k = keys[i];
  if (k >= (uint32_t)N) return;
  if (i == 0 || keys[i - 1] != k) seg_start[k] = i;
  if (i == P - 1 || keys[i + 1] != k) seg_end[k] = i + 1;
}

// ---- plan ----------------------------------------------------------------------
// G lanes per slot (G >= K), 64/G slots per wave. Members are planned one at a
// time: each lane scores its candidate with the members it already holds,
// subtracts the spread penalty of its topo domain, and the group takes the
// (max value, lowest lane).
template <int D, int G>
__global__ __launch_bounds__(256) void k_plan(ScoreParams sp, int32_t A, int32_t U, int32_t pass,
                                              const int32_t *__restrict__ act,
                                              const int32_t *__restrict__ cand,
                                              uint8_t *__restrict__ open,
                                              int32_t *__restrict__ status,
                                              const int64_t *__restrict__ cap,
                                              const int64_t *__restrict__ used,
                                              const uint64_t *__restrict__ R,
                                              const int64_t *__restrict__ base,
                                              const int32_t *__restrict__ topo,
                                              const int64_t *__restrict__ q,
                                              const int32_t *__restrict__ size,
                                              int32_t *__restrict__ planned_out,
                                              int32_t *__restrict__ s0_out,
                                              int32_t *__restrict__ pass_flag) {
  constexpr int SPW = 64 / G;  // slots per wave
  const int lane = threadIdx.x & 63;
  const int gl = lane & (G - 1);           // lane within the group = candidate index
  const int gbase = lane & ~(G - 1);       // first lane of the group
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
  // group size loop bound: max members over the wave's slots
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
    const uint64_t gm = (__ballot(feas) >> gbase) & (G == 64 ? ~0ull : ((1ull << G) - 1));
    if (live && gm == 0) fail = true;
    const int64_t best = group_max_i64<G>(val);
    const uint64_t wm = (__ballot(feas && val == best) >> gbase) & (G == 64 ? ~0ull : ((1ull << G) - 1));
    const int win = wm ? (__ffsll((unsigned long long)wm) - 1) : 0;
    const int32_t wtp = __shfl(tp, gbase + win, kWave);
    if (live && !fail) {
      planned += gl == win ? 1 : 0;
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
  if (gl < K) {
    planned_out[(int64_t)a * K + gl] = planned;
    s0_out[(int64_t)a * K + gl] = s0;
  }
  if (gl == 0) pass_flag[pass] = 1;
}

// ---- accept ----------------------------------------------------------------------
// One wave per node; bidders = CSR entries (slot order = rank order) whose slot is
// open and planned members on this node this pass. Exact parallel first-fit on a
// 64-entry window: lanes that no longer fit alone are rejected; among the rest the
// longest prefix whose running sum fits is accepted and the first lane that breaks
// it is rejected (it cannot fit the reduced remainder); repeat on what is left.
template <int D>
__global__ __launch_bounds__(256) void k_accept(ScoreParams sp, int32_t U,
                                                const int32_t *__restrict__ seg_start,
                                                const int32_t *__restrict__ seg_end,
                                                const uint32_t *__restrict__ csr,
                                                const uint8_t *__restrict__ open,
                                                const int32_t *__restrict__ planned,
                                                const int32_t *__restrict__ act,
                                                const int64_t *__restrict__ q,
                                                const int64_t *__restrict__ cap,
                                                const int64_t *__restrict__ used,
                                                uint8_t *__restrict__ ok) {
  const int lane = threadIdx.x & 63;
  const int node = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int N = sp.N, K = sp.n_cand;
  if (node >= N) return;
  const int32_t s0 = seg_start[node];
  if (s0 < 0) return;
  const int32_t s1 = seg_end[node];
  int64_t rem[D];
#pragma unroll
  for (int d = 0; d < D; ++d) rem[d] = cap[(int64_t)d * N + node] - used[(int64_t)d * N + node];
  for (int base = s0; base < s1; base += 64) {
    const int e = base + lane;
    int64_t idx = -1;
    int64_t need[D];
    int32_t m = 0;
    if (e < s1) {
      const uint32_t v = csr[e];
      const int32_t a = (int32_t)(v >> 5), c = (int32_t)(v & 31u);
      if (open[a]) {
        idx = (int64_t)a * K + c;
        m = planned[idx];
      }
      if (m > 0) {
        const int32_t u = act[a];
#pragma unroll
        for (int d = 0; d < D; ++d) need[d] = (int64_t)m * q[(int64_t)d * U + u];
      }
    }
    if (m <= 0) {
#pragma unroll
      for (int d = 0; d < D; ++d) need[d] = 0;
    }
    bool undecided = m > 0, accepted = false;
    while (__ballot(undecided) != 0) {
      bool fa = undecided;
#pragma unroll
      for (int d = 0; d < D; ++d) fa &= need[d] <= rem[d];
      undecided = fa;  // lanes that do not fit alone are rejected for good
      bool okp = fa;
      int64_t pre[D];
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int64_t x = fa ? need[d] : 0;
        pre[d] = wave_incl_scan_i64(x) - x;  // exclusive
        okp &= pre[d] + need[d] <= rem[d];
      }
      const uint64_t failm = __ballot(fa && !okp);
      if (failm == 0) {
        accepted |= fa;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          const int64_t tot = wave_incl_scan_i64(fa ? need[d] : 0);
          rem[d] -= shfl_i64(tot, 63);
        }
        undecided = false;
      } else {
        const int f = __ffsll((unsigned long long)failm) - 1;
        accepted |= fa && lane < f;
#pragma unroll
        for (int d = 0; d < D; ++d) rem[d] -= shfl_i64(pre[d], f);
        undecided = fa && lane >= f;  // lane f is rejected on the next check
      }
    }
    if (m > 0) ok[idx] = accepted ? 1 : 0;
  }
}

// ---- commit ------------------------------------------------------------------------
__global__ void k_commit(int32_t A, int32_t K, int32_t D, int32_t N, int32_t U,
                         const int32_t *__restrict__ act, const int32_t *__restrict__ cand,
                         const int32_t *__restrict__ planned, const int32_t *__restrict__ s0,
                         const uint8_t *__restrict__ ok, const int64_t *__restrict__ q,
                         const int32_t *__restrict__ leader, uint8_t *__restrict__ open,
                         int32_t *__restrict__ status, int64_t *__restrict__ used,
                         int32_t *__restrict__ job_node, int32_t *__restrict__ job_score) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= A || !open[a]) return;
  const int64_t row = (int64_t)a * K;
  bool any = false, all = true;
  for (int c = 0; c < K; ++c) {
    const int32_t m = planned[row + c];
    if (m > 0) {
      any = true;
      all &= ok[row + c] != 0;
    }
  }
  if (!any || !all) return;  // all-or-nothing: retry next pass
  const int32_t u = act[a];
  int32_t off = leader[u];
  for (int c = 0; c < K; ++c) {
    const int32_t m = planned[row + c];
    if (m <= 0) continue;
    const int32_t node = cand[row + c];
    for (int d = 0; d < D; ++d)
      atomicAdd(reinterpret_cast<unsigned long long *>(&used[(int64_t)d * N + node]),
                (unsigned long long)((int64_t)m * q[(int64_t)d * U + u]));
    const int32_t sc = s0[row + c];
    for (int i = 0; i < m; ++i) {
      job_node[off + i] = node;
      job_score[off + i] = sc;
    }
    off += m;
  }
  status[u] = kPlaced;
  open[a] = 0;
}

// planned[] must read 0 for every (slot, candidate) that a plan did not write this
// pass; the plan writes all K entries of every slot it plans, so only the slots it
// skips matter, and those are closed (open == 0), which accept/commit check first.

template <int D>
struct PlanL {
  static int run(kp_ctx *c, const ScoreParams &sp, int32_t A, int32_t pass) {
    const int K = sp.n_cand;
    if (K <= 16) {
      constexpr int G = 16;
      hipLaunchKernelGGL((k_plan<D, G>), dim3(blocks(A, 4 * (64 / G))), dim3(256), 0, c->stream,
                         sp, A, c->U, pass, c->d.act, c->d.cand, c->d.open, c->d.status,
                         c->d.cap, c->d.used, c->d.R, c->d.base, c->d.topo, c->d.q, c->d.size,
                         c->d.planned, c->d.s0, c->d.pass_flag);
    } else {
      constexpr int G = 32;
      hipLaunchKernelGGL((k_plan<D, G>), dim3(blocks(A, 4 * (64 / G))), dim3(256), 0, c->stream,
                         sp, A, c->U, pass, c->d.act, c->d.cand, c->d.open, c->d.status,
                         c->d.cap, c->d.used, c->d.R, c->d.base, c->d.topo, c->d.q, c->d.size,
                         c->d.planned, c->d.s0, c->d.pass_flag);
    }
    KP_HIP(hipGetLastError());
    return KP_OK;
  }
};

template <int D>
struct AcceptL {
  static int run(kp_ctx *c, const ScoreParams &sp) {
    hipLaunchKernelGGL((k_accept<D>), dim3(blocks(c->N, 4)), dim3(256), 0, c->stream, sp, c->U,
                       c->d.seg_start, c->d.seg_end, c->d.csr_vals, c->d.open, c->d.planned,
                       c->d.act, c->d.q, c->d.cap, c->d.used, c->d.ok);
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

// node -> bidder-slot inverse index of this round's candidates (one sort per round)
int launch_csr_build(kp_ctx *c, int32_t A, int32_t K) {
  const int64_t P = (int64_t)A * K;
  KP_HIP(hipMemsetAsync(c->d.seg_start, 0xFF, sizeof(int32_t) * c->N, c->stream));
  if (P == 0) return KP_OK;
  hipLaunchKernelGGL(k_csr_keys, dim3(blocks(P, 256)), dim3(256), 0, c->stream, A, K, c->N,
                     c->d.cand, c->d.csr_kin, c->d.csr_vin);
  KP_HIP(hipGetLastError());
  unsigned bits = 1;
  while ((1ll << bits) <= c->N) ++bits;  // key N (invalid) must fit too
  size_t tb = c->d.temp_bytes;
  KP_HIP(rocprim::radix_sort_pairs(c->d.temp, tb, c->d.csr_kin, c->d.csr_keys, c->d.csr_vin,
                                   c->d.csr_vals, (size_t)P, 0u, bits, c->stream));
  hipLaunchKernelGGL(k_seg_bounds, dim3(blocks(P, 256)), dim3(256), 0, c->stream, (int32_t)P,
                     c->N, c->d.csr_keys, c->d.seg_start, c->d.seg_end);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

int launch_plan(kp_ctx *c, const ScoreParams &sp, int32_t A, int32_t pass) {
  if (A <= 0) return KP_OK;
  return dispatch_D<PlanL>(c->D, c, sp, A, pass);
}

int launch_accept(kp_ctx *c, const ScoreParams &sp) {
  if (c->N <= 0) return KP_OK;
  return dispatch_D<AcceptL>(c->D, c, sp);
}

int launch_commit(kp_ctx *c, const ScoreParams &sp, int32_t A) {
  if (A <= 0) return KP_OK;
  hipLaunchKernelGGL(k_commit, dim3(blocks(A, 256)), dim3(256), 0, c->stream, A, sp.n_cand, c->D,
                     c->N, c->U, c->d.act, c->d.cand, c->d.planned, c->d.s0, c->d.ok, c->d.q,
                     c->d.leader, c->d.open, c->d.status, c->d.used, c->d.job_node,
                     c->d.job_score);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

}  // namespace kp
