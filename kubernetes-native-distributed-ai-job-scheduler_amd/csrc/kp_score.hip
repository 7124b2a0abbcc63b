// kp_score.hip — gfx950 (CDNA4) filter+score, top-K select and round bookkeeping.
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

#include "kp_device.hpp"
#include "kp_internal.hpp"

namespace kp {
namespace {
using namespace dev;

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

// 32-bit specialisation, chosen by the host when every cap and req is < 2^32
// (then used+q <= cap < 2^32 on every feasible pair). Same result bit for bit:
// util = ((u * R) >> 32) with R = Rh*2^32 + Rl (Rh <= S) is
// mulhi(u, Rl) + u*Rh exactly, since u*Rh*2^32 is a multiple of 2^32.
// Halves the VALU work per pair so the kernel stays on the HBM store roof.
template <int D, int NPL>
__global__ __launch_bounds__(256) void k_score32(ScoreParams sp,
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
  uint32_t f_[NPL][D], u_[NPL][D], rl_[NPL][D], rh_[NPL][D];
  int32_t b_[NPL];
  bool v_[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int n = tile0 + k * 64 + lane;
    v_[k] = n < N;
    const int nn = v_[k] ? n : 0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int64_t cc = cap[(int64_t)d * N + nn], uu = used[(int64_t)d * N + nn];
      const uint64_t rr = R[(int64_t)d * N + nn];
      f_[k][d] = (uint32_t)(cc - uu);
      u_[k][d] = (uint32_t)uu;
      rl_[k][d] = (uint32_t)rr;
      rh_[k][d] = (uint32_t)(rr >> 32);
    }
    b_[k] = (int32_t)base[nn];
  }
  const int words = Ns >> 6;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  if (tile0 >= Ns) return;
  for (int r = r0; r < r1; ++r) {
    const int32_t unit = rows_unit[r];
    uint32_t qq[D];
#pragma unroll
    for (int d = 0; d < D; ++d) qq[d] = (uint32_t)q[(int64_t)d * qstride + unit];
    int32_t *srow = score + (int64_t)r * Ns;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int n = tile0 + k * 64 + lane;
      bool fits = v_[k];
      int32_t acc = 0, fit_bonus = 0;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        fits &= qq[d] <= f_[k][d];
        const uint32_t uu = u_[k][d] + qq[d];
        const uint32_t util = __umulhi(uu, rl_[k][d]) + uu * rh_[k][d];
        acc += sp.w[d] * (int32_t)util;
        if (d == sp.gpu_dim && qq[d] > 0 && f_[k][d] == qq[d]) fit_bonus = sp.w_gpu_fit;
      }
      const int32_t s = (sp.most_allocated ? acc : b_[k] - acc) + fit_bonus;
      if (score && n < Ns) srow[n] = fits ? s : KP_SCORE_INFEASIBLE;
      const uint64_t bits = __ballot(fits);
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
  // one 256-thread workgroup per row: 4 waves split the row, each wave merges
  // its lanes' lists, wave 0 merges the 4 wave lists from LDS
  __shared__ uint64_t part[4][KC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = blockIdx.x;
  if (row >= rows) return;  // block-uniform
  const int K = sp.n_cand;
  const int32_t unit = rows_unit[row];
  const uint32_t sl = sp.tie_rotated ? salt[unit] : 0u;
  const uint32_t mul = sp.tie_rotated ? kTieMul : 1u;
  uint64_t k[KC];
#pragma unroll
  for (int i = 0; i < KC; ++i) k[i] = 0;
  const int4 *row4 = reinterpret_cast<const int4 *>(score + (int64_t)row * Ns);
  const int n4 = Ns >> 2;
  // 4 independent 16-B loads in flight per lane before any is consumed
  constexpr int UNR = 4;
  for (int i0 = threadIdx.x; i0 < n4; i0 += 256 * UNR) {
    int4 v[UNR];
#pragma unroll
    for (int t = 0; t < UNR; ++t) {
      const int i = i0 + 256 * t;
      v[t] = i < n4 ? row4[i] : make_int4(-1, -1, -1, -1);
    }
#pragma unroll
    for (int t = 0; t < UNR; ++t) {
      const int n = (i0 + 256 * t) * 4;
      if (v[t].x >= 0) topk_insert<KC>(k, pack_key(v[t].x, (uint32_t)(n + 0) * mul + sl));
      if (v[t].y >= 0) topk_insert<KC>(k, pack_key(v[t].y, (uint32_t)(n + 1) * mul + sl));
      if (v[t].z >= 0) topk_insert<KC>(k, pack_key(v[t].z, (uint32_t)(n + 2) * mul + sl));
      if (v[t].w >= 0) topk_insert<KC>(k, pack_key(v[t].w, (uint32_t)(n + 3) * mul + sl));
    }
  }
  // wave merge: K times the wave max of the lanes' heads; its owner pops
  for (int it = 0; it < K; ++it) {
    const uint64_t m = wave_max_u64(k[0]);
    if (lane == 0) part[wave][it] = m;
    if (m != 0 && k[0] == m) {  // keys are unique per node: exactly one lane pops
#pragma unroll
      for (int i = 0; i < KC - 1; ++i) k[i] = k[i + 1];
      k[KC - 1] = 0;
    }
  }
  __syncthreads();
  if (wave != 0) return;
  // block merge: lane l holds entries l and l+64 of the 4*K wave results
  const int tot = 4 * K;
  uint64_t h0 = lane < tot ? part[lane / K][lane % K] : 0;
  uint64_t h1 = lane + 64 < tot ? part[(lane + 64) / K][(lane + 64) % K] : 0;
  if (h1 > h0) {
    const uint64_t t = h0;
    h0 = h1;
    h1 = t;
  }
  const uint32_t inv = sp.tie_rotated ? kTieMulInv : 1u;
  for (int it = 0; it < K; ++it) {
    const uint64_t m = wave_max_u64(h0);
    if (lane == 0) {
      int32_t node = -1;
      if (m != 0) {
        const uint32_t tk = ~(uint32_t)m;
        node = (int32_t)((tk - sl) * inv);
      }
      cand[(int64_t)row * K + it] = node;
    }
    if (m != 0 && h0 == m) {
      h0 = h1;
      h1 = 0;
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

template <int D>
struct ScoreL {
  static int run(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit, int32_t rows,
                 int32_t *score, uint64_t *mask, const int64_t *q, int32_t qstride) {
    const int Ns = (c->N + 63) & ~63;
    const int rpb = 32;
    if (c->fits32) {
      constexpr int NPL = D <= 4 ? 4 : 2;
      dim3 grid(blocks(Ns, 256 * NPL), blocks(rows, rpb));
      hipLaunchKernelGGL((k_score32<D, NPL>), grid, dim3(256), 0, c->stream, sp, c->d.cap,
                         c->d.used, c->d.R, c->d.base, q, qstride, rows_unit, rows, rpb, score,
                         mask, Ns);
    } else {
      constexpr int NPL = D <= 4 ? 2 : 1;
      dim3 grid(blocks(Ns, 256 * NPL), blocks(rows, rpb));
      hipLaunchKernelGGL((k_score<D, NPL>), grid, dim3(256), 0, c->stream, sp, c->d.cap,
                         c->d.used, c->d.R, c->d.base, q, qstride, rows_unit, rows, rpb, score,
                         mask, Ns);
    }
    KP_HIP(hipGetLastError());
    return KP_OK;
  }
};

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

int launch_score(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit, int32_t rows,
                 int32_t *score, uint64_t *mask, const int64_t *q, int32_t qstride) {
  if (rows <= 0 || c->N == 0) return KP_OK;
  return dispatch_D<ScoreL>(c->D, c, sp, rows_unit, rows, score, mask, q, qstride);
}

int launch_select(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit, int32_t rows,
                  const int32_t *score, int32_t *cand) {
  if (rows <= 0) return KP_OK;
  const int Ns = (c->N + 63) & ~63;
  dim3 grid(rows), blk(256);  // one workgroup per row
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

// active units of [lo, hi) in rank order -> act_local; count to host
int launch_active(kp_ctx *c, int32_t lo, int32_t hi, int32_t *A_host) {
  *A_host = 0;
  const int32_t n = hi - lo;
  if (n <= 0) return KP_OK;
  int32_t *flag = c->d.flag;
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

int launch_unpack_exchange(kp_ctx *c, int32_t world, int32_t Umax, int32_t K) {
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
