// kp_score.hip — gfx950 (CDNA4) filter+score, top-K select and round bookkeeping.
//
// Every kernel implements one step of DESIGN.md §2 bit-exactly (integer
// arithmetic only; the CPU restatement is oracle/kp_oracle.c). The path is
// integer compare/select/reduce, so no MFMA: what matters is coalesced HBM
// streaming (score matrix stores, row re-reads), keeping the node tile in
// VGPRs across job rows, and 64-lane wave ballots / shuffles for the masks,
// argmax and prefix sums.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "kp_device.hpp"
#include "kp_internal.hpp"

namespace kp {
namespace {
using namespace dev;

// ---------------------------------------------------------------------------
// node prep: exact-division tables (div_prep) and the LeastAllocated base
// ---------------------------------------------------------------------------
__global__ void k_prep_nodes(const int64_t *__restrict__ cap, uint32_t *__restrict__ R32,
                             uint32_t *__restrict__ K32, int64_t *__restrict__ base, int32_t N,
                             int32_t D, int32_t S, int32_t least, ScoreParams sp) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  int64_t b = 0;
  for (int d = 0; d < D; ++d) {
    const int64_t c = cap[(int64_t)d * N + n];
    uint32_t r = 0, k = 0;
    if (c < ((int64_t)1 << 32)) div_prep((uint64_t)c, (uint32_t)S, r, k);
    R32[(int64_t)d * N + n] = r;
    K32[(int64_t)d * N + n] = k;
    if (c > 0) b += (int64_t)sp.w[d] * S;
  }
  base[n] = least ? b : 0;
}

// ---------------------------------------------------------------------------
// filter + score (materialised), 64-bit path (some cap or request >= 2^32).
// One 256-thread workgroup owns a tile of 4 waves x 64 lanes x NPL nodes; the
// tile's cap/used/R stay in VGPRs while the workgroup streams
// `rows_per_block` job rows past it: per row the request is wave-uniform,
// each lane stores NPL int32 scores and the wave ballots the feasibility bits
// straight into the row's mask words.
// Row stride of score/mask = Ns = round_up(N, 64); padding is infeasible.
// ---------------------------------------------------------------------------
// The grid of a device-driven round is sized by a bound on its rows (the
// previous round's count); the actual count (*rows_dev) is spread over every
// launched row block, at least min_rpb rows each, so a shrunken round still
// fills the chip instead of leaving most blocks idle and the rest long.
// rows_per_block only shrinks (the LDS request stage stays in bounds) and
// gridDim.y * rpb >= rows holds either way.
template <int D, int NPL>
__global__ __launch_bounds__(256) void k_score(ScoreParams sp,
                                               const int64_t *__restrict__ cap,
                                               const int64_t *__restrict__ used,
                                               const int32_t *__restrict__ topo,
                                               const int32_t *__restrict__ perm,
                                               const int64_t *__restrict__ q, int32_t qstride,
                                               const int32_t *__restrict__ uaff,
                                               const int32_t *__restrict__ rows_unit,
                                               int32_t rows, int32_t rows_per_block,
                                               int32_t min_rpb, int32_t *__restrict__ score,
                                               uint64_t *__restrict__ mask, int32_t Ns,
                                               const int32_t *__restrict__ rows_dev) {
  if (rows_dev) fit_rows(*rows_dev, min_rpb, rows, rows_per_block);
  if ((int)blockIdx.y * rows_per_block >= rows) return;  // block-uniform
  const int N = sp.N;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile0 = blockIdx.x * (256 * NPL) + wave * (64 * NPL);
  int64_t c_[NPL][D], u_[NPL][D];
  int32_t t_[NPL];
  bool v_[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int n = tile0 + k * 64 + lane;  // column; its node is perm[n] (canonical order)
    v_[k] = n < N;
    const int nn = v_[k] ? (perm ? perm[n] : n) : 0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      c_[k][d] = cap[(int64_t)d * N + nn];
      u_[k][d] = used[(int64_t)d * N + nn];
    }
    t_[k] = topo[nn];
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
    const int32_t af = uaff[unit];
    int32_t *srow = score + (int64_t)r * Ns;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int n = tile0 + k * 64 + lane;
      int64_t s = score_at<D>(sp, qq, c_[k], u_[k], t_[k], af);
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
// (then used+q <= cap < 2^32 on every feasible pair). Same result bit for bit
// as the 64-bit path: the exact division of div_prep (kp_device.hpp), whose
// C and E modes run on full-rate 24-bit multiplies only.
//
// Layout: lane l of wave w owns the NPL CONSECUTIVE nodes tile0 + NPL*l .., so a
// row's scores leave as one 16-B store per lane (1 KiB per wave instruction,
// whole 128-B lines). The 4 per-k ballots are bit-interleaved into the row's
// 4 mask words (word i bit 4j+k = ballot_k bit 16i+j). The requests of the
// workgroup's rows are gathered into LDS once, so the rows_unit -> q load
// chain is paid per workgroup, not per row.
__device__ __forceinline__ uint64_t spread4_16(uint64_t x) {
  // bit j of a 16-bit value -> bit 4j
  x &= 0xFFFFull;
  x = (x | (x << 24)) & 0x000000FF000000FFull;
  x = (x | (x << 12)) & 0x000F000F000F000Full;
  x = (x | (x << 6)) & 0x0303030303030303ull;
  x = (x | (x << 3)) & 0x1111111111111111ull;
  return x;
}

constexpr int kScoreMaxRows = 128;  // rows per workgroup (LDS request stage)

// v_mul_u32_u24 as written: the compiler otherwise fuses the 24-bit product
// with the mulhi sum into a (much slower) v_mad_u64_u32
__device__ __forceinline__ uint32_t mul_u24(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}


// Round-start pack of the node table into the 32-bit form k_score32 /
// k_score_topk consume, column i holding node perm[i] (the canonical order:
// nodes sorted by their capacity vector; identity for
// kp_score) or colnode[i] (the fused solve's class-aligned layout). u32 SoA
// planes [5*d + {0: free, 1: cap, 2: a, 3: R, 4: K}][P] where u*S (+ c - 1
// for LeastAllocated's ceiling) = A*c + a and (R, K) = div_prep(c), then the
// LeastAllocated base, the topo domain and WA = sum_d w_d*A_d in planes 5D,
// 5D+1, 5D+2; padding columns are zero and masked. One 8- or 16-B load per
// lane and plane fetches a lane's consecutive columns. The usage planes (free,
// a, WA) change every round; the capacity planes (cap, R, K, base, topo) only
// with the layout or the node table, so they are written when `full` is set.
// A = floor(u*S / c) through the node's division table (R32, K32 of
// k_prep_nodes: no 64-bit division per node and round).
template <int D>
__device__ __forceinline__ void pack_node(const int64_t *__restrict__ cap,
                                          const int64_t *__restrict__ used,
                                          const uint32_t *__restrict__ R32,
                                          const uint32_t *__restrict__ K32,
                                          const int64_t *__restrict__ base,
                                          const int32_t *__restrict__ topo,
                                          const int32_t *__restrict__ perm,
                                          const int32_t *__restrict__ colnode, int32_t N,
                                          int32_t P, bool full, const ScoreParams &sp,
                                          uint32_t *__restrict__ np, int i,
                                          const uint32_t *__restrict__ ncls) {
  // colnode: column -> node, -1 = padding; the free plane of dim 0 then holds
  // free + 1 (0 on padding), so that the fused kernel's fit test also rejects
  // padding columns
  const int cn = colnode ? colnode[i] : 0;
  const bool v = colnode ? cn >= 0 : i < N;
  const int n = !v ? 0 : colnode ? cn : perm ? perm[i] : i;
  const uint32_t plus1 = colnode && v ? 1u : 0u;
  const uint32_t S = (uint32_t)sp.S;
  uint32_t wa = 0;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const int64_t j = (int64_t)d * N + n;
    const uint32_t cc = v ? (uint32_t)cap[j] : 0u;
    const uint32_t uu = v ? (uint32_t)used[j] : 0u;
    const uint32_t R = v ? R32[j] : 0u, K = v ? K32[j] : (1u | kDivE);
    uint32_t A = 0, a = 0;
    if (cc > 0) {
      bool nz;
      const uint32_t t = div_floor32(uu, cc, R, K & 63u, S, nz);
      const uint32_t r = (uint32_t)((uint64_t)uu * S - (uint64_t)t * cc);
      if (sp.most_allocated) {
        A = t;
        a = r;
      } else {  // (u*S + c - 1) = A*c + a
        A = t + (nz ? 1u : 0u);
        a = nz ? r - 1u : cc - 1u;
      }
    }
    wa += (uint32_t)sp.w[d] * A;
    np[(int64_t)(kPlanes * d + 0) * P + i] = (cc - uu) + (d == 0 ? plus1 : 0u);
    np[(int64_t)(kPlanes * d + 2) * P + i] = a;
    if (full) {
      np[(int64_t)(kPlanes * d + 1) * P + i] = cc;
      np[(int64_t)(kPlanes * d + 3) * P + i] = R;
      np[(int64_t)(kPlanes * d + 4) * P + i] = K;
    }
  }
  if (full) {
    np[(int64_t)(kPlanes * D) * P + i] = v ? (uint32_t)base[n] : 0u;
    np[(int64_t)(kPlanes * D + 1) * P + i] = v ? (uint32_t)topo[n] : 0xFFFFFFFFu;
    // capacity class (k_score32's class form; padding: class 0, masked by N)
    np[(int64_t)(kPlanes * D + 3) * P + i] = v && ncls ? ncls[n] : 0u;
  }
  np[(int64_t)(kPlanes * D + 2) * P + i] = wa;
}

// Round start, one launch: active-unit flags of [lo, hi) (input of the
// compaction) and, when P > 0, the 32-bit node planes of the usage the round
// scores against.
template <int D>
__global__ __launch_bounds__(256) void k_round_start(const int32_t *__restrict__ status,
                                                     int32_t lo, int32_t hi,
                                                     int32_t *__restrict__ flag,
                                                     const int64_t *__restrict__ cap,
                                                     const int64_t *__restrict__ used,
                                                     const uint32_t *__restrict__ R32,
                                                     const uint32_t *__restrict__ K32,
                                                     const int64_t *__restrict__ base,
                                                     const int32_t *__restrict__ topo,
                                                     const int32_t *__restrict__ perm,
                                                     const int32_t *__restrict__ colnode, int32_t N,
                                                     int32_t P, int32_t full, ScoreParams sp,
                                                     uint32_t *__restrict__ np,
                                                     const uint32_t *__restrict__ ncls) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < hi - lo) flag[i] = status[lo + i] == kActive ? 1 : 0;
  if (i < P)
    pack_node<D>(cap, used, R32, K32, base, topo, perm, colnode, N, P, full != 0, sp, np, i, ncls);
}

// bit j of a 32-bit value -> bit 2j
__device__ __forceinline__ uint64_t spread2_32(uint64_t x) {
  x &= 0xFFFFFFFFull;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x << 2)) & 0x3333333333333333ull;
  x = (x | (x << 1)) & 0x5555555555555555ull;
  return x;
}

template <int NPL>
struct Vec;  // NPL consecutive u32 per lane: one 8- or 16-B access
template <>
struct Vec<2> {
  using T = uint2;
  static __device__ __forceinline__ uint32_t at(const T &v, int k) { return k ? v.y : v.x; }
};
template <>
struct Vec<4> {
  using T = uint4;
  static __device__ __forceinline__ uint32_t at(const T &v, int k) {
    return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
  }
};

// Row loop of a wave whose columns all have the same capacity in every dim
// (the canonical node order groups equal capacity vectors, so on a cluster
// of a few node shapes almost every wave qualifies). With u*S = A*c + a per
// node (pack) and q*S = Q*c + rho per row, floor((u+q)*S / c) =
// A + Q + [a >= c - rho]: a pair costs a compare and a select per dim. The
// weighted sums of the A's (WA) come per node from the pack, the per-row
// thresholds c - rho and the weighted sum of the Q's (WQ) from the
// workgroup's staging step (sx: one row of thresholds per wave, computed once
// by one thread, not by every lane).
constexpr uint32_t kRowNoFit = 0x80000000u;  // WQ word flag: no column of the wave fits the row

template <int D, bool MOST, int NPL>
__device__ __forceinline__ void score_rows_uniform(
    const ScoreParams &sp, const uint32_t (&sq)[kScoreMaxRows][D + 2],
    const uint32_t (&sx)[kScoreMaxRows][D + 1], int r0, int r1, const uint32_t (&f_)[NPL][D],
    const uint32_t (&a_)[NPL][D], const int32_t (&wa_)[NPL], const uint32_t (&fg_)[NPL],
    const uint32_t (&tp_)[NPL], const int32_t (&b_)[NPL], int32_t *__restrict__ score,
    uint64_t *__restrict__ mask, int32_t Ns, int tile0, int nb, int lane) {
  const int words = Ns >> 6;
  const bool store_ok = nb < Ns;
  const int32_t wfit = sp.w_gpu_fit, waff = sp.w_affinity;
  for (int r = r0; r < r1; ++r) {
    uint32_t qq[D], thr[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      qq[d] = sq[r - r0][d];
      thr[d] = sx[r - r0][d];
    }
    const uint32_t qg = sq[r - r0][D], af = sq[r - r0][D + 1];
    const uint32_t wqw = sx[r - r0][D];
    const bool row_ok = !(wqw & kRowNoFit);
    const int32_t wq = (int32_t)(wqw & ~kRowNoFit);
    int32_t sv[NPL];
    bool fits[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      bool ft = row_ok;
      int32_t acc = wa_[k] + wq;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        ft &= qq[d] <= f_[k][d];
        acc += a_[k][d] >= thr[d] ? sp.w[d] : 0;
      }
      // GPU-topology fit: the job takes exactly the node's free GPUs;
      // CacheStrategy shared: the node is in the job's affinity domain
      const int32_t bonus = ((qg != 0u && fg_[k] == qg) ? wfit : 0) + (tp_[k] == af ? waff : 0);
      const int32_t sc = (MOST ? acc : b_[k] - acc) + bonus;
      fits[k] = ft;
      sv[k] = ft ? sc : KP_SCORE_INFEASIBLE;
    }
    if (score && store_ok) {
      if constexpr (NPL == 4)
        *reinterpret_cast<int4 *>(score + (int64_t)r * Ns + nb) =
            make_int4(sv[0], sv[1], sv[2], sv[3]);
      else
        *reinterpret_cast<int2 *>(score + (int64_t)r * Ns + nb) = make_int2(sv[0], sv[1]);
    }
    if (mask) {
      uint64_t bal[NPL];
#pragma unroll
      for (int k = 0; k < NPL; ++k) bal[k] = __ballot(fits[k]);
      if (lane < NPL && tile0 + 64 * lane < Ns) {
        uint64_t wd = 0;
        if constexpr (NPL == 4) {
          const int sh = 16 * lane;
          wd = spread4_16(bal[0] >> sh) | (spread4_16(bal[1] >> sh) << 1) |
               (spread4_16(bal[2] >> sh) << 2) | (spread4_16(bal[3] >> sh) << 3);
        } else {
          const int sh = 32 * lane;
          wd = spread2_32(bal[0] >> sh) | (spread2_32(bal[1] >> sh) << 1);
        }
        mask[(int64_t)r * words + (tile0 >> 6) + lane] = wd;
      }
    }
  }
}

// The row loop of k_score32 for a wave with mixed capacities: per row the
// nodes' (c, R, K) planes are re-read (after a compiler memory barrier, so
// they are not hoisted into registers), and each dim takes the full-rate
// 24-bit form or, if a node of the wave needs it, the 64-bit form.
template <int D, bool MOST, int NPL>
__device__ __forceinline__ void score_rows_mixed(
    const ScoreParams &sp, const uint32_t (&sq)[kScoreMaxRows][D + 2], int r0, int r1,
    const typename Vec<NPL>::T *__restrict__ pv, int64_t PV, int64_t iv,
    const uint32_t (&f_)[NPL][D], const uint32_t (&fg_)[NPL], const uint32_t (&tp_)[NPL],
    const int32_t (&b_)[NPL], const bool (&v_)[NPL], int32_t *__restrict__ score,
    uint64_t *__restrict__ mask, int32_t Ns, int tile0, int nb, int lane) {
  using V = Vec<NPL>;
  const int words = Ns >> 6;
  const bool store_ok = nb < Ns;
  const int32_t wfit = sp.w_gpu_fit, waff = sp.w_affinity;
  const uint32_t S = (uint32_t)sp.S;
  for (int r = r0; r < r1; ++r) {
    asm volatile("" ::: "memory");
    uint32_t qq[D];
#pragma unroll
    for (int d = 0; d < D; ++d) qq[d] = sq[r - r0][d];
    const uint32_t qg = sq[r - r0][D], af = sq[r - r0][D + 1];
    bool fits[NPL];
    int32_t acc[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      fits[k] = v_[k];
      acc[k] = 0;
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const typename V::T pc = pv[(kPlanes * d + 1) * PV + iv], pr = pv[(kPlanes * d + 3) * PV + iv],
                          pk = pv[(kPlanes * d + 4) * PV + iv];
      uint32_t wide = 0, nonE = 0;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        wide |= V::at(pk, k) & kDivW;
        nonE |= (V::at(pk, k) & kDivE) ^ kDivE;
      }
      const bool anyW = __ballot(wide != 0) != 0, allE = __ballot(nonE != 0) == 0;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        const uint32_t c = V::at(pc, k), cc = c ? c : 1u, R = V::at(pr, k), kk = V::at(pk, k) & 63u;
        fits[k] &= qq[d] <= f_[k][d];
        // infeasible pairs may compute garbage (operands past 24 bits,
        // wrapped sums): masked below
        const uint32_t x = (c - f_[k][d]) + qq[d];
        uint32_t util;
        if (anyW) {
          bool nz;
          const uint32_t t = div_floor32(x, cc, R, kk, S, nz);
          util = MOST ? t : t + (nz ? 1u : 0u);
        } else {
          uint32_t t = mul_u24(x, R) >> kk;
          if (MOST && allE) {
            util = t;
          } else {
            // r = x*S - t*c lies in [0, 2c) and c < 2^24: exact mod 2^32
            uint32_t rr = mul_u24(x, S) - mul_u24(t, cc);
            const bool up = rr >= cc;
            t += up ? 1u : 0u;
            rr -= up ? cc : 0u;
            util = MOST ? t : t + (rr != 0u ? 1u : 0u);
          }
        }
        acc[k] += (int32_t)__umul24((uint32_t)sp.w[d], util);
      }
    }
    int32_t sv[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int32_t bonus = ((qg != 0u && fg_[k] == qg) ? wfit : 0) + (tp_[k] == af ? waff : 0);
      const int32_t s = (MOST ? acc[k] : b_[k] - acc[k]) + bonus;
      sv[k] = fits[k] ? s : KP_SCORE_INFEASIBLE;
    }
    if (score && store_ok) {
      if constexpr (NPL == 4)
        *reinterpret_cast<int4 *>(score + (int64_t)r * Ns + nb) =
            make_int4(sv[0], sv[1], sv[2], sv[3]);
      else
        *reinterpret_cast<int2 *>(score + (int64_t)r * Ns + nb) = make_int2(sv[0], sv[1]);
    }
    if (mask) {  // wave-uniform: the solve passes no mask (the -1 sentinel is the filter)
      uint64_t bal[NPL];
#pragma unroll
      for (int k = 0; k < NPL; ++k) bal[k] = __ballot(fits[k]);
      // word i of the wave's tile: bit NPL*j + k = ballot_k bit (64/NPL)*i + j
      if (lane < NPL && tile0 + 64 * lane < Ns) {
        uint64_t wd = 0;
        if constexpr (NPL == 4) {
          const int sh = 16 * lane;
          wd = spread4_16(bal[0] >> sh) | (spread4_16(bal[1] >> sh) << 1) |
               (spread4_16(bal[2] >> sh) << 2) | (spread4_16(bal[3] >> sh) << 3);
        } else {
          const int sh = 32 * lane;
          wd = spread2_32(bal[0] >> sh) | (spread2_32(bal[1] >> sh) << 1);
        }
        mask[(int64_t)r * words + (tile0 >> 6) + lane] = wd;
      }
    }
  }
}

template <int D, bool MOST, int NPL>
__global__ __launch_bounds__(256) void k_score32(ScoreParams sp,
                                                 const uint32_t *__restrict__ np, int32_t P,
                                                 const int64_t *__restrict__ q, int32_t qstride,
                                                 const int32_t *__restrict__ uaff,
                                                 const int32_t *__restrict__ rows_unit,
                                                 int32_t rows, int32_t rows_per_block,
                                                 int32_t min_rpb, int32_t *__restrict__ score,
                                                 uint64_t *__restrict__ mask, int32_t Ns,
                                                 const int32_t *__restrict__ rows_dev) {
  static_assert(NPL == 2 || NPL == 4, "2 or 4 nodes per lane");
  using V = Vec<NPL>;
  if (rows_dev) fit_rows(*rows_dev, min_rpb, rows, rows_per_block);
  if ((int)blockIdx.y * rows_per_block >= rows) return;  // block-uniform
  // per row: the D requests, the request in the GPU dim (0 if none) and the
  // affinity domain (0xFFFFFFFF = none: no node has that domain)
  __shared__ uint32_t sq[kScoreMaxRows][D + 2];
  // per wave: its uniform capacities ([D] = 1 if the wave is uniform) and,
  // per row, the thresholds c - rho per dim and WQ (flag kRowNoFit)
  __shared__ uint32_t scu[4][D + 1];
  __shared__ uint32_t sx[4][kScoreMaxRows][D + 1];
  const int N = sp.N;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile0 = blockIdx.x * (256 * NPL) + wave * (64 * NPL);
  const int nb = tile0 + lane * NPL;  // first of this lane's NPL columns
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  const int g = sp.gpu_dim;
  for (int i = threadIdx.x; i < (r1 - r0) * (D + 2); i += blockDim.x) {
    const int rr = i / (D + 2), d = i % (D + 2);
    const int32_t unit = rows_unit[r0 + rr];
    uint32_t v;
    if (d == D + 1) {
      v = (uint32_t)uaff[unit];
    } else {
      const int dd = d < D ? d : g;
      v = dd >= 0 ? (uint32_t)q[(int64_t)dd * qstride + unit] : 0u;
    }
    sq[rr][d] = v;
  }
  const typename V::T *pv = reinterpret_cast<const typename V::T *>(np);
  const int64_t PV = P / NPL, iv = nb / NPL;  // P % 1024 == 0: the tile is inside
  uint32_t f_[NPL][D], a_[NPL][D], fg_[NPL], tp_[NPL];
  int32_t b_[NPL], wa_[NPL];
  bool v_[NPL];
  uint32_t cu[D];
  bool uni = true;
  {
    typename V::T pf[D], pc[D], pa[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      pf[d] = pv[(kPlanes * d + 0) * PV + iv];
      pc[d] = pv[(kPlanes * d + 1) * PV + iv];
      pa[d] = pv[(kPlanes * d + 2) * PV + iv];
    }
    const typename V::T pb = pv[(kPlanes * D) * PV + iv], pt = pv[(kPlanes * D + 1) * PV + iv],
                        pw = pv[(kPlanes * D + 2) * PV + iv];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      v_[k] = nb + k < N;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        f_[k][d] = V::at(pf[d], k);
        a_[k][d] = V::at(pa[d], k);
      }
      b_[k] = (int32_t)V::at(pb, k);
      tp_[k] = V::at(pt, k);
      wa_[k] = (int32_t)V::at(pw, k);
      fg_[k] = 0xFFFFFFFFu;  // free GPUs: never equal to a request when there is no GPU dim
#pragma unroll
      for (int d = 0; d < D; ++d)
        if (d == g) fg_[k] = f_[k][d];
    }
    // one capacity per dim for the whole wave (and no padding column)?
#pragma unroll
    for (int d = 0; d < D; ++d) {
      cu[d] = __builtin_amdgcn_readfirstlane(V::at(pc[d], 0));
      bool differ = false;
#pragma unroll
      for (int k = 0; k < NPL; ++k) differ |= !v_[k] || V::at(pc[d], k) != cu[d];
      uni &= __ballot(differ) == 0;
    }
    if (lane == 0) {
#pragma unroll
      for (int d = 0; d < D; ++d) scu[wave][d] = cu[d];
      scu[wave][D] = uni && tile0 < Ns ? 1u : 0u;
    }
  }
  __syncthreads();  // requests and the waves' capacities staged
  {
    // per (uniform wave, row): q*S = Q*c + rho in every dim, one thread each
    const int nr = r1 - r0;
    const uint64_t S = (uint64_t)sp.S;
    for (int t = threadIdx.x; t < 4 * nr; t += blockDim.x) {
      const int w = t / nr, rr = t - w * nr;
      if (!scu[w][D]) continue;
      uint32_t wq = 0;
      bool ok = true;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const uint32_t c = scu[w][d], qd = sq[rr][d];
        uint32_t thr = 0xFFFFFFFFu;  // cap-0 dim: contributes 0, fits only q = 0
        if (c == 0u) {
          ok &= qd == 0u;
        } else if (qd > c) {
          ok = false;
        } else {
          uint64_t Q, rho;
          udivmod_uniform((uint64_t)qd * S, c, Q, rho);
          thr = c - (uint32_t)rho;  // in (0, c]: carry iff a >= thr
          wq += (uint32_t)sp.w[d] * (uint32_t)Q;
        }
        sx[w][rr][d] = thr;
      }
      sx[w][rr][D] = ok ? wq : kRowNoFit;
    }
  }
  __syncthreads();
  if (tile0 >= Ns) return;  // wave-uniform, after the last barrier
#ifdef KP_SCORE_UNIFORM_ONLY_TIMING  // A/B timing of the uniform path alone (wrong on boundary waves)
  uni = true;
#endif
  if (uni) {
    score_rows_uniform<D, MOST, NPL>(sp, sq, sx[wave], r0, r1, f_, a_, wa_, fg_, tp_, b_, score,
                                     mask, Ns, tile0, nb, lane);
    return;
  }
  // mixed capacities (a class boundary, padding, or an unclustered cluster):
  // the per-node division of div_prep. Such waves are few on a clustered
  // node table, so their node operands are re-read per row (L1/L2) rather
  // than held in registers the uniform path does not need.
#ifndef KP_SCORE_UNIFORM_ONLY_TIMING
  score_rows_mixed<D, MOST, NPL>(sp, sq, r0, r1, pv, PV, iv, f_, fg_, tp_, b_, v_, score, mask, Ns,
                                 tile0, nb, lane);
#endif
}

// Class form of k_score32: node tables with at most kScoreClasses distinct
// capacity vectors (a cluster of a few node shapes: every BASELINE config).
// The workgroup stages, per (row, class), the thresholds c - rho and WQ
// (q*S = Q*c + rho: one exact division per row, class and dim) and every pair
// takes score_rows_uniform's compare-and-select form with its node's class
// (the class plane of the pack, kPlanes*D + 3) — no per-pair division on any
// wave. kp_score returns node order, where the classes interleave, so the
// uniform-wave test of k_score32 fails on almost every wave there.
// Columns are STRIDED over the lanes: a wave owns 256 columns, lane l the
// columns base + 64k + l (k < 4), so each ballot of the fit flags IS a mask
// word (no bit interleaving per row: that per-row chain cost as much as the
// score stores, tools/score_dev_time.py) and every store instruction writes
// 256 contiguous bytes. A workgroup's 1,024 columns are 16 mask words, one
// 128-B line when the row stride is a multiple of 16 words (kp_score_dev).
// Rows are written with the given strides (the internal chunk, or the
// caller's device buffers of kp_score_dev).
constexpr int kScoreClsRows = 64;  // rows per workgroup (LDS: rows x classes x record)
constexpr int kClsCols = 4;        // columns per lane

// a kernel-argument (SGPR) value copied into a VGPR once: a select with a
// compare mask in an SGPR pair may not read a second SGPR (one scalar operand
// per VALU instruction on gfx950), so weights kept in SGPRs cost a v_mov per use
__device__ __forceinline__ int32_t in_vgpr(int32_t s) {
  int32_t v;
  asm("v_mov_b32 %0, %1" : "=v"(v) : "s"(s));
  return v;
}

template <int D, bool MOST, bool WS, bool WM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 6))) void k_score32c(
    ScoreParams sp, const uint32_t *__restrict__ np, int32_t P, const int64_t *__restrict__ q,
    int32_t qstride, const int32_t *__restrict__ uaff, const int32_t *__restrict__ rows_unit,
    int32_t rows, int32_t rows_per_block, int32_t min_rpb, int32_t *__restrict__ score,
    int64_t sstride, uint64_t *__restrict__ mask, int64_t mstride, int32_t Ns,
    const int32_t *__restrict__ rows_dev, const uint32_t *__restrict__ ccap, int32_t ncl) {
  constexpr int NC = kClsCols;
  constexpr int RW = (D + 1 + 3) & ~3;  // per (row, class): D thresholds + WQ, whole 16-B reads
  if (rows_dev) fit_rows(*rows_dev, min_rpb, rows, rows_per_block);
  if ((int)blockIdx.y * rows_per_block >= rows) return;  // block-uniform
  // per row: the D requests, the GPU-dim request (0 if none) and the affinity domain
  __shared__ uint32_t sq[kScoreClsRows][D + 2];
  __shared__ __attribute__((aligned(16))) uint32_t sx[kScoreClsRows][kScoreClasses][RW];
  const int N = sp.N;
  // wave index through readfirstlane: the compiler then knows that every
  // per-wave quantity (tile0, the column groups, the row pointer) is uniform
  // and branches on them with scalar branches (full EXEC: a ballot IS the
  // fit mask, no re-materialisation)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile0 = blockIdx.x * (256 * NC) + wave * (64 * NC);  // this wave's first column
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  const int nr = r1 - r0;
  const int g = sp.gpu_dim;
  for (int i = threadIdx.x; i < nr * (D + 2); i += blockDim.x) {
    const int rr = i / (D + 2), d = i % (D + 2);
    const int32_t unit = rows_unit[r0 + rr];
    uint32_t v;
    if (d == D + 1) {
      v = (uint32_t)uaff[unit];
    } else if (d == D) {
      v = g >= 0 ? (uint32_t)q[(int64_t)g * qstride + unit] : 0u;
    } else {
      v = (uint32_t)q[(int64_t)d * qstride + unit];
    }
    sq[rr][d] = v;
  }
  // the lane's columns tile0 + 64k + lane (P % 1024 == 0: inside the planes)
  uint32_t f_[NC][D], a_[NC][D], fg_[NC], tp_[NC], xo_[NC];
  int32_t b_[NC], wa_[NC];
  bool v_[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int64_t col = tile0 + 64 * k + lane;
    v_[k] = col < N;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      f_[k][d] = np[(int64_t)(kPlanes * d + 0) * P + col];
      a_[k][d] = np[(int64_t)(kPlanes * d + 2) * P + col];
    }
    b_[k] = MOST ? 0 : (int32_t)np[(int64_t)(kPlanes * D) * P + col];
    tp_[k] = np[(int64_t)(kPlanes * D + 1) * P + col];
    wa_[k] = (int32_t)np[(int64_t)(kPlanes * D + 2) * P + col];
    // byte offset of the column's class record in a row of sx
    xo_[k] = min(np[(int64_t)(kPlanes * D + 3) * P + col], (uint32_t)(kScoreClasses - 1)) * (RW * 4);
    fg_[k] = 0xFFFFFFFFu;  // free GPUs: never equal to a request when there is no GPU dim
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (d == g) fg_[k] = f_[k][d];
  }
  __syncthreads();  // requests staged
  {
    // per (row, class): q*S = Q*c + rho in every dim, one thread each
    const uint64_t S = (uint64_t)sp.S;
    for (int t = threadIdx.x; t < ncl * nr; t += blockDim.x) {
      const int k = t / nr, rr = t - k * nr;
      uint32_t wq = 0;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const uint32_t c = ccap[k * D + d], qd = sq[rr][d];
        // cap-0 dim: contributes 0 (fits only q = 0); q > c: fits no node of
        // the class — both rejected by the per-node fit test q <= free <= c
        uint32_t thr = 0xFFFFFFFFu;
        if (c != 0u && qd <= c) {
          uint64_t Q, rho;
          udivmod_uniform((uint64_t)qd * S, c, Q, rho);
          thr = c - (uint32_t)rho;  // in (0, c]: carry iff a >= thr
          wq += (uint32_t)sp.w[d] * (uint32_t)Q;
        }
        sx[rr][k][d] = thr;
      }
      sx[rr][k][D] = wq;
    }
  }
  __syncthreads();
  if (tile0 >= Ns) return;  // wave-uniform, after the last barrier
  const int nk = min(NC, (Ns - tile0) >> 6);  // column groups inside the row stride
  int32_t w_[D];
#pragma unroll
  for (int d = 0; d < D; ++d) w_[d] = in_vgpr(sp.w[d]);
  const int32_t wfit = in_vgpr(sp.w_gpu_fit), waff = in_vgpr(sp.w_affinity);
  const char *sxb = reinterpret_cast<const char *>(&sx[0][0][0]);
  for (int r = r0; r < r1; ++r) {
    const int rr = r - r0;
    // the row's requests are wave-uniform: scalar operands of the compares
    uint32_t qq[D];
#pragma unroll
    for (int d = 0; d < D; ++d) qq[d] = __builtin_amdgcn_readfirstlane(sq[rr][d]);
    const uint32_t qg = __builtin_amdgcn_readfirstlane(sq[rr][D]);
    const uint32_t af = __builtin_amdgcn_readfirstlane(sq[rr][D + 1]);
    const int32_t wfit_r = qg != 0u ? wfit : 0;  // the bonus needs a GPU request
    // every class record of the row's columns first (LDS broadcasts: the lanes
    // of one class read one address), then the arithmetic
    uint32_t x[NC][RW];
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const uint4 *rec = reinterpret_cast<const uint4 *>(sxb + rr * (kScoreClasses * RW * 4) + xo_[k]);
#pragma unroll
      for (int i = 0; i < RW / 4; ++i) {
        const uint4 t4 = rec[i];
        x[k][4 * i] = t4.x;
        x[k][4 * i + 1] = t4.y;
        x[k][4 * i + 2] = t4.z;
        x[k][4 * i + 3] = t4.w;
      }
    }
    int32_t *srow = WS ? score + (int64_t)r * sstride + tile0 : nullptr;  // wave-uniform
    // FULL: all NC column groups inside the row stride (every wave but the
    // last tile's), so the stores need no guard and the ballots stay in
    // SGPRs (a guarded store made the compiler re-materialise each mask
    // through a VGPR); HG / HA: the row has a GPU request / an affinity
    // domain — rows without skip those compares (scalar branches: qg and af
    // are SGPR values)
    auto body = [&](auto full_, auto hg_, auto ha_) {
      constexpr bool FULL = decltype(full_)::value, HG = decltype(hg_)::value,
                     HA = decltype(ha_)::value;
      uint64_t word[NC];
#pragma unroll
      for (int k = 0; k < NC; ++k) {
        bool ft = v_[k];
        int32_t acc = wa_[k] + (int32_t)x[k][D];
#pragma unroll
        for (int d = 0; d < D; ++d) {
          ft &= qq[d] <= f_[k][d];
          acc += a_[k][d] >= x[k][d] ? w_[d] : 0;
        }
        // GPU-topology fit (the job takes exactly the node's free GPUs) and
        // the CacheStrategy=shared affinity domain
        int32_t bonus = 0;
        if constexpr (HG) bonus += fg_[k] == qg ? wfit_r : 0;
        if constexpr (HA) bonus += tp_[k] == af ? waff : 0;
        const int32_t sc = (MOST ? acc : b_[k] - acc) + bonus;
        word[k] = __ballot(ft);  // columns tile0 + 64k .. + 63: mask word (tile0 >> 6) + k
        // the matrix is streamed out once: non-temporal stores (1.10-1.14 ->
        // 1.01-1.04 ms per config #3 call; the mask's 32-B pieces stay cached)
        if (WS && (FULL || k < nk)) __builtin_nontemporal_store(ft ? sc : KP_SCORE_INFEASIBLE, srow + 64 * k + lane);
      }
      if (WM) {  // lane k < nk stores word k (scalar values written into lanes), in
                 // the variant's own block: the masks never leave their SGPRs
        // one asm block led by s_nop 4: the compiler's hazard recognizer
        // does not look inside inline asm, and a ballot's SGPRs written by
        // the VALU just before a v_writelane reads them came out stale
        static_assert(NC == 4, "the writelane block below covers 4 words");
        uint32_t lo = 0u, hi = 0u;
        asm volatile(
            "s_nop 4\n\t"
            "v_writelane_b32 %0, %2, 0\n\tv_writelane_b32 %1, %3, 0\n\t"
            "v_writelane_b32 %0, %4, 1\n\tv_writelane_b32 %1, %5, 1\n\t"
            "v_writelane_b32 %0, %6, 2\n\tv_writelane_b32 %1, %7, 2\n\t"
            "v_writelane_b32 %0, %8, 3\n\tv_writelane_b32 %1, %9, 3"
            : "+v"(lo), "+v"(hi)
            : "s"((uint32_t)word[0]), "s"((uint32_t)(word[0] >> 32)), "s"((uint32_t)word[1]),
              "s"((uint32_t)(word[1] >> 32)), "s"((uint32_t)word[2]), "s"((uint32_t)(word[2] >> 32)),
              "s"((uint32_t)word[3]), "s"((uint32_t)(word[3] >> 32)));
        if (lane < nk) mask[(int64_t)r * mstride + (tile0 >> 6) + lane] = ((uint64_t)hi << 32) | lo;
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    const bool hg = wfit_r != 0, ha = (int32_t)af >= 0;
    if (nk == NC) {
      if (hg) {
        if (ha) body(T_{}, T_{}, T_{}); else body(T_{}, T_{}, F_{});
      } else {
        if (ha) body(T_{}, F_{}, T_{}); else body(T_{}, F_{}, F_{});
      }
    } else {
      body(F_{}, T_{}, T_{});
    }
  }
}

// ---------------------------------------------------------------------------
// Candidate keys (pack_key / key_node, kp_device.hpp)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// ---------------------------------------------------------------------------
// top-K select, threshold form (rows of up to 65536 nodes). One workgroup of
// BS threads per score row; the row is held in registers (V4 16-B loads per
// thread, all issued before any is consumed).
//  1. every thread's best key;
//  2. each wave sorts its 64 thread-bests (bitonic network over lane
//     shuffles); the K-th of them is a lower bound on the row's K-th key
//     (K distinct nodes reach it), so T = their max over the waves is one too;
//  3. keys >= T are appended to an LDS buffer (typically K..4K of them);
//  4. rank counting in LDS gives each survivor its exact position; ranks < K
//     are the candidates, best first.
// If more than `lds_cap` keys survive, T is raised to the K-th largest
// buffered key (again a valid bound: K distinct keys reach it; strictly larger
// than T since the buffer holds > K distinct keys >= T) and step 3 repeats.
// Exact for every input; bit-exact with oracle kpo_round_candidates.
// ---------------------------------------------------------------------------
constexpr int kSelLdsCap = 1024;

template <int V4, int BS>
__global__ __launch_bounds__(BS) void k_select_t(ScoreParams sp,
                                                 const int32_t *__restrict__ score, int32_t Ns,
                                                 const int32_t *__restrict__ rows_unit,
                                                 const uint32_t *__restrict__ salt, int32_t rows,
                                                 int32_t lds_cap, int32_t *__restrict__ cand,
                                                 const int32_t *__restrict__ rows_dev,
                                                 const int32_t *__restrict__ perm) {
  constexpr int NW = BS / 64;
  __shared__ uint64_t buf[kSelLdsCap];
  __shared__ uint64_t wth[NW];
  __shared__ uint64_t raised;
  __shared__ int cnt;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = blockIdx.x;
  if (row >= rows || (rows_dev && row >= *rows_dev)) return;  // block-uniform
  const int K = sp.n_cand;
  const int32_t unit = rows_unit[row];
  const uint32_t sl = sp.tie_rotated ? salt[unit] : 0u;
  const uint32_t mul = sp.tie_rotated ? kTieMul : 1u;
  const uint32_t inv = sp.tie_rotated ? kTieMulInv : 1u;
  const int4 *row4 = reinterpret_cast<const int4 *>(score + (int64_t)row * Ns);
  const int n4 = Ns >> 2;
  int4 v[V4];
#pragma unroll
  for (int t = 0; t < V4; ++t) {
    const int i = tid + BS * t;
    v[t] = i < n4 ? row4[i] : make_int4(-1, -1, -1, -1);
  }
  // tie keys advance by a constant per element: node 4*(tid + BS*t) + j has
  // tk = tk0 + t*step + j*mul (mod 2^32), so no per-element multiply
  const uint32_t tk0 = (uint32_t)(4 * tid) * mul + sl;
  const uint32_t step = (uint32_t)(4 * BS) * mul;
  const uint32_t m1 = mul, m2 = 2u * mul, m3 = 3u * mul;
  // 1. thread best: max score, then the smallest tie key among its holders
  int32_t smax = -1;
#pragma unroll
  for (int t = 0; t < V4; ++t) smax = max(smax, max(max(v[t].x, v[t].y), max(v[t].z, v[t].w)));
  uint32_t tkmin = 0xFFFFFFFFu;
#pragma unroll
  for (int t = 0; t < V4; ++t) {
    const uint32_t tk = tk0 + (uint32_t)t * step;
    tkmin = min(tkmin, v[t].x == smax ? tk : 0xFFFFFFFFu);
    tkmin = min(tkmin, v[t].y == smax ? tk + m1 : 0xFFFFFFFFu);
    tkmin = min(tkmin, v[t].z == smax ? tk + m2 : 0xFFFFFFFFu);
    tkmin = min(tkmin, v[t].w == smax ? tk + m3 : 0xFFFFFFFFu);
  }
  uint64_t x = smax >= 0 ? pack_key(smax, tkmin) : 0ull;
  // bitonic sort of the wave's 64 thread-bests, descending across lanes
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const uint64_t o = shfl_xor_u64(x, j);
      const bool take_max = ((lane & j) == 0) == ((lane & k) == 0);
      x = take_max ? umax64(x, o) : umin64(x, o);
    }
  }
  const uint64_t tw = (uint64_t)shfl_i64((int64_t)x, K - 1);
  if (lane == 0) wth[wave] = tw;
  if (tid == 0) cnt = 0;
  __syncthreads();
  uint64_t T = 1;  // every valid key has bit 63 set
#pragma unroll
  for (int w = 0; w < NW; ++w) T = umax64(T, wth[w]);
  int C;
  while (true) {
    // key >= T  <=>  s >= 0 and (s > Ts or (s == Ts and tk <= Tk)); T == 1
    // (no bound) maps to Ts = -1: every feasible entry
    const int32_t Ts = T == 1 ? -1 : (int32_t)((T >> 32) & 0x7FFFFFFFu);
    const uint32_t Tk = ~(uint32_t)T;
    // branch-free test of every held entry -> one bit each; the (rare)
    // survivors are then appended one at a time, re-reading their score
    constexpr int HW = (V4 + 15) / 16;  // 64-bit hit words (16 int4 = 64 entries each)
    uint64_t hits[HW];
#pragma unroll
    for (int hw = 0; hw < HW; ++hw) hits[hw] = 0;
#pragma unroll
    for (int t = 0; t < V4; ++t) {
      const int32_t sv[4] = {v[t].x, v[t].y, v[t].z, v[t].w};
      const uint32_t tk = tk0 + (uint32_t)t * step;
      const uint32_t tj[4] = {tk, tk + m1, tk + m2, tk + m3};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int32_t s = sv[j];
        const bool h = (s > Ts) | ((s == Ts) & (tj[j] <= Tk));
        hits[t >> 4] |= (uint64_t)(h & (s >= 0)) << (4 * (t & 15) + j);
      }
    }
#pragma unroll
    for (int hw = 0; hw < HW; ++hw)
    while (hits[hw]) {
      const int bpos = __ffsll((unsigned long long)hits[hw]) - 1;
      hits[hw] &= hits[hw] - 1;
      const int t = hw * 16 + (bpos >> 2), j = bpos & 3;
      const int32_t s = score[(int64_t)row * Ns + 4 * (tid + BS * t) + j];
      const uint32_t tk = tk0 + (uint32_t)t * step + (uint32_t)j * m1;
      const int p = atomicAdd(&cnt, 1);
      if (p < lds_cap) buf[p] = pack_key(s, tk);
    }
    __syncthreads();
    C = cnt;
    if (C <= lds_cap) break;  // block-uniform
    // overflow: raise T to the K-th largest buffered key
    for (int i = tid; i < lds_cap; i += BS) {
      const uint64_t ki = buf[i];
      int r = 0;
      for (int jj = 0; jj < lds_cap; ++jj) r += buf[jj] > ki ? 1 : 0;
      if (r == K - 1) raised = ki;
    }
    __syncthreads();
    T = raised;
    if (tid == 0) cnt = 0;
    __syncthreads();
  }
  for (int i = tid; i < C; i += BS) {
    const uint64_t ki = buf[i];
    int r = 0;
    for (int jj = 0; jj < C; ++jj) r += buf[jj] > ki ? 1 : 0;
    if (r < K) {  // column (canonical position) -> node
      const int32_t pos = key_node(ki, sl, inv);
      cand[(int64_t)row * K + r] = perm ? perm[pos] : pos;
    }
  }
  if (tid >= C && tid < K) cand[(int64_t)row * K + tid] = -1;
}

// ---------------------------------------------------------------------------
// top-K select, generic form (rows of any length): one 256-thread workgroup
// per row. Each lane keeps its own descending top-KC list over a strided slice
// of the row (16-B loads: 4 nodes per lane per step), then each wave merges
// its 64 lists K times with a butterfly max and wave 0 merges the 4 wave
// lists from LDS. Exact: every global top-K entry is in its lane's top-K.
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

template <int KC>
__global__ __launch_bounds__(256) void k_select(ScoreParams sp,
                                                const int32_t *__restrict__ score, int32_t Ns,
                                                const int32_t *__restrict__ rows_unit,
                                                const uint32_t *__restrict__ salt,
                                                int32_t rows, int32_t *__restrict__ cand,
                                                const int32_t *__restrict__ rows_dev,
                                                const int32_t *__restrict__ perm) {
  __shared__ uint64_t part[4][KC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = blockIdx.x;
  if (row >= rows || (rows_dev && row >= *rows_dev)) return;  // block-uniform
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
    if (lane == 0) {  // column (canonical position) -> node
      const int32_t pos = m != 0 ? key_node(m, sl, inv) : -1;
      cand[(int64_t)row * K + it] = pos < 0 ? -1 : perm ? perm[pos] : pos;
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
// per-unit salt of the rotated tie-break: fmix32(leader ^ seed)
__device__ __forceinline__ uint32_t fmix32_dev(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

__global__ void k_reset_units(int32_t *__restrict__ status, int32_t U,
                              int32_t *__restrict__ job_node, int32_t *__restrict__ job_score,
                              int32_t J, const int32_t *__restrict__ leader,
                              uint32_t *__restrict__ salt, uint32_t seed) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < U) {
    status[i] = kActive;
    salt[i] = fmix32_dev((uint32_t)leader[i] ^ seed);
  }
  if (i < J) {
    job_node[i] = -1;
    job_score[i] = KP_SCORE_NONE;
  }
}

__global__ void k_finalize(const int32_t *__restrict__ status, const int32_t *__restrict__ leader,
                           const int32_t *__restrict__ size, int32_t U,
                           int32_t *__restrict__ job_node, int32_t *__restrict__ job_score,
                           int32_t *__restrict__ job_status, const int32_t *__restrict__ pass_flag,
                           SolveStats *__restrict__ stats) {
  int u = blockIdx.x * blockDim.x + threadIdx.x;
  // the last round's productive passes (earlier rounds are counted when the
  // next round's index build clears the flags)
  if (u < 64 && pass_flag[u] != 0)
    atomicAdd(reinterpret_cast<unsigned long long *>(&stats->passes), 1ull);
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


// Candidate exchange blocks (multi-GPU): per rank a fixed-size
// block [count, (unit, K candidates) x B] so that every rank calls the same
// all-gather without knowing the counts on the host.
__global__ void k_pack(int32_t B, int32_t K, const int32_t *__restrict__ count,
                       const int32_t *__restrict__ act, const int32_t *__restrict__ cand,
                       int32_t *__restrict__ send) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t A = min(B, *count);
  if (t == 0) send[0] = A;
  if (t >= A) return;
  int32_t *dst = send + 1 + t * (K + 1);
  dst[0] = act[t];
  for (int k = 0; k < K; ++k) dst[1 + k] = cand[t * K + k];
}

// every rank's block -> the global (unit, candidates) list in rank order (=
// unit rank order: shards are contiguous) and its length in *total
__global__ void k_unpack(int32_t world, int32_t B, int32_t K, const int32_t *__restrict__ recv,
                         int32_t *__restrict__ act, int32_t *__restrict__ cand,
                         int32_t *__restrict__ total) {
  const int64_t per = 1 + (int64_t)B * (K + 1);
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int r = (int)(t / B), i = (int)(t % B);
  if (r >= world) return;
  int32_t dst = i, tot = 0;
  for (int k = 0; k < world; ++k) {
    const int32_t ck = recv[k * per];
    if (k < r) dst += ck;
    tot += ck;
  }
  if (t == 0) *total = tot;
  if (i >= recv[r * per]) return;
  const int32_t *src = recv + r * per + 1 + (int64_t)i * (K + 1);
  act[dst] = src[0];
  for (int k = 0; k < K; ++k) cand[(int64_t)dst * K + k] = src[1 + k];
}

// streaming churn: used[d][node[k]] += sign * delta[d*K + k] (int64 atomics,
// several deltas may hit one node), then a check of every touched entry
__global__ void k_delta_apply(int32_t K, int32_t N, int32_t D, const int32_t *__restrict__ node,
                              const int64_t *__restrict__ delta, int64_t sign,
                              int64_t *__restrict__ used) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)K * D) return;
  const int32_t d = (int32_t)(t / K), k = (int32_t)(t % K);
  const int64_t v = sign * delta[t];
  if (v != 0)
    atomicAdd(reinterpret_cast<unsigned long long *>(&used[(int64_t)d * N + node[k]]),
              (unsigned long long)v);
}

__global__ void k_delta_check(int32_t K, int32_t N, int32_t D, const int32_t *__restrict__ node,
                              const int64_t *__restrict__ cap, const int64_t *__restrict__ used,
                              int32_t *__restrict__ bad) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)K * D) return;
  const int32_t d = (int32_t)(t / K), k = (int32_t)(t % K);
  const int64_t i = (int64_t)d * N + node[k];
  const int64_t u = used[i];
  if (u < 0 || u > cap[i]) *bad = 1;
}

// Order-preserving compaction of the active-unit flags in ONE workgroup:
// out = [lo + i for i in [0, n) if flag[i]], *count = its length. Chunks of
// 1024 threads x 16 flags (four 16-B loads per thread), block scan of the
// thread counts, running carry between chunks. Replaces rocprim::select's
// lookback-state init + partition launches (2 kernels, ~13 us per round) for
// the round's few-ten-thousand units.
constexpr int kCompactBS = 1024, kCompactIPT = 16;
// FROM_STATUS: the flags are status[lo + i] == kActive, read straight from the
// unit status (k_round_begin); else the flag array of k_round_start
// The multi-workgroup form (k_compact_count + k_compact_multi: one chunk per
// workgroup, each starting at the sum of the earlier chunks' counts) covers
// any n in two launches; it replaced rocprim::select (lookback init +
// partition) in the compactions above the one-workgroup range and in
// kp_preempt's preemptor list.
constexpr int kCompactChunk = kCompactBS * kCompactIPT;
// FROM_STATUS: the flags are status[lo + i] == kActive, read straight from the
// unit status (k_round_begin); else the flag array of k_round_start.
// Chunks [base_begin, base_end) of the flags, output from position carry0; the
// count (carry0 + the range's flags) is stored when `count` is given.
template <bool FROM_STATUS>
__device__ __forceinline__ void compact_wg(const int32_t *__restrict__ flag, int32_t n,
                                           int32_t lo, int32_t *__restrict__ out,
                                           int32_t *__restrict__ count,
                                           int32_t *__restrict__ host_count,
                                           int32_t base_begin = 0, int32_t base_end = INT32_MAX,
                                           int32_t carry0 = 0) {
  __shared__ int32_t wsum[kCompactBS / kWave];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // 16-B loads need a 16-B aligned start (status + lo: lo % 4 == 0)
  const bool vec = !FROM_STATUS || (lo & 3) == 0;
  const int32_t *src = FROM_STATUS ? flag + lo : flag;
  int32_t carry = carry0;
  const int32_t bend = min(n, base_end);
  for (int32_t base = base_begin; base < bend; base += kCompactChunk) {
    const int32_t i0 = base + t * kCompactIPT;
    int32_t f[kCompactIPT];
    if (vec && i0 + kCompactIPT <= n) {  // 16-B aligned (device allocation), i0 % 16 == 0
      const int4 *p = reinterpret_cast<const int4 *>(src + i0);
#pragma unroll
      for (int v = 0; v < kCompactIPT / 4; ++v) {
        const int4 x = p[v];
        f[4 * v] = x.x; f[4 * v + 1] = x.y; f[4 * v + 2] = x.z; f[4 * v + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kCompactIPT; ++k)
        f[k] = i0 + k < n ? src[i0 + k] : (FROM_STATUS ? -1 : 0);
    }
    if (FROM_STATUS) {
#pragma unroll
      for (int k = 0; k < kCompactIPT; ++k) f[k] = f[k] == kActive ? 1 : 0;
    }
    int32_t c = 0;
#pragma unroll
    for (int k = 0; k < kCompactIPT; ++k) c += f[k] != 0;
    int32_t inc = c;  // wave inclusive scan
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const int32_t o = __shfl_up(inc, d, kWave);
      if (lane >= d) inc += o;
    }
    if (lane == kWave - 1) wsum[w] = inc;
    __syncthreads();
    int32_t before = 0, total = 0;
#pragma unroll
    for (int k = 0; k < kCompactBS / kWave; ++k) {
      const int32_t s = wsum[k];
      before += k < w ? s : 0;
      total += s;
    }
    int32_t pos = carry + before + inc - c;
#pragma unroll
    for (int k = 0; k < kCompactIPT; ++k)
      if (f[k] != 0) out[pos++] = lo + i0 + k;
    carry += total;
    __syncthreads();  // wsum reused by the next chunk
  }
  if (t == 0 && count) {
    *count = carry;
    // the host's copy (pinned, coherent): a system-scope vector store, no
    // copy command and no event in the stream
    if (host_count) __hip_atomic_store(host_count, carry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(kCompactBS) void k_compact(const int32_t *__restrict__ flag, int32_t n,
                                                        int32_t lo, int32_t *__restrict__ out,
                                                        int32_t *__restrict__ count,
                                                        int32_t *__restrict__ host_count) {
  compact_wg<false>(flag, n, lo, out, count, host_count);
}

// set flags of chunk blockIdx.x -> bcount[blockIdx.x]
__global__ __launch_bounds__(kCompactBS) void k_compact_count(const int32_t *__restrict__ flag,
                                                              int32_t n,
                                                              int32_t *__restrict__ bcount) {
  __shared__ int32_t wsum[kCompactBS / kWave];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t i0 = (int64_t)blockIdx.x * kCompactChunk + (int64_t)t * kCompactIPT;
  int32_t c = 0;
#pragma unroll
  for (int k = 0; k < kCompactIPT; ++k) c += i0 + k < n && flag[i0 + k] != 0 ? 1 : 0;
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) c += __shfl_xor(c, d, kWave);
  if (lane == 0) wsum[w] = c;
  __syncthreads();
  if (t == 0) {
    int32_t s = 0;
#pragma unroll
    for (int k = 0; k < kCompactBS / kWave; ++k) s += wsum[k];
    bcount[blockIdx.x] = s;
  }
}

// chunk blockIdx.x compacted at the sum of the earlier chunks' counts; the
// last chunk stores the total count
__global__ __launch_bounds__(kCompactBS) void k_compact_multi(const int32_t *__restrict__ flag,
                                                              int32_t n, int32_t lo,
                                                              const int32_t *__restrict__ bcount,
                                                              int32_t *__restrict__ out,
                                                              int32_t *__restrict__ count,
                                                              int32_t *__restrict__ host_count) {
  __shared__ int32_t psum[kCompactBS / kWave];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int32_t c = 0;
  for (int32_t b = t; b < (int32_t)blockIdx.x; b += kCompactBS) c += bcount[b];
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) c += __shfl_xor(c, d, kWave);
  if (lane == 0) psum[w] = c;
  __syncthreads();
  int32_t carry0 = 0;
#pragma unroll
  for (int k = 0; k < kCompactBS / kWave; ++k) carry0 += psum[k];
  const int32_t base = (int32_t)blockIdx.x * kCompactChunk;
  const bool last = blockIdx.x + 1 == gridDim.x;
  compact_wg<false>(flag, n, lo, out, last ? count : nullptr, last ? host_count : nullptr, base,
                    base + kCompactChunk, carry0);
}

// Round start and compaction in ONE launch (one-workgroup compaction range):
// workgroup 0 compacts the active units of [lo, lo + n) straight from the
// unit status, workgroups 1.. pack the round's 32-bit node planes (the work
// of k_round_start + k_compact, one launch fewer per round).
template <int D>
__global__ __launch_bounds__(kCompactBS) void k_round_begin(
    const int32_t *__restrict__ status, int32_t lo, int32_t n, int32_t *__restrict__ out,
    int32_t *__restrict__ count, int32_t *__restrict__ host_count,
    const int64_t *__restrict__ cap, const int64_t *__restrict__ used,
    const uint32_t *__restrict__ R32, const uint32_t *__restrict__ K32,
    const int64_t *__restrict__ base, const int32_t *__restrict__ topo,
    const int32_t *__restrict__ perm, const int32_t *__restrict__ colnode, int32_t N, int32_t P,
    int32_t full, ScoreParams sp, uint32_t *__restrict__ np, const uint32_t *__restrict__ ncls) {
  if (blockIdx.x == 0) {
    compact_wg<true>(status, n, lo, out, count, host_count);
    return;
  }
  const int i = (blockIdx.x - 1) * kCompactBS + threadIdx.x;
  if (i < P) pack_node<D>(cap, used, R32, K32, base, topo, perm, colnode, N, P, full != 0, sp, np, i, ncls);
}

template <int D>
struct RoundBeginL {
  static int run(kp_ctx *c, int32_t lo, int32_t n, int32_t *host_count) {
    const int32_t P = !c->fits32 || c->N == 0 ? 0 : c->pack_fused ? c->fz_P : (c->N + 1023) & ~1023;
    hipLaunchKernelGGL((k_round_begin<D>), dim3(1 + blocks(P, kCompactBS)), dim3(kCompactBS), 0,
                       c->stream, c->d.status, lo, n, c->d.act_local, c->d.counters, host_count,
                       c->d.cap, c->d.used, c->d.R32, c->d.K32, c->d.base, c->d.topo,
                       c->pack_canonical ? c->d.perm : nullptr,
                       c->pack_fused ? c->d.colnode : nullptr, c->N, P, c->pack_full ? 1 : 0,
                       c->pack_sp, c->d.np32, c->n_classes > 0 ? c->d.ncls : nullptr);
    KP_HIP(hipGetLastError());
    if (P > 0) c->pack_full = false;  // capacity planes in place for this layout
    return KP_OK;
  }
};

template <int D>
struct ScoreL {
  static int run(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit, int32_t rows,
                 int32_t *score, uint64_t *mask, const int64_t *q, int32_t qstride,
                 const int32_t *rows_dev, int64_t sstride, int64_t mstride) {
    const int Ns = (c->N + 63) & ~63;
    if (c->fits32) {
      const int P = (c->N + 1023) & ~1023;  // planes from the round start (launch_pack)
      // rows per workgroup: enough workgroups to cover the 256 CUs several
      // times over, at most kScoreMaxRows (the LDS request stage)
      // nodes per lane: 2 (8-B stores, half the tile registers: twice the
      // resident waves) unless KP_SCORE_NPL=4
      const int npl = c->score_npl;
      const int tiles = blocks(Ns, 256 * npl);
      if (c->n_classes > 0 && c->score_classes) {  // the class form (every wave, either order)
        const int ctiles = blocks(Ns, 256 * kClsCols);
        const int64_t want = ((int64_t)rows * ctiles + c->score_wg_target - 1) / c->score_wg_target;
        const int rpb =
            (int)std::min<int64_t>(kScoreClsRows, std::max<int64_t>(c->score_min_rpb, want));
        const dim3 grid(ctiles, blocks(rows, rpb));
#define KP_SC32C(M, WS_, WM_)                                                                  \
  hipExtLaunchKernelGGL((k_score32c<D, M, WS_, WM_>), grid, dim3(256), 0, c->stream, c->score_ev0,   \
                        c->score_ev1, 0, sp, c->d.np32, P,                                         \
                     q, qstride, c->d.aff, rows_unit, rows, rpb, c->score_min_rpb, score,           \
                     sstride > 0 ? sstride : (int64_t)Ns, mask, mstride > 0 ? mstride : (int64_t)Ns / 64, \
                     Ns, rows_dev, c->d.ccap, c->n_classes)
#define KP_SC32C_M(WS_, WM_)     \
  if (sp.most_allocated)         \
    KP_SC32C(true, WS_, WM_);    \
  else                           \
    KP_SC32C(false, WS_, WM_);
        if (score && mask) {
          KP_SC32C_M(true, true)
        } else if (score) {
          KP_SC32C_M(true, false)
        } else if (mask) {
          KP_SC32C_M(false, true)
        }
#undef KP_SC32C_M
#undef KP_SC32C
        KP_HIP(hipGetLastError());
        return KP_OK;
      }
      // only the class form takes caller row strides (k_score32 / k_score
      // write rows of Ns scores and Ns / 64 mask words)
      if ((sstride > 0 && sstride != Ns) || (mstride > 0 && mstride != Ns / 64))
        { kp_set_error_msg("launch_score: row strides need the capacity-class form"); return KP_EINVAL; }
      const int64_t want = ((int64_t)rows * tiles + c->score_wg_target - 1) / c->score_wg_target;
      const int rpb =
          (int)std::min<int64_t>(kScoreMaxRows, std::max<int64_t>(c->score_min_rpb, want));
      dim3 grid(tiles, blocks(rows, rpb));
#define KP_SC32(M, NP)                                                                      \
  hipLaunchKernelGGL((k_score32<D, M, NP>), grid, dim3(256), 0, c->stream, sp, c->d.np32, P, q, \
                     qstride, c->d.aff, rows_unit, rows, rpb, c->score_min_rpb, score, mask, Ns,  \
                     rows_dev)
      if (sp.most_allocated) {
        if (npl == 4) KP_SC32(true, 4); else KP_SC32(true, 2);
      } else {
        if (npl == 4) KP_SC32(false, 4); else KP_SC32(false, 2);
      }
#undef KP_SC32
    } else {
      if ((sstride > 0 && sstride != Ns) || (mstride > 0 && mstride != Ns / 64))
        { kp_set_error_msg("launch_score: row strides need the capacity-class form"); return KP_EINVAL; }
      constexpr int NPL = D <= 4 ? 2 : 1;
      const int rpb = 32;
      dim3 grid(blocks(Ns, 256 * NPL), blocks(rows, rpb));
      hipLaunchKernelGGL((k_score<D, NPL>), grid, dim3(256), 0, c->stream, sp, c->d.cap,
                         c->d.used, c->d.topo, c->pack_canonical ? c->d.perm : nullptr, q,
                         qstride, c->d.aff, rows_unit, rows, rpb, c->score_min_rpb, score, mask,
                         Ns, rows_dev);
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
                     c->d.R32, c->d.K32, c->d.base, c->N, c->D, S, most_allocated ? 0 : 1, sp);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

int launch_score(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit, int32_t rows,
                 int32_t *score, uint64_t *mask, const int64_t *q, int32_t qstride,
                 const int32_t *rows_dev, int64_t sstride, int64_t mstride) {
  if (rows <= 0 || c->N == 0) return KP_OK;
  return dispatch_D<ScoreL>(c->D, c, sp, rows_unit, rows, score, mask, q, qstride, rows_dev,
                            sstride, mstride);
}

// Threshold-select shapes (V4 16-B loads per thread x BS threads cover
// 4*V4*BS nodes of a row). Per row width the first listed shape of the
// preferred block size that covers the row: few row entries per thread keeps
// the row in fewer VGPRs (more resident waves, more loads in flight).
namespace {
using SelFn = void (*)(dim3, hipStream_t, const ScoreParams &, const int32_t *, int32_t,
                       const int32_t *, const uint32_t *, int32_t, int32_t, int32_t *,
                       const int32_t *, const int32_t *);
template <int V4, int BS>
void sel_t(dim3 grid, hipStream_t st, const ScoreParams &sp, const int32_t *score, int32_t Ns,
           const int32_t *rows_unit, const uint32_t *salt, int32_t rows, int32_t cap,
           int32_t *cand, const int32_t *rows_dev, const int32_t *perm) {
  hipLaunchKernelGGL((k_select_t<V4, BS>), grid, dim3(BS), 0, st, sp, score, Ns, rows_unit, salt,
                     rows, cap, cand, rows_dev, perm);
}
struct SelShape {
  int v4, bs;
  SelFn fn;
};
const SelShape kSelShapes[] = {
    {1, 256, sel_t<1, 256>},    {2, 256, sel_t<2, 256>},    {3, 256, sel_t<3, 256>},
    {4, 256, sel_t<4, 256>},    {6, 256, sel_t<6, 256>},    {8, 256, sel_t<8, 256>},
    {12, 256, sel_t<12, 256>},  {16, 256, sel_t<16, 256>},  {2, 512, sel_t<2, 512>},
    {3, 512, sel_t<3, 512>},    {4, 512, sel_t<4, 512>},    {5, 512, sel_t<5, 512>},
    {6, 512, sel_t<6, 512>},    {8, 512, sel_t<8, 512>},    {4, 1024, sel_t<4, 1024>},
    {5, 1024, sel_t<5, 1024>},  {6, 1024, sel_t<6, 1024>},  {8, 1024, sel_t<8, 1024>},
    {10, 1024, sel_t<10, 1024>}, {17, 768, sel_t<17, 768>},
};
const SelShape *sel_shape(int Ns, int pref_bs) {
  const SelShape *best = nullptr;
  for (const SelShape &s : kSelShapes) {
    if (4 * s.v4 * s.bs < Ns) continue;
    if (pref_bs > 0 && s.bs != pref_bs) continue;
    if (!best) best = &s;
  }
  return best;
}
}  // namespace

int launch_select(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit, int32_t rows,
                  const int32_t *score, int32_t *cand, const int32_t *rows_dev) {
  if (rows <= 0) return KP_OK;
  const int Ns = (c->N + 63) & ~63;
  const int K = sp.n_cand;
  const int lim = c->select_lds_cap > 0 ? std::min(c->select_lds_cap, kSelLdsCap) : kSelLdsCap;
  const int cap = std::max(K + 1, lim);
  dim3 grid(rows);
  // preferred block size: 256 threads up to 4k nodes, 512 up to 16k, 1024
  // up to 40k (at most 128 VGPRs per thread), else 768 (KP_SELECT_BS overrides); rows wider than every
  // shape: generic form
  const int pref = c->select_bs > 0 ? c->select_bs
                   : Ns <= 4096     ? 256
                   : Ns <= 16384    ? 512
                   : Ns <= 40960    ? 1024
                                    : 768;
  const SelShape *sh = c->select_generic ? nullptr : sel_shape(Ns, pref);
  if (!sh && !c->select_generic) sh = sel_shape(Ns, 0);
  if (sh) {
    sh->fn(grid, c->stream, sp, score, Ns, rows_unit, c->d.salt, rows, cap, cand, rows_dev,
           c->d.perm);
  } else if (K <= 4) {
    hipLaunchKernelGGL(k_select<4>, grid, dim3(256), 0, c->stream, sp, score, Ns, rows_unit,
                       c->d.salt, rows, cand, rows_dev, c->d.perm);
  } else if (K <= 8) {
    hipLaunchKernelGGL(k_select<8>, grid, dim3(256), 0, c->stream, sp, score, Ns, rows_unit,
                       c->d.salt, rows, cand, rows_dev, c->d.perm);
  } else if (K <= 16) {
    hipLaunchKernelGGL(k_select<16>, grid, dim3(256), 0, c->stream, sp, score, Ns, rows_unit,
                       c->d.salt, rows, cand, rows_dev, c->d.perm);
  } else {
    hipLaunchKernelGGL(k_select<32>, grid, dim3(256), 0, c->stream, sp, score, Ns, rows_unit,
                       c->d.salt, rows, cand, rows_dev, c->d.perm);
  }
  KP_HIP(hipGetLastError());
  return KP_OK;
}

template <int D>
struct RoundStartL {
  static int run(kp_ctx *c, int32_t lo, int32_t hi, int32_t *flag) {
    const int32_t P = !c->fits32 || c->N == 0 ? 0 : c->pack_fused ? c->fz_P : (c->N + 1023) & ~1023;
    const int64_t n = std::max<int64_t>(hi - lo, P);
    if (n <= 0) return KP_OK;
    hipLaunchKernelGGL((k_round_start<D>), dim3(blocks(n, 256)), dim3(256), 0, c->stream,
                       c->d.status, lo, hi, flag, c->d.cap, c->d.used, c->d.R32, c->d.K32,
                       c->d.base, c->d.topo, c->pack_canonical ? c->d.perm : nullptr,
                       c->pack_fused ? c->d.colnode : nullptr, c->N, P, c->pack_full ? 1 : 0,
                       c->pack_sp, c->d.np32, c->n_classes > 0 ? c->d.ncls : nullptr);
    KP_HIP(hipGetLastError());
    if (P > 0) c->pack_full = false;  // capacity planes in place for this layout
    return KP_OK;
  }
};

// round start: active flags of [lo, hi) + (32-bit path) the node planes
static int launch_round_start(kp_ctx *c, int32_t lo, int32_t hi, int32_t *flag) {
  return dispatch_D<RoundStartL>(c->D, c, lo, hi, flag);
}

int launch_pack(kp_ctx *c) { return launch_round_start(c, 0, 0, nullptr); }

// flags[0, n) -> out (lo + index, rank order; act_local by default), count ->
// counters[0]; one workgroup up to KP_COMPACT_MAX flags (default 65,536),
// the two-launch multi-workgroup form above (chunk counts in `temp`)
int launch_compact_to(kp_ctx *c, const int32_t *flag, int32_t lo, int32_t n, int32_t *out,
                      int32_t *host_count) {
  if (n <= c->compact_max) {
    hipLaunchKernelGGL(k_compact, dim3(1), dim3(kCompactBS), 0, c->stream, flag, n, lo, out,
                       c->d.counters, host_count);
    KP_HIP(hipGetLastError());
    return KP_OK;
  }
  const int chunks = blocks(n, kCompactChunk);
  if ((size_t)chunks * sizeof(int32_t) > c->d.temp_bytes) {
    kp_set_error_msg("launch_compact: chunk counts exceed the scratch buffer");
    return KP_ENOMEM;
  }
  int32_t *bcount = reinterpret_cast<int32_t *>(c->d.temp);
  hipLaunchKernelGGL(k_compact_count, dim3(chunks), dim3(kCompactBS), 0, c->stream, flag, n, bcount);
  KP_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_compact_multi, dim3(chunks), dim3(kCompactBS), 0, c->stream, flag, n, lo,
                     bcount, out, c->d.counters, host_count);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

static int launch_compact(kp_ctx *c, const int32_t *flag, int32_t lo, int32_t n, size_t /*tb*/,
                          int32_t *host_count = nullptr) {
  return launch_compact_to(c, flag, lo, n, c->d.act_local, host_count);
}

// active units of [lo, hi) in rank order -> act_local; count to host
int launch_active(kp_ctx *c, int32_t lo, int32_t hi, int32_t *A_host) {
  *A_host = 0;
  const int32_t n = hi - lo;
  if (n <= 0) return KP_OK;
  int32_t *flag = c->d.flag;
  KP_TRY(launch_round_start(c, lo, hi, flag));
  size_t tb = c->d.temp_bytes;
  KP_TRY(launch_compact(c, flag, lo, n, tb));
  KP_HIP(hipMemcpyAsync(c->pinned, c->d.counters, sizeof(int32_t), hipMemcpyDeviceToHost,
                        c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  *A_host = c->pinned[0];
  return KP_OK;
}

int launch_delta(kp_ctx *c, int32_t K, int32_t *bad_host) {
  const int64_t n = (int64_t)K * c->D;
  int32_t *bad = c->d.dl_bad;
  KP_HIP(hipMemsetAsync(bad, 0, sizeof(int32_t), c->stream));
  hipLaunchKernelGGL(k_delta_apply, dim3(blocks(n, 256)), dim3(256), 0, c->stream, K, c->N, c->D,
                     c->d.dl_node, c->d.dl_delta, (int64_t)1, c->d.used);
  KP_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_delta_check, dim3(blocks(n, 256)), dim3(256), 0, c->stream, K, c->N, c->D,
                     c->d.dl_node, c->d.cap, c->d.used, bad);
  KP_HIP(hipGetLastError());
  KP_HIP(hipMemcpyAsync(c->pinned + 8, bad, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  *bad_host = c->pinned[8];
  if (*bad_host) {  // undo: the call leaves the table unchanged on failure
    hipLaunchKernelGGL(k_delta_apply, dim3(blocks(n, 256)), dim3(256), 0, c->stream, K, c->N,
                       c->D, c->d.dl_node, c->d.dl_delta, (int64_t)-1, c->d.used);
    KP_HIP(hipGetLastError());
    KP_HIP(hipStreamSynchronize(c->stream));
  }
  return KP_OK;
}

// same compaction without the host round trip: the count stays on the device
// (counters[0], read by the round's kernels) and is copied to *count_host
// asynchronously
int launch_active_async(kp_ctx *c, int32_t lo, int32_t hi, int32_t *count_host, bool *direct) {
  const int32_t n = hi - lo;
  if (n <= 0) return KP_EINVAL;
  if (n <= c->compact_max && c->round_begin) {  // one launch: compaction + node planes
    const bool dir = direct && c->count_direct && c->pinned_coh;
    if (direct) *direct = dir;
    if (dir) __atomic_store_n(c->pinned_coh, -1, __ATOMIC_RELAXED);  // the sentinel the host waits on
    KP_TRY(dispatch_D<RoundBeginL>(c->D, c, lo, n, dir ? c->pinned_coh : nullptr));
    if (!dir)
      KP_HIP(hipMemcpyAsync(count_host, c->d.counters, sizeof(int32_t), hipMemcpyDeviceToHost,
                            c->stream));
    return KP_OK;
  }
  KP_TRY(launch_round_start(c, lo, hi, c->d.flag));
  size_t tb = c->d.temp_bytes;
  // the one-workgroup compaction stores the count into coherent pinned
  // memory itself (count_direct); otherwise a copy lands it
  const bool dir = direct && c->count_direct && c->pinned_coh;
  if (direct) *direct = dir;
  if (dir) {
    __atomic_store_n(c->pinned_coh, -1, __ATOMIC_RELAXED);  // the sentinel the host waits on
    KP_TRY(launch_compact(c, c->d.flag, lo, n, tb, c->pinned_coh));
    return KP_OK;
  }
  KP_TRY(launch_compact(c, c->d.flag, lo, n, tb));
  KP_HIP(hipMemcpyAsync(count_host, c->d.counters, sizeof(int32_t), hipMemcpyDeviceToHost,
                        c->stream));
  return KP_OK;
}

int launch_reset_units(kp_ctx *c, uint32_t tie_seed) {
  const int32_t n = c->U > c->J ? c->U : c->J;
  if (n <= 0) return KP_OK;
  hipLaunchKernelGGL(k_reset_units, dim3(blocks(n, 256)), dim3(256), 0, c->stream, c->d.status,
                     c->U, c->d.job_node, c->d.job_score, c->J, c->d.leader, c->d.salt, tie_seed);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

int launch_finalize(kp_ctx *c) {
  const int32_t n = std::max(c->U, 64);
  hipLaunchKernelGGL(k_finalize, dim3(blocks(n, 256)), dim3(256), 0, c->stream, c->d.status,
                     c->d.leader, c->d.size, c->U, c->d.job_node, c->d.job_score,
                     c->d.job_status, c->d.pass_flag, c->d.stats);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

int launch_unpack_exchange(kp_ctx *c, int32_t world, int32_t B, int32_t K) {
  if (B <= 0) return KP_OK;
  hipLaunchKernelGGL(k_unpack, dim3(blocks((int64_t)world * B, 256)), dim3(256), 0, c->stream,
                     world, B, K, c->d.xg_recv, c->d.act, c->d.cand, c->d.counters + 1);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

int launch_pack_exchange(kp_ctx *c, int32_t B, int32_t K) {
  hipLaunchKernelGGL(k_pack, dim3(blocks(std::max(B, 1), 256)), dim3(256), 0, c->stream, B, K,
                     c->d.counters, c->d.act_local, c->d.cand_local, c->d.xg_send);
  KP_HIP(hipGetLastError());
  return KP_OK;
}

}  // namespace kp
