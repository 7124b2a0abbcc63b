// kp_device.hpp — device-side helpers shared by the kplace kernels: 64-lane
// wave reductions / scans (CDNA wavefront = 64, never 32) and the exact
// integer score of DESIGN.md §2.3.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "kp_internal.hpp"

namespace kp {
namespace dev {

constexpr int kWave = 64;

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
// DPP lane move of a 64-bit value (two 32-bit v_mov_dpp); lanes whose
// source is outside the pattern get an unspecified value and must not use it
template <int CTRL>
__device__ __forceinline__ int64_t dpp_i64(int64_t v) {
  const int lo = (int)(uint32_t)(uint64_t)v, hi = (int)(uint32_t)((uint64_t)v >> 32);
  const uint32_t l2 = (uint32_t)__builtin_amdgcn_mov_dpp(lo, CTRL, 0xf, 0xf, false);
  const uint32_t h2 = (uint32_t)__builtin_amdgcn_mov_dpp(hi, CTRL, 0xf, 0xf, false);
  return (int64_t)(((uint64_t)h2 << 32) | l2);
}
// 32-bit wave reductions (OP 0 = OR, 1 = AND, 2 = unsigned max), result in
// every lane: DPP inside each 16-lane row, then the four row results through
// scalar readlanes (VALU-only, no LDS crossbar)
template <int OP>
__device__ __forceinline__ uint32_t wave_red32_op(uint32_t a, uint32_t b) {
  return OP == 0 ? (a | b) : OP == 1 ? (a & b) : (a > b ? a : b);
}
template <int OP>
__device__ __forceinline__ uint32_t wave_red32(uint32_t v) {
  const int rl16 = __lane_id() & 15;
  uint32_t t;
#define KP_STEP(CTRL, SH)                                                 \
  t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false); \
  if (rl16 >= SH) v = wave_red32_op<OP>(v, t);
  KP_STEP(0x111, 1)
  KP_STEP(0x112, 2)
  KP_STEP(0x114, 4)
  KP_STEP(0x118, 8)
#undef KP_STEP
  uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
#pragma unroll
  for (int r = 1; r < 4; ++r)
    m = wave_red32_op<OP>(m, (uint32_t)__builtin_amdgcn_readlane((int)v, 16 * r + 15));
  return m;
}
__device__ __forceinline__ uint32_t wave_or32(uint32_t v) { return wave_red32<0>(v); }
__device__ __forceinline__ uint32_t wave_and32(uint32_t v) { return wave_red32<1>(v); }
__device__ __forceinline__ uint32_t wave_max32(uint32_t v) { return wave_red32<2>(v); }

// 64-bit wave max, result in every lane: DPP max inside each 16-lane row
// (row_shr 1/2/4/8: lane 15 of a row ends with the row max), then the four
// row maxima through scalar readlanes (VALU-only, no LDS crossbar)
__device__ __forceinline__ uint64_t wave_max_u64_dpp(uint64_t v) {
  const int rl16 = __lane_id() & 15;
  uint64_t t;
  t = (uint64_t)dpp_i64<0x111>((int64_t)v);
  if (rl16 >= 1 && t > v) v = t;
  t = (uint64_t)dpp_i64<0x112>((int64_t)v);
  if (rl16 >= 2 && t > v) v = t;
  t = (uint64_t)dpp_i64<0x114>((int64_t)v);
  if (rl16 >= 4 && t > v) v = t;
  t = (uint64_t)dpp_i64<0x118>((int64_t)v);
  if (rl16 >= 8 && t > v) v = t;
  uint64_t m = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 16 * r + 15);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 16 * r + 15);
    const uint64_t x = ((uint64_t)hi << 32) | lo;
    m = x > m ? x : m;
  }
  return m;
}
// inclusive prefix sum over the 64 lanes with DPP (row_shr 1/2/4/8 inside
// each 16-lane row, then row_bcast 15/31 across rows): VALU-only, no LDS
// crossbar round trips
__device__ __forceinline__ int64_t wave_incl_scan_i64(int64_t v) {
  const int l = lane_id(), rl = l & 15;
  int64_t t;
  t = dpp_i64<0x111>(v);
  if (rl >= 1) v += t;
  t = dpp_i64<0x112>(v);
  if (rl >= 2) v += t;
  t = dpp_i64<0x114>(v);
  if (rl >= 4) v += t;
  t = dpp_i64<0x118>(v);
  if (rl >= 8) v += t;
  t = dpp_i64<0x142>(v);  // row_bcast:15
  if ((l & 31) >= 16) v += t;
  t = dpp_i64<0x143>(v);  // row_bcast:31
  if (l >= 32) v += t;
  return v;
}
// 32-bit inclusive prefix sum over the 64 lanes (same DPP pattern)
__device__ __forceinline__ int32_t wave_incl_scan_i32(int32_t v) {
  const int l = lane_id(), rl = l & 15;
  int32_t t;
  t = __builtin_amdgcn_mov_dpp(v, 0x111, 0xf, 0xf, false);
  if (rl >= 1) v += t;
  t = __builtin_amdgcn_mov_dpp(v, 0x112, 0xf, 0xf, false);
  if (rl >= 2) v += t;
  t = __builtin_amdgcn_mov_dpp(v, 0x114, 0xf, 0xf, false);
  if (rl >= 4) v += t;
  t = __builtin_amdgcn_mov_dpp(v, 0x118, 0xf, 0xf, false);
  if (rl >= 8) v += t;
  t = __builtin_amdgcn_mov_dpp(v, 0x142, 0xf, 0xf, false);  // row_bcast:15
  if ((l & 31) >= 16) v += t;
  t = __builtin_amdgcn_mov_dpp(v, 0x143, 0xf, 0xf, false);  // row_bcast:31
  if (l >= 32) v += t;
  return v;
}

// position of the r-th set bit (r < popcount(x)) of x: popcount bisection
__device__ __forceinline__ int select_bit(uint32_t x, int r) {
  int pos = 0;
#pragma unroll
  for (int h = 16; h >= 1; h >>= 1) {
    const int c = __popc(x & ((1u << h) - 1u));
    if (r >= c) {
      r -= c;
      x >>= h;
      pos += h;
    }
  }
  return pos;
}

__device__ __forceinline__ int select_bit64(uint64_t x, int r) {
  const int lo = __popc((uint32_t)x);
  return r < lo ? select_bit((uint32_t)x, r) : 32 + select_bit((uint32_t)(x >> 32), r - lo);
}

// max over aligned groups of G lanes (G = 16, 32 or 64), result in every
// lane of the group: DPP max-scan inside the group, then the group's last
// lane is read back with scalar readlanes (no LDS crossbar)
template <int G>
__device__ __forceinline__ int64_t group_max_i64(int64_t v);

// value of a wave-uniform lane (scalar read, no LDS)
__device__ __forceinline__ int64_t readlane_i64(int64_t v, int lane) {
  const int ln = __builtin_amdgcn_readfirstlane(lane);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, ln);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), ln);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

template <int G>
__device__ __forceinline__ int64_t group_max_i64(int64_t v) {
  static_assert(G == 16 || G == 32 || G == 64, "group size");
  const int l = lane_id(), rl = l & 15;
  int64_t t;
  t = dpp_i64<0x111>(v);
  if (rl >= 1) v = t > v ? t : v;
  t = dpp_i64<0x112>(v);
  if (rl >= 2) v = t > v ? t : v;
  t = dpp_i64<0x114>(v);
  if (rl >= 4) v = t > v ? t : v;
  t = dpp_i64<0x118>(v);
  if (rl >= 8) v = t > v ? t : v;
  if (G >= 32) {
    t = dpp_i64<0x142>(v);  // row_bcast:15
    if ((l & 31) >= 16) v = t > v ? t : v;
  }
  if (G >= 64) {
    t = dpp_i64<0x143>(v);  // row_bcast:31
    if (l >= 32) v = t > v ? t : v;
  }
  if (G == 16) {
    const int64_t m0 = readlane_i64(v, 15), m1 = readlane_i64(v, 31);
    const int64_t m2 = readlane_i64(v, 47), m3 = readlane_i64(v, 63);
    const int g = l >> 4;
    return g == 0 ? m0 : g == 1 ? m1 : g == 2 ? m2 : m3;
  }
  if (G == 32) {
    const int64_t m0 = readlane_i64(v, 31), m1 = readlane_i64(v, 63);
    return l < 32 ? m0 : m1;
  }
  return readlane_i64(v, 63);
}

// ---------------------------------------------------------------------------
// §2.3 exact utilisation, kube-scheduler's integer formulas per dimension:
//   MostAllocated  util = floor(x*S/c)        (mostRequestedScore)
//   LeastAllocated util = floor((c-x)*S/c)    (leastRequestedScore)
//                       = S - ceil(x*S/c)
// for x = used + q <= c, c > 0 (cap-0 dims contribute 0).
//
// 32-bit form (every cap < 2^32): per node and dim a multiplier R and shift
// k (div_prep) make t = (x*R) >> k equal floor(x*S/c) or one less for every
// x <= c (x < 2^k and R = floor(S*2^k/c): x*R/2^k lies in (v - 1, v]); one
// remainder check r = x*S - t*c >= c repairs it. Modes, chosen per node:
//   E (c < 2^12): R = floor(S*2^k/c) + 1 with c^2 < 2^k: t is exact, no
//     check (x*R/2^k = v + x*d/2^k with x*d/2^k < 1/c);
//   C (c < 2^24, S*2^k < 2^32): every product fits 32 bits and every
//     operand 24 bits: full-rate v_mul_u32_u24 throughout;
//   W (otherwise): k = 32, 64-bit products (quarter rate, rare).
// ---------------------------------------------------------------------------
constexpr uint32_t kDivE = 0x100u, kDivW = 0x200u;  // K plane: shift | mode bits

__host__ __device__ inline void div_prep(uint64_t c, uint32_t S, uint32_t &R, uint32_t &K) {
  if (c == 0) {  // feasible x = 0: t = 0
    R = 0;
    K = 1u | kDivE;
    return;
  }
  int fl = 63;
  while (!((c >> fl) & 1ull)) --fl;  // floor(log2 c)
  if (c < (1u << 12)) {
    const int kE = 2 * fl + 2;  // c^2 < 2^kE
    const uint64_t top = (uint64_t)S << kE;
    const uint64_t RE = top / c + 1;
    if (top + c < (1ull << 32) && RE < (1u << 24)) {
      R = (uint32_t)RE;
      K = (uint32_t)kE | kDivE;
      return;
    }
  }
  const int kC = fl + 1;
  if (c < (1u << 24) && ((uint64_t)S << kC) < (1ull << 32)) {
    R = (uint32_t)(((uint64_t)S << kC) / c);
    K = (uint32_t)kC;
    return;
  }
  R = (uint32_t)(((uint64_t)S << 32) / c);  // c >= 2^21 here: R < 2^32
  K = 32u | kDivW;
}

// generic 32-bit form (any mode): floor(x*S/c) for x <= c < 2^32, plus
// whether the remainder is non-zero (LeastAllocated's ceiling)
__device__ __forceinline__ uint32_t div_floor32(uint32_t x, uint32_t c, uint32_t R, uint32_t K,
                                                uint32_t S, bool &rem_nz) {
  uint32_t t = (uint32_t)(((uint64_t)x * R) >> (K & 63u));
  uint64_t r = (uint64_t)x * S - (uint64_t)t * c;
  const uint64_t cc = c ? c : 1;
  if (r >= cc) {
    ++t;
    r -= cc;
  }
  rem_nz = r != 0;
  return t;
}

// the same exact division with its remainder: x·S = t·c + r, 0 <= r < c
// (x <= c < 2^32; c = 0 with x = 0 gives t = r = 0)
__device__ __forceinline__ void divmod32(uint32_t x, uint32_t c, uint32_t R, uint32_t K, uint32_t S,
                                         uint32_t &t, uint32_t &r) {
  t = (uint32_t)(((uint64_t)x * R) >> (K & 63u));
  uint64_t rr = (uint64_t)x * S - (uint64_t)t * c;
  const uint64_t cc = c ? c : 1;
  if (rr >= cc) {
    ++t;
    rr -= cc;
  }
  r = (uint32_t)rr;
}

// 64-bit form (some cap >= 2^32, caps <= 2^56): x*S needs up to 67 bits. A
// double estimate (|error| << 1) corrected with 128-bit remainders.
__device__ __forceinline__ int64_t util64(int64_t x, int64_t c, int32_t S, bool most) {
  if (x > c) x = c;  // infeasible pair: any value (masked by the caller)
  const uint64_t y = most ? (uint64_t)x : (uint64_t)(c - x);
  const unsigned __int128 n = (unsigned __int128)y * (uint32_t)S;
  uint64_t t = (uint64_t)((double)y * (double)S / (double)c);
  __int128 r = (__int128)n - (__int128)((unsigned __int128)t * (uint64_t)c);
  for (int i = 0; i < 4 && r < 0; ++i) {
    --t;
    r += c;
  }
  for (int i = 0; i < 4 && r >= (__int128)c; ++i) {
    ++t;
    r -= c;
  }
  return (int64_t)t;
}

// §2.3: score of one more copy of q on a node whose usage is `used`, in the
// topo domain `topo`, for a unit preferring domain `aff`; -1 when it does not
// fit. 64-bit exact (the int64 path).
template <int D>
__device__ __forceinline__ int64_t score_at(const ScoreParams &sp, const int64_t (&q)[D],
                                            const int64_t (&cap)[D], const int64_t (&used)[D],
                                            int32_t topo, int32_t aff) {
  int64_t acc = 0;
  bool fits = true;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    fits &= q[d] <= cap[d] - used[d];
    if (cap[d] > 0)
      acc += (int64_t)sp.w[d] * util64(used[d] + q[d], cap[d], sp.S, sp.most_allocated != 0);
  }
  int64_t s = acc;
  if (sp.gpu_dim >= 0) {
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (d == sp.gpu_dim && q[d] > 0 && cap[d] - used[d] - q[d] == 0) s += sp.w_gpu_fit;
  }
  if (aff >= 0 && topo == aff) s += sp.w_affinity;
  return fits ? s : -1;
}

// 32-bit group max (same DPP pattern as group_max_i64)
template <int G>
__device__ __forceinline__ int32_t group_max_i32(int32_t v) {
  static_assert(G == 16 || G == 32 || G == 64, "group size");
  const int l = lane_id(), rl = l & 15;
  int32_t t;
  t = __builtin_amdgcn_mov_dpp(v, 0x111, 0xf, 0xf, false);
  if (rl >= 1) v = max(v, t);
  t = __builtin_amdgcn_mov_dpp(v, 0x112, 0xf, 0xf, false);
  if (rl >= 2) v = max(v, t);
  t = __builtin_amdgcn_mov_dpp(v, 0x114, 0xf, 0xf, false);
  if (rl >= 4) v = max(v, t);
  t = __builtin_amdgcn_mov_dpp(v, 0x118, 0xf, 0xf, false);
  if (rl >= 8) v = max(v, t);
  if (G >= 32) {
    t = __builtin_amdgcn_mov_dpp(v, 0x142, 0xf, 0xf, false);  // row_bcast:15
    if ((l & 31) >= 16) v = max(v, t);
  }
  if (G >= 64) {
    t = __builtin_amdgcn_mov_dpp(v, 0x143, 0xf, 0xf, false);  // row_bcast:31
    if (l >= 32) v = max(v, t);
  }
  if (G == 16) {
    const int32_t m0 = __builtin_amdgcn_readlane(v, 15), m1 = __builtin_amdgcn_readlane(v, 31);
    const int32_t m2 = __builtin_amdgcn_readlane(v, 47), m3 = __builtin_amdgcn_readlane(v, 63);
    const int g = l >> 4;
    return g == 0 ? m0 : g == 1 ? m1 : g == 2 ? m2 : m3;
  }
  if (G == 32) {
    const int32_t m0 = __builtin_amdgcn_readlane(v, 31), m1 = __builtin_amdgcn_readlane(v, 63);
    return l < 32 ? m0 : m1;
  }
  return __builtin_amdgcn_readlane(v, 63);
}

// inclusive prefix sum inside aligned groups of G lanes (DPP row shifts, no
// LDS crossbar): row_shr 1/2/4/8, then row_bcast 15 / 31 for G = 32 / 64
template <int G>
__device__ __forceinline__ int32_t group_incl_scan_i32(int32_t v) {
  static_assert(G == 16 || G == 32 || G == 64, "group size");
  const int l = lane_id(), rl = l & 15;
  int32_t t;
  t = __builtin_amdgcn_mov_dpp(v, 0x111, 0xf, 0xf, false);
  if (rl >= 1) v += t;
  t = __builtin_amdgcn_mov_dpp(v, 0x112, 0xf, 0xf, false);
  if (rl >= 2) v += t;
  t = __builtin_amdgcn_mov_dpp(v, 0x114, 0xf, 0xf, false);
  if (rl >= 4) v += t;
  t = __builtin_amdgcn_mov_dpp(v, 0x118, 0xf, 0xf, false);
  if (rl >= 8) v += t;
  if constexpr (G >= 32) {
    t = __builtin_amdgcn_mov_dpp(v, 0x142, 0xf, 0xf, false);  // row_bcast:15
    if ((l & 31) >= 16) v += t;
  }
  if constexpr (G >= 64) {
    t = __builtin_amdgcn_mov_dpp(v, 0x143, 0xf, 0xf, false);  // row_bcast:31
    if (l >= 32) v += t;
  }
  return v;
}

// u32 max over aligned groups of G lanes, returned to every lane of the
// group: a DPP butterfly inside each 16-lane row (quad xor 1, quad xor 2,
// half-row mirror, row mirror — each a max with a DPP operand), then the row
// maxima combined through SGPRs for G = 32 / 64
template <int G>
__device__ __forceinline__ uint32_t group_max_u32(uint32_t v) {
  static_assert(G == 16 || G == 32 || G == 64, "group size");
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false));   // quad [1,0,3,2]
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false));   // quad [2,3,0,1]
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false));  // row_half_mirror
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xf, 0xf, false));  // row_mirror
  if constexpr (G == 16) {
    return v;
  } else {
    const uint32_t r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
    const uint32_t r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
    if constexpr (G == 32) return lane_id() < 32 ? max(r0, r1) : max(r2, r3);
    return max(max(r0, r1), max(r2, r3));
  }
}

// A loaded value that must be in a register here: an empty asm reads it
// (and hands it back opaque, so nothing computed from it moves above this
// point). Put after a group of independent loads, it makes the compiler issue
// them all before its one wait. Without it the latency-bound pass kernels had
// loads sunk below the first branch that did not need them, or waited for
// early by arithmetic hoisted above a branch: one dependent memory level each.
template <typename T>
__device__ __forceinline__ void landed(T &v) {
  static_assert(std::is_arithmetic<T>::value, "a scalar value (one component of a vector load)");
  if constexpr (sizeof(T) < 4) {
    uint32_t t = (uint32_t)v;
    asm volatile("" : "+v"(t));
    v = (T)t;
  } else {
    asm volatile("" : "+v"(v));
  }
}

// u32 planes per dim of the packed 32-bit node tile (kp_score.hip pack_node)
constexpr int kPlanes = 5;

__device__ __forceinline__ void fit_rows(int32_t act, int32_t min_rpb, int32_t &rows,
                                         int32_t &rows_per_block) {
  rows = min(rows, act);
  const int32_t even = (rows + (int32_t)gridDim.y - 1) / (int32_t)gridDim.y;
  rows_per_block = min(rows_per_block, max(min_rpb, even));
}

// floor(n / c) and n mod c for a 64-bit n < 2^53 and c > 0: a double
// estimate corrected by one step each way
__device__ __forceinline__ void udivmod_uniform(uint64_t n, uint32_t c, uint64_t &Q, uint64_t &r) {
  Q = (uint64_t)((double)n / (double)c);
  int64_t rr = (int64_t)n - (int64_t)(Q * c);
  if (rr < 0) {
    --Q;
    rr += c;
  } else if (rr >= (int64_t)c) {
    ++Q;
    rr -= c;
  }
  r = (uint64_t)rr;
}

// Candidate keys: (valid bit | score | ~tie key), unique per node because the
// tie key is a bijection of the canonical position. Larger = better.
__device__ __forceinline__ uint64_t pack_key(int32_t s, uint32_t tk) {
  return (1ull << 63) | ((uint64_t)(uint32_t)s << 32) | (uint64_t)(~tk);
}
__device__ __forceinline__ int32_t key_node(uint64_t key, uint32_t sl, uint32_t inv) {
  const uint32_t tk = ~(uint32_t)key;
  return (int32_t)((tk - sl) * inv);
}
inline int blocks(int64_t n, int b) { return (int)((n + b - 1) / b); }

// rank of this lane among the set lanes of m below it (ballot compaction)
__device__ __forceinline__ int mbcnt64(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// k_csr_keys' per-round state reset, thread t of the extra workgroups of the
// kernel that opens the round's slots (the candidate merge, rk.enabled): round statistics, the previous round's
// productive passes, node segments / flags, window flags and bid minima
__device__ __forceinline__ void round_keys_init(const RoundKeys &rk, int64_t t) {
  if (t == 0) {
    const int32_t Aa = rk.A_dev ? min(rk.A, *rk.A_dev) : rk.A;
    if (Aa > 0) {
      rk.st->rounds += 1;
      rk.st->active_sum += Aa;
    }
    *rk.nl_count = 0;
  }
  if (t < rk.N) {
    rk.seg_start[t] = -1;
    rk.node_flag[t] = -1;
  }
  if (t < rk.nwin) {
    rk.win[t] = -1;
    for (int d = 0; d < rk.D; ++d) rk.bmin[(int64_t)d * rk.nwin + t] = 0;  // no bid yet
  }
  if (t < 64) {
    if (rk.pass_flag[t] != 0)
      atomicAdd(reinterpret_cast<unsigned long long *>(&rk.st->passes), 1ull);
    rk.pass_flag[t] = 0;
  }
}

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

}  // namespace dev
}  // namespace kp
