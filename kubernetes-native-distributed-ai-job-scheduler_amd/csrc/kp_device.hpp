// kp_device.hpp — device-side helpers shared by the kplace kernels: 64-lane
// wave reductions / scans (CDNA wavefront = 64, never 32) and the exact
// integer score of DESIGN.md §2.3.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

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

// §2.3: score of one more copy of q on a node whose usage is `used`;
// -1 when it does not fit. 64-bit exact; util = ((used+q) * R) >> 32 with
// R = floor(S * 2^32 / cap) never overflows because used + q <= cap.
template <int D>
__device__ __forceinline__ int64_t score_at(const ScoreParams &sp, const int64_t (&q)[D],
                                            const int64_t (&cap)[D], const int64_t (&used)[D],
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

}  // namespace dev
}  // namespace kp
