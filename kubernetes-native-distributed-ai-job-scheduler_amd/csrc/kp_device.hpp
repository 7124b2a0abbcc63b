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
// max over aligned groups of G lanes (G a power of two <= 64)
template <int G>
__device__ __forceinline__ int64_t group_max_i64(int64_t v) {
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1) {
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
