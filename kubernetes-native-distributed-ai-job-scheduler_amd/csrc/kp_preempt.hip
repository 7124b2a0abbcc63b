// kp_preempt.hip — gfx950 preemption-candidate scoring (DESIGN.md §2.9,
// BASELINE config #4), bit-exact with oracle/kp_oracle.c kpo_preempt.
//
// Rows = preemptors (NO_FIT singleton units, compacted after the solve),
// columns = nodes. The victim pool is a node-major CSR of the running jobs,
// sorted (node, priority desc, running index asc) once at kp_load_running,
// with per-node suffix sums of their requests so that "free + everything
// evictable" is one load per dim. A workgroup owns RB preemptor rows and
// sweeps every node (thread per node, node data re-read from L2 per tile);
// the reprieve walk is a short per-thread loop over the node's evictable
// running jobs. Each thread keeps its best (victims, cost, node) per row and
// the workgroup reduces them lexicographically.
#include <hip/hip_runtime.h>

#include <cstring>

#include <rocprim/rocprim.hpp>

#include "kp_device.hpp"
#include "kp_internal.hpp"

namespace kp {
namespace {
using namespace dev;

constexpr int kPreRows = 4;  // preemptor rows per workgroup

struct Best {
  int32_t cnt;
  int64_t cost;
  int32_t node;  // -1 = none
};

__device__ __forceinline__ bool better(const Best &a, const Best &b) {
  if (a.node < 0) return false;
  if (b.node < 0) return true;
  if (a.cnt != b.cnt) return a.cnt < b.cnt;
  if (a.cost != b.cost) return a.cost < b.cost;
  return a.node < b.node;
}

template <int D>
__global__ __launch_bounds__(256) void k_preempt(int32_t N, int32_t U, int32_t P, int32_t R,
                                                 const int32_t *__restrict__ plist,
                                                 const int64_t *__restrict__ q,
                                                 const int32_t *__restrict__ uprio,
                                                 const int32_t *__restrict__ leader,
                                                 const int64_t *__restrict__ cap,
                                                 const int64_t *__restrict__ used,
                                                 const int32_t *__restrict__ roff,
                                                 const int64_t *__restrict__ rreq,
                                                 const int64_t *__restrict__ rsuf,
                                                 const int32_t *__restrict__ rprio,
                                                 int32_t *__restrict__ out_node,
                                                 int32_t *__restrict__ out_vict,
                                                 int64_t *__restrict__ out_cost) {
  __shared__ int64_t sq[kPreRows][D];
  __shared__ int32_t spr[kPreRows];
  __shared__ Best wbest[kPreRows][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x * kPreRows;
  const int nrows = min(kPreRows, P - r0);
  if (tid < nrows * D) {
    const int rr = tid / D, d = tid % D;
    sq[rr][d] = q[(int64_t)d * U + plist[r0 + rr]];
  }
  if (tid < nrows) spr[tid] = uprio[plist[r0 + tid]];
  __syncthreads();
  Best best[kPreRows];
#pragma unroll
  for (int rr = 0; rr < kPreRows; ++rr) best[rr] = Best{0, 0, -1};
  for (int n = tid; n < N; n += 256) {
    const int32_t e0 = roff[n], e1 = roff[n + 1];
    int64_t fr[D];
#pragma unroll
    for (int d = 0; d < D; ++d) fr[d] = cap[(int64_t)d * N + n] - used[(int64_t)d * N + n];
#pragma unroll
    for (int rr = 0; rr < kPreRows; ++rr) {
      if (rr >= nrows) break;
      const int32_t p = spr[rr];
      int32_t f = e0;
      while (f < e1 && rprio[f] >= p) ++f;  // evictable = [f, e1)
      int64_t av[D];
      bool ok = true;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        av[d] = fr[d] + (f < e1 ? rsuf[(int64_t)d * R + f] : 0);
        ok &= sq[rr][d] <= av[d];
      }
      if (!ok) continue;
      int32_t cnt = 0;
      int64_t cost = 0;
      for (int32_t e = f; e < e1; ++e) {
        int64_t x[D];
        bool spare = true;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          x[d] = rreq[(int64_t)d * R + e];
          spare &= sq[rr][d] <= av[d] - x[d];
        }
        if (spare) {
#pragma unroll
          for (int d = 0; d < D; ++d) av[d] -= x[d];
        } else {
          ++cnt;
          cost += rprio[e];
        }
      }
      const Best c{cnt, cost, n};
      if (better(c, best[rr])) best[rr] = c;  // n ascends per thread: ties keep the earlier
    }
  }
  // workgroup reduction per row: wave butterfly, then the 4 wave results
#pragma unroll
  for (int rr = 0; rr < kPreRows; ++rr) {
    Best b = best[rr];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      Best o;
      o.cnt = __shfl_xor(b.cnt, m, kWave);
      o.cost = (int64_t)shfl_xor_u64((uint64_t)b.cost, m);
      o.node = __shfl_xor(b.node, m, kWave);
      if (better(o, b)) b = o;
    }
    if (lane == 0) wbest[rr][wave] = b;
  }
  __syncthreads();
  if (tid < nrows) {
    Best b = wbest[tid][0];
    for (int w = 1; w < 4; ++w)
      if (better(wbest[tid][w], b)) b = wbest[tid][w];
    const int32_t j = leader[plist[r0 + tid]];
    out_node[j] = b.node;
    out_vict[j] = b.node >= 0 ? b.cnt : 0;
    out_cost[j] = b.node >= 0 ? b.cost : 0;
  }
}

// Tiled 32-bit form (every cap and request < 2^32, so a node's free capacity
// plus all its running requests stays below its capacity; and (victims,
// cost, node) packs into one ordered 64-bit key, kp_load_running checks the
// bounds). A workgroup owns kPtRows (32) preemptor rows (requests in LDS) and
// sweeps the nodes in tiles of 256, one node per thread: the node's free
// capacity and up to kPreRun (16) running jobs (priority, request) are loaded into
// registers ONCE per tile and evaluated against every row of the block, so
// the node table is read once per kPtRows rows. Per row and tile a wave
// minimum of the packed keys (DPP) and a 4-wave merge into the row's running
// best in LDS. Nodes with more running jobs walk their list in global memory.
// Same order and tie rules as k_preempt: fewest victims, lowest victim
// priority sum, lowest node index.
#ifndef KP_PT_ROWS
#define KP_PT_ROWS 32  // preemptor rows per workgroup (64: +1 ms, 128: +18 ms on config #4, tools/ab_preempt.sh)
#endif
#ifndef KP_PRE_RUN
#define KP_PRE_RUN 16  // running jobs per node in registers (8: +18 ms, 12: +1 ms, 24: +19 ms)
#endif
constexpr int kPtRows = KP_PT_ROWS;
constexpr int kPreRun = KP_PRE_RUN;

__device__ __forceinline__ uint64_t pre_key(int32_t cnt, int64_t cost, int32_t node) {
  return ((uint64_t)cnt << 52) | ((uint64_t)(cost + ((int64_t)1 << 31)) << 20) | (uint64_t)node;
}

template <int D>
__global__ __launch_bounds__(256) void k_preempt_t(int32_t N, int32_t U, int32_t P, int32_t R,
                                                   const int32_t *__restrict__ plist,
                                                   const int64_t *__restrict__ q,
                                                   const int32_t *__restrict__ uprio,
                                                   const int32_t *__restrict__ leader,
                                                   const int64_t *__restrict__ cap,
                                                   const int64_t *__restrict__ used,
                                                   const int32_t *__restrict__ roff,
                                                   const int64_t *__restrict__ rreq,
                                                   const int64_t *__restrict__ rsuf,
                                                   const int32_t *__restrict__ rprio,
                                                   int32_t *__restrict__ out_node,
                                                   int32_t *__restrict__ out_vict,
                                                   int64_t *__restrict__ out_cost) {
  __shared__ uint32_t sq[kPtRows][D];
  __shared__ int32_t spr[kPtRows];
  __shared__ uint64_t sbest[kPtRows];
  __shared__ uint64_t swb[kPtRows][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x * kPtRows;
  const int nrows = min(kPtRows, P - r0);
  for (int i = tid; i < nrows * D; i += 256) {
    const int rr = i / D, d = i % D;
    sq[rr][d] = (uint32_t)q[(int64_t)d * U + plist[r0 + rr]];
  }
  for (int i = tid; i < nrows; i += 256) {
    spr[i] = uprio[plist[r0 + i]];
    sbest[i] = ~0ull;
  }
  __syncthreads();
  for (int t0 = 0; t0 < N; t0 += 256) {
    const int n = t0 + tid;
    const bool valid = n < N;
    const int32_t e0 = valid ? roff[n] : 0, e1 = valid ? roff[n + 1] : 0, cnt = e1 - e0;
    uint32_t fr[D];
#pragma unroll
    for (int d = 0; d < D; ++d)
      fr[d] = valid ? (uint32_t)(cap[(int64_t)d * N + n] - used[(int64_t)d * N + n]) : 0u;
    const bool shortl = cnt <= kPreRun;
    int32_t pr[kPreRun];
    uint32_t rq[kPreRun][D];
#pragma unroll
    for (int k = 0; k < kPreRun; ++k) {
      const bool v = shortl && k < cnt;
      pr[k] = v ? rprio[e0 + k] : INT32_MAX;  // padding: never evictable
#pragma unroll
      for (int d = 0; d < D; ++d) rq[k][d] = v ? (uint32_t)rreq[(int64_t)d * R + e0 + k] : 0u;
    }
    for (int rr = 0; rr < nrows; ++rr) {
      const int32_t p = spr[rr];
      uint32_t qd[D], av[D];
      // free + every evictable request (priority < p): from the registers, or
      // the suffix sum of a long list past its non-evictable prefix
      int32_t f = e0;
      if (!shortl)
        while (f < e1 && rprio[f] >= p) ++f;  // evictable = [f, e1)
      bool ok = valid;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        qd[d] = sq[rr][d];
        av[d] = fr[d];
        if (shortl) {
#pragma unroll
          for (int k = 0; k < kPreRun; ++k) av[d] += pr[k] < p ? rq[k][d] : 0u;
        } else {
          av[d] += f < e1 ? (uint32_t)rsuf[(int64_t)d * R + f] : 0u;
        }
        ok &= qd[d] <= av[d];
      }
      if (__ballot(ok) == 0) {  // no node of this wave qualifies for the row (wave-uniform)
        if (lane == 0) swb[rr][wave] = ~0ull;
        continue;
      }
      int32_t vc = 0;
      int64_t cost = 0;
      if (shortl) {
        // reprieve walk in (priority desc, running index asc) order
#pragma unroll
        for (int k = 0; k < kPreRun; ++k) {
          bool spare = true;
#pragma unroll
          for (int d = 0; d < D; ++d) spare &= qd[d] <= av[d] - rq[k][d];
          const bool ev = ok && pr[k] < p;
#pragma unroll
          for (int d = 0; d < D; ++d) av[d] -= ev && spare ? rq[k][d] : 0u;
          vc += ev && !spare ? 1 : 0;
          cost += ev && !spare ? pr[k] : 0;
        }
      } else {  // a long victim list: walk it in global memory
        for (int32_t e = f; ok && e < e1; ++e) {
          uint32_t x[D];
          bool spare = true;
#pragma unroll
          for (int d = 0; d < D; ++d) {
            x[d] = (uint32_t)rreq[(int64_t)d * R + e];
            spare &= qd[d] <= av[d] - x[d];
          }
          if (spare) {
#pragma unroll
            for (int d = 0; d < D; ++d) av[d] -= x[d];
          } else {
            ++vc;
            cost += rprio[e];
          }
        }
      }
      const uint64_t key = ok ? pre_key(vc, cost, n) : ~0ull;
      const uint64_t m = ~wave_max_u64_dpp(~key);  // the wave's smallest key
      if (lane == 0) swb[rr][wave] = m;
    }
    __syncthreads();
    for (int rr = tid; rr < nrows; rr += 256) {
      uint64_t b = sbest[rr];
#pragma unroll
      for (int w = 0; w < 4; ++w) b = swb[rr][w] < b ? swb[rr][w] : b;
      sbest[rr] = b;
    }
    __syncthreads();  // swb is rewritten by the next tile
  }
  for (int rr = tid; rr < nrows; rr += 256) {
    const uint64_t b = sbest[rr];
    const int32_t j = leader[plist[r0 + rr]];
    const bool has = b != ~0ull;
    out_node[j] = has ? (int32_t)(b & 0xFFFFFull) : -1;
    out_vict[j] = has ? (int32_t)(b >> 52) : 0;
    out_cost[j] = has ? (int64_t)((b >> 20) & 0xFFFFFFFFull) - ((int64_t)1 << 31) : 0;
  }
}

__global__ void k_preempt_flags(const int32_t *__restrict__ status,
                                const int32_t *__restrict__ size, int32_t U,
                                int32_t *__restrict__ flag) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u < U) flag[u] = (status[u] == kNoFit && size[u] == 1) ? 1 : 0;
}

__global__ void k_preempt_init(int32_t J, int32_t *__restrict__ node, int32_t *__restrict__ vict,
                               int64_t *__restrict__ cost) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= J) return;
  node[j] = -1;
  vict[j] = 0;
  cost[j] = 0;
}

template <int D>
struct PreemptL {
  static int run(kp_ctx *c, int32_t lo, int32_t P) {  // preemptor rows [lo, lo + P)
    const int32_t *plist = c->d.plist + lo;
    // the tiled kernel sums free capacity and evictable requests in u32: after
    // kp_apply_delta lowers usage below the running jobs' sum, that sum can
    // reach ~2 x cap, so it needs every cap < 2^31
    if (c->fits32 && c->preempt32 && c->pre_key_ok && c->max_cap < ((int64_t)1 << 31)) {
      hipLaunchKernelGGL((k_preempt_t<D>), dim3(blocks(P, kPtRows)), dim3(256), 0, c->stream, c->N,
                         c->U, P, c->R, plist, c->d.q, c->d.uprio, c->d.leader, c->d.cap,
                         c->d.used, c->d.roff, c->d.rreq, c->d.rsuf, c->d.rprio, c->d.pre_node,
                         c->d.pre_vict, c->d.pre_cost);
      KP_HIP(hipGetLastError());
      return KP_OK;
    }
    hipLaunchKernelGGL((k_preempt<D>), dim3(blocks(P, kPreRows)), dim3(256), 0, c->stream, c->N,
                       c->U, P, c->R, plist, c->d.q, c->d.uprio, c->d.leader, c->d.cap,
                       c->d.used, c->d.roff, c->d.rreq, c->d.rsuf, c->d.rprio, c->d.pre_node,
                       c->d.pre_vict, c->d.pre_cost);
    KP_HIP(hipGetLastError());
    return KP_OK;
  }
};

// Multi-rank preemption: rank r scores the preemptor rows [lo_r, hi_r) of the
// (replicated) preemptor list; the per-row results travel as fixed blocks of
// B = ceil(P / world) rows x {node, victims, cost lo, cost hi} through one
// all-gather, and every rank scatters all of them to the preemptors' jobs.
__global__ void k_preempt_pack(int32_t lo, int32_t hi, const int32_t *__restrict__ plist,
                               const int32_t *__restrict__ leader,
                               const int32_t *__restrict__ node, const int32_t *__restrict__ vict,
                               const int64_t *__restrict__ cost, int32_t *__restrict__ send) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (lo + i >= hi) return;
  const int32_t j = leader[plist[lo + i]];
  const uint64_t cu = (uint64_t)cost[j];
  send[4 * i] = node[j];
  send[4 * i + 1] = vict[j];
  send[4 * i + 2] = (int32_t)(uint32_t)cu;
  send[4 * i + 3] = (int32_t)(uint32_t)(cu >> 32);
}

__global__ void k_preempt_unpack(int32_t P, int32_t world, int32_t B,
                                 const int32_t *__restrict__ plist,
                                 const int32_t *__restrict__ leader,
                                 const int32_t *__restrict__ recv, int32_t *__restrict__ node,
                                 int32_t *__restrict__ vict, int64_t *__restrict__ cost) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;  // preemptor row
  if (r >= P) return;
  // owner rank w of row r: lo_w = floor(P w / world) <= r < lo_{w+1}
  int w = (int)(((int64_t)r * world) / P);
  while (w + 1 < world && ((int64_t)P * (w + 1)) / world <= r) ++w;
  while (w > 0 && ((int64_t)P * w) / world > r) --w;
  const int32_t lo = (int32_t)(((int64_t)P * w) / world);
  const int32_t *x = recv + ((int64_t)w * B + (r - lo)) * 4;
  const int32_t j = leader[plist[r]];
  node[j] = x[0];
  vict[j] = x[1];
  cost[j] = (int64_t)(((uint64_t)(uint32_t)x[3] << 32) | (uint32_t)x[2]);
}

}  // namespace

// preemptor compaction (NO_FIT singletons, rank order) -> count to host; the
// scoring of this rank's rows [*lo, *hi) (all of them on one rank)
int launch_preempt(kp_ctx *c, int32_t *P_host, int32_t *lo, int32_t *hi) {
  *P_host = 0;
  *lo = *hi = 0;
  const int32_t U = c->U, J = c->J;
  if (J > 0) {
    hipLaunchKernelGGL(k_preempt_init, dim3(blocks(J, 256)), dim3(256), 0, c->stream, J,
                       c->d.pre_node, c->d.pre_vict, c->d.pre_cost);
    KP_HIP(hipGetLastError());
  }
  if (U == 0) return KP_OK;
  hipLaunchKernelGGL(k_preempt_flags, dim3(blocks(U, 256)), dim3(256), 0, c->stream, c->d.status,
                     c->d.size, U, c->d.flag);
  KP_HIP(hipGetLastError());
  KP_TRY(launch_compact_to(c, c->d.flag, 0, U, c->d.plist, nullptr));
  KP_HIP(hipMemcpyAsync(c->pinned, c->d.counters, sizeof(int32_t), hipMemcpyDeviceToHost,
                        c->stream));
  KP_HIP(hipStreamSynchronize(c->stream));
  const int32_t P = c->pinned[0];
  *P_host = P;
  *lo = (int32_t)(((int64_t)P * c->rank) / c->world);
  *hi = (int32_t)(((int64_t)P * (c->rank + 1)) / c->world);
  if (*hi == *lo || c->N == 0) return KP_OK;
  return dispatch_D<PreemptL>(c->D, c, *lo, *hi - *lo);
}

int launch_preempt_pack(kp_ctx *c, int32_t lo, int32_t hi, int32_t *send) {
  if (hi > lo) {
    hipLaunchKernelGGL(k_preempt_pack, dim3(blocks(hi - lo, 256)), dim3(256), 0, c->stream, lo, hi,
                       c->d.plist, c->d.leader, c->d.pre_node, c->d.pre_vict, c->d.pre_cost, send);
    KP_HIP(hipGetLastError());
  }
  return KP_OK;
}

int launch_preempt_unpack(kp_ctx *c, int32_t P, int32_t B, const int32_t *recv) {
  if (P > 0) {
    hipLaunchKernelGGL(k_preempt_unpack, dim3(blocks(P, 256)), dim3(256), 0, c->stream, P, c->world,
                       B, c->d.plist, c->d.leader, recv, c->d.pre_node, c->d.pre_vict,
                       c->d.pre_cost);
    KP_HIP(hipGetLastError());
  }
  return KP_OK;
}

}  // namespace kp
