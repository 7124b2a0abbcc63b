// kp_incr.hip — gfx950 incremental candidate phase: rounds
// after the first re-score only the nodes whose usage the previous round's
// passes changed, against a per-unit list of its best KL >= K nodes.
//
// Exactness: a unit's key on a node (score, tie key) is a
// function of that node's usage alone, and usage changes only where an accept
// committed. Every unit keeps its top-KL keys and nodes from its last full
// scan or update, their count and a bound B: every node NOT in the list has a
// key below B (B = 0: the list holds every feasible node). At round r the
// list minus the changed nodes C still holds the exact best keys of the
// unchanged nodes above B; the changed nodes are re-scored exactly; the union
// above B, truncated to KL (B raised to the smallest kept key when
// truncated), is again a valid list. Its first K entries are the round's
// exact top-K candidates whenever it holds at least K keys or B = 0;
// otherwise the row is rescanned in full (k_score_topk over the round's
// rescan rows, whose merge rewrites the list). Keys are the candidate
// phase's (pack_key: unique per node), so the order is the same total order.
//
// k_cand_update: one wave per slot, 8 slots per workgroup; per slot one load
// level for the list, C / 64 re-scoring sweeps (C is the same short list for
// every slot: L2-resident gathers), the union ranked in LDS. More changed
// nodes than N / incr_cthr_div (the first rounds of a large queue): every
// slot is rescanned (a full candidate phase).
#include <hip/hip_runtime.h>

#include "kp_device.hpp"
#include "kp_internal.hpp"

namespace kp {
namespace {
using namespace dev;

constexpr int kIncWaves = 8;   // slots (waves) per workgroup
constexpr int kIncBuf = 192;   // per-wave union buffer: 128 re-scored keys + the kept list (KL <= 32)
constexpr int kIncRescored = kIncBuf - 64;

struct IncrArgs {
  ScoreParams sp;  // n_cand = the solve's K
  int32_t KL, rows, U, serial_prev, cthr;
  const int32_t *rows_dev, *act;
  uint64_t *ukey, *ubound;
  int32_t *unode, *ucnt;
  const int32_t *chg, *clist, *ccount;
  int32_t *ccount_next, *rs_count, *rs_count_next;
  const int64_t *cap, *used, *q;
  const uint32_t *R32, *K32, *salt;
  const int32_t *topo, *npos, *aff;
  int32_t *cand, *rs_slot, *rs_unit;
  RoundKeys rk;  // enabled: k_csr_keys' work for the completed slots (+ init workgroups)
};

// S(q | n, usage) exactly as the candidate phase (§2.3), -1 when q does not
// fit: W32 (every cap and request < 2^32) through the node's division tables,
// else the 64-bit form
template <int D, bool W32>
__device__ __forceinline__ int32_t rescore(const IncrArgs &a, int32_t n, const int64_t (&q)[D],
                                           int32_t af) {
  const ScoreParams &sp = a.sp;
  const int32_t N = sp.N;
  int64_t c[D], u[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    c[d] = a.cap[(int64_t)d * N + n];
    u[d] = a.used[(int64_t)d * N + n];
  }
  const int32_t tp = a.topo[n];
  if constexpr (W32) {
    bool fits = true;
#pragma unroll
    for (int d = 0; d < D; ++d) fits &= q[d] <= c[d] - u[d];
    if (!fits) return -1;
    int32_t acc = 0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (c[d] == 0) continue;  // cap-0 dims contribute 0 (q = 0 there)
      const uint32_t x = (uint32_t)(u[d] + q[d]), cc = (uint32_t)c[d];
      bool nz;
      const uint32_t t = div_floor32(x, cc, a.R32[(int64_t)d * N + n], a.K32[(int64_t)d * N + n] & 63u,
                                     (uint32_t)sp.S, nz);
      // LeastAllocated: floor((c - x) S / c) = S - ceil(x S / c)
      const int32_t util = sp.most_allocated ? (int32_t)t : sp.S - (int32_t)t - (nz ? 1 : 0);
      acc += sp.w[d] * util;
    }
    const int g = sp.gpu_dim;
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (d == g && q[d] > 0 && c[d] - u[d] - q[d] == 0) acc += sp.w_gpu_fit;
    if (af >= 0 && tp == af) acc += sp.w_affinity;
    return acc;
  } else {
    return (int32_t)score_at<D>(sp, q, c, u, tp, af);
  }
}

template <int D, bool W32>
__global__ __launch_bounds__(64 * kIncWaves) void k_cand_update(IncrArgs a) {
  __shared__ uint64_t sk[kIncWaves][kIncBuf];
  __shared__ int32_t sn[kIncWaves][kIncBuf];
  __shared__ int32_t s_need[kIncWaves];
  __shared__ int32_t s_base;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rblocks = (a.rows + kIncWaves - 1) / kIncWaves;
  if ((int)blockIdx.x >= rblocks) {  // extra workgroups: the round state (k_csr_keys' init part)
    round_keys_init(a.rk, (int64_t)(blockIdx.x - rblocks) * (64 * kIncWaves) + threadIdx.x);
    return;
  }
  const ScoreParams &sp = a.sp;
  const int K = sp.n_cand, KL = a.KL;
  const int32_t A = a.rows_dev ? min(a.rows, *a.rows_dev) : a.rows;
  const int32_t nc = *a.ccount;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // the next round's counters (their last readers ran in the previous round)
    *a.ccount_next = 0;
    *a.rs_count_next = 0;
  }
  const int row = blockIdx.x * kIncWaves + wave;
  const bool in = row < A;
  if (nc > a.cthr) {  // too many changed nodes: every slot is rescanned (workgroup-uniform)
    if (in && lane == 0) {
      a.rs_slot[row] = row;
      a.rs_unit[row] = a.act[row];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.rs_count = A;
    return;
  }
  bool need = false;
  int32_t u = 0;
  if (in) {
    u = a.act[row];
    const int64_t lb = (int64_t)u * KL;
    const int32_t cnt = a.ucnt[u];
    const uint64_t B = a.ubound[u];
    uint64_t lk = 0;
    int32_t ln = -1;
    if (lane < cnt) {
      lk = a.ukey[lb + lane];
      ln = a.unode[lb + lane];
    }
    int64_t q[D];
#pragma unroll
    for (int d = 0; d < D; ++d) q[d] = a.q[(int64_t)d * a.U + u];
    const int32_t af = a.aff[u];
    const uint32_t sl = sp.tie_rotated ? a.salt[u] : 0u;
    // list entries on changed nodes leave; the changed nodes come back re-scored
    const bool keep = lane < cnt && a.chg[ln] != a.serial_prev;
    int m = 0;
    for (int i0 = 0; i0 < nc; i0 += 64) {  // wave-uniform
      const int i = i0 + lane;
      bool hit = false;
      uint64_t key = 0;
      int32_t n = -1;
      if (i < nc) {
        n = a.clist[i];
        const int32_t s = rescore<D, W32>(a, n, q, af);
        if (s >= 0) {
          const uint32_t pos = (uint32_t)a.npos[n];
          key = pack_key(s, sp.tie_rotated ? pos * kTieMul + sl : pos);
          hit = key >= B;  // a key below B may sit below unlisted nodes
        }
      }
      const uint64_t hm = __ballot(hit);
      const int p = m + mbcnt64(hm);
      if (hit && p < kIncRescored) {
        sk[wave][p] = key;
        sn[wave][p] = n;
      }
      m += __popcll(hm);
    }
    if (m > kIncRescored) {
      need = true;  // more re-scored keys above B than the buffer holds: rescan
    } else {
      const uint64_t km = __ballot(keep);
      if (keep) {
        const int p = m + mbcnt64(km);
        sk[wave][p] = lk;
        sn[wave][p] = ln;
      }
      const int T = m + __popcll(km);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // rank of every union element (keys are unique): lane holds elements
      // lane, lane + 64, lane + 128
      uint64_t e[3];
      int32_t en[3], r[3] = {0, 0, 0};
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int idx = lane + 64 * t;
        e[t] = idx < T ? sk[wave][idx] : 0ull;
        en[t] = idx < T ? sn[wave][idx] : -1;
      }
      for (int j = 0; j < T; ++j) {  // broadcast LDS reads
        const uint64_t x = sk[wave][j];
#pragma unroll
        for (int t = 0; t < 3; ++t) r[t] += x > e[t] ? 1 : 0;
      }
      const int ncnt = min(T, KL);
      // truncated: the bound rises to the smallest kept key
      uint64_t B2 = B;
      if (T > KL) {
        uint64_t bk = 0;
#pragma unroll
        for (int t = 0; t < 3; ++t)
          if (lane + 64 * t < T && r[t] == KL - 1) bk = e[t];
        B2 = wave_max_u64_dpp(bk);
      }
      if (ncnt < K && B2 != 0) {
        need = true;  // fewer than K known keys above the bound: rescan
      } else {
        int32_t *out = a.cand + (int64_t)row * K;
#pragma unroll
        for (int t = 0; t < 3; ++t)
          if (lane + 64 * t < T && r[t] < KL) {
            a.ukey[lb + r[t]] = e[t];
            a.unode[lb + r[t]] = en[t];
            if (r[t] < K) out[r[t]] = en[t];
          }
        if (lane >= ncnt && lane < K) out[lane] = -1;  // every feasible node listed, fewer than K
        if (lane == 0) {
          a.ucnt[u] = ncnt;
          a.ubound[u] = B2;
        }
        if (a.rk.enabled) {
          // candidate `lane` of the slot: the holder of rank j hands its node
          // to lane j through LDS (every lane read its elements above)
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
          for (int t = 0; t < 3; ++t)
            if (lane + 64 * t < T && r[t] < K) sn[wave][r[t]] = en[t];
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          const int32_t cn = lane < ncnt && lane < K ? sn[wave][lane] : -1;
          round_keys_slot(a.rk, row, u, K, cn, lane);
        }
      }
    }
  }
  // the rows to rescan: one counter add per workgroup
  if (lane == 0) s_need[wave] = in && need ? 1 : 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t tot = 0;
    for (int w = 0; w < kIncWaves; ++w) tot += s_need[w];
    s_base = tot ? atomicAdd(a.rs_count, tot) : 0;
  }
  __syncthreads();
  if (in && need && lane == 0) {
    int32_t idx = s_base;
    for (int w = 0; w < wave; ++w) idx += s_need[w];
    a.rs_slot[idx] = row;
    a.rs_unit[idx] = u;
  }
}

template <int D>
struct IncrL {
  static int run(kp_ctx *c, const IncrArgs &a, int32_t rows, bool keys) {
    const unsigned grid = (unsigned)(blocks(rows, kIncWaves) +
                                     (keys ? blocks(a.rk.init_n, 64 * kIncWaves) : 0));
    if (c->fits32)
      hipLaunchKernelGGL((k_cand_update<D, true>), dim3(grid), dim3(64 * kIncWaves), 0, c->stream, a);
    else
      hipLaunchKernelGGL((k_cand_update<D, false>), dim3(grid), dim3(64 * kIncWaves), 0, c->stream, a);
    KP_HIP(hipGetLastError());
    return KP_OK;
  }
};

}  // namespace

int launch_cand_update(kp_ctx *c, const ScoreParams &sp, int32_t KL, int32_t rows,
                       const int32_t *rows_dev, int32_t round, bool keys) {
  if (rows <= 0 || c->N == 0) return KP_OK;
  const int par = round & 1;
  IncrArgs a{};
  a.sp = sp;
  a.KL = KL;
  a.rows = rows;
  a.U = c->U;
  a.serial_prev = c->cur_serial - 1;
  a.cthr = std::max(64, c->N / std::max(1, c->incr_cthr_div));
  a.rows_dev = rows_dev;
  a.act = c->d.act_local;
  a.ukey = c->d.ukey;
  a.ubound = c->d.ubound;
  a.unode = c->d.unode;
  a.ucnt = c->d.ucnt;
  a.chg = c->d.chg;
  a.clist = c->d.clist + (size_t)par * c->cap_N;
  a.ccount = c->d.counters + kCCount + par;
  a.ccount_next = c->d.counters + kCCount + (par ^ 1);
  a.rs_count = c->d.counters + kRsCount + par;
  a.rs_count_next = c->d.counters + kRsCount + (par ^ 1);
  a.cap = c->d.cap;
  a.used = c->d.used;
  a.q = c->d.q;
  a.R32 = c->d.R32;
  a.K32 = c->d.K32;
  a.salt = c->d.salt;
  a.topo = c->d.topo;
  a.npos = c->d.npos;
  a.aff = c->d.aff;
  a.cand = c->d.cand_local;
  a.rs_slot = c->d.rs_slot;
  a.rs_unit = c->d.rs_unit;
  if (keys) a.rk = round_keys_args(c, rows, sp.n_cand, c->d.counters);
  return dispatch_D<IncrL>(c->D, c, a, rows, keys);
}

}  // namespace kp
