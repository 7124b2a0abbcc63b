// kp_topk.hip — gfx950 fused filter + score + top-K of the solve's candidate
// phase: the J x N scores never reach HBM.
//
// The node table is packed in the class-aligned canonical layout (pack_node
// with colnode: nodes sorted by capacity vector, every capacity class
// starting on a 128-column wave tile, padding columns infeasible), so the 128
// columns of a wave share one capacity vector and a pair's exact utilisation
// is the compare-and-select form of k_score32's uniform path.
//
// k_score_topk: a 512-thread workgroup owns 1,024 columns (8 waves x 64 lanes
// x 2 columns, tile operands in VGPRs) and streams its rows in chunks of 8:
//   1. score — the chunk's row records (thresholds c - rho of the wave's
//      capacity class, WQ, requests: k_unit_rec, once per solve; without
//      them each wave computes its class's thresholds with one exact division
//      per (row, dim) lane) reach LDS by DMA one chunk ahead; each wave
//      writes its 128 scores of every row into the LDS tile (16-bit, double
//      buffered when every score fits);
//   2. select — wave w reads row w of the chunk back (16 columns per lane,
//      4-column groups strided over the tile; rows padded so that no LDS
//      access conflicts): lane best of 32-bit truncated keys (and its best per
//      group), T = the K-th lane best by a radix search over ballots (a lower
//      bound of the tile's K-th key: K distinct columns reach it; truncation
//      only keeps more), the survivors >= T of the groups whose best reached
//      T appended to LDS, exact ranks from LDS broadcast reads; the tile's
//      top-K exact keys, best first, go to part[row][tile]. More than 128
//      survivors (adversarial ties) switch to an exact bisection for the K-th
//      64-bit key.
// k_merge_tour merges a row's per-tile lists into its K candidates, mapping
// canonical position -> node through perm. Bit-exact with the materialised
// path (k_score32 + k_select_t) and oracle kpo_round_candidates: every
// global top-K key is in its tile's exact top-K.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "kp_device.hpp"
#include "kp_internal.hpp"

// KP_FZ_EXP=1: a measurement-only build (tools/build_variant.sh, the VALU
// split of tools/gpu_evidence.sh) whose k_score_topk skips the select phase;
// never the product
#ifndef KP_FZ_EXP
#define KP_FZ_EXP 0
#endif
// KP_FZ_PROFILE: per-phase shader-clock sums (s_memtime deltas of every
// wave, lane 0 adds them into prof[phase]); a timing build only
#ifdef KP_FZ_PROFILE
#define KP_FZ_PROF_MARK(ph)                           \
  do {                                                \
    const uint64_t now_ = __builtin_amdgcn_s_memtime(); \
    pacc_[ph] += now_ - t_prev_;                      \
    t_prev_ = now_;                                   \
  } while (0)
#define KP_FZ_PROF_FLUSH()                                                               \
  do {                                                                                   \
    if (prof && lane == 0)                                                               \
      for (int p_ = 0; p_ < 9; ++p_)                                                     \
        atomicAdd((unsigned long long *)&prof[p_], (unsigned long long)pacc_[p_]);       \
  } while (0)
#else
#define KP_FZ_PROF_MARK(ph) \
  do {                      \
  } while (0)
#define KP_FZ_PROF_FLUSH() \
  do {                     \
  } while (0)
#endif
#ifndef KP_FZ_RANK_UNROLL
#define KP_FZ_RANK_UNROLL 2  // survivor rank loop unroll (4: +10 ms on config #4, spills)
#endif
#ifndef KP_FZ_ROW_UNROLL
#define KP_FZ_ROW_UNROLL 2  // rows of the score loop interleaved (1: config #4 +2 ms, r05)
#endif

namespace kp {
namespace {
using namespace dev;

#ifndef KP_MERGE_WPB
#define KP_MERGE_WPB 4  // k_merge_tour rows (waves) per workgroup
#endif
constexpr int kMergeWPB = KP_MERGE_WPB;
constexpr int kMergeLoadBatch = 8;  // k_merge_tour: list loads per lane in flight
constexpr int kFzMaxRows = 128;          // rows per workgroup (request stage)
constexpr int kFzSurv = 128;             // survivor slots per wave (2 per lane)
// Workgroup shape of k_score_topk: NW waves x 128 columns (2 per lane) =
// the tile whose exact top-K one select per row produces. NW = 8: 1,024
// columns, 3 workgroups per CU. (NW = 16 — 2,048 columns, one workgroup per
// CU, half the per-(row, tile) select and merge work — measured slower in
// r05: config #3 +0.2-1.5 ms, config #4 620 vs 552 ms)
template <int NW>
struct FzShape {
  static constexpr int BS = 64 * NW;     // threads
  static constexpr int TILE = 128 * NW;  // columns per workgroup
  static constexpr int RC = NW;          // rows per LDS chunk: one per wave in the select
  static constexpr int GPL = NW / 2;     // 4-column groups per lane in the select
  static_assert(kFzTileMax % TILE == 0, "the tile width divides the layout's alignment");
};

template <int D>
constexpr int fz_dp() {
  return D <= 1 ? 1 : D <= 2 ? 2 : D <= 4 ? 4 : 8;
}

__device__ __forceinline__ uint32_t rl(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}

// value of lane ^ M (M = 1, 2, 4) through DPP: quad permutes for 1 and 2,
// row shifts by 4 for 4 (VALU only, no LDS crossbar)
template <int M>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
  if constexpr (M == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);  // [1,0,3,2]
  } else if constexpr (M == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);  // [2,3,0,1]
  } else {
    static_assert(M == 4, "xor 1, 2 or 4");
    const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x104, 0xf, 0xf, false);  // row_shl:4
    const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    return (__lane_id() & 4) ? dn : up;
  }
}

template <int W>
struct RowRec {  // one LDS row record in registers (W % 4 == 0 words)
  uint4 v[W / 4];
  __device__ __forceinline__ void load(const uint32_t *p) {
#pragma unroll
    for (int i = 0; i < W / 4; ++i) v[i] = reinterpret_cast<const uint4 *>(p)[i];
  }
  __device__ __forceinline__ uint32_t operator[](int j) const {
    const uint4 &x = v[j >> 2];
    return (j & 3) == 0 ? x.x : (j & 3) == 1 ? x.y : (j & 3) == 2 ? x.z : x.w;
  }
};

// a wave-uniform value held in a VGPR (VOP3 compares / selects read at most
// one scalar operand: the lane mask)
__device__ __forceinline__ int32_t in_vgpr(int32_t x) {
  int32_t r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
  return r;
}

// the 4 scores of 4-column group g of an LDS score row (u32 or packed u16)
template <bool H16>
__device__ __forceinline__ void load_group(const uint32_t *row, int g, uint32_t (&v)[4]) {
  if constexpr (H16) {
    const uint2 x = reinterpret_cast<const uint2 *>(row)[g];
    v[0] = x.x & 0xFFFFu;
    v[1] = x.x >> 16;
    v[2] = x.y & 0xFFFFu;
    v[3] = x.y >> 16;
  } else {
    const uint4 x = reinterpret_cast<const uint4 *>(row)[g];
    v[0] = x.x;
    v[1] = x.y;
    v[2] = x.z;
    v[3] = x.w;
  }
}

template <bool H16>
__device__ __forceinline__ uint32_t load_one(const uint32_t *row, int col) {
  if constexpr (H16)
    return reinterpret_cast<const uint16_t *>(row)[col];
  else
    return row[col];
}


#ifndef KP_FZ_WAVES_PER_EU
#define KP_FZ_WAVES_PER_EU 6  // NW = 8: 80 VGPRs, 3 workgroups of 8 waves per CU (a small spill is cheaper than 2)
#endif
template <int D, bool MOST, bool H16, int NW, bool PRE>
__global__ __launch_bounds__(64 * NW)
__attribute__((amdgpu_waves_per_eu(NW == 8 ? KP_FZ_WAVES_PER_EU : 4, NW == 8 ? KP_FZ_WAVES_PER_EU : 4)))
void k_score_topk(
    ScoreParams sp, const uint32_t *__restrict__ np, int32_t P, const int64_t *__restrict__ q,
    int32_t qstride, const int32_t *__restrict__ uaff, const uint32_t *__restrict__ salt,
    const int32_t *__restrict__ rows_unit, int32_t rows, int32_t rows_per_block, int32_t min_rpb,
    const int32_t *__restrict__ rows_dev, const int32_t *__restrict__ wshift, int32_t ksh, int32_t tbits,
    uint64_t *__restrict__ part, uint64_t *__restrict__ prof, const uint32_t *__restrict__ crec,
    const int32_t *__restrict__ tcls, int32_t nfc) {
  using FS = FzShape<NW>;
  constexpr int kFzBS = FS::BS, kFzTile = FS::TILE, kFzRC = FS::RC, GPL = FS::GPL;
  constexpr int DP = fz_dp<D>();  // lanes per row in the threshold stage
  constexpr int RPI = 64 / DP;    // rows per iteration of the threshold stage
  constexpr int SQW = D + 3;      // per row: requests, GPU request, affinity domain, tie salt
  static_assert(DP <= 64, "threshold stage: one lane per (row, dim)");
  // the chunk's scores s + 1 (0 = infeasible): 16-bit and double-buffered
  // (one barrier per chunk) when every score + 1 fits 16 bits and the tile
  // is 1,024 columns, else single-buffered with a second barrier before the
  // tile is rewritten
  constexpr int NB = H16 && NW == 8 ? 2 : 1;  // buffers
  // A row of the LDS tile: 4-column groups of GW words (one 8- or 16-B
  // access), one padding group after every 64: the select reads group
  // lane + 64k in its first pass (consecutive across lanes) and the 4·GPL
  // columns of one candidate lane (groups L + 64k) in its survivor scan,
  // which without the padding would all sit in one LDS bank
  constexpr int GW = H16 ? 2 : 4, NG = kFzTile / 4;
  constexpr int RWD = (NG + NG / 64) * GW;  // words per row
  constexpr int TB = NW == 8 ? 10 : 11;     // log2 of the tile width (tie mode 0)
  __shared__ __attribute__((aligned(16))) uint32_t ssc[NB][kFzRC][RWD];
  // PRE keeps only the tie salt per row (the LDS for the second record buffer)
  constexpr int SALT = PRE ? 0 : D + 2;
  __shared__ uint32_t sq[kFzMaxRows][PRE ? 1 : SQW];
  __shared__ __attribute__((aligned(16))) uint64_t sbuf[NW][kFzSurv];
  // per group (padded like the tile rows): [0] pos·mul, [1] tie mode 0's
  // select-phase tie bits (one LDS object: a pointer chosen between two
  // objects made the compiler wait for the record DMA before reading it)
  __shared__ uint32_t sposb[2][NG + NG / 64];
  uint32_t *const spos = sposb[0];
  __shared__ uint8_t scand[NW][64 * GPL];  // per wave: the (lane, group) pairs whose best reached T
  constexpr int RW = (2 * D + 4 + 3) & ~3;  // row record words, whole 16-B reads
  // PRE: the next chunk's records are copied by the memory unit straight
  // into the wave's LDS records (through VGPRs they spilled at the 80-VGPR
  // budget) once the chunk's scores are in, so the copy is in flight during
  // the select phase. (Issued at the chunk start into a second buffer, the
  // copy was waited for at the chunk's first record read: the compiler's
  // LDS-DMA wait covers every buffer of one LDS array.)
  __shared__ __attribute__((aligned(16))) uint32_t srec[1][NW][kFzRC][RW];
  __shared__ int32_t su[PRE ? kFzMaxRows : 1];  // PRE: the rows' units
  auto pgi = [](int g) { return g + (g >> 6); };  // padded group index
  if (rows_dev) fit_rows(*rows_dev, min_rpb, rows, rows_per_block);
  const int r0 = blockIdx.y * rows_per_block;
  if (r0 >= rows) return;  // block-uniform
  const int nr = min(rows, r0 + rows_per_block) - r0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntiles = gridDim.x, tile = blockIdx.x;
#ifdef KP_FZ_PROFILE
  uint64_t t_prev_ = __builtin_amdgcn_s_memtime(), pacc_[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#else
  (void)prof;
#endif
  const int tile0 = tile * kFzTile;
  // this lane's word (H16) / 8-B pair (32-bit scores) of a tile row, padded:
  // the lane's 2 columns are half of group (wave*64 + lane) / 2
  const int wix = (wave * 64 + lane) + 2 * ((wave * 64 + lane) >> 7);
  const int g = sp.gpu_dim;
  const int K = sp.n_cand;
  if constexpr (PRE) {  // the row records come precomputed: units and tie salts only
    for (int i = tid; i < nr; i += kFzBS) {
      const int32_t unit = rows_unit[r0 + i];
      su[i] = unit;
      sq[i][SALT] = sp.tie_rotated ? salt[unit] : 0u;
    }
  } else {
    for (int i = tid; i < nr * SQW; i += kFzBS) {
      const int rr = i / SQW, d = i - rr * SQW;
      const int32_t unit = rows_unit[r0 + rr];
      uint32_t v;
      if (d == D + 2) {
        v = sp.tie_rotated ? salt[unit] : 0u;
      } else if (d == D + 1) {
        v = (uint32_t)uaff[unit];
      } else {
        const int dd = d < D ? d : g;
        v = dd >= 0 ? (uint32_t)q[(int64_t)dd * qstride + unit] : 0u;
      }
      sq[rr][d] = v;
    }
  }
  // the wave's 128 columns: 2 per lane, one 8-B load per plane
  const uint2 *pv = reinterpret_cast<const uint2 *>(np);
  const int64_t PV = P / 2, iv = (tile0 + wave * 128) / 2 + lane;
  uint32_t f_[2][D], a_[2][D], fg_[2], tp_[2], cu[D], cR[D], cK[D];
  int32_t b_[2], wa_[2];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const uint2 pf = pv[(kPlanes * d + 0) * PV + iv], pa = pv[(kPlanes * d + 2) * PV + iv];
    f_[0][d] = pf.x;
    f_[1][d] = pf.y;
    a_[0][d] = pa.x;
    a_[1][d] = pa.y;
    // the class capacity: the wave's first column is always a node of its
    // class (classes start on a wave tile); an all-padding wave reads 0
    cu[d] = __builtin_amdgcn_readfirstlane(pv[(kPlanes * d + 1) * PV + iv].x);
    cR[d] = __builtin_amdgcn_readfirstlane(pv[(kPlanes * d + 3) * PV + iv].x);
    cK[d] = __builtin_amdgcn_readfirstlane(pv[(kPlanes * d + 4) * PV + iv].x);
  }
  {
    const uint2 pb = pv[(kPlanes * D) * PV + iv], pt = pv[(kPlanes * D + 1) * PV + iv],
                pw = pv[(kPlanes * D + 2) * PV + iv];
    b_[0] = (int32_t)pb.x;
    b_[1] = (int32_t)pb.y;
    tp_[0] = pt.x;
    tp_[1] = pt.y;
    wa_[0] = (int32_t)pw.x;
    wa_[1] = (int32_t)pw.y;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      fg_[k] = 0xFFFFFFFFu;  // no GPU dim: never equal to a request
#pragma unroll
      for (int d = 0; d < D; ++d)
        if (d == g) fg_[k] = d == 0 ? f_[k][0] - 1u : f_[k][d];  // dim 0 holds free + 1
    }
  }
  // select-phase column groups c = tile0 + 4*g (4 columns inside one wave
  // tile): their canonical positions times the tie multiplier (padding
  // columns get garbage, they are never feasible)
  const uint32_t mul = sp.tie_rotated ? kTieMul : 1u;
  // Tie mode 0 (tie = position): the tile's real columns hold positions
  // p0 .. p0 + 1023 (p0 = its first column's), so the select phase ranks
  // ties by p0 + 1023 - pos in the top 10 bits, not by the top bits of
  // ~pos (which are equal across the tile and send ties to the bisection).
  // Monotone in the exact key, so the survivor bound stays exact; padding
  // columns wrap mod 1024 and stay below 1 << ksh.
  const bool tie0 = !sp.tie_rotated;
  if (tid < NG) {
    const int c = tile0 + 4 * tid;
    const uint32_t pos = (uint32_t)(c - wshift[c >> 7]);
    spos[pgi(tid)] = pos * mul;
    sposb[1][pgi(tid)] = pos << (32 - TB);
  }
  KP_FZ_PROF_MARK(0);
  __syncthreads();  // requests and positions staged
  KP_FZ_PROF_MARK(1);
  const uint32_t S = (uint32_t)sp.S;
  int32_t wv[D];
#pragma unroll
  for (int d = 0; d < D; ++d) wv[d] = in_vgpr(sp.w[d]);
  const int32_t waffv = in_vgpr(sp.w_affinity);
  const int rsh = 32 - tbits;  // select-phase tie bits: tbits <= ksh (= ksh but in tests)
  // PRE: this wave's class (wave-uniform: scalar) and its row records
  // (kp_score.hip k_unit_rec), RW/4 16-B pieces per row, one per lane, the
  // next chunk's loaded during the current chunk's select
  constexpr int Q4 = RW / 4;
  static_assert(!PRE || kFzRC * Q4 <= 64, "one record piece per lane");
  const int cls = PRE ? tcls[(tile0 >> 7) + __builtin_amdgcn_readfirstlane(wave)] : 0;
  const uint4 *crec4 = reinterpret_cast<const uint4 *>(crec) + cls * Q4;
  // rows c .. c + kFzRC - 1 into srec[0][wave]: lane l copies 16-B piece l % Q4
  // of row l / Q4 to byte 16·l of the buffer (the LDS DMA's lane layout). The
  // lane terms are recomputed per call (hoisted out of the chunk loop they
  // were spilled)
  auto rec_dma = [&](int c) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    if (ln < min(kFzRC, nr - c) * Q4)
      __builtin_amdgcn_global_load_lds(crec4 + (int64_t)su[c + ln / Q4] * (nfc * Q4) + ln % Q4,
                                       (void __attribute__((address_space(3))) *)&srec[0][wave][0][0], 16, 0, 0);
  };
  if (PRE) rec_dma(0);
  for (int c0 = 0; c0 < nr; c0 += kFzRC) {
    const int cr = min(kFzRC, nr - c0);
    const int buf = NB == 2 ? (c0 / kFzRC) & 1 : 0;
    if constexpr (PRE) {  // 1a. the chunk's row records: one 16-B piece per lane
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this chunk's copy has landed
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else
    // 1a. the thresholds of this wave's class: lane -> (row lane/DP, dim
    //     lane%DP), into the wave's LDS row records [q (dim 0: q + 1), GPU
    //     request, affinity domain, thresholds, WQ, GPU-fit bonus]
#pragma unroll
    for (int rb = 0; rb < kFzRC; rb += RPI) {
      const int rr = rb + lane / DP, d = lane % DP;
      uint32_t *rec = srec[0][wave][rr];
      uint32_t tthr = 0xFFFFFFFFu, twq = 0, tok = 1u;
      if (rr < cr && d < D) {
        const uint32_t qd = sq[c0 + rr][d];
        uint32_t c = 0, wd = 0;
#pragma unroll
        for (int dd = 0; dd < D; ++dd)
          if (d == dd) {
            c = cu[dd];
            wd = (uint32_t)sp.w[dd];
          }
        if (c == 0u) {
          tok = qd == 0u ? 1u : 0u;  // cap-0 dim: contributes 0, fits only q = 0
        } else if (qd > c) {
          tok = 0u;
        } else {  // q*S = Q*c + rho: carry iff a >= c - rho (the class's division table)
          uint32_t R = 0, Kd = 0;
#pragma unroll
          for (int dd = 0; dd < D; ++dd)
            if (d == dd) {
              R = cR[dd];
              Kd = cK[dd];
            }
          bool nz;
          const uint32_t Q = div_floor32(qd, c, R, Kd, S, nz);
          const uint32_t rho = (uint32_t)((uint64_t)qd * S - (uint64_t)Q * c);
          tthr = c - rho;
          twq = wd * Q;
        }
        if (d > 0) rec[d] = qd;
        rec[D + 2 + d] = tthr;
      }
      if constexpr (DP >= 2) {
        twq += lane_xor<1>(twq);
        tok &= lane_xor<1>(tok);
      }
      if constexpr (DP >= 4) {
        twq += lane_xor<2>(twq);
        tok &= lane_xor<2>(tok);
      }
      if constexpr (DP >= 8) {
        twq += lane_xor<4>(twq);
        tok &= lane_xor<4>(tok);
      }
      if (rr < cr && d == 0) {
        // dim 0 holds q + 1 against free + 1 (padding columns hold 0), or a
        // request no column can meet when no column of the class fits
        rec[0] = tok ? sq[c0 + rr][0] + 1u : 0x7FFFFFFFu;
        const uint32_t qg = sq[c0 + rr][D];
        rec[D] = qg;
        rec[D + 1] = sq[c0 + rr][D + 1];
        rec[2 * D + 2] = twq;
        rec[2 * D + 3] = qg != 0u ? (uint32_t)sp.w_gpu_fit : 0u;  // the row's GPU-fit bonus
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    KP_FZ_PROF_MARK(2);
    // 1b. this wave's 128 scores of every row of the chunk -> LDS (the row
    //     record is a broadcast read)
    {
#if KP_FZ_ROW_UNROLL == 2
#pragma unroll 2
#else
#pragma unroll 1
#endif
      for (int i = 0; i < cr; ++i) {
        RowRec<RW> cur;
        cur.load(srec[0][wave][i]);
        const uint32_t wq = cur[2 * D + 2], qg = cur[D], af = cur[D + 1];
        const int32_t wfr = (int32_t)cur[2 * D + 3];
        // the row's terms, wave-uniform: a request no column of the wave's
        // class can meet scores nothing; the GPU-fit bonus only exists for a
        // GPU request (wfr != 0) and the affinity bonus for an affinity
        // domain (af >= 0), so rows without them skip those compares
        // dims past DL whose request is 0 are skipped: they always fit
        // (free >= 0) and add no carry (q = 0: threshold c > every a); dim 0
        // is always tested (padding columns fail it)
        auto score = [&](auto hasg, auto hasa, auto dl) {
          constexpr int DL = decltype(dl)::value;
          int32_t sv[2];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            // fit: every free - q >= 0; operands < 2^30, so the signed
            // differences are exact and one min replaces D compares
            int32_t mn = (int32_t)(f_[k][0] - cur[0]);
#pragma unroll
            for (int d = 1; d < DL; ++d) mn = min(mn, (int32_t)(f_[k][d] - cur[d]));
            int32_t acc = wa_[k] + (int32_t)wq + 1;  // s + 1
#pragma unroll
            for (int d = 0; d < DL; ++d) acc += a_[k][d] >= cur[D + 2 + d] ? wv[d] : 0;
            // GPU-topology fit and the CacheStrategy=shared affinity bonus
            int32_t bonus = 0;
            if constexpr (decltype(hasg)::value) bonus += fg_[k] == qg ? wfr : 0;
            if constexpr (decltype(hasa)::value) bonus += tp_[k] == af ? waffv : 0;
            const int32_t sc = (MOST ? acc : b_[k] + 2 - acc) + bonus;
            sv[k] = mn >= 0 ? sc : 0;  // s + 1, 0 = infeasible
          }
          if constexpr (H16)
            ssc[buf][i][wix] = (uint32_t)sv[0] | ((uint32_t)sv[1] << 16);
          else
            reinterpret_cast<int2 *>(ssc[0][i])[wix] = make_int2(sv[0], sv[1]);
        };
        using T_ = std::true_type;
        using F_ = std::false_type;
        using DA = std::integral_constant<int, D>;
        using D2 = std::integral_constant<int, 2>;  // D = 4: no GPU request in dims 2, 3
        const bool hasg = wfr != 0, hasa = (int32_t)af >= 0;
        bool hi0 = false;
        if constexpr (D == 4) hi0 = (cur[2] | cur[3]) == 0u;
        if (cur[0] == 0x7FFFFFFFu) {  // no column of this class fits the row
          if constexpr (H16)
            ssc[buf][i][wix] = 0u;
          else
            reinterpret_cast<int2 *>(ssc[0][i])[wix] = make_int2(0, 0);
        } else if (hasg) {  // a GPU-fit bonus implies a GPU request: all dims
          if (hasa) score(T_{}, T_{}, DA{}); else score(T_{}, F_{}, DA{});
        } else if (hi0) {
          if (hasa) score(F_{}, T_{}, D2{}); else score(F_{}, F_{}, D2{});
        } else {
          if (hasa) score(F_{}, T_{}, DA{}); else score(F_{}, F_{}, DA{});
        }
      }
    }
    KP_FZ_PROF_MARK(3);
    __syncthreads();  // the chunk's scores are in LDS
    // the next chunk's records (the wave's own LDS records, read by the score
    // loop above): in flight during the select phase, which reads other LDS
    if constexpr (PRE)
      if (c0 + kFzRC < nr) rec_dma(c0 + kFzRC);
    KP_FZ_PROF_MARK(4);
    // 2. top-K of this tile for row `wave` of the chunk. LDS holds s + 1
    //    (0 = infeasible); a column's 32-bit key is (s + 1) << ksh | the top
    //    bits of ~tk, ~tk = ~(pos*mul + salt) = ~salt - pos*mul
#if KP_FZ_EXP == 1  // timing experiment: no select phase
    if (wave < cr && lane < K)  // no candidates (keeps the merge in bounds)
      // (0 at run time: n_cand < 2^16; an opaque mask keeps the LDS tile's
      // stores alive — with a literal & 0 the compiler dropped them and the
      // whole score stage with them)
      part[((r0 + c0 + wave) * ntiles + tile) * K + lane] =
          (uint64_t)(ssc[buf][wave][lane] & (uint32_t)(sp.n_cand >> 16));
    if (false)
#endif
    if (wave < cr) {
      const int i = wave;
      const int64_t row = r0 + c0 + i;
      const uint32_t nsl = ~sq[c0 + i][SALT];
      // select-phase tie bits: (nst - tsp[g] - j * mt) >> rsh
      const uint32_t *tsp = sposb[tie0 ? 1 : 0];
      const uint32_t nst = tie0 ? (spos[0] + (uint32_t)(kFzTile - 1)) << (32 - TB) : nsl,
                     mt = tie0 ? 1u << (32 - TB) : mul;
      // lane L's 16 columns are the 4-column groups L + 64k, k < GPL
      // (strided: the tile's best keys spread over the lanes; the padded rows
      // keep both this pass and the survivor scan free of bank conflicts)
      // 16-bit scores: the select key is (s + 1) << 16 | the top 16 tie
      // bits, built from the packed LDS word by one v_alignbit (low column)
      // or v_perm (high column) per column; tests with fewer tie bits
      // (KP_FZ_TIE_BITS < 16) mask the low key bits per group (max commutes
      // with the mask). 32-bit scores: (s + 1) << ksh | tie >> rsh
      const int kss = H16 ? 16 : ksh;
      const uint32_t kmask = H16 && tbits < 16 ? ~((1u << (16 - tbits)) - 1u) : 0xFFFFFFFFu;
      auto key32 = [&](uint32_t s1, uint32_t tk) {
        return H16 ? (((s1 << 16) | (tk >> 16)) & kmask) : ((s1 << ksh) | (tk >> rsh));
      };
      uint32_t best = 0;
      uint32_t gb[GPL];  // the lane's best key per group
#pragma unroll
      for (int k = 0; k < GPL; ++k) {
        const int gk = pgi(lane + 64 * k);
        const uint32_t npk = nst - tsp[gk];
        uint32_t b4 = 0;
        if constexpr (H16) {
          const uint2 x = reinterpret_cast<const uint2 *>(ssc[buf][i])[gk];
          const uint32_t k0 = __builtin_amdgcn_alignbit(x.x, npk, 16);
          const uint32_t k1 = __builtin_amdgcn_perm(x.x, npk - mt, 0x07060302u);
          const uint32_t k2 = __builtin_amdgcn_alignbit(x.y, npk - 2u * mt, 16);
          const uint32_t k3 = __builtin_amdgcn_perm(x.y, npk - 3u * mt, 0x07060302u);
          b4 = max(max(k0, k1), max(k2, k3)) & kmask;
        } else {
          uint32_t v4[4];
          load_group<H16>(ssc[buf][i], gk, v4);
#pragma unroll
          for (int j = 0; j < 4; ++j) b4 = max(b4, key32(v4[j], npk - (uint32_t)j * mt));
        }
        best = max(best, b4);
        gb[k] = b4;
      }
      // T = the K-th largest lane best (radix select over ballots; lower
      // bound of the tile's K-th key), at least 1 << kss: every key >= T is
      // feasible
      KP_FZ_PROF_MARK(5);
      uint32_t T = 0;
      // fewer than K lanes with a feasible best: the K-th lane best is below
      // 1 << kss and T is 1 << kss without the search (wave-uniform)
      if (__popcll(__ballot(best >= (1u << kss))) >= K)
#pragma unroll
      for (int bb = 31; bb >= 0; --bb) {
        const uint32_t cb = T | (1u << bb);
        T = __popcll(__ballot(best >= cb)) >= K ? cb : T;
      }
      T = max(T, 1u << kss);
      KP_FZ_PROF_MARK(6);
      // survivors (keys >= T) -> LDS as exact 64-bit keys. Only the groups
      // whose best reached T hold any (at least K of them, typically about
      // K): their (lane, k) go to LDS in order and the whole wave scans just
      // their 4 columns each (a lane-granular list scanned 16 columns per
      // listed lane, 4x the work)
      int m = 0;
#pragma unroll
      for (int k = 0; k < GPL; ++k) {
        const uint64_t Mk = __ballot(gb[k] >= T);
        if (gb[k] >= T)
          scand[wave][m + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(Mk >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)Mk, 0u))] =
              (uint8_t)(lane | (k << 6));
        m += __popcll(Mk);
      }
      constexpr int CPL = 4;        // columns per listed entry
      constexpr int CPB = 4 * GPL;  // columns per lane (the bisection re-reads them all)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint32_t *srow = ssc[buf][i];
      int C = 0;
      for (int e0 = 0; e0 < CPL * m; e0 += 64) {  // wave-uniform
        const int e = e0 + lane;
        bool hit = false;
        uint32_t s1 = 0, ntk = 0;
        if (e < CPL * m) {
          const int ent = scand[wave][e >> 2];  // listed (lane, group k)
          const int g = pgi((ent & 63) + 64 * (ent >> 6)), jj = e & 3;
          s1 = load_one<H16>(srow, 4 * g + jj);
          ntk = nsl - spos[g] - (uint32_t)jj * mul;
          hit = key32(s1, nst - tsp[g] - (uint32_t)jj * mt) >= T;
        }
        const uint64_t mm = __ballot(hit);
        const int p = C + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
        if (hit && p < kFzSurv) sbuf[wave][p] = ((uint64_t)(0x80000000u | (s1 - 1u)) << 32) | ntk;
        C += __popcll(mm);
      }
      if (C > kFzSurv) {
        // exact K-th largest 64-bit key by bisection (> 128 keys reached T:
        // adversarial ties; the columns are re-read from LDS)
        uint64_t pre = 0;
#pragma unroll 1
        for (int bb = 63; bb >= 0; --bb) {
          const uint64_t cb = pre | (1ull << bb);
          int c = 0;
#pragma unroll 1
          for (int e = 0; e < CPB; ++e) {
            const int k = e >> 2, j = e & 3;
            const uint32_t s1 = load_one<H16>(srow, 4 * pgi(lane + 64 * k) + j);
            const uint32_t ntk = nsl - spos[pgi(lane + 64 * k)] - (uint32_t)j * mul;
            c += (s1 != 0u && (((uint64_t)(0x80000000u | (s1 - 1u)) << 32) | ntk) >= cb) ? 1 : 0;
          }
          c = (int)rl((uint32_t)wave_incl_scan_i32(c), 63);
          if (c >= K) pre = cb;
        }
        C = 0;
#pragma unroll 1
        for (int e = 0; e < CPB; ++e) {
          const int k = e >> 2, j = e & 3;
          const uint32_t s1 = load_one<H16>(srow, 4 * pgi(lane + 64 * k) + j);
          const uint32_t ntk = nsl - spos[pgi(lane + 64 * k)] - (uint32_t)j * mul;
          const uint64_t key = ((uint64_t)(0x80000000u | (s1 - 1u)) << 32) | ntk;
          const bool hit = s1 != 0u && key >= pre;
          const uint64_t m = __ballot(hit);
          const int p = C + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          if (hit) sbuf[wave][p] = key;
          C += __popcll(m);  // = min(K, feasible) <= 32 in the end
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      KP_FZ_PROF_MARK(7);
      // exact rank of each survivor (one per lane, two past 64; keys
      // broadcast with v_readlane, no LDS round trip per step); ranks < K
      // are the list
      uint64_t *dst = part + (row * ntiles + tile) * K;
      if (C <= 64) {
        const uint64_t my = lane < C ? sbuf[wave][lane] : 0ull;
        int r = 0;
        // the other keys as LDS broadcast reads, two per 16-B read (a
        // v_readlane pair per key cost config #4 +25 ms)
        const ulonglong2 *sb2 = reinterpret_cast<const ulonglong2 *>(sbuf[wave]);
#pragma unroll KP_FZ_RANK_UNROLL
        for (int j = 0; j < C / 2; ++j) {
          const ulonglong2 o = sb2[j];
          r += (o.x > my ? 1 : 0) + (o.y > my ? 1 : 0);
        }
        if (C & 1) r += sbuf[wave][C - 1] > my ? 1 : 0;
        if (lane < C && r < K) dst[r] = my;
        if (lane >= C && lane < K) dst[lane] = 0ull;
      } else {  // 64 < C <= 128 (K <= 64 < C: every slot is filled)
        const uint64_t my0 = sbuf[wave][lane];
        const uint64_t my1 = lane + 64 < C ? sbuf[wave][lane + 64] : 0ull;
        const ulonglong2 *sb2 = reinterpret_cast<const ulonglong2 *>(sbuf[wave]);
        int r0 = 0, r1 = 0;
#pragma unroll KP_FZ_RANK_UNROLL
        for (int j = 0; j < C / 2; ++j) {
          const ulonglong2 o = sb2[j];
          r0 += (o.x > my0 ? 1 : 0) + (o.y > my0 ? 1 : 0);
          r1 += (o.x > my1 ? 1 : 0) + (o.y > my1 ? 1 : 0);
        }
        if (C & 1) {
          const uint64_t o = sbuf[wave][C - 1];
          r0 += o > my0 ? 1 : 0;
          r1 += o > my1 ? 1 : 0;
        }
        if (r0 < K) dst[r0] = my0;
        if (lane + 64 < C && r1 < K) dst[r1] = my1;
      }
    }
    KP_FZ_PROF_MARK(8);
    if constexpr (NB == 1) __syncthreads();  // the single LDS tile is rewritten next
  }
  KP_FZ_PROF_FLUSH();
}

// Tournament form: the row's ntiles sorted lists are staged in LDS, lane t
// holds the heads of lists t, t+64, ... (LPL per lane); K times the wave
// max of the heads, and only the owner of the max advances its list (one LDS
// read). K x (one wave max + one LDS read) per row instead of K passes over
// all ntiles*K keys. Returns the canonical position of candidate `lane`
// (-1 past the row's feasible nodes). L = the row's lists in LDS.
template <int LPL>
__device__ __forceinline__ int32_t merge_tour_row(const uint64_t *L, int32_t ntiles, int32_t K,
                                                  uint32_t sl, uint32_t inv, int lane) {
  int h[LPL];
  uint64_t v[LPL];
#pragma unroll
  for (int j = 0; j < LPL; ++j) {
    const int t = lane + 64 * j;
    h[j] = 0;
    v[j] = t < ntiles ? L[t * K] : 0ull;
  }
  // lane it keeps the canonical position of candidate it; the positions are
  // mapped to nodes after the loop with ONE load per lane (a perm load + store
  // inside the loop serialises K memory latencies)
  int32_t mypos = -1;
  for (int it = 0; it < K; ++it) {
    uint64_t b = v[0];
#pragma unroll
    for (int j = 1; j < LPL; ++j) b = v[j] > b ? v[j] : b;
    const uint32_t mhi = wave_max32((uint32_t)(b >> 32));
    const uint32_t mlo = wave_max32((uint32_t)(b >> 32) == mhi ? (uint32_t)b : 0u);
    const uint64_t m = ((uint64_t)mhi << 32) | mlo;
    if (m == 0) break;  // fewer than K feasible nodes: lanes >= it keep -1
#pragma unroll
    for (int j = 0; j < LPL; ++j)
      if (v[j] == m) {  // keys are unique: one list of one lane
        const int t = lane + 64 * j;
        ++h[j];
        v[j] = h[j] < K ? L[t * K + h[j]] : 0ull;
      }
    if (lane == it) mypos = key_node(m, sl, inv);
  }
  return mypos;
}

// One wave per row: the row's ntiles sorted per-tile lists staged in LDS and
// merged by the tournament; the candidates' canonical positions mapped to
// nodes through perm. Dynamic LDS: KP_MERGE_WPB rows x ntiles*K keys. (A
// threshold merge — T = the largest K-th key of the tile lists, the keys >= T
// ranked exactly — measured equal in r05 and was dropped.)
template <int LPL>
__global__ __launch_bounds__(64 * KP_MERGE_WPB) void k_merge_tour(ScoreParams sp, const uint64_t *__restrict__ part,
                                                    int32_t ntiles,
                                                    const int32_t *__restrict__ rows_unit,
                                                    const uint32_t *__restrict__ salt, int32_t rows,
                                                    const int32_t *__restrict__ rows_dev,
                                                    const int32_t *__restrict__ perm,
                                                    int32_t *__restrict__ cand, RoundKeys rk) {
  extern __shared__ uint64_t slist[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rblocks = (rows + kMergeWPB - 1) / kMergeWPB;
  if ((int)blockIdx.x >= rblocks) {  // rk.enabled: the extra workgroups
    round_keys_init(rk, (int64_t)(blockIdx.x - rblocks) * (64 * kMergeWPB) + threadIdx.x);
    return;
  }
  const int row = blockIdx.x * kMergeWPB + wave;
  const int K = sp.n_cand, M = ntiles * K;
  int32_t unit = 0, mine = -1;
  uint32_t sl = 0u;  // the unit's tie salt (rotated ties)
  bool live = false;
  if (row < rows) {  // wave-uniform
    // the device row count and the row's unit are loaded with the first keys
    // (then the unit's tie salt while the keys go to LDS): no dependent
    // memory level before the staging
    int32_t rdev = rows_dev ? *rows_dev : rows;
    int32_t u0 = rows_unit[row];
    uint64_t *L = slist + (int64_t)wave * M;
    const uint64_t *src = part + (int64_t)row * M;  // readable for every row < rows
    // the row's lists staged in batches of 8 loads per lane issued together (a
    // load-then-store loop waited one memory latency per 64 keys)
    for (int b0 = 0; b0 < M; b0 += 64 * kMergeLoadBatch) {
      uint64_t x[kMergeLoadBatch];
#pragma unroll
      for (int u = 0; u < kMergeLoadBatch; ++u)  // unmasked (clamped): exact wait counts below
        x[u] = src[min(b0 + 64 * u + lane, M - 1)];
      if (b0 == 0) {
        landed(rdev);  // issued before the keys: the keys stay in flight
        landed(u0);
        if (sp.tie_rotated && row < rdev) sl = salt[u0];  // a live row's unit only
      }
#pragma unroll
      for (int u = 0; u < kMergeLoadBatch; ++u) {
        const int e = b0 + 64 * u + lane;
        if (e < M) L[e] = x[u];
      }
    }
    live = row < rdev;
    unit = u0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (live) {
    const uint64_t *L = slist + (int64_t)wave * M;
    const uint32_t inv = sp.tie_rotated ? kTieMulInv : 1u;
    const int32_t mypos = merge_tour_row<LPL>(L, ntiles, K, sl, inv, lane);
    // canonical position -> node (a position is always < N)
    mine = (uint32_t)mypos < (uint32_t)sp.N ? perm[mypos] : -1;
    if (lane < K) cand[(int64_t)row * K + lane] = mine;
  }
  if (rk.enabled) {  // k_csr_keys' work for the workgroup's slots
    // the slots of a workgroup share one bitmap word (kMergeWPB divides 32):
    // the first wave with node n at candidate index j sets the bits of every
    // wave with n at j in one atomic (herded rounds: consecutive slots list
    // the same nodes in the same order)
    static_assert(32 % kMergeWPB == 0, "a workgroup's slots in one bitmap word");
    __shared__ int32_t snode[kMergeWPB][64];
    snode[wave][lane] = live ? mine : -1;
    __syncthreads();
    if (live) {
      if (lane < K) {
        rk.bid[(int64_t)row * K + lane] = 0xFFFFFFFFu;  // kNoBid
        if (mine >= 0) {
          bool first = true;
          uint32_t bits = 0;
#pragma unroll
          for (int w2 = 0; w2 < kMergeWPB; ++w2)
            if (snode[w2][lane] == mine) {
              first = first && w2 >= wave;
              bits |= 1u << ((blockIdx.x * kMergeWPB + w2) & 31);
            }
          if (first && atomicOr(&rk.bm[(int64_t)mine * rk.Wb + (row >> 5)], bits) == 0u)
            atomicOr(&rk.bms[(int64_t)mine * rk.Ws + (row >> 10)], 1u << ((row >> 5) & 31));
        }
      }
      const int32_t first_node = __shfl(mine, 0, 64);
      if (lane == 0) {
        rk.open[row] = first_node >= 0 ? 1 : 0;
        if (first_node < 0) rk.status[unit] = kNoFit;
      }
    }
  }
}

template <int D>
struct TopkL {
  template <int NW>
  static int run_nw(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit, int32_t rows,
                    int32_t ksh, int32_t *cand, const int32_t *rows_dev, bool init_wgs) {
    using FS = FzShape<NW>;
    const int P = c->fz_P, ntiles = P / FS::TILE;
    const int64_t want = ((int64_t)rows * ntiles + c->fz_wg_target - 1) / c->fz_wg_target;
    const int rpb = (int)std::min<int64_t>(kFzMaxRows, std::max<int64_t>(FS::RC, want));
    const dim3 grid(ntiles, blocks(rows, rpb));
    const int32_t tb = c->fz_tie_bits > 0 ? std::min(ksh, c->fz_tie_bits) : ksh;
#define KP_FZ_(M, H, PR)                                                                             \
  hipLaunchKernelGGL((k_score_topk<D, M, H, NW, PR>), grid, dim3(FS::BS), 0, c->stream, sp, c->d.np32, \
                     P, c->d.q, c->U, c->d.aff, c->d.salt, rows_unit, rows, rpb, FS::RC, rows_dev,      \
                     c->d.wshift, ksh, tb, c->d.part, c->d.fz_prof, c->d.crec, c->d.tcls, c->nfc)
#define KP_FZ(M, H)          \
  if (c->crec_ok)            \
    KP_FZ_(M, H, true);      \
  else                       \
    KP_FZ_(M, H, false)
    // 16-bit LDS scores when every score + 1 < 2^16 (ksh >= 16)
    const bool h16 = ksh >= 16 && c->fz_h16;
    if (sp.most_allocated) {
      if (h16) KP_FZ(true, true); else KP_FZ(true, false);
    } else {
      if (h16) KP_FZ(false, true); else KP_FZ(false, false);
    }
#undef KP_FZ
#undef KP_FZ_
    KP_HIP(hipGetLastError());
    if (c->fz_end_event) KP_HIP(hipEventRecord(c->fz_end_event, c->stream));
    const int M = ntiles * sp.n_cand;
    RoundKeys rk{};
    if (c->keys_in_merge) rk = round_keys_args(c, rows, sp.n_cand, c->d.counters);
    const dim3 mg(blocks(rows, kMergeWPB) +
                  (rk.enabled && init_wgs ? blocks(rk.init_n, 64 * kMergeWPB) : 0));
    const size_t lds = (size_t)kMergeWPB * M * sizeof(uint64_t);  // <= 16 KB per row (M <= 2,048)
#define KP_MG(LPL)                                                                       \
  hipLaunchKernelGGL((k_merge_tour<LPL>), mg, dim3(64 * kMergeWPB), lds, c->stream, sp, c->d.part, \
                     ntiles, rows_unit, c->d.salt, rows, rows_dev, c->d.perm, cand, rk)
    if (ntiles <= 64)
      KP_MG(1);
    else if (ntiles <= 128)
      KP_MG(2);
    else if (ntiles <= 256)
      KP_MG(4);
    else if (ntiles <= 512)
      KP_MG(8);
    else if (ntiles <= 1024)
      KP_MG(16);
    else
      KP_MG(32);
#undef KP_MG
    KP_HIP(hipGetLastError());
    return KP_OK;
  }
  static int run(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit, int32_t rows,
                 int32_t ksh, int32_t *cand, const int32_t *rows_dev, bool init_wgs) {
    return run_nw<kFzWaves>(c, sp, rows_unit, rows, ksh, cand, rows_dev, init_wgs);
  }
};

// Row records of the fused candidate phase, once per solve: for unit u and
// fused capacity class k (capacities c_d), the words k_score_topk's stage 1a
// computed per chunk and wave before — [q_0 + 1 (0x7FFFFFFF: no column of
// the class fits), q_1 .. q_{D-1}, GPU request, affinity domain, thresholds
// c_d - rho_d (q_d·S = Q_d·c_d + rho_d; 0xFFFFFFFF: cap-0 dim or q > c),
// WQ = sum_d w_d·Q_d, GPU-fit bonus] — with exact 64-bit divisions.
template <int D>
__global__ void k_unit_rec(ScoreParams sp, const int64_t *__restrict__ q, int32_t U,
                           const int32_t *__restrict__ uaff, const uint32_t *__restrict__ fccap,
                           int32_t nfc, uint32_t *__restrict__ crec) {
  constexpr int RW = (2 * D + 4 + 3) & ~3;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)U * nfc) return;
  const int32_t u = (int32_t)(t / nfc), k = (int32_t)(t - (int64_t)u * nfc);
  uint32_t rec[RW];
#pragma unroll
  for (int i = 0; i < RW; ++i) rec[i] = 0u;
  const uint64_t S = (uint64_t)sp.S;
  uint32_t wq = 0;
  bool ok = true;
  uint32_t q0 = 0;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const uint32_t qd = (uint32_t)q[(int64_t)d * U + u], c = fccap[(int64_t)k * D + d];
    uint32_t thr = 0xFFFFFFFFu;
    if (c == 0u) {
      ok &= qd == 0u;
    } else if (qd > c) {
      ok = false;
    } else {
      const uint64_t x = (uint64_t)qd * S, Q = x / c;
      thr = c - (uint32_t)(x - Q * c);
      wq += (uint32_t)sp.w[d] * (uint32_t)Q;
    }
    if (d == 0) q0 = qd;
    else rec[d] = qd;
    rec[D + 2 + d] = thr;
  }
  const int g = sp.gpu_dim;
  const uint32_t qg = g >= 0 ? (uint32_t)q[(int64_t)g * U + u] : 0u;
  rec[0] = ok ? q0 + 1u : 0x7FFFFFFFu;
  rec[D] = qg;
  rec[D + 1] = (uint32_t)uaff[u];
  rec[2 * D + 2] = wq;
  rec[2 * D + 3] = qg != 0u ? (uint32_t)sp.w_gpu_fit : 0u;
  uint4 *dst = reinterpret_cast<uint4 *>(crec + t * RW);
#pragma unroll
  for (int i = 0; i < RW / 4; ++i) dst[i] = make_uint4(rec[4 * i], rec[4 * i + 1], rec[4 * i + 2], rec[4 * i + 3]);
}

template <int D>
struct UnitRecL {
  static int run(kp_ctx *c, const ScoreParams &sp) {
    const int64_t n = (int64_t)c->U * c->nfc;
    if (n <= 0) return KP_OK;
    hipLaunchKernelGGL(k_unit_rec<D>, dim3(blocks(n, 256)), dim3(256), 0, c->stream, sp, c->d.q,
                       c->U, c->d.aff, c->d.fccap, c->nfc, c->d.crec);
    KP_HIP(hipGetLastError());
    return KP_OK;
  }
};

}  // namespace

int launch_unit_rec(kp_ctx *c, const ScoreParams &sp) { return dispatch_D<UnitRecL>(c->D, c, sp); }

int launch_score_topk(kp_ctx *c, const ScoreParams &sp, const int32_t *rows_unit, int32_t rows,
                      int32_t ksh, int32_t *cand, const int32_t *rows_dev, bool init_wgs) {
  if (rows <= 0 || c->N == 0) return KP_OK;
  return dispatch_D<TopkL>(c->D, c, sp, rows_unit, rows, ksh, cand, rows_dev, init_wgs);
}

}  // namespace kp
