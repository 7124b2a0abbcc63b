// Microbenchmark (r05): store-pattern ceilings of the materialised score
// matrix + feasibility mask at config #3's full size (100k rows x 10,048
// columns, int32 scores + 1 bit per pair), to decide the layout and work
// decomposition of k_score32c:
//   kernel "tiles": a workgroup = 4 waves x 256 columns (lane l owns columns
//     base + 64k + l, k < 4, as k_score32c), its rows from blockIdx.y, each
//     wave writes its 4 mask words per row (32-B pieces);
//   kernel "wide":  a wave owns all 1,024 columns of the tile (16 per lane),
//     the workgroup's 4 waves take interleaved rows, each row's 16 mask words
//     are ONE 128-B store of 16 lanes;
//   grid: "chunk4" = 4 launches of 25k rows (as kp_score_dev's cap_U chunks),
//     "one" = one launch over every row, "persist" = exactly the resident
//     workgroups, each a fixed column tile and a contiguous row range;
//   mask row stride 157 words (= Ns/64, lines straddle workgroups) or 160
//     (a workgroup's 16 words are one aligned 128-B line);
//   `work` dependent v_mad_u32_u24 per pair stand in for the score VALU.
// Bytes = rows x Ns x 4 (scores) + rows x Ns / 8 (mask); no validation (a
// throughput probe; every index is bounded by rows x Ns / rows x mstride).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

enum { M_SCORE = 1, M_MASK = 2, M_MASK_NT = 4 };

__device__ __forceinline__ uint32_t chain(uint32_t v, uint32_t r, int work) {
  for (int i = 0; i < work; ++i) v = __umul24(v, 0x9E37u) + r;
  return v;
}

struct Range {
  int tile, ra, rb, step, first;
};

// which tile and rows this workgroup/wave covers
__device__ __forceinline__ Range wg_range(int rows, int ctiles, int rpb, int persist, int nslots) {
  Range g;
  if (persist) {
    g.tile = blockIdx.x % ctiles;
    const int slot = blockIdx.x / ctiles;
    g.ra = (int)((int64_t)rows * slot / nslots);
    g.rb = (int)((int64_t)rows * (slot + 1) / nslots);
  } else {
    g.tile = blockIdx.x;
    g.ra = blockIdx.y * rpb;
    g.rb = min(rows, g.ra + rpb);
  }
  return g;
}

__global__ __launch_bounds__(256) void k_tiles(int32_t *score, uint64_t *mask, int rows, int Ns,
                                               int64_t mstride, int rpb, int work, int mode,
                                               int persist, int nslots, int ctiles, int row0) {
  extern __shared__ int dyn[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const Range g = wg_range(rows, ctiles, rpb, persist, nslots);
  const int tile0 = g.tile * 1024 + wave * 256;
  if (tile0 >= Ns) return;
  if (work < 0) dyn[threadIdx.x] = 0;  // never: keeps the dynamic LDS (occupancy limiter)
  for (int r = g.ra; r < g.rb; ++r) {
    const int rr = r + row0;
    int32_t *srow = score + (int64_t)rr * Ns + tile0 + lane;
    uint64_t word[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int col = tile0 + 64 * k + lane;
      const uint32_t v = chain((uint32_t)col ^ (uint32_t)rr, (uint32_t)rr, work);
      const bool ft = (v & 15u) != 0u && col < Ns;
      if ((mode & M_SCORE) && tile0 + 64 * k < Ns)
        __builtin_nontemporal_store(ft ? (int32_t)(v >> 1) : -1, srow + 64 * k);
      word[k] = __ballot(ft);
    }
    if ((mode & M_MASK) && lane < 4 && tile0 + 64 * lane < Ns) {
      uint64_t wd = word[0];
#pragma unroll
      for (int k = 1; k < 4; ++k) wd = lane == k ? word[k] : wd;
      uint64_t *dst = mask + (int64_t)rr * mstride + (tile0 >> 6) + lane;
      if (mode & M_MASK_NT)
        __builtin_nontemporal_store(wd, dst);
      else
        *dst = wd;
    }
  }
}

__global__ __launch_bounds__(256) void k_wide(int32_t *score, uint64_t *mask, int rows, int Ns,
                                              int64_t mstride, int rpb, int work, int mode,
                                              int persist, int nslots, int ctiles, int row0) {
  extern __shared__ int dyn[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const Range g = wg_range(rows, ctiles, rpb, persist, nslots);
  const int base = g.tile * 1024;
  if (work < 0) dyn[threadIdx.x] = 0;
  for (int r = g.ra + wave; r < g.rb; r += 4) {
    const int rr = r + row0;
    int32_t *srow = score + (int64_t)rr * Ns + base + lane;
    uint64_t word[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int col = base + 64 * k + lane;
      const uint32_t v = chain((uint32_t)col ^ (uint32_t)rr, (uint32_t)rr, work);
      const bool ft = (v & 15u) != 0u && col < Ns;
      if ((mode & M_SCORE) && base + 64 * k < Ns)
        __builtin_nontemporal_store(ft ? (int32_t)(v >> 1) : -1, srow + 64 * k);
      word[k] = __ballot(ft);
    }
    if ((mode & M_MASK) && lane < 16 && base + 64 * lane < Ns) {
      uint64_t wd = word[0];
#pragma unroll
      for (int k = 1; k < 16; ++k) wd = lane == k ? word[k] : wd;
      uint64_t *dst = mask + (int64_t)rr * mstride + (base >> 6) + lane;
      if (mode & M_MASK_NT)
        __builtin_nontemporal_store(wd, dst);
      else
        *dst = wd;
    }
  }
}

int main() {
  const int rows = 100000, Ns = 10048, ctiles = (Ns + 1023) / 1024;
  const int64_t mstride_max = 160;
  int32_t *score;
  uint64_t *mask;
  CK(hipMalloc(&score, (size_t)rows * Ns * 4));
  CK(hipMalloc(&mask, (size_t)rows * mstride_max * 8));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::printf("CUs %d, rows %d, Ns %d, scores %.3f GB, mask %.3f GB\n", cus, rows, Ns,
              (double)rows * Ns * 4 / 1e9, (double)rows * Ns / 8 / 1e9);
  struct ModeDef {
    const char *name;
    int mode;
    int64_t mstride;
  };
  const ModeDef modes[] = {{"score", M_SCORE, 157},
                           {"score+mask157", M_SCORE | M_MASK, 157},
                           {"score+mask160", M_SCORE | M_MASK, 160},
                           {"score+mask160nt", M_SCORE | M_MASK | M_MASK_NT, 160},
                           {"mask157", M_MASK, 157},
                           {"mask160", M_MASK, 160}};
  for (int kern = 0; kern < 2; ++kern) {
    for (int lds : {0, 26 * 1024}) {  // 26 KB: at most 6 workgroups per CU (k_score32c's occupancy)
      for (int grid_kind = 0; grid_kind < 3; ++grid_kind) {
        for (const ModeDef &m : modes) {
          for (int work : {0, 16, 32}) {
            if (kern == 1 && lds == 0 && grid_kind == 0 && work == 32) continue;
            float best = 1e9f;
            for (int rep = 0; rep < 4; ++rep) {
              CK(hipEventRecord(a, 0));
              const int rpb = 64;
              if (grid_kind == 2) {
                int nb = 0;
                if (kern == 0)
                  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tiles, 256, lds));
                else
                  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_wide, 256, lds));
                const int nslots = nb * cus / ctiles;
                const dim3 gr(nslots * ctiles);
                if (kern == 0)
                  hipLaunchKernelGGL(k_tiles, gr, dim3(256), lds, 0, score, mask, rows, Ns, m.mstride,
                                     rpb, work, m.mode, 1, nslots, ctiles, 0);
                else
                  hipLaunchKernelGGL(k_wide, gr, dim3(256), lds, 0, score, mask, rows, Ns, m.mstride,
                                     rpb, work, m.mode, 1, nslots, ctiles, 0);
              } else {
                const int chunk = grid_kind == 0 ? 25000 : rows;
                for (int r0 = 0; r0 < rows; r0 += chunk) {
                  const int nr = rows - r0 < chunk ? rows - r0 : chunk;
                  const dim3 gr(ctiles, (nr + rpb - 1) / rpb);
                  if (kern == 0)
                    hipLaunchKernelGGL(k_tiles, gr, dim3(256), lds, 0, score, mask, nr, Ns,
                                       m.mstride, rpb, work, m.mode, 0, 0, ctiles, r0);
                  else
                    hipLaunchKernelGGL(k_wide, gr, dim3(256), lds, 0, score, mask, nr, Ns,
                                       m.mstride, rpb, work, m.mode, 0, 0, ctiles, r0);
                }
              }
              CK(hipGetLastError());
              CK(hipEventRecord(b, 0));
              CK(hipEventSynchronize(b));
              float ms;
              CK(hipEventElapsedTime(&ms, a, b));
              if (rep > 0 && ms < best) best = ms;
            }
            double bytes = 0;
            if (m.mode & M_SCORE) bytes += (double)rows * Ns * 4;
            if (m.mode & M_MASK) bytes += (double)rows * Ns / 8;
            std::printf("%-5s lds%-5d %-7s %-16s work %2d: %7.1f us %6.0f GB/s (%.3f of 8 TB/s)\n",
                        kern ? "wide" : "tiles", lds, grid_kind == 0 ? "chunk4" : grid_kind == 1 ? "one" : "persist",
                        m.name, work, best * 1e3, bytes / (best * 1e-3) / 1e9, bytes / (best * 1e-3) / 8e12);
            std::fflush(stdout);
          }
        }
      }
    }
  }
  return 0;
}
