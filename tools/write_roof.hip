// Microbenchmark: achievable HBM write and read bandwidth on this MI355X for
// the score-matrix shapes (16-B stores / loads per lane, 1.07 GB = round 0 of
// config #3, and 120 MB = a mid round). Sets the practical ceiling for the
// k_score32 / k_select_t roofline fractions.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_store(int4 *p, long n4, int v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    p[i] = make_int4(v, v + 1, v + 2, v + 3);
}

__global__ void k_store_nt(int4 *p, long n4, int v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    __builtin_nontemporal_store((v4i){v, v + 1, v + 2, v + 3}, reinterpret_cast<v4i *>(p + i));
}

// the score-matrix pattern: WG (x, y) writes rows [y*rpb, (y+1)*rpb) of a
// 1024-column tile x (4 KB per row, row stride Ns*4 bytes)
__global__ void k_store_tiles(int *p, int rows, int Ns, int rpb, int v, int nt) {
  const int nb = blockIdx.x * 1024 + threadIdx.x * 4;
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  if (nb >= Ns) return;
  for (int r = r0; r < r1; ++r) {
    int4 x = make_int4(v + r, v, v, v);
    if (nt) __builtin_nontemporal_store((v4i){v + r, v, v, v}, reinterpret_cast<v4i *>(p + (long)r * Ns + nb));
    else *reinterpret_cast<int4 *>(p + (long)r * Ns + nb) = x;
  }
}

// same pattern with `work` x 16 independent full-rate VALU ops per row per lane
// (4 accumulators x 4 nodes), to see whether the VALU of a row overlaps its store
__global__ void k_store_tiles_valu(int *p, int rows, int Ns, int rpb, int v, int work) {
  const int nb = blockIdx.x * 1024 + threadIdx.x * 4;
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  if (nb >= Ns) return;
  unsigned a0 = nb, a1 = nb + 1, a2 = nb + 2, a3 = nb + 3;
  for (int r = r0; r < r1; ++r) {
    unsigned x0 = a0 + r, x1 = a1 + r, x2 = a2 + r, x3 = a3 + r;
    for (int i = 0; i < work; ++i) {
      x0 = x0 * 0x9E37u + (unsigned)i; x1 = x1 * 0x9E37u + (unsigned)i;
      x2 = x2 * 0x9E37u + (unsigned)i; x3 = x3 * 0x9E37u + (unsigned)i;
    }
    *reinterpret_cast<int4 *>(p + (long)r * Ns + nb) = make_int4(x0, x1, x2, x3);
  }
}

__global__ void k_load(const int4 *p, long n4, int *out) {
  int acc = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    int4 x = p[i];
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

int main() {
  const long bytes_max = 1066092800L;
  int4 *p;
  int *o;
  CK(hipMalloc(&p, bytes_max));
  CK(hipMalloc(&o, 64));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (long bytes : {bytes_max}) {
    const long n4 = bytes / 16;
    for (int grid : {32768}) {
      for (int kind = 0; kind < 3; ++kind) {
        float best = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
          CK(hipEventRecord(a, 0));
          if (kind == 0)
            hipLaunchKernelGGL(k_store, dim3(grid), dim3(256), 0, 0, p, n4, rep);
          else if (kind == 2)
            hipLaunchKernelGGL(k_store_nt, dim3(grid), dim3(256), 0, 0, p, n4, rep);
          else
            hipLaunchKernelGGL(k_load, dim3(grid), dim3(256), 0, 0, p, n4, o);
          CK(hipEventRecord(b, 0));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          if (ms < best) best = ms;
        }
        std::printf("%-8s %8.1f MB grid %6d: %7.1f us  %6.0f GB/s\n", kind == 1 ? "load" : kind == 2 ? "store_nt" : "store",
                    bytes / 1e6, grid, best * 1e3, bytes / (best * 1e-3) / 1e9);
      }
    }
  }
  const int Ns = 10048;
  for (int rows : {26525}) {
    for (int rpb : {128}) {
      for (int nt = 0; nt < 2; ++nt) {
        float best = 1e9f;
        dim3 g((Ns + 1023) / 1024, (rows + rpb - 1) / rpb);
        for (int rep = 0; rep < 5; ++rep) {
          CK(hipEventRecord(a, 0));
          hipLaunchKernelGGL(k_store_tiles, g, dim3(256), 0, 0, (int *)p, rows, Ns, rpb, rep, nt);
          CK(hipEventRecord(b, 0));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          if (ms < best) best = ms;
        }
        const double bytes = (double)rows * Ns * 4;
        std::printf("tiles%s rows %6d rpb %3d (%6d WGs): %7.1f us  %6.0f GB/s\n", nt ? "_nt" : "   ", rows, rpb,
                    g.x * g.y, best * 1e3, bytes / (best * 1e-3) / 1e9);
      }
    }
  }
  for (int work : {0, 4, 8, 16, 32}) {
    const int rows = 26525, rpb = 128;
    dim3 g((Ns + 1023) / 1024, (rows + rpb - 1) / rpb);
    float best = 1e9f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(k_store_tiles_valu, g, dim3(256), 0, 0, (int *)p, rows, Ns, rpb, rep, work);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    std::printf("tiles+valu work %2d (~%3d VALU/row/wave): %7.1f us  %6.0f GB/s\n", work, work * 8,
                best * 1e3, (double)rows * Ns * 4 / (best * 1e-3) / 1e9);
  }
  return 0;
}
