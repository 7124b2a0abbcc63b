// Microbenchmark (r05): the int32 VALU issue rate of gfx950 for the
// instruction mixes of the candidate-phase kernels (bench.py's VALU roofline
// peak): every CU busy, 8 waves per SIMD, 8 independent chains per lane.
//   add:    v_add_u32 chains
//   cmpsel: v_cmp_ge_u32 + v_cndmask_b32 + v_add_u32 (the carry step of a
//           score: acc += a >= thr ? w : 0)
//   minsub: v_sub_u32 + v_min_i32 (the fit test's signed minimum)
// lane-ops/s = 64 x (VALU instructions of the loop, counted from the ISA by
// the caller or from the unroll below) x waves / time.
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

constexpr int kChains = 8;

__global__ __launch_bounds__(256) void k_add(uint32_t *out, int iters, uint32_t s) {
  uint32_t a[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) a[c] = threadIdx.x * (c + 1);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int c = 0; c < kChains; ++c) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(a[(c + 1) % kChains]));
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) r ^= a[c];
  if (r == s) out[0] = r;
}

__global__ __launch_bounds__(256) void k_cmpsel(uint32_t *out, int iters, uint32_t s) {
  uint32_t a[kChains], t[kChains], w = threadIdx.x | 1u;
#pragma unroll
  for (int c = 0; c < kChains; ++c) {
    a[c] = threadIdx.x * (c + 3);
    t[c] = threadIdx.x ^ (c * 77);
  }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int c = 0; c < kChains; ++c) {
        uint32_t x;
        asm volatile(
            "v_cmp_ge_u32 vcc, %1, %2\n\t"
            "v_cndmask_b32 %0, 0, %3, vcc\n\t"
            "v_add_u32 %1, %1, %0"
            : "=&v"(x), "+v"(a[c])
            : "v"(t[c]), "v"(w)
            : "vcc");
      }
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) r ^= a[c];
  if (r == s) out[0] = r;
}

__global__ __launch_bounds__(256) void k_minsub(uint32_t *out, int iters, uint32_t s) {
  int32_t m[kChains], f[kChains];
  const int32_t q = (int32_t)threadIdx.x;
#pragma unroll
  for (int c = 0; c < kChains; ++c) {
    m[c] = (int32_t)threadIdx.x * (c + 5);
    f[c] = (int32_t)(threadIdx.x ^ (c * 31));
  }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int c = 0; c < kChains; ++c) {
        int32_t x;
        asm volatile(
            "v_sub_u32 %0, %2, %3\n\t"
            "v_min_i32 %1, %1, %0"
            : "=&v"(x), "+v"(m[c])
            : "v"(f[c]), "v"(q));
      }
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) r ^= (uint32_t)m[c];
  if (r == s) out[0] = r;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *out;
  CK(hipMalloc(&out, 64));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int iters = 2000;
  const int grid = cus * 8;  // 8 workgroups of 4 waves per CU = 8 waves per SIMD
  struct K {
    const char *name;
    void (*fn)(uint32_t *, int, uint32_t);
    int insts;  // VALU instructions per (u, c) step
  };
  const K ks[] = {{"add", k_add, 1}, {"cmpsel", k_cmpsel, 3}, {"minsub", k_minsub, 2}};
  for (const K &k : ks) {
    float best = 1e9f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(k.fn, dim3(grid), dim3(256), 0, 0, out, iters, 0x12345u);
      CK(hipGetLastError());
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep > 0 && ms < best) best = ms;
    }
    const double insts = (double)iters * 8 * kChains * k.insts;  // per wave
    const double waves = (double)grid * 4;
    const double lane_ops = insts * 64 * waves;
    std::printf("%-7s %8.3f ms  %7.2f Tlane-ops/s  (%.1f lanes/clk/SIMD at 2.4 GHz)\n", k.name, best,
                lane_ops / (best * 1e-3) / 1e12, lane_ops / (best * 1e-3) / (cus * 4 * 2.4e9));
  }
  return 0;
}
