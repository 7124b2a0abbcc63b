// Microbenchmark for the persistent pass loop: the cost of one
// grid barrier among P resident workgroups of 1,024 threads (atomic arrival
// counter, relaxed sc1 poll, bounded spin), alone and with a dependent level
// of sc1 loads of data other workgroups stored sc1 in the previous phase.
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

__device__ __forceinline__ bool grid_barrier(unsigned *bar, unsigned target, unsigned *err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {  // 200 ms
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        break;
      }
    }
  }
  __shared__ int s_ok;
  if (threadIdx.x == 0) s_ok = ok;
  __syncthreads();
  return s_ok;
}

// mode 0: barriers only; mode 1: each wave stores one 8-B word sc1, barrier,
// then every wave loads another workgroup's word sc1 (one dependent level)
__global__ __launch_bounds__(1024) void k_loop(unsigned *bar, unsigned *err, uint64_t *buf,
                                               int phases, int mode) {
  const int P = gridDim.x;
  const int wv = blockIdx.x * 16 + (threadIdx.x >> 6), W = P * 16;
  uint64_t acc = 0;
  for (int ph = 0; ph < phases; ++ph) {
    if (mode == 1 && (threadIdx.x & 63) == 0)
      __hip_atomic_store(&buf[(size_t)(ph & 1) * W + wv], (uint64_t)ph + acc, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    if (!grid_barrier(bar, (unsigned)(P * (ph + 1)), err)) return;
    if (mode == 1) {
      const int src = (wv + 16 * 3 + 1) % W;  // another workgroup's word
      acc += __hip_atomic_load(&buf[(size_t)(ph & 1) * W + src], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT) & 1;
    }
  }
  if (acc == 12345678) buf[0] = acc;
}

int main() {
  unsigned *bar, *err;
  uint64_t *buf;
  CK(hipMalloc(&bar, 64));
  CK(hipMalloc(&err, 64));
  CK(hipMalloc(&buf, 2 * 256 * 16 * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int phases = 2000;
  for (int mode = 0; mode < 2; ++mode)
    for (int P : {1, 2, 4, 8, 16, 32, 64, 128}) {
      float best = 1e9f;
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemset(bar, 0, 64));
        CK(hipMemset(err, 0, 64));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_loop, dim3(P), dim3(1024), 0, 0, bar, err, buf, phases, mode);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        unsigned e = 0;
        CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
        if (e) {
          std::printf("timeout P=%d\n", P);
          return 1;
        }
        best = ms < best ? ms : best;
      }
      std::printf("mode %d P %3d: %.3f us per phase\n", mode, P, best * 1e3 / phases);
    }
  return 0;
}
