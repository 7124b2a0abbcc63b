// Microbenchmark: cost of cooperative_groups grid.sync() inside one
// cooperative launch, for small grids (the candidate design for running all
// acceptance passes of a small round in one launch).
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <cstdio>

namespace cg = cooperative_groups;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

__global__ void k_syncs(int *x, int nsync) {
  cg::grid_group g = cg::this_grid();
  for (int i = 0; i < nsync; ++i) {
    if (threadIdx.x == 0) atomicAdd(&x[(blockIdx.x + i) % gridDim.x], 1);
    g.sync();
  }
}

int main() {
  int *x;
  CK(hipMalloc(&x, 4096 * sizeof(int)));
  CK(hipMemset(x, 0, 4096 * sizeof(int)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int threads : {256, 1024}) {
    for (int grid : {8, 16, 32, 64, 128}) {
      float t[2];
      for (int v = 0; v < 2; ++v) {
        int nsync = v ? 64 : 0;
        void *args[] = {&x, &nsync};
        CK(hipLaunchCooperativeKernel((void *)k_syncs, dim3(grid), dim3(threads), args, 0, s));
        CK(hipStreamSynchronize(s));
        float best = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
          CK(hipEventRecord(a, s));
          CK(hipLaunchCooperativeKernel((void *)k_syncs, dim3(grid), dim3(threads), args, 0, s));
          CK(hipEventRecord(b, s));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          if (ms < best) best = ms;
        }
        t[v] = best * 1e3f;
      }
      std::printf("threads %4d grid %4d: launch %.2f us, per grid.sync %.2f us\n", threads, grid,
                  t[0], (t[1] - t[0]) / 64);
    }
  }
  return 0;
}
