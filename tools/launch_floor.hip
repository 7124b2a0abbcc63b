// Microbenchmark: per-launch floor of dependent kernels on one stream, eager
// vs hipGraph replay, for grids of 1 / 42 / 2500 workgroups, plus a kernel
// with a short dependent load chain. Informs the pass-loop design.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void k_trivial(int *p, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n && p[t] == 12345) p[t] = 0;
}

__global__ void k_chain(const int *__restrict__ a, int *__restrict__ out, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  int x = a[t];
  int y = a[(x * 7 + t) & (n - 1)];
  int z = a[(y * 13 + t) & (n - 1)];
  out[t] = x + y + z;
}

int main() {
  const int n = 1 << 20;
  int *p, *q;
  CK(hipMalloc(&p, n * sizeof(int)));
  CK(hipMalloc(&q, n * sizeof(int)));
  CK(hipMemset(p, 0, n * sizeof(int)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int L = 2000;
  for (int grid : {1, 42, 172, 2500}) {
    for (int kind = 0; kind < 2; ++kind) {
      auto launch = [&]() {
        if (kind == 0)
          hipLaunchKernelGGL(k_trivial, dim3(grid), dim3(256), 0, s, p, grid * 256);
        else
          hipLaunchKernelGGL(k_chain, dim3(grid), dim3(256), 0, s, p, q, grid * 256 < n ? grid * 256 : n);
      };
      for (int i = 0; i < 50; ++i) launch();
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(a, s));
      for (int i = 0; i < L; ++i) launch();
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      // graph
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < L; ++i) launch();
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(a, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float gms;
      CK(hipEventElapsedTime(&gms, a, b));
      std::printf("%-8s grid %5d: eager %.2f us/launch, graph %.2f us/launch\n",
                  kind ? "chain" : "trivial", grid, ms * 1e3 / L, gms * 1e3 / L);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
