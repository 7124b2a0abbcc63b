// Microbenchmark: cost of one dependent global-load level in a short kernel
// that reads data the previous kernel (all CUs) just wrote — the situation of
// every plan/accept pass. Graph replay of (writer, reader) pairs;
// reader = L dependent loads per lane (p = X[p]) for L = 0..6.
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

__global__ void k_write(int *x, int n, int salt) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x)
    x[t] = (int)(((unsigned)t * 2654435761u + (unsigned)salt) % (unsigned)n);
}

__global__ void k_read(const int *x, int *out, int n, int L) {
  int p = (blockIdx.x * blockDim.x + threadIdx.x) * 97 % n;
  for (int i = 0; i < L; ++i) p = x[p];
  if (p == -1) out[0] = p;
}

int main() {
  const int n = 4 << 20;  // 16 MB
  int *x, *o;
  CK(hipMalloc(&x, n * sizeof(int)));
  CK(hipMalloc(&o, 64));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 200;
  for (int grid : {4, 170}) {
    float base = 0;
    for (int L = -1; L <= 6; ++L) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < reps; ++i) {
        hipLaunchKernelGGL(k_write, dim3(1024), dim3(256), 0, s, x, n, i);
        if (L >= 0) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, s, x, o, n, L);
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(a, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      const float us = ms * 1e3f / reps;
      if (L < 0)
        base = us;
      else
        std::printf("grid %4d  levels %d: reader adds %.2f us (writer alone %.2f us)\n", grid, L,
                    us - base, base);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
