// Microbenchmark: does data a previous kernel only READ stay in the XCD L2
// across a kernel boundary? Per dependent load level (p = X[p], a 64 KB table)
// of a short reader kernel, in three sequences (graph replay, 200 pairs each):
//   written: writer(X) -> reader(X)   (the reader's data was just written)
//   reread : reader(X) -> reader(X)   (only read since the last write)
//   other  : writer(Y) -> reader(X)   (an unrelated kernel wrote other data)
// The slope in L (us per level) says what a static operand costs the pass
// kernels.
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
    x[t] = (int)(((unsigned)t * 2654435761u + 977u) % (unsigned)n) + 0 * salt;
}

__global__ void k_read(const int *x, int *out, int n, int L) {
  int p = (blockIdx.x * blockDim.x + threadIdx.x) * 97 % n;
  for (int i = 0; i < L; ++i) p = x[p];
  if (p == -1) out[0] = p;
}

int main() {
  const int n = 16 << 10;  // 64 KB: L2-resident
  int *x, *y, *o;
  CK(hipMalloc(&x, n * sizeof(int)));
  CK(hipMalloc(&y, n * sizeof(int)));
  CK(hipMalloc(&o, 64));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_write, dim3(64), dim3(256), 0, s, x, n, 0);
  CK(hipStreamSynchronize(s));
  const int reps = 200, grid = 128;
  const char *names[3] = {"written", "reread", "other"};
  for (int mode = 0; mode < 3; ++mode) {
    float base = 0;
    for (int L = 0; L <= 6; L += 2) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < reps; ++i) {
        if (mode == 0) hipLaunchKernelGGL(k_write, dim3(64), dim3(256), 0, s, x, n, i);
        if (mode == 1) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, s, x, o, n, 2);
        if (mode == 2) hipLaunchKernelGGL(k_write, dim3(64), dim3(256), 0, s, y, n, i);
        hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, s, x, o, n, L);
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
      if (L == 0) base = us;
      std::printf("%-7s L=%d: %.2f us per pair, %.3f us per level\n", names[mode], L, us,
                  L ? (us - base) / L : 0.f);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
