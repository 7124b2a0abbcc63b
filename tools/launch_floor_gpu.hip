// Microbenchmark: GPU-side per-launch cost of dependent kernels on one stream
// when the host is far ahead (a 30 ms spin kernel first lets the host enqueue
// every launch before the GPU reaches them): eager vs hipGraph replay, small
// vs 400-B kernargs, trivial vs a 3-level dependent-load chain.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void k_spin(uint64_t ticks) {  // s_memrealtime runs at 100 MHz
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}
__global__ void k_trivial(int *p, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n && p[t] == 12345) p[t] = 0;
}
struct Big { int *p; int n; int pad[100]; };
__global__ void k_big(Big b) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < b.n && b.p[t] == 12345) b.p[t] = b.pad[t & 63];
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
  for (int grid : {1, 64, 2500}) {
    for (int kind = 0; kind < 3; ++kind) {
      auto launch = [&]() {
        if (kind == 0) {
          hipLaunchKernelGGL(k_trivial, dim3(grid), dim3(256), 0, s, p, grid * 256);
        } else if (kind == 2) {
          Big bb{};
          bb.p = p;
          bb.n = grid * 256;
          hipLaunchKernelGGL(k_big, dim3(grid), dim3(256), 0, s, bb);
        } else {
          hipLaunchKernelGGL(k_chain, dim3(grid), dim3(256), 0, s, p, q, grid * 256 < n ? grid * 256 : n);
        }
      };
      for (int i = 0; i < 50; ++i) launch();
      CK(hipStreamSynchronize(s));
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, (uint64_t)3000000);  // 30 ms
      CK(hipEventRecord(a, s));
      const auto h0 = std::chrono::steady_clock::now();
      for (int i = 0; i < L; ++i) launch();
      const double host_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < L; ++i) launch();
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, (uint64_t)1000000);
      CK(hipEventRecord(a, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float gms;
      CK(hipEventElapsedTime(&gms, a, b));
      std::printf("%-8s grid %5d: GPU eager %.2f us/launch (host enqueue %.2f, %s), graph %.2f us/launch\n",
                  kind == 2 ? "big-arg" : kind ? "chain" : "trivial", grid, ms * 1e3 / L, host_us / L,
                  host_us < 30000 ? "ahead" : "NOT ahead", gms * 1e3 / L);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
