// Same-address float atomic contention: G workgroups x 256 threads, each thread adds one
// float to dst[(blockIdx % R) * 256 + tid]  (R = replicas; R = G -> no sharing).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void add_kernel(float* dst, int R) {
  atomicAdd(dst + (blockIdx.x % R) * 256 + threadIdx.x, 1.0f);
}
int main() {
  float* d;
  hipMalloc(&d, 64 << 20);
  hipMemset(d, 0, 64 << 20);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const int Gs[] = {256, 1024, 4096};
  const int Rs[] = {1, 8, 32, 256, 4096};
  for (int G : Gs)
    for (int R : Rs) {
      if (R > G) continue;
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(add_kernel, dim3(G), dim3(256), 0, 0, d, R);
      hipEventRecord(a);
      const int N = 20;
      for (int i = 0; i < N; ++i) hipLaunchKernelGGL(add_kernel, dim3(G), dim3(256), 0, 0, d, R);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("G=%5d R=%5d adders/addr=%5d : %8.2f us/launch\n", G, R, G / R, ms * 1000 / N);
    }
  hipFree(d);
  return 0;
}
