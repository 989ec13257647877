// Weight-stream rate of the fused user head's access pattern (ttmi_head.hip WFrags): each wave
// loads its weight fragments one stage ahead into VGPRs; per workgroup ~368 KB of bf16 weights
// (Wo 32 KB, W1 128 KB, W2 128 KB, Wf0 48 KB, Wf3 32 KB) read from L2 (every workgroup reads the
// same weights).  MODE 0: the kernel's addressing (lane group g reads 16 B at k = 32c + 8g of
// output row n0 + 16t + (lane & 15): 16 rows per instruction); MODE 1: the same bytes laid out in
// fragment order (each wave instruction reads 1 KB contiguous).  Prints us per launch.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int NST = 6;
__constant__ int kStageN[NST] = {8, 16, 16, 32, 12, 8};     // uint4 per lane per stage
__constant__ int kStageNT[NST] = {2, 4, 4, 2, 2, 2};        // column tiles (MODE 0 rows)
__constant__ int kStageK[NST] = {128, 128, 128, 512, 192, 128};
__constant__ int kStageOff[NST] = {0, 32768, 98304, 163840, 294912, 344064};   // bytes

template <int MODE>
__device__ __forceinline__ void load_stage(const char* W, int s, int w, int lane, uint4 (&f)[32]) {
  const int n = kStageN[s], nt = kStageNT[s], K = kStageK[s];
  const char* base = W + kStageOff[s];
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    if (i < n) {
      int64_t off;
      if (MODE == 0) {
        const int c = i / nt, t = i % nt;
        const int row = w * 16 * nt + 16 * t + (lane & 15);
        off = (int64_t)row * K * 2 + (c * 32 + (lane >> 4) * 8) * 2;
      } else {
        off = ((int64_t)(w * n + i) * 64 + lane) * 16;
      }
      f[i] = *reinterpret_cast<const uint4*>(base + off);
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void stream_kernel(const char* W, uint32_t* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint4 a[32], b[32];
  uint32_t acc = 0;
  load_stage<MODE>(W, 0, w, lane, a);
#pragma unroll
  for (int s = 0; s < NST; s += 2) {
    if (s + 1 < NST) load_stage<MODE>(W, s + 1, w, lane, b);
#pragma unroll
    for (int i = 0; i < 32; ++i) if (i < kStageN[s]) acc ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
    __syncthreads();
    if (s + 2 < NST) load_stage<MODE>(W, s + 2, w, lane, a);
#pragma unroll
    for (int i = 0; i < 32; ++i) if (i < kStageN[s + 1]) acc ^= b[i].x ^ b[i].y ^ b[i].z ^ b[i].w;
    __syncthreads();
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
  char* W;
  uint32_t* out;
  hipMalloc(&W, 1 << 20);
  hipMemset(W, 1, 1 << 20);
  hipMalloc(&out, 1 << 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int G : {32, 64, 128, 256}) {
    for (int mode = 0; mode < 2; ++mode) {
      auto run = [&]() {
        if (mode == 0) hipLaunchKernelGGL(stream_kernel<0>, dim3(G), dim3(256), 0, 0, W, out);
        else hipLaunchKernelGGL(stream_kernel<1>, dim3(G), dim3(256), 0, 0, W, out);
      };
      for (int i = 0; i < 5; ++i) run();
      hipEventRecord(e0);
      const int N = 50;
      for (int i = 0; i < N; ++i) run();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1000.0 / N;
      printf("G=%4d mode=%d (%s): %7.2f us/launch, %6.1f GB/s per CU\n", G, mode,
             mode ? "fragment-ordered" : "head layout", us, 368.0 * 1024 / us / 1e3);
    }
  }
  return 0;
}
