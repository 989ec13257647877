// Micro-benchmark: is the per-XCD start offset seen in the phase stamps (XCDs 0-1 first, 4-5
// ~4.5 us later) a real dispatch stagger or a clock offset between XCDs?  Each workgroup spins
// for SPIN_US (s_memrealtime, 100 MHz) and records its start; the launch is timed with hip
// events.  Real stagger: launch time ~ SPIN_US + the start spread.  Clock offset: ~ SPIN_US.
// Also a dynamic-tile variant: NT tiles of SPIN_US / 8 each taken from an atomic counter.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/xcd_stagger.hip -o tools/micro/xcd_stagger
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void spin_kernel(unsigned long long* starts, int us) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) starts[blockIdx.x] = t0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)us * 100) __builtin_amdgcn_s_sleep(1);
}

__global__ void tiles_kernel(int* ctr, int ntiles, int tile_us, int* done_by_xcd) {
  __shared__ int t;
  int mine = 0;
  for (;;) {
    if (threadIdx.x == 0) t = atomicAdd(ctr, 1);
    __syncthreads();
    const int tt = t;
    __syncthreads();
    if (tt >= ntiles) break;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)tile_us * 100) __builtin_amdgcn_s_sleep(1);
    ++mine;
  }
  if (threadIdx.x == 0) atomicAdd(done_by_xcd + (blockIdx.x & 7), mine);
}

__global__ void static_tiles_kernel(int ntiles, int tile_us) {
  for (int tt = blockIdx.x; tt < ntiles; tt += gridDim.x) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)tile_us * 100) __builtin_amdgcn_s_sleep(1);
  }
}

static float time_it(void (*fn)(hipStream_t), hipStream_t s, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  fn(s);
  hipStreamSynchronize(s);
  hipEventRecord(a, s);
  for (int i = 0; i < reps; ++i) fn(s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

static unsigned long long* g_starts;
static int* g_ctr;
static int* g_done;
static int g_blocks = 256, g_us = 10, g_ntiles = 2048, g_tile_us = 1;

int main() {
  hipMalloc(&g_starts, 4096 * 8);
  hipMalloc(&g_ctr, 4);
  hipMalloc(&g_done, 32);
  hipStream_t s;
  hipStreamCreate(&s);
  for (int us : {0, 5, 10}) {
    g_us = us;
    for (int nb : {8, 256, 1024}) {
      g_blocks = nb;
      const float t = time_it([](hipStream_t st) { spin_kernel<<<g_blocks, 64, 0, st>>>(g_starts, g_us); }, s, 50);
      std::vector<unsigned long long> h(nb);
      hipMemcpy(h.data(), g_starts, nb * 8, hipMemcpyDeviceToHost);
      const unsigned long long mn = *std::min_element(h.begin(), h.end());
      double xs[8] = {0};
      for (int x = 0; x < 8; ++x) {
        unsigned long long m = ~0ull;
        for (int i = x; i < nb; i += 8) m = std::min(m, h[i]);
        xs[x] = (m - mn) / 100.0;
      }
      printf("spin %2d us, %4d blocks: launch %6.2f us; first start per xcd (us): %.2f %.2f %.2f %.2f %.2f %.2f %.2f %.2f\n",
             us, nb, t, xs[0], xs[1], xs[2], xs[3], xs[4], xs[5], xs[6], xs[7]);
    }
  }
  // 2048 tiles of 1 us on 256 workgroups: static round-robin vs an atomic tile counter
  g_ntiles = 2048; g_tile_us = 1;
  const float ts = time_it([](hipStream_t st) { static_tiles_kernel<<<256, 64, 0, st>>>(g_ntiles, g_tile_us); }, s, 20);
  float td = 0;
  int done[8] = {0};
  for (int r = 0; r < 21; ++r) {
    hipMemsetAsync(g_ctr, 0, 4, s);
    hipMemsetAsync(g_done, 0, 32, s);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, s);
    tiles_kernel<<<256, 64, 0, s>>>(g_ctr, g_ntiles, g_tile_us, g_done);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (r) td += ms * 1000.f / 20;
    hipMemcpy(done, g_done, 32, hipMemcpyDeviceToHost);
  }
  printf("2048 x 1 us tiles on 256 WGs: static %.2f us, atomic counter %.2f us; tiles per xcd %d %d %d %d %d %d %d %d\n",
         ts, td, done[0], done[1], done[2], done[3], done[4], done[5], done[6], done[7]);
  return 0;
}
