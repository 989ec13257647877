// ttmi_infonce.hip — symmetric in-batch InfoNCE of TwoTowerModel.forward
// (reference two_tower.py:98-140), fp32 end to end (1/τ = 14.3 amplifies any logit error).
//
// forward : l2norm(u), l2norm(i)                       [1 launch, wave per row]
//           S = û·îᵀ/τ                                [f32-MFMA GEMM]
//           collision mask + row LSE (wave per row) ∥ column LSE (thread per column,
//           online max/sum, mask recomputed on the fly)  [1 launch]
//           loss = (Σ CE_row + Σ CE_col) / 2B          [1 block, fixed order: deterministic]
// backward: dS = g/2B·[(softmax_row − I) + (softmax_col − I)], 0 at masked entries
//           dû' = dS·î/τ, dî' = dSᵀ·û/τ               [2 f32-MFMA GEMMs]
//           normalize backward                          [1 launch]
#include "ttmi_common.h"

namespace {

constexpr float NORM_EPS = 1e-12f;   // F.normalize default
constexpr float MASK_FILL = -1e4f;   // two_tower.py:121

__global__ __launch_bounds__(256) void l2norm_kernel(int B, int D, const float* __restrict__ u,
                                                     const float* __restrict__ it,
                                                     float* __restrict__ uh, float* __restrict__ ih,
                                                     float* __restrict__ norms) {
  const int lane = threadIdx.x & 63;
  const int row = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (row >= 2 * B) return;
  const bool isu = row < B;
  const int r = isu ? row : row - B;
  const float* x = (isu ? u : it) + (int64_t)r * D;
  float* y = (isu ? uh : ih) + (int64_t)r * D;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) s += x[c] * x[c];
  const float nrm = sqrtf(wave_sum(s));
  const float inv = 1.f / fmaxf(nrm, NORM_EPS);
  for (int c = lane; c < D; c += 64) y[c] = x[c] * inv;
  if (lane == 0) norms[row] = nrm;
}

TTMI_DEV bool collide(const int64_t* uid, int i, int j) {
  return uid && i != j && uid[i] == uid[j];
}

// blocks [0, nrb): rows (wave per row; masks the logits in place);
// blocks [nrb, ...): columns — 32 columns x 8 row groups per block, online max/sum-exp per
// thread, partials merged through LDS (the mask is recomputed, so row and column blocks
// need no ordering).
constexpr int LC = 32, LRG = 8;

__global__ __launch_bounds__(256) void lse_kernel(int B, float* __restrict__ S,
                                                  const int64_t* __restrict__ uid,
                                                  float* __restrict__ lse, float* __restrict__ ce,
                                                  int nrb) {
  if ((int)blockIdx.x < nrb) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= B) return;
    float* row = S + (int64_t)i * B;
    float m = -INFINITY;
    for (int j = lane; j < B; j += 64) {
      float v = row[j];
      if (collide(uid, i, j)) { v = MASK_FILL; row[j] = v; }
      m = fmaxf(m, v);
    }
    m = wave_max(m);
    float s = 0.f;
    for (int j = lane; j < B; j += 64) {
      const float v = collide(uid, i, j) ? MASK_FILL : row[j];
      s += expf(v - m);
    }
    s = wave_sum(s);
    if (lane == 0) {
      const float l = m + logf(s);
      lse[i] = l;
      ce[i] = l - row[i];
    }
    return;
  }
  __shared__ float pm[LRG][LC], ps[LRG][LC], pd[LRG][LC];
  const int cl = threadIdx.x % LC, rg = threadIdx.x / LC;
  const int j = (blockIdx.x - nrb) * LC + cl;
  float m = -INFINITY, s = 0.f, diag = 0.f;
  if (j < B) {
    for (int i = rg; i < B; i += LRG) {
      const float v = collide(uid, i, j) ? MASK_FILL : S[(int64_t)i * B + j];
      if (i == j) diag = v;
      if (v > m) { s = s * expf(m - v) + 1.f; m = v; }
      else s += expf(v - m);
    }
  }
  pm[rg][cl] = m;
  ps[rg][cl] = s;
  pd[rg][cl] = diag;
  __syncthreads();
  if (rg == 0 && j < B) {
    float M = -INFINITY, D = 0.f;
#pragma unroll
    for (int k = 0; k < LRG; ++k) { M = fmaxf(M, pm[k][cl]); D += pd[k][cl]; }
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < LRG; ++k) tot += ps[k][cl] * expf(pm[k][cl] - M);
    const float l = M + logf(tot);
    lse[B + j] = l;
    ce[B + j] = l - D;
  }
}

__global__ __launch_bounds__(256) void loss_kernel(int n, const float* __restrict__ ce, float scale,
                                                   float* __restrict__ loss) {
  __shared__ float red[256];
  float s = 0.f;
  for (int k = threadIdx.x; k < n; k += 256) s += ce[k];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = red[0] * scale;
}

__global__ __launch_bounds__(256) void dlogits_kernel(int B, const float* __restrict__ S,
                                                      const float* __restrict__ lse,
                                                      const int64_t* __restrict__ uid,
                                                      const float* __restrict__ dloss, float scale,
                                                      float* __restrict__ dS) {
  const int64_t n = (int64_t)B * B;
  const float g = (dloss ? dloss[0] : 1.f) * scale;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(k / B), j = (int)(k % B);
    float d = 0.f;
    if (!collide(uid, i, j)) {
      const float v = S[k];
      const float diag = i == j ? 1.f : 0.f;
      d = g * ((expf(v - lse[i]) - diag) + (expf(v - lse[B + j]) - diag));
    }
    dS[k] = d;
  }
}

__global__ __launch_bounds__(256) void l2norm_bwd_kernel(int B, int D, const float* __restrict__ uh,
                                                         const float* __restrict__ ih,
                                                         const float* __restrict__ norms,
                                                         const float* __restrict__ duh,
                                                         const float* __restrict__ dih,
                                                         float* __restrict__ du,
                                                         float* __restrict__ di) {
  const int lane = threadIdx.x & 63;
  const int row = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (row >= 2 * B) return;
  const bool isu = row < B;
  const int r = isu ? row : row - B;
  const float* y = (isu ? uh : ih) + (int64_t)r * D;
  const float* dy = (isu ? duh : dih) + (int64_t)r * D;
  float* dx = (isu ? du : di) + (int64_t)r * D;
  const float nrm = norms[row];
  if (nrm > NORM_EPS) {
    float s = 0.f;
    for (int c = lane; c < D; c += 64) s += y[c] * dy[c];
    s = wave_sum(s);
    const float inv = 1.f / nrm;
    for (int c = lane; c < D; c += 64) dx[c] = (dy[c] - y[c] * s) * inv;
  } else {
    for (int c = lane; c < D; c += 64) dx[c] = dy[c] / NORM_EPS;
  }
}

// Single-tensor forms (wave per row) for the distributed InfoNCE pieces.
__global__ __launch_bounds__(256) void rows_l2norm_kernel(int n, int D, const float* __restrict__ x,
                                                          float* __restrict__ y,
                                                          float* __restrict__ norms) {
  const int lane = threadIdx.x & 63;
  const int r = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (r >= n) return;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) s += x[(int64_t)r * D + c] * x[(int64_t)r * D + c];
  const float nrm = sqrtf(wave_sum(s));
  const float inv = 1.f / fmaxf(nrm, NORM_EPS);
  for (int c = lane; c < D; c += 64) y[(int64_t)r * D + c] = x[(int64_t)r * D + c] * inv;
  if (lane == 0) norms[r] = nrm;
}

__global__ __launch_bounds__(256) void rows_l2norm_bwd_kernel(int n, int D, const float* __restrict__ y,
                                                              const float* __restrict__ norms,
                                                              const float* __restrict__ dy,
                                                              const float* __restrict__ dy2,
                                                              float* __restrict__ dx) {
  const int lane = threadIdx.x & 63;
  const int r = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (r >= n) return;
  const float* yr = y + (int64_t)r * D;
  const float* dyr = dy + (int64_t)r * D;
  const float* dy2r = dy2 ? dy2 + (int64_t)r * D : nullptr;
  float* dxr = dx + (int64_t)r * D;
  const float nrm = norms[r];
  auto g = [&](int c) { return dyr[c] + (dy2r ? dy2r[c] : 0.f); };
  if (nrm > NORM_EPS) {
    float s = 0.f;
    for (int c = lane; c < D; c += 64) s += yr[c] * g(c);
    s = wave_sum(s);
    const float inv = 1.f / nrm;
    for (int c = lane; c < D; c += 64) dxr[c] = (g(c) - yr[c] * s) * inv;
  } else {
    for (int c = lane; c < D; c += 64) dxr[c] = g(c) / NORM_EPS;
  }
}

// ---------------------------------------------------------------- rectangular row CE
// Global in-batch negatives (BASELINE cfg 5): each rank scores its R query rows against all
// C = world·B gathered keys.  Row i's positive is column row0 + i; column j is masked to
// MASK_FILL when uid_q[i] == uid_k[j] and j != row0 + i (two_tower.py:111-124 applied to the
// concatenated global batch).  One wave per row: masked logits written back, LSE, CE.
__global__ __launch_bounds__(256) void rowce_lse_kernel(int R, int C, int64_t row0,
                                                        float* __restrict__ S,
                                                        const int64_t* __restrict__ uq,
                                                        const int64_t* __restrict__ uk,
                                                        float* __restrict__ lse,
                                                        float* __restrict__ ce) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= R) return;
  float* row = S + (int64_t)i * C;
  const int64_t tgt = row0 + i;
  const bool mask = uq != nullptr && uk != nullptr;
  const int64_t me = mask ? uq[i] : 0;
  float m = -INFINITY;
  for (int j = lane; j < C; j += 64) {
    float v = row[j];
    if (mask && j != tgt && uk[j] == me) { v = MASK_FILL; row[j] = v; }
    m = fmaxf(m, v);
  }
  m = wave_max(m);
  float sum = 0.f;
  for (int j = lane; j < C; j += 64) sum += expf(row[j] - m);
  sum = wave_sum(sum);
  if (lane == 0) {
    const float l = m + logf(sum);
    lse[i] = l;
    ce[i] = l - row[tgt];
  }
}

// dS[i,j] = g·scale·(softmax_ij − [j == row0+i]), 0 at masked entries.
__global__ __launch_bounds__(256) void rowce_dlogits_kernel(int R, int C, int64_t row0,
                                                            const float* __restrict__ S,
                                                            const float* __restrict__ lse,
                                                            const int64_t* __restrict__ uq,
                                                            const int64_t* __restrict__ uk,
                                                            const float* __restrict__ dloss,
                                                            float scale, float* __restrict__ dS) {
  const int64_t n = (int64_t)R * C;
  const float g = (dloss ? dloss[0] : 1.f) * scale;
  const bool mask = uq != nullptr && uk != nullptr;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(k / C), j = (int)(k % C);
    const bool pos = j == row0 + i;
    float d = 0.f;
    if (!(mask && !pos && uk[j] == uq[i])) d = g * (expf(S[k] - lse[i]) - (pos ? 1.f : 0.f));
    dS[k] = d;
  }
}

// ------------------------------------------------------------ fused local InfoNCE
// Both CE directions as rows: direction 0 scores û_i against every î_j (rows of S),
// direction 1 scores î_j against every û_i (rows of Sᵀ = columns of S).  A workgroup owns 16
// query rows of one direction and one of NSPLIT key ranges (2·(B/16)·NSPLIT workgroups);
// f32 MFMA (16x16x4, exact fp32 products) gives the 16x16 logit tiles, each lane keeps an
// online (max, sum-exp) over its keys; partials are merged by nce_combine_kernel.
constexpr int NQ = 16, NSPLIT = 4;

TTMI_DEV void online_add(float& m, float& s, float v) {
  if (v == -INFINITY) return;
  if (v > m) { s = s * expf(m - v) + 1.f; m = v; }
  else s += expf(v - m);
}
TTMI_DEV void online_merge(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;
  if (m == -INFINITY) { m = m2; s = s2; return; }
  const float M = fmaxf(m, m2);
  // explicit fma: the contraction is otherwise the backend's per-context choice, and the
  // in-launch combine must match nce_combine_kernel bit for bit
  s = fmaf(s, expf(m - M), s2 * expf(m2 - M));
  m = M;
}

// Agent-scope relaxed atomic store / load of a float (visible to every XCD without a cache
// writeback fence).
TTMI_DEV void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
TTMI_DEV float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int DC, bool VEC>
__global__ __launch_bounds__(256) void nce_fwd_kernel(int B, const float* __restrict__ uh,
                                                      const float* __restrict__ ih,
                                                      const int64_t* __restrict__ uid,
                                                      float inv_tau, float* __restrict__ logits,
                                                      float* __restrict__ part, int* __restrict__ cnt,
                                                      float* __restrict__ qsum, float* __restrict__ lse,
                                                      float* __restrict__ loss,
                                                      float* __restrict__ loss_acc) {
  constexpr int D = 16 * DC, QP = D * 4 + 16;
  __shared__ __attribute__((aligned(16))) char sq[NQ * QP];
  __shared__ float sm[4][NQ], ss[4][NQ], st[4][NQ];
  TTMI_TSTAMP(0);
  const int nb = (B + NQ - 1) / NQ;
  const int split = blockIdx.x % NSPLIT;
  const int qb = blockIdx.x / NSPLIT;
  const int dir = qb >= nb;
  const int i0 = (qb - dir * nb) * NQ;
  const float* Q = dir ? ih : uh;
  const float* Kp = dir ? uh : ih;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lg = lane >> 4;
  for (int idx = tid; idx < NQ * D / 4; idx += 256) {
    const int r = idx / (D / 4), c4 = idx % (D / 4);
    const int row = i0 + r;
    const float4 v = row < B ? *reinterpret_cast<const float4*>(Q + (int64_t)row * D + 4 * c4)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(sq + r * QP + c4 * 16) = v;
  }
  __syncthreads();
  TTMI_TSTAMP(1);
  const int i = i0 + li;
  const bool iok = i < B;
  const int64_t ui = (uid && iok) ? uid[i] : 0;
  float m = -INFINITY, sum = 0.f, tgt = 0.f;
  const int nkt = (B + 15) / 16;
  const int kt0 = (int)((int64_t)nkt * split / NSPLIT), kt1 = (int)((int64_t)nkt * (split + 1) / NSPLIT);
  // the key tile's fragments and user ids are loaded one tile ahead (each tile was a K load
  // round trip, then a dependent uid round trip: 4 serial round trips per wave at B = 512)
  uint4 a[DC];
  int64_t uk[4];
  auto load_tile = [&](int t) {
    const float* kp = Kp + (int64_t)min(16 * t + li, B - 1) * D + 4 * lg;   // clamped; masked below
#pragma unroll
    for (int c = 0; c < DC; ++c) a[c] = *reinterpret_cast<const uint4*>(kp + 16 * c);
#pragma unroll
    for (int r = 0; r < 4; ++r) uk[r] = uid ? uid[min(16 * t + 4 * lg + r, B - 1)] : 0;
  };
  if (kt0 + wave < kt1) load_tile(kt0 + wave);
  for (int t = kt0 + wave; t < kt1; t += 4) {
    f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
    uint4 ac[DC];
    int64_t ukc[4];
#pragma unroll
    for (int c = 0; c < DC; ++c) ac[c] = a[c];
#pragma unroll
    for (int r = 0; r < 4; ++r) ukc[r] = uk[r];
    if (t + 4 < kt1) load_tile(t + 4);
#pragma unroll
    for (int c = 0; c < DC; ++c) {
      const uint4 b = lds16(sq + li * QP + (16 * c + 4 * lg) * 4);
      Mma<float>::run(acc, ac[c], b);
    }
    // this lane: query row li, keys 16t + 4lg + r
    float o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * t + 4 * lg + r;
      float v = acc[r] * inv_tau;
      if (j >= B) v = -INFINITY;
      else if (uid && j != i && ukc[r] == ui) v = MASK_FILL;
      if (j == i) tgt = v;
      o[r] = v;
      online_add(m, sum, v);
    }
    if (dir == 0 && iok && 16 * t + 4 * lg < B) {
      if constexpr (VEC) {
        *reinterpret_cast<float4*>(logits + (int64_t)i * B + 16 * t + 4 * lg) = make_float4(o[0], o[1], o[2], o[3]);
      } else {   // ragged B (row pitch not 16-byte aligned): element stores inside the row
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (16 * t + 4 * lg + r < B) logits[(int64_t)i * B + 16 * t + 4 * lg + r] = o[r];
      }
    }
  }
  TTMI_TSTAMP(2);
  // merge the 4 lane groups holding row li, then the 4 waves
#pragma unroll
  for (int off = 16; off <= 32; off <<= 1) {
    const float m2 = __shfl_xor(m, off, 64), s2 = __shfl_xor(sum, off, 64);
    online_merge(m, sum, m2, s2);
    tgt += __shfl_xor(tgt, off, 64);
  }
  if (lg == 0) { sm[wave][li] = m; ss[wave][li] = sum; st[wave][li] = tgt; }
  __syncthreads();
  if (tid < NQ && i0 + tid < B) {
    float M = sm[0][tid], S_ = ss[0][tid], T = st[0][tid];
#pragma unroll
    for (int w = 1; w < 4; ++w) { online_merge(M, S_, sm[w][tid], ss[w][tid]); T += st[w][tid]; }
    const int64_t row = (int64_t)dir * B + i0 + tid;
    if (cnt == nullptr) {
      part[(0 * NSPLIT + split) * 2 * (int64_t)B + row] = M;
      part[(1 * NSPLIT + split) * 2 * (int64_t)B + row] = S_;
      part[(2 * NSPLIT + split) * 2 * (int64_t)B + row] = T;
    } else {                                         // read by another XCD's workgroup
      st_agent(part + (0 * NSPLIT + split) * 2 * (int64_t)B + row, M);
      st_agent(part + (1 * NSPLIT + split) * 2 * (int64_t)B + row, S_);
      st_agent(part + (2 * NSPLIT + split) * 2 * (int64_t)B + row, T);
    }
  }
  if (cnt == nullptr) return;                        // nce_combine_kernel follows
  // ---- the combine in the same launch (ABI 15): the last of a query block's NSPLIT
  // workgroups (arrival count) merges its 16 rows into lse and their CE sum; the last query
  // block adds the per-block sums in block order (deterministic).  Each last arriver resets
  // its counter.  Cross-XCD visibility without fences: the exchanged values are agent-scope
  // relaxed atomic stores / loads (coherent at the memory side, sc1), the stores are retired
  // (vmcnt(0)) before the arrival increment.  (A __threadfence pair instead wrote back the
  // whole L2 per workgroup: 8.7 -> 43 us.)
  __shared__ int s_last;
  const int nqb = 2 * nb;
  __builtin_amdgcn_s_waitcnt(0);                     // every counter at zero: stores retired
  __syncthreads();
  TTMI_TSTAMP(3);
  if (tid == 0)
    s_last = __hip_atomic_fetch_add(cnt + qb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == NSPLIT - 1;
  __syncthreads();
  TTMI_TSTAMP(4);
  if (!s_last) return;
  if (tid < 64) {
    float c = 0.f;
    if (tid < NQ && i0 + tid < B) {
      const int64_t n2 = 2 * (int64_t)B, row = (int64_t)dir * B + i0 + tid;
      float pm[NSPLIT], ps[NSPLIT], T = 0.f;
#pragma unroll
      for (int k = 0; k < NSPLIT; ++k) {
        pm[k] = ld_agent(part + (0 * NSPLIT + k) * n2 + row);
        ps[k] = ld_agent(part + (1 * NSPLIT + k) * n2 + row);
        T += ld_agent(part + (2 * NSPLIT + k) * n2 + row);
      }
      float M = -INFINITY, S_ = 0.f;
#pragma unroll
      for (int k = 0; k < NSPLIT; ++k) online_merge(M, S_, pm[k], ps[k]);
      const float l = M + logf(S_);
      lse[row] = l;
      c = l - T;
    }
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if (tid == 0) {
      st_agent(qsum + qb, c);
      __hip_atomic_store(cnt + qb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  TTMI_TSTAMP(5);
  if (tid == 0)
    s_last = __hip_atomic_fetch_add(cnt + nqb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nqb - 1;
  __syncthreads();
  if (!s_last) return;
  TTMI_TSTAMP(6);
  if (tid < 64) {
    float c = 0.f;
    for (int q = tid; q < nqb; q += 64) c += ld_agent(qsum + q);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if (tid == 0) {
      const float lv = c * (0.5f / (float)B);
      loss[0] = lv;
      if (loss_acc) loss_acc[0] += lv;               // the caller's running sum (epoch mean)
      __hip_atomic_store(cnt + nqb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// lse[2B], loss = Σ CE / 2B (one block of 1024 threads, fixed order: deterministic).
__global__ __launch_bounds__(1024) void nce_combine_kernel(int B, const float* __restrict__ part,
                                                           float* __restrict__ lse,
                                                           float* __restrict__ loss) {
  __shared__ float red[1024];
  const int64_t n = 2 * (int64_t)B;
  float acc = 0.f;
  for (int64_t r = threadIdx.x; r < n; r += 1024) {
    float pm[NSPLIT], ps[NSPLIT], T = 0.f;
#pragma unroll
    for (int k = 0; k < NSPLIT; ++k) {
      pm[k] = part[(0 * NSPLIT + k) * n + r];
      ps[k] = part[(1 * NSPLIT + k) * n + r];
      T += part[(2 * NSPLIT + k) * n + r];
    }
    float M = -INFINITY, S_ = 0.f;
#pragma unroll
    for (int k = 0; k < NSPLIT; ++k) online_merge(M, S_, pm[k], ps[k]);
    const float l = M + logf(S_);
    lse[r] = l;
    acc += l - T;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = red[0] * (0.5f / (float)B);
}

// Backward.  G[i,j] = g/2B·(e^(S_ij − lse_i) + e^(S_ij − lse'_j) − 2δ_ij) (masked S = −1e4 gives
// 0); dû_i = Σ_j G_ij î_j /τ (direction 0), dî_j = Σ_i G_ij û_i /τ (direction 1).  A
// workgroup owns 16 output rows of one direction and one of NSPLIT key ranges, walked in
// blocks of 64 keys: the workgroup stages the key block of V (16-byte loads) and the 16 x 64
// block of G (computed once per workgroup, not per wave) in LDS, then each wave runs its
// d-tiles' MFMAs D[d][row] = Σ_k Vᵀ[d][k] G[row][k] from LDS; partial rows go to part.
constexpr int NKB = 64;   // keys per staged block

// Four consecutive floats p[k .. k+3] of a row of n: one 16-byte load when the row pitch keeps
// it aligned (VEC, n % 4 == 0, k clamped to n - 4), else element loads clamped to n - 1.
template <bool VEC>
TTMI_DEV void load4(const float* __restrict__ p, int k, int n, float (&v)[4]) {
  if constexpr (VEC) {
    const float4 q = *reinterpret_cast<const float4*>(p + min(k, n - 4));
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = p[min(k + e, n - 1)];
  }
}

// The finish's arguments when it runs inside the backward launch (ttmi_infonce_bwd_fused).
struct NceFinish {
  const float* norms; float inv_tau; float* du; float* di; bf16_t* du16; int* cnt;
};

template <int DC, bool VEC, bool FIN>
__global__ __launch_bounds__(256) void nce_bwd_kernel(int B, const float* __restrict__ uh,
                                                      const float* __restrict__ ih,
                                                      const float* __restrict__ S,
                                                      const float* __restrict__ lse,
                                                      const float* __restrict__ dloss,
                                                      float* __restrict__ part, NceFinish fin) {
  constexpr int D = 16 * DC, TPW = DC / 4;
  static_assert(DC % 4 == 0, "D % 64 == 0");
  constexpr int VP = D + 4, GP = NKB + 4;          // LDS pitches (floats)
  __shared__ __attribute__((aligned(16))) float sV[NKB * VP];
  __shared__ __attribute__((aligned(16))) float sG[NQ * GP];
  TTMI_TSTAMP(0);
  const int nb = (B + NQ - 1) / NQ;
  const int split = blockIdx.x % NSPLIT;
  const int qb = blockIdx.x / NSPLIT;
  const int dir = qb >= nb;
  const int r0 = (qb - dir * nb) * NQ;
  const float* V = dir ? uh : ih;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lg = lane >> 4;
  const float coef = (dloss ? dloss[0] : 1.f) * (0.5f / (float)B);
  const float* lse_q = lse + (int64_t)dir * B;     // the output rows' direction
  const float* lse_k = lse + (int64_t)(1 - dir) * B;
  f32x4_t acc[TPW];
#pragma unroll
  for (int q = 0; q < TPW; ++q) acc[q] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int kbeg = (int)((int64_t)B * split / NSPLIT) / 4 * 4;
  const int kend = split == NSPLIT - 1 ? B : (int)((int64_t)B * (split + 1) / NSPLIT) / 4 * 4;
  // the next key block's V rows, S values and lse terms are loaded while this block's G and
  // MFMAs run (each block was a load round trip before its LDS staging: 2 per workgroup at
  // B = 512, serial)
  constexpr int VQ = NKB * D / 4 / 256;            // float4 per thread
  float4 v[VQ];
  float sv[4], l4[4], l1;
  auto load_blk = [&](int k0) {
#pragma unroll
    for (int j = 0; j < VQ; ++j) {
      const int idx = tid + 256 * j, kr = idx / (D / 4), c4 = idx % (D / 4);
      v[j] = *reinterpret_cast<const float4*>(V + (int64_t)min(k0 + kr, B - 1) * D + 4 * c4);
    }
    if (dir == 0) {      // thread -> row tid/16, keys 4·(tid%16) .. +3 (one float4 of S's row)
      const int row = r0 + (tid >> 4), k = k0 + (tid & 15) * 4;
      load4<VEC>(S + (int64_t)min(row, B - 1) * B, k, B, sv);
      load4<VEC>(lse_k, k, B, l4);
      l1 = lse_q[min(row, B - 1)];
    } else {             // thread -> key tid/4, rows 4·(tid%4) .. +3 (one float4 of S's row k)
      const int k = k0 + (tid >> 2), row = r0 + (tid & 3) * 4;
      load4<VEC>(S + (int64_t)min(k, B - 1) * B, row, B, sv);
      load4<VEC>(lse_q, row, B, l4);
      l1 = lse_k[min(k, B - 1)];
    }
  };
  if (kbeg < kend) load_blk(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += NKB) {
    // ---- stage V[k0 .. k0+64) (rows past kend zero) and G[16][64]
    float4 vc[VQ];
    float svv[4], lv[4];
#pragma unroll
    for (int j = 0; j < VQ; ++j) vc[j] = v[j];
#pragma unroll
    for (int e = 0; e < 4; ++e) { svv[e] = sv[e]; lv[e] = l4[e]; }
    const float lc = l1;
    if (k0 + NKB < kend) load_blk(k0 + NKB);
    float g[4];
    int gr[4], gk[4];
    if (dir == 0) {
      const int r = tid >> 4, kq = (tid & 15) * 4;
      const int row = r0 + r, k = k0 + kq;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gr[e] = r;
        gk[e] = kq + e;
        const bool ok = row < B && k + e < kend;
        g[e] = ok ? coef * (__expf(svv[e] - lc) + __expf(svv[e] - lv[e]) - (k + e == row ? 2.f : 0.f)) : 0.f;
      }
    } else {
      const int kk = tid >> 2, rq = (tid & 3) * 4;
      const int k = k0 + kk, row = r0 + rq;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gr[e] = rq + e;
        gk[e] = kk;
        const bool ok = row + e < B && k < kend;
        g[e] = ok ? coef * (__expf(svv[e] - lv[e]) + __expf(svv[e] - lc) - (k == row + e ? 2.f : 0.f)) : 0.f;
      }
    }
    __syncthreads();                               // previous block's MFMAs done with LDS
#pragma unroll
    for (int j = 0; j < VQ; ++j) {
      const int idx = tid + 256 * j, kr = idx / (D / 4), c4 = idx % (D / 4);
      *reinterpret_cast<float4*>(sV + kr * VP + 4 * c4) =
          k0 + kr < kend ? vc[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) sG[gr[e] * GP + gk[e]] = g[e];
    __syncthreads();
    // ---- MFMAs: A = Vᵀ fragment (lane li = d, k = 16c + 4lg + e), B = G fragment
#pragma unroll
    for (int c = 0; c < NKB / 16; ++c) {
      const int kb = 16 * c + 4 * lg;
      const uint4 gf = *reinterpret_cast<const uint4*>(sG + li * GP + kb);
#pragma unroll
      for (int q = 0; q < TPW; ++q) {
        const int d = (wave + 4 * q) * 16 + li;
        const uint4 xf = make_uint4(__float_as_uint(sV[(kb + 0) * VP + d]), __float_as_uint(sV[(kb + 1) * VP + d]),
                                    __float_as_uint(sV[(kb + 2) * VP + d]), __float_as_uint(sV[(kb + 3) * VP + d]));
        Mma<float>::run(acc[q], xf, gf);
      }
    }
  }
  TTMI_TSTAMP(1);
  // lane holds D[d = dtile*16 + 4lg + r][row = r0 + li]
  const int row = r0 + li;
  if constexpr (!FIN) {
    if (row < B) {
      float* pr = part + ((int64_t)split * 2 * B + (int64_t)dir * B + row) * D;
#pragma unroll
      for (int q = 0; q < TPW; ++q)
        *reinterpret_cast<float4*>(pr + (wave + 4 * q) * 16 + 4 * lg) =
            make_float4(acc[q][0], acc[q][1], acc[q][2], acc[q][3]);
    }
    return;
  } else {
    // ---- the finish in the same launch: the last of a row block's NSPLIT workgroups sums the
    // NSPLIT partial rows in split order (the separate finish kernel's order: bit-identical)
    // and runs the normalise backward.  Hand-off (MI355X_MICROARCH.md, valid forms, row 1):
    // every partial byte is stored write-through (sc1, 16 B per lane), every storing wave
    // drains vmcnt before the workgroup barrier, one lane's agent-scope add is the arrival, the
    // last arriver (told by the returned count) reads the partials with sc1 loads only.
    if (row < B) {
      const uint32_t base = (uint32_t)(((int64_t)split * 2 * B + (int64_t)dir * B + row) * D * 4);
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(part, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
      for (int q = 0; q < TPW; ++q) {
        const i32x4_t v = {(int)__float_as_uint(acc[q][0]), (int)__float_as_uint(acc[q][1]),
                           (int)__float_as_uint(acc[q][2]), (int)__float_as_uint(acc[q][3])};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, base + ((wave + 4 * q) * 16 + 4 * lg) * 4, 0, 16);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __shared__ int s_last;
    __syncthreads();
    TTMI_TSTAMP(2);
    if (tid == 0)
      s_last = __hip_atomic_fetch_add(fin.cnt + qb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == NSPLIT - 1;
    __syncthreads();
    TTMI_TSTAMP(3);
    if (!s_last) return;
    if (tid == 0) __hip_atomic_store(fin.cnt + qb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    constexpr int CPL = (D + 63) / 64;               // columns per lane (c = lane + 64q)
    constexpr int RPW = NQ / 4;                      // rows per wave: r0 + wave + 4k
    const float* Y = dir ? ih : uh;
    float* dX = dir ? fin.di : fin.du;
    float pv[RPW][NSPLIT][CPL];                      // every partial load in flight first
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      const int64_t prow = (int64_t)dir * B + min(r0 + wave + 4 * k, B - 1);
#pragma unroll
      for (int sp = 0; sp < NSPLIT; ++sp)
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
          const int c = min(lane + 64 * q, D - 1);
          pv[k][sp][q] = __hip_atomic_load(part + ((int64_t)sp * 2 * B + prow) * D + c, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
        }
    }
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      const int rr = r0 + wave + 4 * k;
      if (rr >= B) break;
      const int64_t prow = (int64_t)dir * B + rr;
      const float nrm = fin.norms[prow];
      float v[CPL], y[CPL];
      float sdot = 0.f;
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        const int c = lane + 64 * q;
        float t = 0.f;
        y[q] = 0.f;
        if (c < D) {
#pragma unroll
          for (int sp = 0; sp < NSPLIT; ++sp) t += pv[k][sp][q];
          t *= fin.inv_tau;
          y[q] = Y[(int64_t)rr * D + c];
          sdot += y[q] * t;
        }
        v[q] = t;
      }
      sdot = wave_sum(sdot);
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        const int c = lane + 64 * q;
        if (c < D) {
          const float g = nrm > NORM_EPS ? (v[q] - y[q] * sdot) / nrm : v[q] / NORM_EPS;
          dX[(int64_t)rr * D + c] = g;
          if (dir == 0 && fin.du16) fin.du16[(int64_t)rr * D + c] = f2bf(g);
        }
      }
    }
    TTMI_TSTAMP(4);
  }
}

// dx = normalize-backward(Σ_split part / τ); wave per row of the 2B rows.
__global__ __launch_bounds__(256) void nce_bwd_finish_kernel(int B, int D, const float* __restrict__ uh,
                                                             const float* __restrict__ ih,
                                                             const float* __restrict__ norms,
                                                             const float* __restrict__ part,
                                                             float inv_tau, float* __restrict__ du,
                                                             float* __restrict__ di,
                                                             bf16_t* __restrict__ du16) {
  const int lane = threadIdx.x & 63;
  const int row = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (row >= 2 * B) return;
  const bool isu = row < B;
  const int r = isu ? row : row - B;
  const float* y = (isu ? uh : ih) + (int64_t)r * D;
  float* dx = (isu ? du : di) + (int64_t)r * D;
  const float nrm = norms[row];
  float dy[4];
  float sdot = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = lane + 64 * q;
    float v = 0.f;
    if (c < D) {
#pragma unroll
      for (int k = 0; k < NSPLIT; ++k) v += part[((int64_t)k * 2 * B + row) * D + c];
      v *= inv_tau;
      sdot += y[c] * v;
    }
    dy[q] = v;
  }
  sdot = wave_sum(sdot);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = lane + 64 * q;
    if (c < D) {
      const float g = nrm > NORM_EPS ? (dy[q] - y[c] * sdot) / nrm : dy[q] / NORM_EPS;
      dx[c] = g;
      if (isu && du16) du16[(int64_t)r * D + c] = f2bf(g);   // the user tower's bf16 operand
    }
  }
}

struct Ws {
  float* dS; float* ce; float* duh; float* dih;
};
Ws carve(void* ws, int B, int D) {
  Ws w;
  char* p = static_cast<char*>(ws);
  auto take = [&](int64_t bytes) { char* q = p; p += (bytes + 255) / 256 * 256; return q; };
  w.dS = (float*)take((int64_t)B * B * 4);
  w.ce = (float*)take((int64_t)2 * B * 4);
  w.duh = (float*)take((int64_t)B * D * 4);
  w.dih = (float*)take((int64_t)B * D * 4);
  return w;
}

ttmi_gemm_desc f32_gemm(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, int ak,
                        const float* Bm, int64_t ldb, int bk, float* C, int64_t ldc, float alpha) {
  ttmi_gemm_desc d = {};
  d.dtype = TTMI_F32;
  d.M = M; d.N = N; d.K = K;
  d.A = A; d.lda = lda; d.a_kmajor = ak;
  d.B = Bm; d.ldb = ldb; d.b_kmajor = bk;
  d.C = C; d.ldc = ldc; d.c_dtype = TTMI_F32; d.c_mode = 0;
  d.alpha = alpha;
  d.split_k = 1;
  return d;
}

}  // namespace

bool fused_ok(int B, int D) { return D % 64 == 0 && D <= 256; }

extern "C" int64_t ttmi_infonce_workspace(int B, int D) {
  auto al = [](int64_t b) { return (b + 255) / 256 * 256; };
  if (fused_ok(B, D))   // fwd partials (3·NSPLIT·2B) + bwd partial rows (NSPLIT·2B·D)
    return al((int64_t)3 * NSPLIT * 2 * B * 4) + al((int64_t)NSPLIT * 2 * B * D * 4);
  // dS [B,B] + ce [2B] + dû', dî' [B,D], each 256-B aligned
  return al((int64_t)B * B * 4) + al((int64_t)2 * B * 4) + 2 * al((int64_t)B * D * 4);
}

namespace {
int infonce_fwd_impl(int B, int D, const float* u, const float* it, const int64_t* user_idx,
                     float inv_tau, float* u_hat, float* i_hat, float* norms, float* logits,
                     float* lse, float* loss, void* ws, bool normalise, int32_t* counters,
                     float* loss_acc, hipStream_t s) {
  TTMI_REQUIRE(B > 0 && D > 0 && D <= 4096 && D % 4 == 0 && (B % 4 == 0 || fused_ok(B, D)),
               "ttmi_infonce_fwd: need D %% 4 == 0, D <= 4096, and B %% 4 == 0 unless D %% 64 == 0 and D <= 256");
  TTMI_REQUIRE((!normalise || (u && it)) && u_hat && i_hat && norms && logits && lse && loss && ws,
               "ttmi_infonce_fwd: null argument");
  int rc = TTMI_OK;
  if (normalise) {
    hipLaunchKernelGGL(l2norm_kernel, dim3((2 * B + 3) / 4), dim3(256), 0, s, B, D, u, it, u_hat, i_hat,
                       norms);
    rc = ttmi_check_launch("ttmi_infonce_fwd/l2norm");
    if (rc) return rc;
  }
  if (fused_ok(B, D)) {
    float* part = static_cast<float*>(ws);
    const int nb = (B + NQ - 1) / NQ;
    const dim3 grid(2 * nb * NSPLIT);
    // per-query-block CE sums of the fused combine: scratch in the backward's partial region
    float* qsum = reinterpret_cast<float*>(static_cast<char*>(ws) + (((int64_t)3 * NSPLIT * 2 * B * 4 + 255) / 256 * 256));
#define TTMI_NCE_FWD(DC, V) hipLaunchKernelGGL((nce_fwd_kernel<DC, V>), grid, dim3(256), 0, s, B, u_hat, i_hat, user_idx, inv_tau, logits, part, counters, qsum, lse, loss, loss_acc)
#define TTMI_NCE_FWD2(DC) do { if (B % 4 == 0) TTMI_NCE_FWD(DC, true); else TTMI_NCE_FWD(DC, false); } while (0)
    switch (D / 16) {
      case 4: TTMI_NCE_FWD2(4); break;
      case 8: TTMI_NCE_FWD2(8); break;
      case 12: TTMI_NCE_FWD2(12); break;
      default: TTMI_NCE_FWD2(16); break;
    }
#undef TTMI_NCE_FWD2
#undef TTMI_NCE_FWD
    rc = ttmi_check_launch("ttmi_infonce_fwd/rows");
    if (rc || counters) return rc;
    hipLaunchKernelGGL(nce_combine_kernel, dim3(1), dim3(1024), 0, s, B, part, lse, loss);
    return ttmi_check_launch("ttmi_infonce_fwd/combine");
  }
  Ws w = carve(ws, B, D);
  ttmi_gemm_desc g = f32_gemm(B, B, D, u_hat, D, 1, i_hat, D, 1, logits, B, inv_tau);
  rc = ttmi_gemm(&g, s);
  if (rc) return rc;
  const int nrb = (B + 3) / 4;
  hipLaunchKernelGGL(lse_kernel, dim3(nrb + (B + LC - 1) / LC), dim3(256), 0, s, B, logits, user_idx,
                     lse, w.ce, nrb);
  rc = ttmi_check_launch("ttmi_infonce_fwd/lse");
  if (rc) return rc;
  hipLaunchKernelGGL(loss_kernel, dim3(1), dim3(256), 0, s, 2 * B, w.ce, 0.5f / (float)B, loss);
  return ttmi_check_launch("ttmi_infonce_fwd/loss");
}
}  // namespace

extern "C" int ttmi_infonce_fwd(int B, int D, const float* u, const float* it,
                                const int64_t* user_idx, float inv_tau, float* u_hat,
                                float* i_hat, float* norms, float* logits, float* lse, float* loss,
                                void* ws, hipStream_t s) {
  return infonce_fwd_impl(B, D, u, it, user_idx, inv_tau, u_hat, i_hat, norms, logits, lse, loss,
                          ws, true, nullptr, nullptr, s);
}

// ttmi_infonce_fwd with the combine inside the logits launch and the loss accumulator (ABI 19):
// the normalise launch + one launch, for callers whose rows are not normalised by their producers
// (the unfused heads, D = 256).
extern "C" int ttmi_infonce_fwd_acc(int B, int D, const float* u, const float* it,
                                    const int64_t* user_idx, float inv_tau, float* u_hat, float* i_hat,
                                    float* norms, float* logits, float* lse, float* loss, void* ws,
                                    int32_t* counters, float* loss_acc, hipStream_t s) {
  TTMI_REQUIRE(counters && ((uintptr_t)counters & 3) == 0 && fused_ok(B, D),
               "ttmi_infonce_fwd_acc: needs 4-byte aligned counters and D %% 64 == 0, D <= 256");
  return infonce_fwd_impl(B, D, u, it, user_idx, inv_tau, u_hat, i_hat, norms, logits, lse, loss,
                          ws, true, counters, loss_acc, s);
}

extern "C" int64_t ttmi_infonce_counter_bytes(int B) {
  return B > 0 ? (int64_t)(2 * ((B + NQ - 1) / NQ) + 1) * 4 : 0;
}

extern "C" int ttmi_infonce_fwd_pre(int B, int D, const int64_t* user_idx, float inv_tau,
                                    const float* u_hat, const float* i_hat, const float* norms,
                                    float* logits, float* lse, float* loss, void* ws,
                                    int32_t* counters, float* loss_acc, hipStream_t s) {
  TTMI_REQUIRE(((uintptr_t)counters & 3) == 0, "ttmi_infonce_fwd_pre: counters need 4-byte alignment");
  TTMI_REQUIRE(!loss_acc || (counters && fused_ok(B, D)), "ttmi_infonce_fwd_pre: loss_acc needs the fused combine");
  return infonce_fwd_impl(B, D, nullptr, nullptr, user_idx, inv_tau, const_cast<float*>(u_hat),
                          const_cast<float*>(i_hat), const_cast<float*>(norms), logits, lse, loss,
                          ws, false, counters, loss_acc, s);
}

extern "C" int ttmi_infonce_bwd16(int B, int D, const float* u_hat, const float* i_hat,
                                  const float* norms, const float* logits, const float* lse,
                                  const int64_t* user_idx, float inv_tau, const float* dloss,
                                  float* du, float* di, uint16_t* du16, void* ws, hipStream_t s);

extern "C" int ttmi_infonce_bwd(int B, int D, const float* u_hat, const float* i_hat,
                                const float* norms, const float* logits, const float* lse,
                                const int64_t* user_idx, float inv_tau, const float* dloss,
                                float* du, float* di, void* ws, hipStream_t s) {
  return ttmi_infonce_bwd16(B, D, u_hat, i_hat, norms, logits, lse, user_idx, inv_tau, dloss, du, di,
                            nullptr, ws, s);
}

extern "C" int ttmi_infonce_bwd16(int B, int D, const float* u_hat, const float* i_hat,
                                  const float* norms, const float* logits, const float* lse,
                                  const int64_t* user_idx, float inv_tau, const float* dloss,
                                  float* du, float* di, uint16_t* du16, void* ws, hipStream_t s) {
  TTMI_REQUIRE(B > 0 && D > 0 && D <= 4096 && D % 4 == 0 && (B % 4 == 0 || fused_ok(B, D)),
               "ttmi_infonce_bwd: need D %% 4 == 0, D <= 4096, and B %% 4 == 0 unless D %% 64 == 0 and D <= 256");
  TTMI_REQUIRE(u_hat && i_hat && norms && logits && lse && du && di && ws,
               "ttmi_infonce_bwd: null argument");
  if (fused_ok(B, D)) {
    float* part = reinterpret_cast<float*>(static_cast<char*>(ws) +
                                           ((int64_t)3 * NSPLIT * 2 * B * 4 + 255) / 256 * 256);
    const int nb = (B + NQ - 1) / NQ;
    const dim3 grid(2 * nb * NSPLIT);
#define TTMI_NCE_BWD(DC, V) hipLaunchKernelGGL((nce_bwd_kernel<DC, V, false>), grid, dim3(256), 0, s, B, u_hat, i_hat, logits, lse, dloss, part, NceFinish{})
#define TTMI_NCE_BWD2(DC) do { if (B % 4 == 0) TTMI_NCE_BWD(DC, true); else TTMI_NCE_BWD(DC, false); } while (0)
    switch (D / 16) {
      case 4: TTMI_NCE_BWD2(4); break;
      case 8: TTMI_NCE_BWD2(8); break;
      case 12: TTMI_NCE_BWD2(12); break;
      default: TTMI_NCE_BWD2(16); break;
    }
#undef TTMI_NCE_BWD2
#undef TTMI_NCE_BWD
    int rc = ttmi_check_launch("ttmi_infonce_bwd/rows");
    if (rc) return rc;
    hipLaunchKernelGGL(nce_bwd_finish_kernel, dim3((2 * B + 3) / 4), dim3(256), 0, s, B, D, u_hat, i_hat,
                       norms, part, inv_tau, du, di, (bf16_t*)du16);
    return ttmi_check_launch("ttmi_infonce_bwd/finish");
  }
  Ws w = carve(ws, B, D);
  const int64_t n = (int64_t)B * B;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(dlogits_kernel, dim3(grid), dim3(256), 0, s, B, logits, lse, user_idx, dloss,
                     0.5f / (float)B, w.dS);
  int rc = ttmi_check_launch("ttmi_infonce_bwd/dlogits");
  if (rc) return rc;
  ttmi_gemm_desc g1 = f32_gemm(B, D, B, w.dS, B, 1, i_hat, D, 0, w.duh, D, inv_tau);
  rc = ttmi_gemm(&g1, s);
  if (rc) return rc;
  ttmi_gemm_desc g2 = f32_gemm(B, D, B, w.dS, B, 0, u_hat, D, 0, w.dih, D, inv_tau);
  rc = ttmi_gemm(&g2, s);
  if (rc) return rc;
  hipLaunchKernelGGL(l2norm_bwd_kernel, dim3((2 * B + 3) / 4), dim3(256), 0, s, B, D, u_hat, i_hat,
                     norms, w.duh, w.dih, du, di);
  rc = ttmi_check_launch("ttmi_infonce_bwd/l2norm_bwd");
  if (rc || !du16) return rc;
  return ttmi_cast_f32_bf16((int64_t)B * D, du, du16, s);
}

extern "C" int64_t ttmi_infonce_bwd_counter_bytes(int B) {
  return B > 0 ? (int64_t)(2 * ((B + NQ - 1) / NQ)) * 4 : 0;
}

extern "C" int ttmi_infonce_bwd_fused(int B, int D, const float* u_hat, const float* i_hat,
                                      const float* norms, const float* logits, const float* lse,
                                      const int64_t* user_idx, float inv_tau, const float* dloss,
                                      float* du, float* di, uint16_t* du16, void* ws, int32_t* counters,
                                      hipStream_t s) {
  if (counters == nullptr || !fused_ok(B, D))
    return ttmi_infonce_bwd16(B, D, u_hat, i_hat, norms, logits, lse, user_idx, inv_tau, dloss, du, di, du16,
                              ws, s);
  TTMI_REQUIRE(B > 0 && u_hat && i_hat && norms && logits && lse && du && di && ws,
               "ttmi_infonce_bwd_fused: null argument");
  TTMI_REQUIRE(((uintptr_t)counters & 3) == 0, "ttmi_infonce_bwd_fused: counters need 4-byte alignment");
  TTMI_REQUIRE((int64_t)NSPLIT * 2 * B * D * 4 < 0x7FFFFFFF, "ttmi_infonce_bwd_fused: batch too large");
  float* part = reinterpret_cast<float*>(static_cast<char*>(ws) +
                                         ((int64_t)3 * NSPLIT * 2 * B * 4 + 255) / 256 * 256);
  TTMI_REQUIRE(((uintptr_t)part & 15) == 0, "ttmi_infonce_bwd_fused: workspace needs 16-byte alignment");
  const int nb = (B + NQ - 1) / NQ;
  const dim3 grid(2 * nb * NSPLIT);
  const NceFinish fin{norms, inv_tau, du, di, (bf16_t*)du16, counters};
#define TTMI_NCE_BWDF(DC, V) hipLaunchKernelGGL((nce_bwd_kernel<DC, V, true>), grid, dim3(256), 0, s, B, u_hat, i_hat, logits, lse, dloss, part, fin)
#define TTMI_NCE_BWDF2(DC) do { if (B % 4 == 0) TTMI_NCE_BWDF(DC, true); else TTMI_NCE_BWDF(DC, false); } while (0)
  switch (D / 16) {
    case 4: TTMI_NCE_BWDF2(4); break;
    case 8: TTMI_NCE_BWDF2(8); break;
    case 12: TTMI_NCE_BWDF2(12); break;
    default: TTMI_NCE_BWDF2(16); break;
  }
#undef TTMI_NCE_BWDF2
#undef TTMI_NCE_BWDF
  return ttmi_check_launch("ttmi_infonce_bwd_fused");
}

// ------------------------------------------------------------ building blocks (cfg 5)
extern "C" int ttmi_l2norm_fwd(int n, int D, const float* x, float* y, float* norms,
                               hipStream_t s) {
  TTMI_REQUIRE(n >= 0 && D > 0, "ttmi_l2norm_fwd: bad sizes");
  if (n == 0) return TTMI_OK;
  TTMI_REQUIRE(x && y && norms, "ttmi_l2norm_fwd: null argument");
  hipLaunchKernelGGL(rows_l2norm_kernel, dim3((n + 3) / 4), dim3(256), 0, s, n, D, x, y, norms);
  return ttmi_check_launch("ttmi_l2norm_fwd");
}

extern "C" int ttmi_l2norm_bwd(int n, int D, const float* y, const float* norms, const float* dy,
                               const float* dy2, float* dx, hipStream_t s) {
  TTMI_REQUIRE(n >= 0 && D > 0, "ttmi_l2norm_bwd: bad sizes");
  if (n == 0) return TTMI_OK;
  TTMI_REQUIRE(y && norms && dy && dx, "ttmi_l2norm_bwd: null argument");
  hipLaunchKernelGGL(rows_l2norm_bwd_kernel, dim3((n + 3) / 4), dim3(256), 0, s, n, D, y, norms, dy,
                     dy2, dx);
  return ttmi_check_launch("ttmi_l2norm_bwd");
}

extern "C" int ttmi_rowce_fwd(int R, int C, int D, const float* q, const float* k,
                              const int64_t* uid_q, const int64_t* uid_k, int64_t row0,
                              float inv_tau, float* logits, float* lse, float* ce, hipStream_t s) {
  TTMI_REQUIRE(R > 0 && C > 0 && D > 0 && D % 4 == 0 && row0 >= 0 && row0 + R <= C,
               "ttmi_rowce_fwd: need D %% 4 == 0 and 0 <= row0, row0 + R <= C");
  TTMI_REQUIRE(q && k && logits && lse && ce, "ttmi_rowce_fwd: null argument");
  TTMI_REQUIRE(C % 4 == 0, "ttmi_rowce_fwd: C must be a multiple of 4");
  ttmi_gemm_desc g = f32_gemm(R, C, D, q, D, 1, k, D, 1, logits, C, inv_tau);
  int rc = ttmi_gemm(&g, s);
  if (rc) return rc;
  hipLaunchKernelGGL(rowce_lse_kernel, dim3((R + 3) / 4), dim3(256), 0, s, R, C, row0, logits, uid_q,
                     uid_k, lse, ce);
  return ttmi_check_launch("ttmi_rowce_fwd");
}

extern "C" int64_t ttmi_rowce_workspace(int R, int C) { return ((int64_t)R * C * 4 + 255) / 256 * 256; }

extern "C" int ttmi_rowce_bwd(int R, int C, int D, const float* q, const float* k,
                              const float* logits, const float* lse, const int64_t* uid_q,
                              const int64_t* uid_k, int64_t row0, float inv_tau,
                              const float* dloss, float scale, float* dq, float* dk, void* ws,
                              hipStream_t s) {
  TTMI_REQUIRE(R > 0 && C > 0 && D > 0 && D % 4 == 0 && C % 4 == 0 && row0 >= 0 && row0 + R <= C,
               "ttmi_rowce_bwd: bad sizes");
  TTMI_REQUIRE(q && k && logits && lse && dq && dk && ws, "ttmi_rowce_bwd: null argument");
  float* dS = static_cast<float*>(ws);
  const int64_t n = (int64_t)R * C;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(rowce_dlogits_kernel, dim3(grid), dim3(256), 0, s, R, C, row0, logits, lse,
                     uid_q, uid_k, dloss, scale, dS);
  int rc = ttmi_check_launch("ttmi_rowce_bwd/dlogits");
  if (rc) return rc;
  ttmi_gemm_desc g1 = f32_gemm(R, D, C, dS, C, 1, k, D, 0, dq, D, inv_tau);   // dq = dS·k
  rc = ttmi_gemm(&g1, s);
  if (rc) return rc;
  ttmi_gemm_desc g2 = f32_gemm(C, D, R, dS, C, 0, q, D, 0, dk, D, inv_tau);   // dk = dSᵀ·q
  return ttmi_gemm(&g2, s);
}

extern "C" int ttmi_sum_scaled(int n, const float* x, float scale, float* out, hipStream_t s) {
  TTMI_REQUIRE(n >= 0 && x && out, "ttmi_sum_scaled: bad argument");
  hipLaunchKernelGGL(loss_kernel, dim3(1), dim3(256), 0, s, n, x, scale, out);
  return ttmi_check_launch("ttmi_sum_scaled");
}

TTMI_STAMP_DUMP(infonce)
