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

extern "C" int64_t ttmi_infonce_workspace(int B, int D) {
  // dS [B,B] + ce [2B] + dû', dî' [B,D], each 256-B aligned
  return ((int64_t)B * B * 4 + 255) / 256 * 256 + ((int64_t)2 * B * 4 + 255) / 256 * 256 +
         2 * (((int64_t)B * D * 4 + 255) / 256 * 256);
}

extern "C" int ttmi_infonce_fwd(int B, int D, const float* u, const float* it,
                                const int64_t* user_idx, float inv_tau, float* u_hat,
                                float* i_hat, float* norms, float* logits, float* lse, float* loss,
                                void* ws, hipStream_t s) {
  TTMI_REQUIRE(B > 0 && D > 0 && D <= 4096 && D % 4 == 0 && B % 4 == 0,
               "ttmi_infonce_fwd: need B %% 4 == 0, D %% 4 == 0, D <= 4096");
  TTMI_REQUIRE(u && it && u_hat && i_hat && norms && logits && lse && loss && ws,
               "ttmi_infonce_fwd: null argument");
  Ws w = carve(ws, B, D);
  hipLaunchKernelGGL(l2norm_kernel, dim3((2 * B + 3) / 4), dim3(256), 0, s, B, D, u, it, u_hat, i_hat,
                     norms);
  int rc = ttmi_check_launch("ttmi_infonce_fwd/l2norm");
  if (rc) return rc;
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

extern "C" int ttmi_infonce_bwd(int B, int D, const float* u_hat, const float* i_hat,
                                const float* norms, const float* logits, const float* lse,
                                const int64_t* user_idx, float inv_tau, const float* dloss,
                                float* du, float* di, void* ws, hipStream_t s) {
  TTMI_REQUIRE(B > 0 && D > 0 && D <= 4096 && D % 4 == 0 && B % 4 == 0,
               "ttmi_infonce_bwd: need B %% 4 == 0, D %% 4 == 0, D <= 4096");
  TTMI_REQUIRE(u_hat && i_hat && norms && logits && lse && du && di && ws,
               "ttmi_infonce_bwd: null argument");
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
  return ttmi_check_launch("ttmi_infonce_bwd/l2norm_bwd");
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
