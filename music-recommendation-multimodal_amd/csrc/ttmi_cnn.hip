// ttmi_cnn.hip — ResNet-18 non-GEMM layers over NHWC bf16 activations (torchvision
// resnet18 as used by reference item_tower.py:9-39): BatchNorm2d in train mode (batch
// statistics, running-stat update), residual add + ReLU, max-pool 3x3/2 and the global
// average pool, with their backwards.
//
// BatchNorm2d forward takes the per-channel Σx and Σx² that the producing convolution
// accumulated in its epilogue (ttmi_conv2d FWD; int64 fixed point, so order-independent), so
// it is one element-wise pass:
//   y = act(w·(x − μ)·rstd + b + residual),  μ = Σx/M, var = Σx²/M − μ² (biased),
//   running stats with momentum and the unbiased variance (nn.BatchNorm2d).
// Its backward is a reduction pass (Σg, Σg·x̂ per channel, g = dy ⊙ ReLU gate, optionally
// writing g for the residual branch) and an element-wise pass
//   dx = w·rstd·(g − Σg/M − x̂·Σg x̂/M).
// Element-wise passes move 8 channels (16 bytes) per thread.
#include "ttmi_common.h"

namespace {

constexpr int MAXC = 512;

int grid_for(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096)); }
constexpr int EW_U = 4;     // 16-byte items per thread per trip in the element-wise BN passes
int grid_ew(int64_t n) { return grid_for((n + EW_U - 1) / EW_U); }

// ---------------------------------------------------------------- BatchNorm2d forward
__global__ __launch_bounds__(256) void bn2d_fwd_kernel(int64_t M, int C, const bf16_t* __restrict__ x,
                                                       const int64_t* __restrict__ csum,
                                                       const int64_t* __restrict__ csq,
                                                       const float* __restrict__ w,
                                                       const float* __restrict__ b, float eps,
                                                       float momentum, float* running_mean,
                                                       float* running_var, int64_t* nbt,
                                                       const bf16_t* __restrict__ res, int relu,
                                                       bf16_t* __restrict__ y, float* save_mean,
                                                       float* save_rstd) {
  __shared__ float sa[MAXC], sb[MAXC];      // y = x·sa + sb
  const bool eval = csum == nullptr;        // eval mode: normalise with the running statistics
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    long long q1 = 0, q2 = 0;
    if (!eval)
      for (int r = 0; r < TTMI_CONV_STAT_REPS; ++r) {   // replica rows of the conv epilogue
        q1 += csum[r * C + c];
        q2 += csq[r * C + c];
      }
    // fixed-point sums -> double moments (E[x²] − E[x]² without fp32 cancellation)
    const double dmu = fx_to_d(q1, TTMI_FX_STAT) / (double)M;
    const double dvar = fx_to_d(q2, TTMI_FX_STAT) / (double)M - dmu * dmu;
    const float mu = eval ? running_mean[c] : (float)dmu;
    const float var = eval ? running_var[c] : (float)fmax(dvar, 0.0);
    const float rs = 1.f / sqrtf(var + eps);
    sa[c] = w[c] * rs;
    sb[c] = b[c] - mu * w[c] * rs;
    if (blockIdx.x == 0) {
      save_mean[c] = mu;
      save_rstd[c] = rs;
      if (running_mean && !eval) {
        const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mu;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt && !eval) *nbt += 1;
  __syncthreads();
  const int cpr = C / 8;
  const int64_t n = M * cpr;
  // EW_U 16-byte items per thread per trip, every load issued before any math (one load per
  // trip left the pass latency-bound at ~half the HBM rate)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * EW_U;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x * EW_U + threadIdx.x; i0 < n; i0 += stride) {
    uint4 qx[EW_U], qr[EW_U];
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const int64_t i = min(i0 + (int64_t)u * blockDim.x, n - 1);
      qx[u] = reinterpret_cast<const uint4*>(x)[i];
      qr[u] = res ? reinterpret_cast<const uint4*>(res)[i] : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i >= n) break;
      const int c0 = (int)(i % cpr) * 8;
      float v[8], r[8];
      unpack8(qx[u], v);
      unpack8(qr[u], r);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] = v[e] * sa[c0 + e] + sb[c0 + e] + r[e];
        if (relu) v[e] = fmaxf(v[e], 0.f);
      }
      reinterpret_cast<uint4*>(y)[i] = pack8(v);
    }
  }
}

// ---------------------------------------------------------------- BatchNorm2d backward
// Reduction: sums[r][c] += Σ g, sums[r][C + c] += Σ g·x̂ (g = dy ⊙ (gate > 0) when gate
// given) with r = block % TTMI_CONV_STAT_REPS; g is written (bf16) when gout != NULL.  Block =
// 256 threads over row slabs; per thread 8 channels of strided rows, then an LDS reduction (a
// fixed order) and one int64 fixed-point add (TTMI_FX_GRAD) per channel per block into its
// replica row (spread: no single hot address; order-independent: deterministic).
__global__ __launch_bounds__(256) void bn2d_bwd_reduce_kernel(int64_t M, int C, const bf16_t* __restrict__ dy,
                                                              const bf16_t* __restrict__ gate,
                                                              const bf16_t* __restrict__ x,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ rstd,
                                                              bf16_t* __restrict__ gout,
                                                              int64_t* __restrict__ sums,
                                                              int64_t rows_per_block) {
  __shared__ float red[2][256][8];
  const int cpr = C / 8;
  const int tpr = 256 / cpr > 0 ? 256 / cpr : 1;     // row lanes per block (C <= 2048)
  const int t = threadIdx.x;
  const int cg = t % cpr, rl = t / cpr;
  const int c0 = cg * 8;
  float s1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, s2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float mu[8], rs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { mu[e] = cg < cpr ? mean[c0 + e] : 0.f; rs[e] = cg < cpr ? rstd[c0 + e] : 0.f; }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  if (rl < tpr && cg < cpr) {
    // U rows per step, every load of the step issued before any arithmetic (a thread walks
    // ~25 rows: one dependent memory latency per row made this a latency chain)
    constexpr int U = 4;
    for (int64_t mb = r0 + rl; mb < r1; mb += U * tpr) {
      uint4 qd[U], qg[U], qx[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = min(mb + u * tpr, r1 - 1) * cpr + cg;
        qd[u] = reinterpret_cast<const uint4*>(dy)[i];
        qg[u] = gate ? reinterpret_cast<const uint4*>(gate)[i] : make_uint4(0u, 0u, 0u, 0u);
        qx[u] = reinterpret_cast<const uint4*>(x)[i];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t m = mb + u * tpr;
        if (m >= r1) break;
        const int64_t i = m * cpr + cg;
        float g[8], xv[8];
        unpack8(qd[u], g);
        if (gate) {
          float gv[8];
          unpack8(qg[u], gv);
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] = gv[e] > 0.f ? g[e] : 0.f;
        }
        if (gout) reinterpret_cast<uint4*>(gout)[i] = pack8(g);
        unpack8(qx[u], xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s1[e] += g[e];
          s2[e] += g[e] * (xv[e] - mu[e]) * rs[e];
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][t][e] = s1[e]; red[1][t][e] = s2[e]; }
  __syncthreads();
  if (t < cpr) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < tpr; ++r) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { a[e] += red[0][r * cpr + t][e]; bb[e] += red[1][r * cpr + t][e]; }
    }
    int64_t* rep = sums + (int64_t)(blockIdx.x % TTMI_CONV_STAT_REPS) * 2 * C;   // replica row
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      fx_add(rep + t * 8 + e, a[e], TTMI_FX_GRAD);
      fx_add(rep + C + t * 8 + e, bb[e], TTMI_FX_GRAD);
    }
  }
}

// dx = w·rstd·(g − Σg/M − x̂·Σgx̂/M) (+ addend); block 0 also adds the sums into dw/db.
__global__ __launch_bounds__(256) void bn2d_bwd_apply_kernel(int64_t M, int C, const bf16_t* __restrict__ dy,
                                                             const bf16_t* __restrict__ gate,
                                                             const bf16_t* __restrict__ x,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ w,
                                                             const int64_t* __restrict__ sums,
                                                             bf16_t* __restrict__ dx,
                                                             float* dw, float* db) {
  __shared__ float sk[MAXC], sm1[MAXC], sm2[MAXC], smu[MAXC], srs[MAXC];
  const float invM = 1.f / (float)M;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    long long q1 = 0, q2 = 0;
    for (int r = 0; r < TTMI_CONV_STAT_REPS; ++r) {
      q1 += sums[(int64_t)r * 2 * C + c];
      q2 += sums[(int64_t)r * 2 * C + C + c];
    }
    const float t1 = fx_to_f(q1, TTMI_FX_GRAD), t2 = fx_to_f(q2, TTMI_FX_GRAD);
    sk[c] = w[c] * rstd[c];
    sm1[c] = t1 * invM;
    sm2[c] = t2 * invM;
    smu[c] = mean[c];
    srs[c] = rstd[c];
    if (blockIdx.x == 0) {
      if (db) db[c] += t1;
      if (dw) dw[c] += t2;
    }
  }
  __syncthreads();
  const int cpr = C / 8;
  const int64_t n = M * cpr;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * EW_U;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x * EW_U + threadIdx.x; i0 < n; i0 += stride) {
    uint4 qd[EW_U], qg[EW_U], qx[EW_U];
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const int64_t i = min(i0 + (int64_t)u * blockDim.x, n - 1);
      qd[u] = reinterpret_cast<const uint4*>(dy)[i];
      qg[u] = gate ? reinterpret_cast<const uint4*>(gate)[i] : make_uint4(0u, 0u, 0u, 0u);
      qx[u] = reinterpret_cast<const uint4*>(x)[i];
    }
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i >= n) break;
      const int c0 = (int)(i % cpr) * 8;
      float g[8], xv[8], o[8];
      unpack8(qd[u], g);
      if (gate) {
        float gv[8];
        unpack8(qg[u], gv);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = gv[e] > 0.f ? g[e] : 0.f;
      }
      unpack8(qx[u], xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + e;
        const float xh = (xv[e] - smu[c]) * srs[c];
        o[e] = sk[c] * (g[e] - sm1[c] - xh * sm2[c]);
      }
      reinterpret_cast<uint4*>(dx)[i] = pack8(o);
    }
  }
}

// ---------------------------------------------------------------- pools
// max-pool k x k / s, padding p (-inf), NHWC; idx = window tap of the max (first on ties).
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(int N, int H, int W, int C, int Ho, int Wo, int k,
                                                          int s, int p, const bf16_t* __restrict__ x,
                                                          bf16_t* __restrict__ y, uint8_t* __restrict__ idx) {
  const int cpr = C / 8;
  const int n = N * Ho * Wo * cpr;                    // < 2^31 (host-checked): 32-bit math
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int cg = i % cpr;
    int t = i / cpr;
    const int wo = t % Wo; t /= Wo;
    const int ho = t % Ho;
    const int b = t / Ho;
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
    for (int kh = 0; kh < k; ++kh) {
      const int h = ho * s - p + kh;
      if (h < 0 || h >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int w = wo * s - p + kw;
        if (w < 0 || w >= W) continue;
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(x + (((int64_t)b * H + h) * W + w) * C + cg * 8), v);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > best[e]) { best[e] = v[e]; arg[e] = (uint8_t)(kh * k + kw); }
      }
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(best);
    uint2 a;
    a.x = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) | ((uint32_t)arg[3] << 24);
    a.y = (uint32_t)arg[4] | ((uint32_t)arg[5] << 8) | ((uint32_t)arg[6] << 16) | ((uint32_t)arg[7] << 24);
    reinterpret_cast<uint2*>(idx)[i] = a;
  }
}

// dx[h, w] = Σ over the windows that chose (h, w) of dy (gather form: deterministic).
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(int N, int H, int W, int C, int Ho, int Wo, int k,
                                                          int s, int p, const bf16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ idx,
                                                          bf16_t* __restrict__ dx) {
  const int cpr = C / 8;
  const int n = N * H * W * cpr;                      // < 2^31 (host-checked): 32-bit math
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int cg = i % cpr;
    int t = i / cpr;
    const int w = t % W; t /= W;
    const int h = t % H;
    const int b = t / H;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // windows (ho, wo) with ho*s - p <= h <= ho*s - p + k - 1
    const int ho_lo = max(0, (h + p - k + s) / s), ho_hi = min(Ho - 1, (h + p) / s);
    const int wo_lo = max(0, (w + p - k + s) / s), wo_hi = min(Wo - 1, (w + p) / s);
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      const int kh = h - (ho * s - p);
      if (kh < 0 || kh >= k) continue;
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const int kw = w - (wo * s - p);
        if (kw < 0 || kw >= k) continue;
        const int64_t o = ((((int64_t)b * Ho + ho) * Wo + wo) * cpr + cg);
        const uint2 a = reinterpret_cast<const uint2*>(idx)[o];
        float g[8];
        unpack8(reinterpret_cast<const uint4*>(dy)[o], g);
        const uint8_t tap = (uint8_t)(kh * k + kw);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint8_t ae = (uint8_t)(((e < 4 ? a.x : a.y) >> (8 * (e & 3))) & 0xFF);
          if (ae == tap) acc[e] += g[e];
        }
      }
    }
    reinterpret_cast<uint4*>(dx)[i] = pack8(acc);
  }
}

// y[n, c] = mean over H·W of x[n, :, :, c] (fp32 accumulate; out bf16).  Block per (n, 64-ch).
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(int N, int HW, int C, const bf16_t* __restrict__ x,
                                                          bf16_t* __restrict__ y) {
  __shared__ float red[4][64];
  const int b = blockIdx.x / ((C + 63) / 64), c = (blockIdx.x % ((C + 63) / 64)) * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  float s = 0.f;
  if (c < C)
    for (int p = rl; p < HW; p += 4) s += bf2f(x[((int64_t)b * HW + p) * C + c]);
  red[rl][threadIdx.x & 63] = s;
  __syncthreads();
  if (rl == 0 && c < C) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    y[(int64_t)b * C + c] = f2bf(t / (float)HW);
  }
}

// dx[n, p, c] = dy[n, c] / HW (dy fp32 or bf16), optionally gated by (gate > 0): the ReLU at
// the end of the last block.
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(int N, int HW, int C, const void* __restrict__ dy,
                                                          int dy_f32, const bf16_t* __restrict__ gate,
                                                          bf16_t* __restrict__ dx) {
  const int64_t n = (int64_t)N * HW * C;
  const float inv = 1.f / (float)HW;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int b = (int)(i / ((int64_t)HW * C));
    float g = ld_dyn(dy, (int64_t)b * C + c, dy_f32) * inv;
    if (gate && bf2f(gate[i]) <= 0.f) g = 0.f;
    dx[i] = f2bf(g);
  }
}

// ---------------------------------------------------------------- stem: BN + ReLU + max-pool
// resnet18's conv1 → bn1 → relu → maxpool(3, 2, 1) with the BN output never stored: the
// forward normalises each window element on the fly (a = bf16(relu(x·sa + sb)), the exact
// value bn2d_fwd would store, so the window max and its first-on-ties tap are the unfused
// ones) and writes only the pooled map + taps; the backward gathers the pooled gradient onto
// each conv output (as maxpool_bwd), re-derives the ReLU gate from x, and runs the BN
// backward's two passes on it.  Saves the 4x-larger pre-pool map's write and its re-reads.
struct StemBn {
  float sa[MAXC], sb[MAXC];
};
// sa/sb from the batch statistics (train) or the running ones (eval), as bn2d_fwd_kernel
TTMI_DEV void stem_bn_coeffs(StemBn& s, int64_t M, int C, const int64_t* csum, const int64_t* csq,
                             const float* w, const float* b, float eps, float momentum,
                             float* running_mean, float* running_var, int64_t* nbt, float* save_mean,
                             float* save_rstd) {
  const bool eval = csum == nullptr;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    long long q1 = 0, q2 = 0;
    if (!eval)
      for (int r = 0; r < TTMI_CONV_STAT_REPS; ++r) {
        q1 += csum[r * C + c];
        q2 += csq[r * C + c];
      }
    const double dmu = fx_to_d(q1, TTMI_FX_STAT) / (double)M;
    const double dvar = fx_to_d(q2, TTMI_FX_STAT) / (double)M - dmu * dmu;
    const float mu = eval ? running_mean[c] : (float)dmu;
    const float var = eval ? running_var[c] : (float)fmax(dvar, 0.0);
    const float rs = 1.f / sqrtf(var + eps);
    s.sa[c] = w[c] * rs;
    s.sb[c] = b[c] - mu * w[c] * rs;
    if (blockIdx.x == 0) {
      save_mean[c] = mu;
      save_rstd[c] = rs;
      if (running_mean && !eval) {
        const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mu;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt && !eval) *nbt += 1;
}
// the stored-BN value of 8 channels (bf16-rounded, as bn2d_fwd writes it)
TTMI_DEV void stem_act8(const StemBn& s, int c0, const uint4& q, float* a) {
  float v[8];
  unpack8(q, v);
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = bf2f(f2bf(fmaxf(v[e] * s.sa[c0 + e] + s.sb[c0 + e], 0.f)));
}

__global__ __launch_bounds__(256) void stem_pool_fwd_kernel(int N, int H, int W, int C, int Ho, int Wo,
                                                            const bf16_t* __restrict__ x,
                                                            const int64_t* __restrict__ csum,
                                                            const int64_t* __restrict__ csq,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ b, float eps,
                                                            float momentum, float* running_mean,
                                                            float* running_var, int64_t* nbt,
                                                            bf16_t* __restrict__ y, uint8_t* __restrict__ idx,
                                                            float* save_mean, float* save_rstd) {
  __shared__ StemBn s;
  stem_bn_coeffs(s, (int64_t)N * H * W, C, csum, csq, w, b, eps, momentum, running_mean, running_var, nbt,
                 save_mean, save_rstd);
  __syncthreads();
  const int cpr = C / 8;
  const int n = N * Ho * Wo * cpr;                    // < 2^31 (host-checked)
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int cg = i % cpr;
    int t = i / cpr;
    const int wo = t % Wo; t /= Wo;
    const int ho = t % Ho;
    const int bb = t / Ho;
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
    for (int kh = 0; kh < 3; ++kh) {
      const int h = ho * 2 - 1 + kh;
      if (h < 0 || h >= H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int ww = wo * 2 - 1 + kw;
        if (ww < 0 || ww >= W) continue;
        float v[8];
        stem_act8(s, cg * 8, *reinterpret_cast<const uint4*>(x + (((int64_t)bb * H + h) * W + ww) * C + cg * 8), v);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > best[e]) { best[e] = v[e]; arg[e] = (uint8_t)(kh * 3 + kw); }
      }
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(best);
    uint2 a;
    a.x = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) | ((uint32_t)arg[3] << 24);
    a.y = (uint32_t)arg[4] | ((uint32_t)arg[5] << 8) | ((uint32_t)arg[6] << 16) | ((uint32_t)arg[7] << 24);
    reinterpret_cast<uint2*>(idx)[i] = a;
  }
}

// g (8 channels at conv-output element i) = Σ over the pool windows that chose it of dy,
// zeroed where the recomputed BN+ReLU output is 0; xv = the conv output there.  For the 3/2/1
// pool, input row h lies in window ho = (h+1)/2 (tap kh = h+1−2ho) and, for odd h, also in
// ho − 1: the 2 x 2 candidate windows are loaded unconditionally (clamped, then masked), so a
// row's five loads are independent and in flight together.
TTMI_DEV void stem_grad8(const StemBn& s, int64_t i, int cpr, int H, int W, int Ho, int Wo,
                         const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                         const bf16_t* __restrict__ x, float* g, float* xv) {
  const int cg = (int)(i % cpr);
  int64_t t = i / cpr;
  const int w = (int)(t % W); t /= W;
  const int h = (int)(t % H);
  const int bb = (int)(t / H);
  const uint4 qx = reinterpret_cast<const uint4*>(x)[i];
  const int hh = (h + 1) >> 1, wh = (w + 1) >> 1;
  uint4 qd[2][2];
  uint2 qa[2][2];
  int tap[2][2];
  bool ok[2][2];
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int dw = 0; dw < 2; ++dw) {
      const int ho = hh - dh, wo = wh - dw;
      const int kh = h + 1 - 2 * ho, kw = w + 1 - 2 * wo;
      ok[dh][dw] = ho >= 0 && ho < Ho && wo >= 0 && wo < Wo && kh < 3 && kw < 3;
      const int64_t o = (((int64_t)bb * Ho + min(max(ho, 0), Ho - 1)) * Wo + min(max(wo, 0), Wo - 1)) * cpr + cg;
      qd[dh][dw] = reinterpret_cast<const uint4*>(dy)[o];
      qa[dh][dw] = reinterpret_cast<const uint2*>(idx)[o];
      tap[dh][dw] = kh * 3 + kw;
    }
#pragma unroll
  for (int e = 0; e < 8; ++e) g[e] = 0.f;
  // windows in (ho, wo) ascending order, as maxpool_bwd adds them
#pragma unroll
  for (int dh = 1; dh >= 0; --dh)
#pragma unroll
    for (int dw = 1; dw >= 0; --dw) {
      if (!ok[dh][dw]) continue;
      float d[8];
      unpack8(qd[dh][dw], d);
      const uint2 a = qa[dh][dw];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ae = (int)(((e < 4 ? a.x : a.y) >> (8 * (e & 3))) & 0xFF);
        if (ae == tap[dh][dw]) g[e] += d[e];
      }
    }
  float av[8];
  stem_act8(s, cg * 8, qx, av);
  unpack8(qx, xv);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    g[e] = bf2f(f2bf(g[e]));                          // maxpool_bwd stores dpool in bf16
    if (!(av[e] > 0.f)) g[e] = 0.f;
  }
}

// Even H, W: a thread owns a 2x2 quad of conv-output pixels (2t+dh, 2u+dw) x 8 channels.
// The quad's pixels lie in the pool windows (t or t+1) x (u or u+1) only — row 2t in window
// t (tap 1), row 2t+1 in t (tap 2) and t+1 (tap 0) — so 4 window loads serve 4 pixels (the
// per-pixel gather issued 9 for the same quad).  Sums run in (ho, wo) order as maxpool_bwd's.
template <typename F>
TTMI_DEV void stem_quad_grad(const StemBn& s, int64_t q, int cpr, int H, int W, int Ho, int Wo,
                             const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                             const bf16_t* __restrict__ x, F&& use) {   // use(pix, g[8], xv[8])
  const int cg = (int)(q % cpr);
  int64_t t = q / cpr;
  const int W2 = W >> 1, H2 = H >> 1;
  const int u = (int)(t % W2); t /= W2;
  const int tq = (int)(t % H2);
  const int bb = (int)(t / H2);
  uint4 qx[4], qd[2][2];
  uint2 qa[2][2];
  int64_t pix[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int h = 2 * tq + (p >> 1), w = 2 * u + (p & 1);
    pix[p] = (((int64_t)bb * H + h) * W + w) * cpr + cg;
    qx[p] = reinterpret_cast<const uint4*>(x)[pix[p]];
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2) {
      const int ho = min(tq + a, Ho - 1), wo = min(u + b2, Wo - 1);
      const int64_t o = (((int64_t)bb * Ho + ho) * Wo + wo) * cpr + cg;
      qd[a][b2] = reinterpret_cast<const uint4*>(dy)[o];
      qa[a][b2] = reinterpret_cast<const uint2*>(idx)[o];
    }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int dh = p >> 1, dw = p & 1;
    float g[8], xv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = 0.f;
    // windows of this pixel, ascending: row a = 0 (tap 1 + dh) and, for dh = 1, a = 1 (tap 0)
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      if (a == 1 && (dh == 0 || tq + 1 >= Ho)) continue;
      const int kh = a == 0 ? 1 + dh : 0;
#pragma unroll
      for (int b2 = 0; b2 < 2; ++b2) {
        if (b2 == 1 && (dw == 0 || u + 1 >= Wo)) continue;
        const int kw = b2 == 0 ? 1 + dw : 0;
        const uint8_t tap = (uint8_t)(kh * 3 + kw);
        float d[8];
        unpack8(qd[a][b2], d);
        const uint2 aa = qa[a][b2];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint8_t ae = (uint8_t)(((e < 4 ? aa.x : aa.y) >> (8 * (e & 3))) & 0xFF);
          if (ae == tap) g[e] += d[e];
        }
      }
    }
    float av[8];
    stem_act8(s, cg * 8, qx[p], av);
    unpack8(qx[p], xv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      g[e] = bf2f(f2bf(g[e]));                        // maxpool_bwd stores dpool in bf16
      if (!(av[e] > 0.f)) g[e] = 0.f;
    }
    use(pix[p], g, xv);
  }
}

TTMI_DEV void stem_coeffs_bwd(StemBn& s, int C, const float* mean, const float* rstd, const float* w,
                              const float* b) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float mu = mean[c], rs = rstd[c];
    s.sa[c] = w[c] * rs;
    s.sb[c] = b[c] - mu * w[c] * rs;
  }
}

__global__ __launch_bounds__(256) void stem_pool_bwd_reduce_kernel(int N, int H, int W, int C, int Ho, int Wo,
                                                                   const bf16_t* __restrict__ dy,
                                                                   const uint8_t* __restrict__ idx,
                                                                   const bf16_t* __restrict__ x,
                                                                   const float* __restrict__ mean,
                                                                   const float* __restrict__ rstd,
                                                                   const float* __restrict__ w,
                                                                   const float* __restrict__ b,
                                                                   int64_t* __restrict__ sums,
                                                                   int64_t rows_per_block) {
  __shared__ StemBn s;
  __shared__ float red[2][256][8];
  stem_coeffs_bwd(s, C, mean, rstd, w, b);
  __syncthreads();
  const int64_t M = (int64_t)N * H * W;
  const int cpr = C / 8;
  const int tpr = 256 / cpr > 0 ? 256 / cpr : 1;
  const int t = threadIdx.x;
  const int cg = t % cpr, rl = t / cpr;
  const int c0 = cg * 8;
  float s1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, s2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float mu[8], rs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { mu[e] = cg < cpr ? mean[c0 + e] : 0.f; rs[e] = cg < cpr ? rstd[c0 + e] : 0.f; }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  if (rl < tpr && cg < cpr) {
#pragma unroll 2
    for (int64_t m = r0 + rl; m < r1; m += tpr) {
      float g[8], xv[8];
      stem_grad8(s, m * cpr + cg, cpr, H, W, Ho, Wo, dy, idx, x, g, xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += g[e];
        s2[e] += g[e] * (xv[e] - mu[e]) * rs[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][t][e] = s1[e]; red[1][t][e] = s2[e]; }
  __syncthreads();
  if (t < cpr) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < tpr; ++r) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { a[e] += red[0][r * cpr + t][e]; bb[e] += red[1][r * cpr + t][e]; }
    }
    int64_t* rep = sums + (int64_t)(blockIdx.x % TTMI_CONV_STAT_REPS) * 2 * C;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      fx_add(rep + t * 8 + e, a[e], TTMI_FX_GRAD);
      fx_add(rep + C + t * 8 + e, bb[e], TTMI_FX_GRAD);
    }
  }
}

__global__ __launch_bounds__(256) void stem_pool_bwd_apply_kernel(int N, int H, int W, int C, int Ho, int Wo,
                                                                  const bf16_t* __restrict__ dy,
                                                                  const uint8_t* __restrict__ idx,
                                                                  const bf16_t* __restrict__ x,
                                                                  const float* __restrict__ mean,
                                                                  const float* __restrict__ rstd,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ b,
                                                                  const int64_t* __restrict__ sums,
                                                                  bf16_t* __restrict__ dx, float* dw, float* db) {
  __shared__ StemBn s;
  __shared__ float sk[MAXC], sm1[MAXC], sm2[MAXC], smu[MAXC], srs[MAXC];
  const int64_t M = (int64_t)N * H * W;
  const float invM = 1.f / (float)M;
  stem_coeffs_bwd(s, C, mean, rstd, w, b);
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    long long q1 = 0, q2 = 0;
    for (int r = 0; r < TTMI_CONV_STAT_REPS; ++r) {
      q1 += sums[(int64_t)r * 2 * C + c];
      q2 += sums[(int64_t)r * 2 * C + C + c];
    }
    const float t1 = fx_to_f(q1, TTMI_FX_GRAD), t2 = fx_to_f(q2, TTMI_FX_GRAD);
    sk[c] = w[c] * rstd[c];
    sm1[c] = t1 * invM;
    sm2[c] = t2 * invM;
    smu[c] = mean[c];
    srs[c] = rstd[c];
    if (blockIdx.x == 0) {
      if (db) db[c] += t1;
      if (dw) dw[c] += t2;
    }
  }
  __syncthreads();
  const int cpr = C / 8;
  const int64_t n = M * cpr;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cpr) * 8;
    float g[8], xv[8], o[8];
    stem_grad8(s, i, cpr, H, W, Ho, Wo, dy, idx, x, g, xv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c0 + e;
      const float xh = (xv[e] - smu[c]) * srs[c];
      o[e] = sk[c] * (g[e] - sm1[c] - xh * sm2[c]);
    }
    reinterpret_cast<uint4*>(dx)[i] = pack8(o);
  }
}

__global__ __launch_bounds__(256) void stem_quad_bwd_reduce_kernel(int N, int H, int W, int C, int Ho, int Wo,
                                                                   const bf16_t* __restrict__ dy,
                                                                   const uint8_t* __restrict__ idx,
                                                                   const bf16_t* __restrict__ x,
                                                                   const float* __restrict__ mean,
                                                                   const float* __restrict__ rstd,
                                                                   const float* __restrict__ w,
                                                                   const float* __restrict__ b,
                                                                   int64_t* __restrict__ sums,
                                                                   int64_t quads_per_block) {
  __shared__ StemBn s;
  __shared__ float red[2][256][8];
  stem_coeffs_bwd(s, C, mean, rstd, w, b);
  __syncthreads();
  const int64_t NQ = (int64_t)N * (H / 2) * (W / 2);
  const int cpr = C / 8;
  const int tpr = 256 / cpr > 0 ? 256 / cpr : 1;
  const int t = threadIdx.x;
  const int cg = t % cpr, rl = t / cpr;
  const int c0 = cg * 8;
  float s1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, s2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float mu[8], rs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { mu[e] = cg < cpr ? mean[c0 + e] : 0.f; rs[e] = cg < cpr ? rstd[c0 + e] : 0.f; }
  const int64_t q0 = (int64_t)blockIdx.x * quads_per_block, q1 = min(NQ, q0 + quads_per_block);
  if (rl < tpr && cg < cpr) {
    for (int64_t qq = q0 + rl; qq < q1; qq += tpr) {
      stem_quad_grad(s, qq * cpr + cg, cpr, H, W, Ho, Wo, dy, idx, x,
                     [&](int64_t, const float* g, const float* xv) {
#pragma unroll
                       for (int e = 0; e < 8; ++e) {
                         s1[e] += g[e];
                         s2[e] += g[e] * (xv[e] - mu[e]) * rs[e];
                       }
                     });
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][t][e] = s1[e]; red[1][t][e] = s2[e]; }
  __syncthreads();
  if (t < cpr) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < tpr; ++r) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { a[e] += red[0][r * cpr + t][e]; bb[e] += red[1][r * cpr + t][e]; }
    }
    int64_t* rep = sums + (int64_t)(blockIdx.x % TTMI_CONV_STAT_REPS) * 2 * C;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      fx_add(rep + t * 8 + e, a[e], TTMI_FX_GRAD);
      fx_add(rep + C + t * 8 + e, bb[e], TTMI_FX_GRAD);
    }
  }
}

__global__ __launch_bounds__(256) void stem_quad_bwd_apply_kernel(int N, int H, int W, int C, int Ho, int Wo,
                                                                  const bf16_t* __restrict__ dy,
                                                                  const uint8_t* __restrict__ idx,
                                                                  const bf16_t* __restrict__ x,
                                                                  const float* __restrict__ mean,
                                                                  const float* __restrict__ rstd,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ b,
                                                                  const int64_t* __restrict__ sums,
                                                                  bf16_t* __restrict__ dx, float* dw, float* db) {
  __shared__ StemBn s;
  __shared__ float sk[MAXC], sm1[MAXC], sm2[MAXC], smu[MAXC], srs[MAXC];
  const int64_t M = (int64_t)N * H * W;
  const float invM = 1.f / (float)M;
  stem_coeffs_bwd(s, C, mean, rstd, w, b);
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    long long q1 = 0, q2 = 0;
    for (int r = 0; r < TTMI_CONV_STAT_REPS; ++r) {
      q1 += sums[(int64_t)r * 2 * C + c];
      q2 += sums[(int64_t)r * 2 * C + C + c];
    }
    const float t1 = fx_to_f(q1, TTMI_FX_GRAD), t2 = fx_to_f(q2, TTMI_FX_GRAD);
    sk[c] = w[c] * rstd[c];
    sm1[c] = t1 * invM;
    sm2[c] = t2 * invM;
    smu[c] = mean[c];
    srs[c] = rstd[c];
    if (blockIdx.x == 0) {
      if (db) db[c] += t1;
      if (dw) dw[c] += t2;
    }
  }
  __syncthreads();
  const int cpr = C / 8;
  const int64_t n = (int64_t)N * (H / 2) * (W / 2) * cpr;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cpr) * 8;
    stem_quad_grad(s, i, cpr, H, W, Ho, Wo, dy, idx, x, [&](int64_t pix, const float* g, const float* xv) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + e;
        const float xh = (xv[e] - smu[c]) * srs[c];
        o[e] = sk[c] * (g[e] - sm1[c] - xh * sm2[c]);
      }
      reinterpret_cast<uint4*>(dx)[pix] = pack8(o);
    });
  }
}

}  // namespace

extern "C" int ttmi_bn2d_fwd(int64_t M, int C, const uint16_t* x, const int64_t* colsum,
                             const int64_t* colsumsq, const float* w, const float* b, float eps,
                             float momentum, float* running_mean, float* running_var,
                             int64_t* num_batches_tracked, const uint16_t* residual, int relu,
                             uint16_t* y, float* save_mean, float* save_rstd, hipStream_t s) {
  TTMI_REQUIRE(M > 0 && C > 0 && C % 8 == 0 && C <= MAXC, "ttmi_bn2d_fwd: need 0 < C <= %d, C %% 8 == 0", MAXC);
  TTMI_REQUIRE(x && w && b && y && save_mean && save_rstd, "ttmi_bn2d_fwd: null argument");
  TTMI_REQUIRE(!running_mean == !running_var, "ttmi_bn2d_fwd: running_mean/var go together");
  TTMI_REQUIRE(!colsum == !colsumsq, "ttmi_bn2d_fwd: colsum/colsumsq go together");
  TTMI_REQUIRE(colsum || running_mean, "ttmi_bn2d_fwd: eval mode (no colsum) needs running stats");
  hipLaunchKernelGGL(bn2d_fwd_kernel, dim3(grid_ew(M * C / 8)), dim3(256), 0, s, M, C, (const bf16_t*)x,
                     colsum, colsumsq, w, b, eps, momentum, running_mean, running_var,
                     num_batches_tracked, (const bf16_t*)residual, relu, (bf16_t*)y, save_mean, save_rstd);
  return ttmi_check_launch("ttmi_bn2d_fwd");
}

extern "C" int ttmi_bn2d_bwd_reduce(int64_t M, int C, const uint16_t* dy, const uint16_t* gate,
                                    const uint16_t* x, const float* mean, const float* rstd, int64_t* sums,
                                    uint16_t* g_out, hipStream_t s) {
  TTMI_REQUIRE(M > 0 && C > 0 && C % 8 == 0 && C <= MAXC, "ttmi_bn2d_bwd_reduce: need 0 < C <= %d, C %% 8 == 0",
               MAXC);
  TTMI_REQUIRE(dy && x && mean && rstd && sums, "ttmi_bn2d_bwd_reduce: null argument");
  const int cpr = C / 8;
  const int tpr = std::max(1, 256 / cpr);
  int64_t blocks = std::min<int64_t>(1024, (M + tpr * 8 - 1) / (tpr * 8));
  blocks = std::max<int64_t>(blocks, 1);
  const int64_t rpb = (M + blocks - 1) / blocks;
  hipLaunchKernelGGL(bn2d_bwd_reduce_kernel, dim3((unsigned)((M + rpb - 1) / rpb)), dim3(256), 0, s, M, C,
                     (const bf16_t*)dy, (const bf16_t*)gate, (const bf16_t*)x, mean, rstd, (bf16_t*)g_out,
                     sums, rpb);
  return ttmi_check_launch("ttmi_bn2d_bwd_reduce");
}

extern "C" int ttmi_bn2d_bwd_apply(int64_t M, int C, const uint16_t* dy, const uint16_t* gate,
                                   const uint16_t* x, const float* mean, const float* rstd, const float* w,
                                   const int64_t* sums, uint16_t* dx, float* dw, float* db, hipStream_t s) {
  TTMI_REQUIRE(M > 0 && C > 0 && C % 8 == 0 && C <= MAXC, "ttmi_bn2d_bwd_apply: need 0 < C <= %d, C %% 8 == 0",
               MAXC);
  TTMI_REQUIRE(dy && x && mean && rstd && w && sums && dx, "ttmi_bn2d_bwd_apply: null argument");
  hipLaunchKernelGGL(bn2d_bwd_apply_kernel, dim3(grid_ew(M * C / 8)), dim3(256), 0, s, M, C,
                     (const bf16_t*)dy, (const bf16_t*)gate, (const bf16_t*)x, mean, rstd, w, sums,
                     (bf16_t*)dx, dw, db);
  return ttmi_check_launch("ttmi_bn2d_bwd_apply");
}

extern "C" int ttmi_bn2d_bwd(int64_t M, int C, const uint16_t* dy, const uint16_t* gate,
                             const uint16_t* x, const float* mean, const float* rstd,
                             const float* w, int64_t* sums, uint16_t* g_out, uint16_t* dx,
                             float* dw, float* db, hipStream_t s) {
  TTMI_REQUIRE(dy && x && mean && rstd && w && sums && dx, "ttmi_bn2d_bwd: null argument");
  int rc = ttmi_bn2d_bwd_reduce(M, C, dy, gate, x, mean, rstd, sums, g_out, s);
  if (rc) return rc;
  return ttmi_bn2d_bwd_apply(M, C, dy, gate, x, mean, rstd, w, sums, dx, dw, db, s);
}

extern "C" int ttmi_maxpool_fwd(int N, int H, int W, int C, int k, int stride, int pad,
                                const uint16_t* x, uint16_t* y, uint8_t* idx, hipStream_t s) {
  TTMI_REQUIRE(N >= 0 && H > 0 && W > 0 && C > 0 && C % 8 == 0 && k > 0 && k * k <= 255 && stride > 0 &&
                   pad >= 0 && pad < k, "ttmi_maxpool_fwd: bad shape");
  TTMI_REQUIRE(x && y && idx, "ttmi_maxpool_fwd: null argument");
  const int Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  if (N == 0) return TTMI_OK;
  TTMI_REQUIRE((int64_t)N * H * W * C < (1ll << 31), "ttmi_maxpool_fwd: tensor too large");
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for((int64_t)N * Ho * Wo * C / 8)), dim3(256), 0, s, N, H,
                     W, C, Ho, Wo, k, stride, pad, (const bf16_t*)x, (bf16_t*)y, idx);
  return ttmi_check_launch("ttmi_maxpool_fwd");
}

extern "C" int ttmi_maxpool_bwd(int N, int H, int W, int C, int k, int stride, int pad,
                                const uint16_t* dy, const uint8_t* idx, uint16_t* dx, hipStream_t s) {
  TTMI_REQUIRE(N >= 0 && H > 0 && W > 0 && C > 0 && C % 8 == 0 && k > 0 && stride > 0 && pad >= 0,
               "ttmi_maxpool_bwd: bad shape");
  TTMI_REQUIRE(dy && idx && dx, "ttmi_maxpool_bwd: null argument");
  const int Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  if (N == 0) return TTMI_OK;
  TTMI_REQUIRE((int64_t)N * H * W * C < (1ll << 31), "ttmi_maxpool_bwd: tensor too large");
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for((int64_t)N * H * W * C / 8)), dim3(256), 0, s, N, H, W,
                     C, Ho, Wo, k, stride, pad, (const bf16_t*)dy, idx, (bf16_t*)dx);
  return ttmi_check_launch("ttmi_maxpool_bwd");
}

extern "C" int ttmi_avgpool_fwd(int N, int HW, int C, const uint16_t* x, uint16_t* y, hipStream_t s) {
  TTMI_REQUIRE(N >= 0 && HW > 0 && C > 0, "ttmi_avgpool_fwd: bad shape");
  TTMI_REQUIRE(x && y, "ttmi_avgpool_fwd: null argument");
  if (N == 0) return TTMI_OK;
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(N * ((C + 63) / 64)), dim3(256), 0, s, N, HW, C, (const bf16_t*)x,
                     (bf16_t*)y);
  return ttmi_check_launch("ttmi_avgpool_fwd");
}

extern "C" int ttmi_avgpool_bwd(int N, int HW, int C, const void* dy, int dy_dtype, const uint16_t* gate,
                                uint16_t* dx, hipStream_t s) {
  TTMI_REQUIRE(N >= 0 && HW > 0 && C > 0, "ttmi_avgpool_bwd: bad shape");
  TTMI_REQUIRE(dy && dx, "ttmi_avgpool_bwd: null argument");
  if (N == 0) return TTMI_OK;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for((int64_t)N * HW * C)), dim3(256), 0, s, N, HW, C, dy,
                     dy_dtype == TTMI_F32, (const bf16_t*)gate, (bf16_t*)dx);
  return ttmi_check_launch("ttmi_avgpool_bwd");
}

extern "C" int ttmi_stem_pool_fwd(int N, int H, int W, int C, const uint16_t* x, const int64_t* colsum,
                                  const int64_t* colsumsq, const float* w, const float* b, float eps,
                                  float momentum, float* running_mean, float* running_var,
                                  int64_t* num_batches_tracked, uint16_t* y, uint8_t* idx, float* save_mean,
                                  float* save_rstd, hipStream_t s) {
  TTMI_REQUIRE(N > 0 && H > 0 && W > 0 && C > 0 && C % 8 == 0 && C <= MAXC,
               "ttmi_stem_pool_fwd: need 0 < C <= %d, C %% 8 == 0", MAXC);
  TTMI_REQUIRE(x && w && b && y && idx && save_mean && save_rstd, "ttmi_stem_pool_fwd: null argument");
  TTMI_REQUIRE(!running_mean == !running_var, "ttmi_stem_pool_fwd: running_mean/var go together");
  TTMI_REQUIRE(!colsum == !colsumsq, "ttmi_stem_pool_fwd: colsum/colsumsq go together");
  TTMI_REQUIRE(colsum || running_mean, "ttmi_stem_pool_fwd: eval mode (no colsum) needs running stats");
  TTMI_REQUIRE((int64_t)N * H * W * C < (1ll << 31), "ttmi_stem_pool_fwd: tensor too large");
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  hipLaunchKernelGGL(stem_pool_fwd_kernel, dim3(grid_for((int64_t)N * Ho * Wo * C / 8)), dim3(256), 0, s, N, H,
                     W, C, Ho, Wo, (const bf16_t*)x, colsum, colsumsq, w, b, eps, momentum, running_mean,
                     running_var, num_batches_tracked, (bf16_t*)y, idx, save_mean, save_rstd);
  return ttmi_check_launch("ttmi_stem_pool_fwd");
}

extern "C" int ttmi_stem_pool_bwd(int N, int H, int W, int C, const uint16_t* dy, const uint8_t* idx,
                                  const uint16_t* x, const float* mean, const float* rstd, const float* w,
                                  const float* b, int64_t* sums, uint16_t* dx, float* dw, float* db,
                                  hipStream_t s) {
  TTMI_REQUIRE(N > 0 && H > 0 && W > 0 && C > 0 && C % 8 == 0 && C <= MAXC,
               "ttmi_stem_pool_bwd: need 0 < C <= %d, C %% 8 == 0", MAXC);
  TTMI_REQUIRE(dy && idx && x && mean && rstd && w && b && sums && dx, "ttmi_stem_pool_bwd: null argument");
  TTMI_REQUIRE((int64_t)N * H * W * C < (1ll << 31), "ttmi_stem_pool_bwd: tensor too large");
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  const int64_t M = (int64_t)N * H * W;
  const int cpr = C / 8;
  const int tpr = std::max(1, 256 / cpr);
  if (H % 2 == 0 && W % 2 == 0) {                   // 2x2 quads per thread
    const int64_t NQ = M / 4;
    int64_t qb = std::min<int64_t>(8192, (NQ + tpr - 1) / tpr);
    qb = std::max<int64_t>(qb, 1);
    const int64_t qpb = (NQ + qb - 1) / qb;
    hipLaunchKernelGGL(stem_quad_bwd_reduce_kernel, dim3((unsigned)((NQ + qpb - 1) / qpb)), dim3(256), 0, s, N, H,
                       W, C, Ho, Wo, (const bf16_t*)dy, idx, (const bf16_t*)x, mean, rstd, w, b, sums, qpb);
    int rc = ttmi_check_launch("ttmi_stem_pool_bwd/reduce");
    if (rc) return rc;
    hipLaunchKernelGGL(stem_quad_bwd_apply_kernel, dim3(grid_for(NQ * C / 8)), dim3(256), 0, s, N, H, W, C, Ho,
                       Wo, (const bf16_t*)dy, idx, (const bf16_t*)x, mean, rstd, w, b, sums, (bf16_t*)dx, dw, db);
    return ttmi_check_launch("ttmi_stem_pool_bwd/apply");
  }
  int64_t blocks = std::min<int64_t>(8192, (M + tpr * 4 - 1) / (tpr * 4));
  blocks = std::max<int64_t>(blocks, 1);
  const int64_t rpb = (M + blocks - 1) / blocks;
  hipLaunchKernelGGL(stem_pool_bwd_reduce_kernel, dim3((unsigned)((M + rpb - 1) / rpb)), dim3(256), 0, s, N, H, W,
                     C, Ho, Wo, (const bf16_t*)dy, idx, (const bf16_t*)x, mean, rstd, w, b, sums, rpb);
  int rc = ttmi_check_launch("ttmi_stem_pool_bwd/reduce");
  if (rc) return rc;
  hipLaunchKernelGGL(stem_pool_bwd_apply_kernel, dim3(grid_for(M * C / 8)), dim3(256), 0, s, N, H, W, C, Ho, Wo,
                     (const bf16_t*)dy, idx, (const bf16_t*)x, mean, rstd, w, b, sums, (bf16_t*)dx, dw, db);
  return ttmi_check_launch("ttmi_stem_pool_bwd/apply");
}
