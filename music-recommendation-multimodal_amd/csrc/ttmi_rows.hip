// ttmi_rows.hip — last-layer pruning primitives.
//
// The user tower consumes ONE token per sequence from the last encoder layer (the
// last-valid gather, reference user_tower.py:118-132), and nothing after the last layer's
// attention mixes tokens.  So the last layer only needs K/V for every token and everything
// else (Q, attention output, out_proj, FFN, both residuals) for the gathered token:
//   ttmi_last_rows      rows[b] = b*L + max(len_b - 1, 0)
//   ttmi_gather_rows    out[b] = x[rows[b]]
//   ttmi_scatter_add_rows dst[rows[b]] += src[b]
//   ttmi_mha_q1_fwd/bwd single-query causal attention for the gathered row of each sequence
// Dropout masks keep the full-tensor flat indices (row-mapped), so the pruned layer draws
// exactly the masks the unpruned layer would: outputs and gradients are identical.
#include "ttmi_common.h"

namespace {

__global__ void last_rows_kernel(int B, int L, const int64_t* __restrict__ len_src,
                                 int32_t* __restrict__ rows) {
  const int lane = threadIdx.x & 63;
  const int b = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (b >= B) return;
  float cnt = 0.f;
  for (int l = lane; l < L; l += 64) cnt += len_src[(int64_t)b * L + l] != 0 ? 1.f : 0.f;
  const int len = (int)(wave_sum(cnt) + 0.5f);
  if (lane == 0) rows[b] = (int32_t)((int64_t)b * L + max(len - 1, 0));
}

// last_rows + gather_rows in one launch: wave per sequence counts its valid positions, then
// copies that row (16-byte lanes when D % 4 == 0).
__global__ void last_rows_gather_kernel(int B, int L, int D, const int64_t* __restrict__ len_src,
                                        const float* __restrict__ x, int32_t* __restrict__ rows,
                                        float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int b = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (b >= B) return;
  float cnt = 0.f;
  for (int l = lane; l < L; l += 64) cnt += len_src[(int64_t)b * L + l] != 0 ? 1.f : 0.f;
  const int len = (int)(wave_sum(cnt) + 0.5f);
  const int64_t r = (int64_t)b * L + max(len - 1, 0);
  if (lane == 0) rows[b] = (int32_t)r;
  if (D % 4 == 0) {
    for (int c = lane * 4; c < D; c += 256)
      *reinterpret_cast<float4*>(out + (int64_t)b * D + c) = *reinterpret_cast<const float4*>(x + r * D + c);
  } else {
    for (int c = lane; c < D; c += 64) out[(int64_t)b * D + c] = x[r * D + c];
  }
}

__global__ void gather_rows_kernel(int B, int D, const float* __restrict__ x,
                                   const int32_t* __restrict__ rows, float* __restrict__ out) {
  const int b = blockIdx.x;
  const int64_t r = rows[b];
  for (int c = threadIdx.x; c < D; c += blockDim.x) out[(int64_t)b * D + c] = x[r * D + c];
}

__global__ void scatter_add_rows_kernel(int B, int D, const float* __restrict__ src,
                                        const int32_t* __restrict__ rows, float* __restrict__ dst) {
  const int b = blockIdx.x;
  const int64_t r = rows[b];
  for (int c = threadIdx.x; c < D; c += blockDim.x) dst[r * D + c] += src[(int64_t)b * D + c];
}

// Dot product of an LDS fp32 vector with a global row of Dh (multiple of 8 for bf16 / 4 for
// f32) elements, loaded 16 bytes at a time.
template <typename T>
TTMI_DEV float dot_row(const float* __restrict__ v, const T* __restrict__ row, int Dh) {
  constexpr int E = 16 / sizeof(T);
  float acc = 0.f;
  for (int d0 = 0; d0 < Dh; d0 += E) {
    const uint4 q = *reinterpret_cast<const uint4*>(row + d0);
    const T* e = reinterpret_cast<const T*>(&q);
#pragma unroll
    for (int k = 0; k < E; ++k) acc += v[d0 + k] * ldf<T>(e, k);
  }
  return acc;
}

// 16-byte vector of E = 16 / sizeof(T) elements from fp32 values.
template <typename T>
TTMI_DEV void st16(T* p, const float* v) {
  constexpr int E = 16 / sizeof(T);
  T tmp[E];
#pragma unroll
  for (int i = 0; i < E; ++i) stf<T>(tmp, i, v[i]);
  *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(tmp);
}

// Row-vector lane layout of one wave over [rows][Dh]: lane = (row group, 16-byte chunk).
template <typename T>
struct RowLanes {
  static constexpr int E = 16 / sizeof(T);
  int lpr, ngrp, grp, cv;
  TTMI_DEV explicit RowLanes(int Dh) {
    lpr = Dh / E;
    ngrp = 64 / lpr;
    grp = (int)threadIdx.x / lpr;
    cv = (int)threadIdx.x % lpr;
  }
  TTMI_DEV bool active() const { return grp < ngrp; }
};

// out[t] = Σ_{k<n} coef[k]·rows[k][t] for lane t < Dh: lanes split over (row group, 16-byte
// chunk) so each lane issues ceil(n / groups) independent 16-byte loads; partials meet in LDS
// (red: 64·E floats).
template <typename T>
TTMI_DEV float rows_combine(const float* coef, const T* __restrict__ base, int64_t ld, int n,
                            int Dh, float* red) {
  constexpr int E = RowLanes<T>::E;
  const RowLanes<T> rl(Dh);
  float acc[E];
#pragma unroll
  for (int i = 0; i < E; ++i) acc[i] = 0.f;
  if (rl.active()) {
    for (int k = rl.grp; k < n; k += rl.ngrp) {
      const uint4 q = *reinterpret_cast<const uint4*>(base + (int64_t)k * ld + rl.cv * E);
      const T* e = reinterpret_cast<const T*>(&q);
      const float c = coef[k];
#pragma unroll
      for (int i = 0; i < E; ++i) acc[i] += c * ldf<T>(e, i);
    }
#pragma unroll
    for (int i = 0; i < E; ++i) red[rl.grp * Dh + rl.cv * E + i] = acc[i];
  }
  __syncthreads();
  const int t = threadIdx.x;
  float s = 0.f;
  if (t < Dh)
    for (int g = 0; g < rl.ngrp; ++g) s += red[g * Dh + t];
  return s;
}

// One 64-lane wave per (b, h), XCD-contiguous so the H heads of a sequence share an L2;
// lane j owns key j (L <= 64) for the score/softmax phase; lanes own (row group, 16-byte
// chunk) pairs for the P·V / dS·K reductions and the row stores.
// GATHER: the wave also finds the sequence's last valid row itself (rows[b] = b·L +
// max(len - 1, 0), len = the count of non-zero key_valid entries: the right-padding convention
// of last_rows_gather_kernel) and the head-0 wave writes rows[b] and x_rows[b] = x[rows[b]]
// (the pruned layer's residual rows), so no separate gather launch precedes it.
template <typename T, bool GATHER>
__global__ __launch_bounds__(64) void mha_q1_fwd_kernel(int B, int L, int H, int Dh,
                                                        const T* __restrict__ qkv,
                                                        const int64_t* __restrict__ kvalid,
                                                        int32_t* __restrict__ rows,
                                                        const float* __restrict__ x,
                                                        float* __restrict__ x_rows,
                                                        DropParams dp, T* __restrict__ ctx,
                                                        float* __restrict__ lse, float scale) {
  __shared__ float sq[64], sp[64], red[64 * 8];
  const int j = threadIdx.x;
  const int bh = xcd_contiguous(blockIdx.x, gridDim.x), b = bh / H, h = bh % H;
  const int D = H * Dh;
  const int64_t ld = 3LL * D;
  int64_t r;
  if constexpr (GATHER) {
    const float cnt = (j < L && kvalid[(int64_t)b * L + j] != 0) ? 1.f : 0.f;
    const int len = (int)(wave_sum(cnt) + 0.5f);
    r = (int64_t)b * L + max(len - 1, 0);
    if (h == 0) {
      if (j == 0) rows[b] = (int32_t)r;
      for (int c = j; c < D; c += 64) x_rows[(int64_t)b * D + c] = x[r * D + c];
    }
  } else {
    r = rows[b];
  }
  const int p = (int)(r - (int64_t)b * L);
  const T* seq = qkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  if (j < Dh) sq[j] = ldf<T>(qkv, r * ld + (int64_t)h * Dh + j);
  __syncthreads();
  const bool ok = j < L && j <= p && kvalid[(int64_t)b * L + j] != 0;
  const float s = ok ? dot_row<T>(sq, seq + (int64_t)j * ld + D, Dh) * scale : -INFINITY;
  const float m = wave_max(s);
  const float e = (ok && m != -INFINITY) ? expf(s - m) : 0.f;
  const float sum = wave_sum(e);
  float pj = sum > 0.f ? e / sum : 0.f;
  const DropKeys dk = resolve_drop(dp);
  if (dk.on && ok) pj = drop_apply(dk, (uint32_t)((((int64_t)bh * L) + p) * L + j), pj);
  sp[j] = pj;
  if (j == 0) lse[bh] = m == -INFINITY ? INFINITY : m + logf(sum);
  __syncthreads();
  const float acc = rows_combine<T>(sp, seq + 2 * D, ld, min(p, L - 1) + 1, Dh, red);
  if (j < Dh) stf<T>(ctx, (int64_t)b * D + (int64_t)h * Dh + j, acc);
}

template <typename T>
__global__ __launch_bounds__(64) void mha_q1_bwd_kernel(int B, int L, int H, int Dh,
                                                        const T* __restrict__ qkv,
                                                        const int64_t* __restrict__ kvalid,
                                                        const int32_t* __restrict__ rows,
                                                        const float* __restrict__ lse,
                                                        const T* __restrict__ dctx, DropParams dp,
                                                        T* __restrict__ dqkv, float scale) {
  constexpr int E = RowLanes<T>::E;
  __shared__ float sq[64], sdo[64], sds[64], spd[64], red[64 * 8];
  const int t = threadIdx.x;
  const int bh = xcd_contiguous(blockIdx.x, gridDim.x), b = bh / H, h = bh % H;
  const int D = H * Dh;
  const int64_t ld = 3LL * D;
  const int64_t r = rows[b];
  const int p = (int)(r - (int64_t)b * L);
  const T* seq = qkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  T* dseq = dqkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  if (t < Dh) {
    sq[t] = ldf<T>(qkv, r * ld + (int64_t)h * Dh + t);
    sdo[t] = ldf<T>(dctx, (int64_t)b * D + (int64_t)h * Dh + t);
  }
  __syncthreads();
  // ---- per key j = t: probabilities and gradients of the scores
  const int j = t;
  const bool ok = j < L && j <= p && kvalid[(int64_t)b * L + j] != 0;
  const DropKeys dk = resolve_drop(dp);
  float pj = 0.f, dP = 0.f, keep = 1.f;
  if (ok) {
    const float sd = dot_row<T>(sq, seq + (int64_t)j * ld + D, Dh);
    const float dv = dot_row<T>(sdo, seq + (int64_t)j * ld + 2 * D, Dh);
    pj = expf(sd * scale - lse[bh]);
    if (dk.on) keep = drop_keep(dk, (uint32_t)((((int64_t)bh * L) + p) * L + j)) ? dk.scale : 0.f;
    dP = dv * keep;
  }
  const float Dsum = wave_sum(pj * dP);
  sds[j] = pj * (dP - Dsum) * scale;
  spd[j] = pj * keep;
  __syncthreads();
  // ---- row stores as 16-byte vectors: dK_j = dS_j q, dV_j = Pd_j dO, Q slice zero except
  //      the query row; dQ_p = Σ_j dS_j k_j
  const RowLanes<T> rl(Dh);
  if (rl.active()) {
    float qv[E], ov[E], z[E], v[E];
#pragma unroll
    for (int i = 0; i < E; ++i) {
      qv[i] = sq[rl.cv * E + i];
      ov[i] = sdo[rl.cv * E + i];
      z[i] = 0.f;
    }
    for (int jj = rl.grp; jj < L; jj += rl.ngrp) {
      T* row = dseq + (int64_t)jj * ld + rl.cv * E;
      if (jj != p) st16<T>(row, z);
      const float a = sds[jj], c = spd[jj];
#pragma unroll
      for (int i = 0; i < E; ++i) v[i] = a * qv[i];
      st16<T>(row + D, v);
#pragma unroll
      for (int i = 0; i < E; ++i) v[i] = c * ov[i];
      st16<T>(row + 2 * D, v);
    }
  }
  const float acc = rows_combine<T>(sds, seq + D, ld, min(p, L - 1) + 1, Dh, red);
  if (t < Dh) stf<T>(dseq + (int64_t)p * ld, t, acc);
}

}  // namespace

extern "C" int ttmi_last_rows(int B, int L, const int64_t* len_src, int32_t* rows, hipStream_t s) {
  TTMI_REQUIRE(B >= 0 && L > 0 && len_src && rows, "ttmi_last_rows: bad args");
  if (B == 0) return TTMI_OK;
  hipLaunchKernelGGL(last_rows_kernel, dim3((B + 3) / 4), dim3(256), 0, s, B, L, len_src, rows);
  return ttmi_check_launch("ttmi_last_rows");
}

extern "C" int ttmi_last_rows_gather(int B, int L, int D, const int64_t* len_src, const float* x,
                                     int32_t* rows, float* out, hipStream_t s) {
  TTMI_REQUIRE(B >= 0 && L > 0 && D > 0 && len_src && x && rows && out, "ttmi_last_rows_gather: bad args");
  TTMI_REQUIRE(D % 4 != 0 || (((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0),
               "ttmi_last_rows_gather: x/out need 16-byte alignment");
  if (B == 0) return TTMI_OK;
  hipLaunchKernelGGL(last_rows_gather_kernel, dim3((B + 3) / 4), dim3(256), 0, s, B, L, D, len_src, x,
                     rows, out);
  return ttmi_check_launch("ttmi_last_rows_gather");
}

extern "C" int ttmi_gather_rows(int B, int D, const float* x, const int32_t* rows, float* out,
                                hipStream_t s) {
  TTMI_REQUIRE(B >= 0 && D > 0 && x && rows && out, "ttmi_gather_rows: bad args");
  if (B == 0) return TTMI_OK;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(B), dim3(128), 0, s, B, D, x, rows, out);
  return ttmi_check_launch("ttmi_gather_rows");
}

extern "C" int ttmi_scatter_add_rows(int B, int D, const float* src, const int32_t* rows,
                                     float* dst, hipStream_t s) {
  TTMI_REQUIRE(B >= 0 && D > 0 && src && rows && dst, "ttmi_scatter_add_rows: bad args");
  if (B == 0) return TTMI_OK;
  hipLaunchKernelGGL(scatter_add_rows_kernel, dim3(B), dim3(128), 0, s, B, D, src, rows, dst);
  return ttmi_check_launch("ttmi_scatter_add_rows");
}

extern "C" int ttmi_mha_q1_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                               const int64_t* key_valid, const int32_t* rows, float drop_p,
                               const uint64_t* drop_seed, void* ctx, float* lse, hipStream_t s) {
  TTMI_REQUIRE(dtype == TTMI_F32 || dtype == TTMI_BF16, "ttmi_mha_q1_fwd: bad dtype");
  TTMI_REQUIRE(B >= 0 && L > 0 && L <= TTMI_ATTN_LMAX && H > 0 && Dh > 0 && Dh <= 64 && Dh % 8 == 0 &&
                   (int64_t)B * H * L * L < (1LL << 32),
               "ttmi_mha_q1_fwd: need L <= %d, Dh <= 64, Dh %% 8 == 0", TTMI_ATTN_LMAX);
  TTMI_REQUIRE(((uintptr_t)qkv & 15) == 0, "ttmi_mha_q1_fwd: qkv must be 16-byte aligned");
  TTMI_REQUIRE(qkv && key_valid && rows && ctx && lse, "ttmi_mha_q1_fwd: null argument");
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || drop_seed),
               "ttmi_mha_q1_fwd: bad dropout");
  if (B == 0) return TTMI_OK;
  DropParams dp = make_drop(drop_p, drop_seed);
  const float scale = 1.f / sqrtf((float)Dh);
  int32_t* rw = const_cast<int32_t*>(rows);          // read only (GATHER = false)
  if (L > 64) return attn_long_q1_fwd(dtype, B, L, H, Dh, qkv, key_valid, rw, nullptr, nullptr, false, dp, ctx, lse, s);
  if (dtype == TTMI_BF16)
    hipLaunchKernelGGL((mha_q1_fwd_kernel<bf16_t, false>), dim3(B * H), dim3(64), 0, s, B, L, H, Dh,
                       (const bf16_t*)qkv, key_valid, rw, nullptr, nullptr, dp, (bf16_t*)ctx, lse, scale);
  else
    hipLaunchKernelGGL((mha_q1_fwd_kernel<float, false>), dim3(B * H), dim3(64), 0, s, B, L, H, Dh,
                       (const float*)qkv, key_valid, rw, nullptr, nullptr, dp, (float*)ctx, lse, scale);
  return ttmi_check_launch("ttmi_mha_q1_fwd");
}

extern "C" int ttmi_mha_q1_gather_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                                      const int64_t* key_valid, const float* x, int32_t* rows,
                                      float* x_rows, float drop_p, const uint64_t* drop_seed,
                                      void* ctx, float* lse, hipStream_t s) {
  TTMI_REQUIRE(dtype == TTMI_F32 || dtype == TTMI_BF16, "ttmi_mha_q1_gather_fwd: bad dtype");
  TTMI_REQUIRE(B >= 0 && L > 0 && L <= TTMI_ATTN_LMAX && H > 0 && Dh > 0 && Dh <= 64 && Dh % 8 == 0 &&
                   (int64_t)B * H * L * L < (1LL << 32),
               "ttmi_mha_q1_gather_fwd: need L <= %d, Dh <= 64, Dh %% 8 == 0", TTMI_ATTN_LMAX);
  TTMI_REQUIRE(((uintptr_t)qkv & 15) == 0, "ttmi_mha_q1_gather_fwd: qkv must be 16-byte aligned");
  TTMI_REQUIRE(qkv && key_valid && x && rows && x_rows && ctx && lse, "ttmi_mha_q1_gather_fwd: null argument");
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || drop_seed),
               "ttmi_mha_q1_gather_fwd: bad dropout");
  if (B == 0) return TTMI_OK;
  DropParams dp = make_drop(drop_p, drop_seed);
  const float scale = 1.f / sqrtf((float)Dh);
  if (L > 64) return attn_long_q1_fwd(dtype, B, L, H, Dh, qkv, key_valid, rows, x, x_rows, true, dp, ctx, lse, s);
  if (dtype == TTMI_BF16)
    hipLaunchKernelGGL((mha_q1_fwd_kernel<bf16_t, true>), dim3(B * H), dim3(64), 0, s, B, L, H, Dh,
                       (const bf16_t*)qkv, key_valid, rows, x, x_rows, dp, (bf16_t*)ctx, lse, scale);
  else
    hipLaunchKernelGGL((mha_q1_fwd_kernel<float, true>), dim3(B * H), dim3(64), 0, s, B, L, H, Dh,
                       (const float*)qkv, key_valid, rows, x, x_rows, dp, (float*)ctx, lse, scale);
  return ttmi_check_launch("ttmi_mha_q1_gather_fwd");
}

extern "C" int ttmi_mha_q1_bwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                               const int64_t* key_valid, const int32_t* rows, const float* lse,
                               const void* dctx, float drop_p, const uint64_t* drop_seed,
                               void* dqkv, hipStream_t s) {
  TTMI_REQUIRE(dtype == TTMI_F32 || dtype == TTMI_BF16, "ttmi_mha_q1_bwd: bad dtype");
  TTMI_REQUIRE(B >= 0 && L > 0 && L <= TTMI_ATTN_LMAX && H > 0 && Dh > 0 && Dh <= 64 && Dh % 8 == 0 &&
                   (int64_t)B * H * L * L < (1LL << 32),
               "ttmi_mha_q1_bwd: need L <= %d, Dh <= 64, Dh %% 8 == 0", TTMI_ATTN_LMAX);
  TTMI_REQUIRE(((uintptr_t)qkv & 15) == 0, "ttmi_mha_q1_bwd: qkv must be 16-byte aligned");
  TTMI_REQUIRE(qkv && key_valid && rows && lse && dctx && dqkv, "ttmi_mha_q1_bwd: null argument");
  TTMI_REQUIRE(((uintptr_t)dqkv & 15) == 0, "ttmi_mha_q1_bwd: dqkv must be 16-byte aligned");
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || drop_seed),
               "ttmi_mha_q1_bwd: bad dropout");
  if (B == 0) return TTMI_OK;
  DropParams dp = make_drop(drop_p, drop_seed);
  const float scale = 1.f / sqrtf((float)Dh);
  if (L > 64) return attn_long_q1_bwd(dtype, B, L, H, Dh, qkv, key_valid, rows, lse, dctx, dp, dqkv, s);
  if (dtype == TTMI_BF16)
    hipLaunchKernelGGL(mha_q1_bwd_kernel<bf16_t>, dim3(B * H), dim3(64), 0, s, B, L, H, Dh,
                       (const bf16_t*)qkv, key_valid, rows, lse, (const bf16_t*)dctx, dp,
                       (bf16_t*)dqkv, scale);
  else
    hipLaunchKernelGGL(mha_q1_bwd_kernel<float>, dim3(B * H), dim3(64), 0, s, B, L, H, Dh,
                       (const float*)qkv, key_valid, rows, lse, (const float*)dctx, dp,
                       (float*)dqkv, scale);
  return ttmi_check_launch("ttmi_mha_q1_bwd");
}
