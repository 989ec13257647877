// ttmi_q1.h — device bodies shared by the one-query attention launches of the pruned last
// encoder layer (ttmi_rows.hip) and the launches that carry independent item-head work on
// the same grid (ttmi_head.hip: item stage A beside the forward; ttmi_rows.hip: the item
// BatchNorm1d backward beside the backward).
//
// One 64-lane wave owns one (sequence b, head h) and synchronises only with itself (LDS
// traffic of one wave is performed in program order), so a 256-thread workgroup runs four
// (b, h) pairs independently and a workgroup of other work can sit in the same grid.
#pragma once
#include "ttmi_common.h"

// Wave-level ordering of LDS traffic: a wave's LDS operations complete in issue order, so the
// only hazard is the compiler moving them; these fences are compiler-only at wavefront scope.
TTMI_DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Host: the one-query entry points' shared argument check (ttmi_rows.hip).
int q1_validate(const char* who, int dtype, int B, int L, int H, int Dh, const void* qkv, float drop_p,
                const uint64_t* drop_seed);

struct Q1Args {
  int B, L, H, Dh;
  float scale;
  const void* qkv; const int64_t* kvalid;
  int32_t* rows; const float* x; float* x_rows;      // fwd (x / x_rows: GATHER only)
  DropParams dp;
  void* ctx; float* lse;                             // fwd outputs / bwd: lse input
  const void* dctx; void* dqkv;                      // bwd
  // ABI 21, fwd (bf16, H·Dh = 128, Dh = 32): the query row's projection is computed here,
  // q = a_in[row]·wq[h·Dh ..]ᵀ + bq (wq: in_proj's first D rows), and written into qkv's Q
  // columns of that row only (the pruned layer projects K / V alone for the other rows)
  const bf16_t* qa; const bf16_t* wq; const float* bq;
};

// Per-wave LDS of the one-query bodies (2.5 KB).
struct Q1Lds {
  float sq[64], sd[64], s1[64], s2[64];
  float red[64 * 8];
};

// Dot product of an LDS fp32 vector with a global row of Dh elements (16-byte loads).
template <typename T>
TTMI_DEV float q1_dot_row(const float* __restrict__ v, const T* __restrict__ row, int Dh) {
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

template <typename T>
TTMI_DEV void q1_st16(T* p, const float* v) {
  constexpr int E = 16 / sizeof(T);
  T tmp[E];
#pragma unroll
  for (int i = 0; i < E; ++i) stf<T>(tmp, i, v[i]);
  *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(tmp);
}

// out[t] = Σ_{k<n} coef[k]·rows[k][t] for lane t < Dh: the wave's lanes split over (row group,
// 16-byte chunk), each lane issues ceil(n / groups) independent 16-byte loads; partials meet
// in the wave's LDS (red: 64·E floats).
template <typename T>
TTMI_DEV float q1_rows_combine(const float* coef, const T* __restrict__ base, int64_t ld, int n,
                               int Dh, float* red, int lane) {
  constexpr int E = 16 / sizeof(T);
  const int lpr = Dh / E, ngrp = 64 / lpr, grp = lane / lpr, cv = lane % lpr;
  float acc[E];
#pragma unroll
  for (int i = 0; i < E; ++i) acc[i] = 0.f;
  if (grp < ngrp) {
    for (int k = grp; k < n; k += ngrp) {
      const uint4 q = *reinterpret_cast<const uint4*>(base + (int64_t)k * ld + cv * E);
      const T* e = reinterpret_cast<const T*>(&q);
      const float c = coef[k];
#pragma unroll
      for (int i = 0; i < E; ++i) acc[i] += c * ldf<T>(e, i);
    }
#pragma unroll
    for (int i = 0; i < E; ++i) red[grp * Dh + cv * E + i] = acc[i];
  }
  wave_lds_sync();
  float s = 0.f;
  if (lane < Dh)
    for (int g = 0; g < ngrp; ++g) s += red[g * Dh + lane];
  return s;
}

// Forward of one (b, h): lane j owns key j (L <= 64).  GATHER: the wave finds the sequence's
// last valid row itself (rows[b] = b·L + max(len - 1, 0), len = the count of non-zero
// key_valid entries) and the head-0 wave writes rows[b] and x_rows[b] = x[rows[b]].
template <typename T, bool GATHER>
TTMI_DEV void q1_fwd_wave(const Q1Args& a, int bh, Q1Lds& S) {
  const int j = threadIdx.x & 63;
  const int b = bh / a.H, h = bh % a.H, L = a.L, Dh = a.Dh;
  const int D = a.H * Dh;
  const int64_t ld = 3LL * D;
  const T* qkv = static_cast<const T*>(a.qkv);
  int64_t r;
  if constexpr (GATHER) {
    const float cnt = (j < L && a.kvalid[(int64_t)b * L + j] != 0) ? 1.f : 0.f;
    const int len = (int)(wave_sum(cnt) + 0.5f);
    r = (int64_t)b * L + max(len - 1, 0);
    if (h == 0) {
      if (j == 0) a.rows[b] = (int32_t)r;
      for (int c = j; c < D; c += 64) a.x_rows[(int64_t)b * D + c] = a.x[r * D + c];
    }
  } else {
    r = a.rows[b];
  }
  const int p = (int)(r - (int64_t)b * L);
  const T* seq = qkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  bool proj = false;
  if constexpr (sizeof(T) == 2) proj = a.qa != nullptr;
  if (proj) {
    // two lanes per output d (64 of the 128 k each), fp32 sums, rounded to bf16 as the
    // projection GEMM's output would be
    const int d = j >> 1, hf = j & 1;
    const uint4* wr = reinterpret_cast<const uint4*>(a.wq + (int64_t)(h * Dh + d) * D + hf * 64);
    const uint4* ar = reinterpret_cast<const uint4*>(a.qa + r * D + hf * 64);
    uint4 wv[8], av[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) { wv[c] = wr[c]; av[c] = ar[c]; }
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint32_t wx[4] = {wv[c].x, wv[c].y, wv[c].z, wv[c].w}, ax[4] = {av[c].x, av[c].y, av[c].z, av[c].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc = fmaf(__uint_as_float(ax[e] << 16), __uint_as_float(wx[e] << 16), acc);
        acc = fmaf(__uint_as_float(ax[e] & 0xFFFF0000u), __uint_as_float(wx[e] & 0xFFFF0000u), acc);
      }
    }
    acc += __shfl_xor(acc, 1, 64);
    const bf16_t qb = f2bf(acc + a.bq[h * Dh + d]);
    if (hf == 0) {
      S.sq[d] = __uint_as_float((uint32_t)qb << 16);
      reinterpret_cast<bf16_t*>(const_cast<void*>(a.qkv))[r * ld + (int64_t)h * Dh + d] = qb;
    }
  } else if (j < Dh) {
    S.sq[j] = ldf<T>(qkv, r * ld + (int64_t)h * Dh + j);
  }
  wave_lds_sync();
  const bool ok = j < L && j <= p && a.kvalid[(int64_t)b * L + j] != 0;
  const float s = ok ? q1_dot_row<T>(S.sq, seq + (int64_t)j * ld + D, Dh) * a.scale : -INFINITY;
  const float m = wave_max(s);
  const float e = (ok && m != -INFINITY) ? expf(s - m) : 0.f;
  const float sum = wave_sum(e);
  float pj = sum > 0.f ? e / sum : 0.f;
  const DropKeys dk = resolve_drop(a.dp);
  if (dk.on && ok) pj = drop_apply(dk, (uint32_t)((((int64_t)bh * L) + p) * L + j), pj);
  S.s1[j] = pj;
  if (j == 0) a.lse[bh] = m == -INFINITY ? INFINITY : m + logf(sum);
  wave_lds_sync();
  const float acc = q1_rows_combine<T>(S.s1, seq + 2 * D, ld, min(p, L - 1) + 1, Dh, S.red, j);
  if (j < Dh) stf<T>(static_cast<T*>(a.ctx), (int64_t)b * D + (int64_t)h * Dh + j, acc);
}

// Backward of one (b, h): writes the (b, h) slices of dqkv for all L rows (dQ zero except the
// query row, dK_j = dS_j q, dV_j = Pd_j dO) and dQ_p = Σ_j dS_j k_j.  KV (ABI 21,
// ttmi_mha_q1_kv_bwd): dqkv's Q columns are left alone and dQ_p goes to sdq[h·Dh + t] (the
// workgroup's query-row gradient, for the caller's dq·W_q) instead.
template <typename T, bool KV = false>
TTMI_DEV void q1_bwd_wave(const Q1Args& a, int bh, Q1Lds& S, float* sdq = nullptr) {
  constexpr int E = 16 / sizeof(T);
  const int t = threadIdx.x & 63;
  const int b = bh / a.H, h = bh % a.H, L = a.L, Dh = a.Dh;
  const int D = a.H * Dh;
  const int64_t ld = 3LL * D;
  const T* qkv = static_cast<const T*>(a.qkv);
  const int64_t r = a.rows[b];
  const int p = (int)(r - (int64_t)b * L);
  const T* seq = qkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  T* dseq = static_cast<T*>(a.dqkv) + (int64_t)b * L * ld + (int64_t)h * Dh;
  if (t < Dh) {
    S.sq[t] = ldf<T>(qkv, r * ld + (int64_t)h * Dh + t);
    S.sd[t] = ldf<T>(static_cast<const T*>(a.dctx), (int64_t)b * D + (int64_t)h * Dh + t);
  }
  wave_lds_sync();
  const int j = t;
  const bool ok = j < L && j <= p && a.kvalid[(int64_t)b * L + j] != 0;
  const DropKeys dk = resolve_drop(a.dp);
  float pj = 0.f, dP = 0.f, keep = 1.f;
  if (ok) {
    const float sd = q1_dot_row<T>(S.sq, seq + (int64_t)j * ld + D, Dh);
    const float dv = q1_dot_row<T>(S.sd, seq + (int64_t)j * ld + 2 * D, Dh);
    pj = expf(sd * a.scale - a.lse[bh]);
    if (dk.on) keep = drop_keep(dk, (uint32_t)((((int64_t)bh * L) + p) * L + j)) ? dk.scale : 0.f;
    dP = dv * keep;
  }
  const float Dsum = wave_sum(pj * dP);
  S.s1[j] = pj * (dP - Dsum) * a.scale;
  S.s2[j] = pj * keep;
  wave_lds_sync();
  const int lpr = Dh / E, ngrp = 64 / lpr, grp = t / lpr, cv = t % lpr;
  if (grp < ngrp) {
    float qv[E], ov[E], z[E], v[E];
#pragma unroll
    for (int i = 0; i < E; ++i) {
      qv[i] = S.sq[cv * E + i];
      ov[i] = S.sd[cv * E + i];
      z[i] = 0.f;
    }
    for (int jj = grp; jj < L; jj += ngrp) {
      T* row = dseq + (int64_t)jj * ld + cv * E;
      if (!KV && jj != p) q1_st16<T>(row, z);
      const float c1 = S.s1[jj], c2 = S.s2[jj];
#pragma unroll
      for (int i = 0; i < E; ++i) v[i] = c1 * qv[i];
      q1_st16<T>(row + D, v);
#pragma unroll
      for (int i = 0; i < E; ++i) v[i] = c2 * ov[i];
      q1_st16<T>(row + 2 * D, v);
    }
  }
  const float acc = q1_rows_combine<T>(S.s1, seq + D, ld, min(p, L - 1) + 1, Dh, S.red, t);
  if constexpr (KV) {
    if (t < Dh) sdq[h * Dh + t] = acc;
  } else {
    if (t < Dh) stf<T>(dseq + (int64_t)p * ld, t, acc);
  }
}

// ------------------------------------------------------------ BatchNorm1d backward body
// Register-resident BatchNorm1d backward (ttmi_batchnorm_bwd's B <= 16·RG path): COLS x RG
// threads, every thread holds RPT rows of one column (all loads issued first); the two column
// sums through LDS in row-group order.  dw / db get ONE add per column per launch (plain
// atomics on addresses no other workgroup touches: order-free).
struct BnrBwdArgs {
  int B, C;
  const float* dy; const float* z; const float* w; const float* mean; const float* rstd;
  const void* y;                 // gate operand (T), may be NULL when !gated
  float gate_scale; int gated;
  float* dz; float* dw; float* db; bf16_t* dz16;
};

template <int COLS, int RG>
struct BnrLds {
  float red[RG][COLS];
};

template <int COLS, int RG>
TTMI_DEV float bnr_colsum_t(float v, BnrLds<COLS, RG>& L, int rg, int cl) {
  __syncthreads();
  L.red[rg][cl] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < RG; ++k) s += L.red[k][cl];
  return s;
}

template <typename T, int COLS, int RG, int RPT>
TTMI_DEV void bnr_bwd_body(const BnrBwdArgs& a, int blk, BnrLds<COLS, RG>& L) {
  const int cl = threadIdx.x % COLS, rg = threadIdx.x / COLS;
  const int B = a.B, C = a.C;
  const int c = blk * COLS + cl;
  const int cc = min(c, C - 1);
  const T* y = static_cast<const T*>(a.y);
  float d[RPT], xh[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int64_t o = (int64_t)min(rg + RG * j, B - 1) * C + cc;
    d[j] = a.dy[o];
    xh[j] = a.z[o];
    if (a.gated) d[j] = ldf<T>(y, o) > 0.f ? d[j] * a.gate_scale : 0.f;
  }
  const float mu = a.mean[cc], rs = a.rstd[cc], wc = a.w[cc];
  float s1 = 0.f, s2 = 0.f;   // Σ dy', Σ dy'·x̂
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    xh[j] = (xh[j] - mu) * rs;
    if (rg + RG * j < B) {
      s1 += d[j];
      s2 += d[j] * xh[j];
    }
  }
  const float S1 = bnr_colsum_t(s1, L, rg, cl);
  const float S2 = bnr_colsum_t(s2, L, rg, cl);
  if (c >= C) return;
  const float invB = 1.f / (float)B;
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int r = rg + RG * j;
    if (r < B) {
      const float v = wc * rs * (d[j] - S1 * invB - xh[j] * S2 * invB);
      a.dz[(int64_t)r * C + c] = v;
      if (a.dz16) a.dz16[(int64_t)r * C + c] = f2bf(v);   // the next GEMM's bf16 operand
    }
  }
  if (rg == 0) {
    if (a.dw) atomicAdd(a.dw + c, S2);
    if (a.db) atomicAdd(a.db + c, S1);
  }
}
