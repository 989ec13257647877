// ttmi_norm.hip — row/column normalisation kernels of the two-tower step:
//   LayerNorm fwd/bwd (one wave per row, D <= 1024 held in registers, fp32 statistics),
//   the SASRec input block (embedding gather + position add + LN + dropout) fwd/bwd,
//   the last-valid-row gather + demographics concat fwd/bwd, BatchNorm1d train fwd/bwd.
#include "ttmi_common.h"

namespace {

constexpr int MAXV = 16;   // D <= 64 * MAXV
constexpr int LN_REPL = 32;   // replicas of the LayerNorm-backward weight/bias column sums

// Instantiate a kernel template for the smallest NV (64-wide column chunks per row) that
// covers D: NV in {1, 2, 4, 8, 16}.
#define TTMI_NV_DISPATCH(D, ...)                 \
  do {                                          \
    if ((D) <= 64) { constexpr int NV = 1; __VA_ARGS__; }        \
    else if ((D) <= 128) { constexpr int NV = 2; __VA_ARGS__; }  \
    else if ((D) <= 256) { constexpr int NV = 4; __VA_ARGS__; }  \
    else if ((D) <= 512) { constexpr int NV = 8; __VA_ARGS__; }  \
    else { constexpr int NV = 16; __VA_ARGS__; }                 \
  } while (0)

// ------------------------------------------------------------------------------ LayerNorm
template <typename TY, int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int64_t M, int D, const float* __restrict__ x,
                                                     int64_t ldx, const float* __restrict__ w,
                                                     const float* __restrict__ b, float eps,
                                                     int relu, DropParams dp, TY* __restrict__ y,
                                                     int64_t ldy, float* __restrict__ mean,
                                                     float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const float invD = 1.f / (float)D;
  const DropKeys dk = resolve_drop(dp);
  for (int64_t row = wid; row < M; row += nw) {
    float v[NV];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      v[i] = c < D ? x[row * ldx + c] : 0.f;
      s += v[i];
    }
    const float mu = wave_sum(s) * invD;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      const float dlt = c < D ? v[i] - mu : 0.f;
      q += dlt * dlt;
    }
    const float rs = 1.f / sqrtf(wave_sum(q) * invD + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      if (c < D) {
        float o = (v[i] - mu) * rs * w[c] + b[c];
        if (relu) o = fmaxf(o, 0.f);
        if (dk.on) o = drop_apply(dk, (uint32_t)(row * D + c), o);
        stf<TY>(y, row * ldy + c, o);
      }
    }
    if (lane == 0) {
      if (mean) mean[row] = mu;
      if (rstd) rstd[row] = rs;
    }
  }
}

// Per-block reduction of per-lane column partials (W waves, in wave order) followed by one
// fixed-point atomic per column (order-independent: the sum's bits do not depend on which
// block adds first).
template <int NV, int W>
TTMI_DEV void block_col_fx(float (&acc)[NV], int D, int64_t* dst, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < D) red[wave * 64 * NV + c] = acc[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < W; ++k) t += red[k * 64 * NV + c];
    fx_add(dst + c, t, TTMI_FX_GRAD);
  }
}

template <int NV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    int64_t M, int D, const float* __restrict__ dy, int64_t lddy, const float* __restrict__ x,
    int64_t ldx, const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ w, const void* __restrict__ gate, int gate_f32, int64_t ldg,
    float gate_scale, const float* res, float* dx, int64_t lddx, int64_t* __restrict__ cw,
    int64_t* __restrict__ cb, int nrep, int64_t rstride, bf16_t* __restrict__ dx16, int64_t ld16,
    DropParams dp16) {
  __shared__ float red[4 * 64 * NV];
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const float invD = 1.f / (float)D;
  float aw[NV], ab[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) aw[i] = ab[i] = 0.f;
  const DropKeys dk16 = resolve_drop(dp16);
  // U rows per wave per pass (rows row0 + u·nw), every load of all U rows issued before any
  // arithmetic: with the column sums the grid is capped (1,024 blocks), so a wave walks
  // M / 4,096 rows and a row-at-a-time loop paid one dependent memory round trip per row.
  // Rows are accumulated in the same order as one at a time (deterministic, unchanged sums).
  constexpr int U = 4;
  for (int64_t row0 = wid; row0 < M; row0 += U * nw) {
    int64_t row[U];
    bool live[U];
    float mu[U], rs[U], d[U][NV], xv[U][NV], rv[U][NV];
#pragma unroll
    for (int u = 0; u < U; ++u) {          // clamped rows and columns: unconditional loads
      live[u] = row0 + (int64_t)u * nw < M;
      row[u] = live[u] ? row0 + (int64_t)u * nw : M - 1;
      mu[u] = mean[row[u]];
      rs[u] = rstd[row[u]];
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = min(lane + 64 * i, D - 1);
        d[u][i] = dy[row[u] * lddy + c];
        if (gate) d[u][i] = ld_dyn(gate, row[u] * ldg + c, gate_f32) > 0.f ? d[u][i] * gate_scale : 0.f;
        xv[u][i] = x[row[u] * ldx + c];
        rv[u][i] = res ? res[row[u] * lddx + c] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!live[u]) continue;                // wave-uniform
      float g[NV], xh[NV];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = lane + 64 * i;
        g[i] = 0.f; xh[i] = 0.f;
        if (c < D) {
          xh[i] = (xv[u][i] - mu[u]) * rs[u];
          aw[i] += d[u][i] * xh[i];
          ab[i] += d[u][i];
          g[i] = d[u][i] * w[c];
          s1 += g[i];
          s2 += g[i] * xh[i];
        }
      }
      const float c1 = wave_sum(s1) * invD, c2 = wave_sum(s2) * invD;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = lane + 64 * i;
        if (c < D) {
          const float o = rs[u] * (g[i] - c1 - xh[i] * c2);
          const float v = rv[u][i] + o;
          dx[row[u] * lddx + c] = v;
          if (dx16) dx16[row[u] * ld16 + c] = f2bf(drop_apply(dk16, (uint32_t)(row[u] * D + c), v));
        }
      }
    }
  }
  if (cw) {   // LN weight / bias partials: fixed-point adds into this block's replica row
    const int64_t o = (int64_t)(blockIdx.x % nrep) * rstride;
    block_col_fx<NV, 4>(aw, D, cw + o, red);
    block_col_fx<NV, 4>(ab, D, cb + o, red);
  }
}

// Wide rows (D % 256 == 0, no gate, no column sums: the frozen text-encoder LayerNorms,
// D = 768): one wave per row, each lane 4 consecutive columns per 16-byte access (Q4 = D/256
// float4 per lane) — the 4-byte-per-lane form streamed at ~3 TB/s.
template <int Q4>
__global__ __launch_bounds__(256) void ln_bwd_vec_kernel(int64_t M, int D, const float* __restrict__ dy,
                                                         int64_t lddy, const float* __restrict__ x,
                                                         int64_t ldx, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd,
                                                         const float* __restrict__ w,
                                                         const float* res, float* dx, int64_t lddx,
                                                         bf16_t* __restrict__ dx16, int64_t ld16,
                                                         DropParams dp16) {
  const int lane = threadIdx.x & 63;
  const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (row >= M) return;
  const DropKeys dk16 = resolve_drop(dp16);
  const float invD = 1.f / (float)D;
  const float mu = mean[row], rs = rstd[row];
  float4 g[Q4], xh[Q4], r[Q4];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < Q4; ++i) {
    const int c = (lane + 64 * i) * 4;
    const float4 d = *reinterpret_cast<const float4*>(dy + row * lddy + c);
    const float4 xv = *reinterpret_cast<const float4*>(x + row * ldx + c);
    const float4 wv = *reinterpret_cast<const float4*>(w + c);
    r[i] = res ? *reinterpret_cast<const float4*>(res + row * lddx + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    xh[i] = make_float4((xv.x - mu) * rs, (xv.y - mu) * rs, (xv.z - mu) * rs, (xv.w - mu) * rs);
    g[i] = make_float4(d.x * wv.x, d.y * wv.y, d.z * wv.z, d.w * wv.w);
    s1 += g[i].x + g[i].y + g[i].z + g[i].w;
    s2 += g[i].x * xh[i].x + g[i].y * xh[i].y + g[i].z * xh[i].z + g[i].w * xh[i].w;
  }
  const float c1 = wave_sum(s1) * invD, c2 = wave_sum(s2) * invD;
#pragma unroll
  for (int i = 0; i < Q4; ++i) {
    const int c = (lane + 64 * i) * 4;
    float4 o = make_float4(r[i].x + rs * (g[i].x - c1 - xh[i].x * c2), r[i].y + rs * (g[i].y - c1 - xh[i].y * c2),
                           r[i].z + rs * (g[i].z - c1 - xh[i].z * c2), r[i].w + rs * (g[i].w - c1 - xh[i].w * c2));
    *reinterpret_cast<float4*>(dx + row * lddx + c) = o;
    if (dx16) {          // bf16(dropout(dx)): the next GEMM's operand (dropout backward fused)
      drop_apply_vec<4>(dk16, (uint32_t)(row * D + c), &o.x);
      ushort4 h;
      h.x = f2bf(o.x); h.y = f2bf(o.y); h.z = f2bf(o.z); h.w = f2bf(o.w);
      *reinterpret_cast<ushort4*>(dx16 + row * ld16 + c) = h;
    }
  }
}

// dst0[i] += Σ_r ws[r][i] (i < n0), dst1[i - n0] += ... (n0 <= i < n) over int64 fixed-point
// replicas (exact integer sum, converted once); zeroes the replicas.
__global__ __launch_bounds__(256) void colsum_fold_kernel(int n, int n0, int R, int64_t* __restrict__ ws,
                                                          float* __restrict__ dst0,
                                                          float* __restrict__ dst1) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  long long s = 0;
  constexpr int U = 8;
  for (int r0 = 0; r0 < R; r0 += U) {
    long long v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = r0 + u < R ? ws[(int64_t)(r0 + u) * n + i] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      s += v[u];
      if (r0 + u < R) ws[(int64_t)(r0 + u) * n + i] = 0;
    }
  }
  const float f = fx_to_f(s, TTMI_FX_GRAD);
  if (i < n0) { if (dst0) dst0[i] += f; }
  else if (dst1) dst1[i - n0] += f;
}

// ------------------------------------------------------------------- SASRec input block
// Forward: one wave per token row.  With LN2 the row also goes through the first encoder
// layer's norm1 (norm_first) while it is in registers: y1 = bf16(LN1(x)), mean1 / rstd1.
template <int NV, bool LN2>
__global__ __launch_bounds__(256) void seq_embed_fwd_kernel(
    int B, int L, int D, const int64_t* __restrict__ ids, const float* __restrict__ E, int64_t V,
    const float* __restrict__ P, const float* __restrict__ w, const float* __restrict__ b,
    float eps, DropParams dp, float* __restrict__ x, float* __restrict__ mean,
    float* __restrict__ rstd, const float* __restrict__ w1, const float* __restrict__ b1,
    float eps1, bf16_t* __restrict__ y1, float* __restrict__ mean1, float* __restrict__ rstd1,
    int32_t* __restrict__ id_err) {
  const int lane = threadIdx.x & 63;
  const int64_t M = (int64_t)B * L;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const float invD = 1.f / (float)D;
  const DropKeys dk = resolve_drop(dp);
  for (int64_t row = wid; row < M; row += nw) {
    const int l = (int)(row % L);
    const int64_t id = ids[row];
    const bool ok = id >= 0 && id < V;      // an id outside the table reads a zero row and flags
    if (!ok) raise_id_err(id_err, TTMI_IDERR_HISTORY);
    float v[NV];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      v[i] = c < D ? (ok ? E[id * D + c] : 0.f) + P[(int64_t)l * D + c] : 0.f;
      s += v[i];
    }
    const float mu = wave_sum(s) * invD;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      const float dlt = c < D ? v[i] - mu : 0.f;
      q += dlt * dlt;
    }
    const float rs = 1.f / sqrtf(wave_sum(q) * invD + eps);
    float s1 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      if (c < D) {
        float o = (v[i] - mu) * rs * w[c] + b[c];
        if (dk.on) o = drop_apply(dk, (uint32_t)(row * D + c), o);
        x[row * D + c] = o;
        v[i] = o;
        s1 += o;
      }
    }
    if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
    if constexpr (LN2) {
      const float mu1 = wave_sum(s1) * invD;
      float q1 = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = lane + 64 * i;
        const float dlt = c < D ? v[i] - mu1 : 0.f;
        q1 += dlt * dlt;
      }
      const float rs1 = 1.f / sqrtf(wave_sum(q1) * invD + eps1);
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = lane + 64 * i;
        if (c < D) stf<bf16_t>(y1, row * D + c, (v[i] - mu1) * rs1 * w1[c] + b1[c]);
      }
      if (lane == 0) { mean1[row] = mu1; rstd1[row] = rs1; }
    }
  }
}

// Forward, 16-byte lanes (D = 128 or 256): a row is LPR = D / 4 lanes holding 4 consecutive
// columns each (2 rows per wave at D = 128), and a wave keeps U row groups in flight with every
// load issued before any arithmetic (the one-row-per-wave kernel above ran a dependent
// ids -> E[id] -> reduce -> store chain per row with 4-byte loads: ~1.8 TB/s at cfg 2).
template <int LPR>
TTMI_DEV float lane_group_sum(float v) {
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int D, bool LN2, int U>
__global__ __launch_bounds__(256) void seq_embed_fwd_vec_kernel(
    int B, int L, const int64_t* __restrict__ ids, const float* __restrict__ E, int64_t V,
    const float* __restrict__ P, const float* __restrict__ w, const float* __restrict__ b,
    float eps, DropParams dp, float* __restrict__ x, float* __restrict__ mean,
    float* __restrict__ rstd, const float* __restrict__ w1, const float* __restrict__ b1,
    float eps1, bf16_t* __restrict__ y1, float* __restrict__ mean1, float* __restrict__ rstd1,
    int32_t* __restrict__ id_err) {
  constexpr int LPR = D / 4, RPW = 64 / LPR;          // lanes per row, rows per wave instruction
  const int lane = threadIdx.x & 63, j = lane % LPR, sub = lane / LPR;
  const int64_t M = (int64_t)B * L;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  constexpr float invD = 1.f / (float)D;
  const DropKeys dk = resolve_drop(dp);
  const float4 wv = reinterpret_cast<const float4*>(w)[j], bv = reinterpret_cast<const float4*>(b)[j];
  float4 w1v = make_float4(0.f, 0.f, 0.f, 0.f), b1v = w1v;
  if constexpr (LN2) { w1v = reinterpret_cast<const float4*>(w1)[j]; b1v = reinterpret_cast<const float4*>(b1)[j]; }
  for (int64_t g0 = wid * (U * RPW); g0 < M; g0 += nw * (U * RPW)) {
    int64_t row[U], id[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      row[u] = g0 + u * RPW + sub;
      id[u] = ids[min(row[u], M - 1)];              // clamped: unconditional loads
    }
    float4 e[U], pv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = id[u] >= 0 && id[u] < V;   // outside the table: a zero row, flagged
      if (!ok) raise_id_err(id_err, TTMI_IDERR_HISTORY);
      const int l = (int)(min(row[u], M - 1) % L);
      e[u] = reinterpret_cast<const float4*>(E + (ok ? id[u] : 0) * D)[j];
      if (!ok) e[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      pv[u] = reinterpret_cast<const float4*>(P + (int64_t)l * D)[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float v[4] = {e[u].x + pv[u].x, e[u].y + pv[u].y, e[u].z + pv[u].z, e[u].w + pv[u].w};
      const float mu = lane_group_sum<LPR>(v[0] + v[1] + v[2] + v[3]) * invD;
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) q += (v[k] - mu) * (v[k] - mu);
      const float rs = 1.f / sqrtf(lane_group_sum<LPR>(q) * invD + eps);
      const float wa[4] = {wv.x, wv.y, wv.z, wv.w}, ba[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = (v[k] - mu) * rs * wa[k] + ba[k];
      drop_apply_vec<4>(dk, (uint32_t)(row[u] * D + 4 * j), v);
      if (row[u] >= M) continue;
      reinterpret_cast<float4*>(x + row[u] * D)[j] = make_float4(v[0], v[1], v[2], v[3]);
      if (j == 0) { mean[row[u]] = mu; rstd[row[u]] = rs; }
      if constexpr (LN2) {
        const float mu1 = lane_group_sum<LPR>(v[0] + v[1] + v[2] + v[3]) * invD;
        float q1 = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) q1 += (v[k] - mu1) * (v[k] - mu1);
        const float rs1 = 1.f / sqrtf(lane_group_sum<LPR>(q1) * invD + eps1);
        const float wa1[4] = {w1v.x, w1v.y, w1v.z, w1v.w}, ba1[4] = {b1v.x, b1v.y, b1v.z, b1v.w};
        ushort4 o;
        o.x = f2bf((v[0] - mu1) * rs1 * wa1[0] + ba1[0]);
        o.y = f2bf((v[1] - mu1) * rs1 * wa1[1] + ba1[1]);
        o.z = f2bf((v[2] - mu1) * rs1 * wa1[2] + ba1[2]);
        o.w = f2bf((v[3] - mu1) * rs1 * wa1[3] + ba1[3]);
        reinterpret_cast<ushort4*>(y1 + row[u] * D)[j] = o;
        if (j == 0) { mean1[row[u]] = mu1; rstd1[row[u]] = rs1; }
      }
    }
  }
}

// Backward: block (l, b-chunk) of SEB_W waves; each wave walks b = chunk*bpc + wave,
// + SEB_W, ... so the position gradient dP[l] accumulates in registers (one add per column
// per block).  A wave makes SEB_R passes of U rows whose loads are all in flight at once (the
// dependent gather ids -> E[id]: two memory round trips per wave), so the grid is one round.
// Every cross-block sum goes to int64 fixed-point accumulators (ABI 16): the item-embedding
// rows accE[V][D] (one add per token and column) and accL[3][L][D] (dP, and the LayerNorm
// weight / bias partials per position), converted into the fp32 gradients by the fold
// (ttmi_seq_embed_bwd_folds): the gradient is bit-identical run to run (the fp32 atomics it
// replaces summed in arrival order).  TTMI_SEB_R = 2 measured ~2.5 us a step faster in round 6
// (profiles/r06/seq_embed_bwd_passes.txt) but is not the default: its validation run hit a host
// segfault in an unrelated cfg-4 graph replay whose cause was not established before the round
// closed, so the build that passed the full suite twice is kept.
#ifndef TTMI_SEB_R
#define TTMI_SEB_R 4
#endif
constexpr int SEB_W = 4, SEB_R = TTMI_SEB_R;
template <int NV>
__global__ __launch_bounds__(64 * SEB_W) void seq_embed_bwd_kernel(
    int B, int L, int D, const int64_t* __restrict__ ids, const float* __restrict__ E,
    const float* __restrict__ P, const float* __restrict__ w, const float* __restrict__ mean,
    const float* __restrict__ rstd, DropParams dp, const float* __restrict__ dx,
    int64_t* __restrict__ accE, int64_t* __restrict__ accL, int64_t padding_idx, int64_t V, int bpc) {
  __shared__ float red[SEB_W * 64 * NV];
  TTMI_TSTAMP(0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l = blockIdx.x;
  const int b0 = blockIdx.y * bpc;
  const int b1 = min(B, b0 + bpc);
  const float invD = 1.f / (float)D;
  const DropKeys dk = resolve_drop(dp);
  float ap[NV], aw[NV], ab[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) ap[i] = aw[i] = ab[i] = 0.f;
  // two rows per wave per pass, SEB_R passes
  constexpr int U = 2, STEP = SEB_W * U;
  struct Rows { int64_t row[U], id[U]; float mu[U], rs[U], d[U][NV], e[U][NV]; };
  auto load_ids = [&](int bq, int64_t (&row)[U], int64_t (&id)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {       // rows past the chunk clamped: harmless re-loads
      row[u] = (int64_t)min(bq + SEB_W * u, b1 - 1) * L + l;
      id[u] = ids[row[u]];
    }
  };
  // the padding row E[padding_idx], read once: about half the tokens are padding, and every
  // wave gathering that one 512-byte row queued on the same L2 channel of its XCD
  const bool pad_ok = padding_idx >= 0 && padding_idx < V;
  float epad[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) epad[i] = pad_ok ? E[padding_idx * D + min(lane + 64 * i, D - 1)] : 0.f;
  // r.e: the row's embedding value (E[id], the padding row, or 0 for an id outside [0, V))
  auto load_rows = [&](const int64_t (&row)[U], const int64_t (&id)[U], Rows& r) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      r.row[u] = row[u];
      r.id[u] = id[u];
      const bool ok = id[u] >= 0 && id[u] < V;
      r.mu[u] = mean[row[u]];
      r.rs[u] = rstd[row[u]];
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = min(lane + 64 * i, D - 1);
        r.d[u][i] = dx[row[u] * D + c];
        r.e[u][i] = id[u] == padding_idx ? epad[i] : 0.f;
      }
      if (ok && id[u] != padding_idx) {          // wave-uniform (one row per wave)
#pragma unroll
        for (int i = 0; i < NV; ++i) r.e[u][i] = E[id[u] * D + min(lane + 64 * i, D - 1)];
      }
    }
  };
  float pl[NV], wl[NV];                  // this block's position row and LayerNorm weight
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = min(lane + 64 * i, D - 1);
    pl[i] = P[(int64_t)l * D + c];
    wl[i] = w[c];
  }
  // all SEB_R passes' ids, then all their rows, in flight at once: two memory round trips per
  // wave (under the kernel's load a round trip is ~3 us: a one-pass-ahead pipeline still paid
  // about one per pass)
  Rows rr[SEB_R];
  {
    int64_t row0[SEB_R][U], id0[SEB_R][U];
#pragma unroll
    for (int k = 0; k < SEB_R; ++k) load_ids(b0 + wave + k * STEP, row0[k], id0[k]);
#pragma unroll
    for (int k = 0; k < SEB_R; ++k) load_rows(row0[k], id0[k], rr[k]);
  }
#pragma unroll
  for (int k = 0; k < SEB_R; ++k) {
    TTMI_TSTAMP(1 + k);                          // (diagnostic build: pass k starts)
    const int bq = b0 + wave + k * STEP;
    const Rows& cur = rr[k];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (bq + SEB_W * u >= b1) continue;
      const int64_t row = cur.row[u], id = cur.id[u];
      const bool ok = id >= 0 && id < V;
      float g[NV], xh[NV];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = lane + 64 * i;
        g[i] = 0.f; xh[i] = 0.f;
        if (c < D) {
          float dd = cur.d[u][i];
          if (dk.on) dd = drop_keep(dk, (uint32_t)(row * D + c)) ? dd * dk.scale : 0.f;
          const float ev = cur.e[u][i] + pl[i];
          xh[i] = (ev - cur.mu[u]) * cur.rs[u];
          aw[i] += dd * xh[i];
          ab[i] += dd;
          g[i] = dd * wl[i];
          s1 += g[i];
          s2 += g[i] * xh[i];
        }
      }
      const float c1 = wave_sum_dpp(s1) * invD, c2 = wave_sum_dpp(s2) * invD;
      const bool emb = ok && id != padding_idx;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = lane + 64 * i;
        if (c < D) {
          const float o = cur.rs[u] * (g[i] - c1 - xh[i] * c2);
          ap[i] += o;
#ifndef TTMI_DIAG_NOATOM
          if (emb) fx_add(accE + id * D + c, o, TTMI_FX_GRAD);
#else
          if (emb && o == 12345.f) accE[id * D + c] = 1;   // diagnostic build: no scatter
#endif
        }
      }
    }
  }
  TTMI_TSTAMP(1 + SEB_R);
  const int64_t LD = (int64_t)L * D;
  block_col_fx<NV, SEB_W>(ap, D, accL + (int64_t)l * D, red);
  block_col_fx<NV, SEB_W>(aw, D, accL + LD + (int64_t)l * D, red);
  block_col_fx<NV, SEB_W>(ab, D, accL + 2 * LD + (int64_t)l * D, red);
  TTMI_TSTAMP(2 + SEB_R);
}

// ------------------------------------------------------------ last-valid gather + concat
template <typename T>
__global__ void user_concat_fwd_kernel(int B, int L, int D, const float* __restrict__ x,
                                       const int64_t* __restrict__ len_src,
                                       const int64_t* __restrict__ gender,
                                       const float* __restrict__ G, int dg,
                                       const int64_t* __restrict__ country,
                                       const float* __restrict__ C, int dc, T* __restrict__ comb,
                                       int32_t* __restrict__ rows, int ng, int nc,
                                       int32_t* __restrict__ id_err) {
  const int lane = threadIdx.x & 63;
  const int b = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (b >= B) return;
  float cnt = 0.f;
  if (len_src)
    for (int l = lane; l < L; l += 64) cnt += len_src[(int64_t)b * L + l] != 0 ? 1.f : 0.f;
  const int len = len_src ? (int)(wave_sum(cnt) + 0.5f) : 1;
  const int64_t row = (int64_t)b * L + max(len - 1, 0);
  const int W = D + dg + dc;
  const int64_t g = clamp_id(gender[b], ng, id_err, TTMI_IDERR_GENDER);
  const int64_t c = clamp_id(country[b], nc, id_err, TTMI_IDERR_COUNTRY);
  for (int k = lane; k < W; k += 64) {
    float v;
    if (k < D) v = x[row * D + k];
    else if (k < D + dg) v = G[g * dg + (k - D)];
    else v = C[c * dc + (k - D - dg)];
    stf<T>(comb, (int64_t)b * W + k, v);
  }
  if (lane == 0) rows[b] = (int32_t)row;
}

__global__ void user_concat_bwd_kernel(int B, int D, const float* __restrict__ dcomb,
                                       const int32_t* __restrict__ rows,
                                       const int64_t* __restrict__ gender, int dg,
                                       const int64_t* __restrict__ country, int dc,
                                       float* __restrict__ dx, int64_t* __restrict__ dG,
                                       int64_t* __restrict__ dC, int accumulate, int ng, int nc) {
  const int lane = threadIdx.x & 63;
  const int b = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (b >= B) return;
  const int W = D + dg + dc;
  const int64_t row = rows[b];
  const int64_t g = clamp_id(gender[b], ng, nullptr, 0), c = clamp_id(country[b], nc, nullptr, 0);
  for (int k = lane; k < W; k += 64) {
    const float v = dcomb[(int64_t)b * W + k];
    if (k < D) {
      if (accumulate) dx[row * D + k] += v;   // rows distinct: each dx row has one writer
      else dx[row * D + k] = v;
    }   // demographic rows shared by users: fixed-point adds (order-independent)
    else if (k < D + dg) { if (dG) fx_add(dG + g * dg + (k - D), v, TTMI_FX_GRAD); }
    else if (dC) fx_add(dC + c * dc + (k - D - dg), v, TTMI_FX_GRAD);
  }
}

// ---------------------------------------------------------------------- BatchNorm1d
// Block: 256 threads = BN_COLS columns x BN_RG row groups; per-column statistics reduced
// through LDS (no atomics: one block owns its columns).
constexpr int BN_COLS = 16, BN_RG = 16;

template <typename T>
__global__ __launch_bounds__(256) void bn_fwd_kernel(int B, int C, const float* __restrict__ z,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ b, float eps,
                                                     float momentum, float* running_mean,
                                                     float* running_var, int64_t* nbt,
                                                     int training, int relu, DropParams dp,
                                                     T* __restrict__ y, float* __restrict__ mean,
                                                     float* __restrict__ rstd) {
  __shared__ float red[BN_RG][BN_COLS];
  const int cl = threadIdx.x % BN_COLS, rg = threadIdx.x / BN_COLS;
  const int c = blockIdx.x * BN_COLS + cl;
  const bool ok = c < C;
  float mu, var;
  if (training) {
    float s = 0.f;
    if (ok) for (int r = rg; r < B; r += BN_RG) s += z[(int64_t)r * C + c];
    red[rg][cl] = s;
    __syncthreads();
    s = 0.f;
#pragma unroll
    for (int k = 0; k < BN_RG; ++k) s += red[k][cl];
    mu = s / (float)B;
    __syncthreads();
    float q = 0.f;
    if (ok) for (int r = rg; r < B; r += BN_RG) { const float d = z[(int64_t)r * C + c] - mu; q += d * d; }
    red[rg][cl] = q;
    __syncthreads();
    q = 0.f;
#pragma unroll
    for (int k = 0; k < BN_RG; ++k) q += red[k][cl];
    var = q / (float)B;
  } else {                                     // eval: running statistics, no update
    mu = ok ? running_mean[c] : 0.f;
    var = ok ? running_var[c] : 1.f;
  }
  const float rs = 1.f / sqrtf(var + eps);
  const DropKeys dk = resolve_drop(dp);
  if (ok) {
    const float wc = w[c], bc = b[c];
    for (int r = rg; r < B; r += BN_RG) {
      float o = (z[(int64_t)r * C + c] - mu) * rs * wc + bc;
      if (relu) o = fmaxf(o, 0.f);
      if (dk.on) o = drop_apply(dk, (uint32_t)((int64_t)r * C + c), o);
      stf<T>(y, (int64_t)r * C + c, o);
    }
    if (rg == 0) {
      if (mean) mean[c] = mu;
      if (rstd) rstd[c] = rs;
      if (training && running_mean)
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mu;
      if (training && running_var)
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * var * ((float)B / (float)(B - 1));
    }
  }
  if (training && nbt && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
}

template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_kernel(int B, int C, const float* __restrict__ dy,
                                                     const float* __restrict__ z,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd,
                                                     const T* __restrict__ y, float gate_scale,
                                                     int gated, float* __restrict__ dz,
                                                     float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float red[2][BN_RG][BN_COLS];
  const int cl = threadIdx.x % BN_COLS, rg = threadIdx.x / BN_COLS;
  const int c = blockIdx.x * BN_COLS + cl;
  const bool ok = c < C;
  const float mu = ok ? mean[c] : 0.f, rs = ok ? rstd[c] : 0.f, wc = ok ? w[c] : 0.f;
  float s1 = 0.f, s2 = 0.f;   // Σ dy', Σ dy'·x̂
  if (ok) {
    for (int r = rg; r < B; r += BN_RG) {
      const int64_t o = (int64_t)r * C + c;
      float d = dy[o];
      if (gated) d = ldf<T>(y, o) > 0.f ? d * gate_scale : 0.f;
      const float xh = (z[o] - mu) * rs;
      s1 += d;
      s2 += d * xh;
    }
  }
  red[0][rg][cl] = s1;
  red[1][rg][cl] = s2;
  __syncthreads();
  float S1 = 0.f, S2 = 0.f;
#pragma unroll
  for (int k = 0; k < BN_RG; ++k) { S1 += red[0][k][cl]; S2 += red[1][k][cl]; }
  if (!ok) return;
  const float invB = 1.f / (float)B;
  for (int r = rg; r < B; r += BN_RG) {
    const int64_t o = (int64_t)r * C + c;
    float d = dy[o];
    if (gated) d = ldf<T>(y, o) > 0.f ? d * gate_scale : 0.f;
    const float xh = (z[o] - mu) * rs;
    dz[o] = wc * rs * (d - S1 * invB - xh * S2 * invB);
  }
  if (rg == 0) {
    if (dw) atomicAdd(dw + c, S2);
    if (db) atomicAdd(db + c, S1);
  }
}

// Register-resident BatchNorm1d for B <= BNR_RG * RPT (the fusion / tabular heads, B = 256-512):
// 512 threads = BNR_COLS columns x BNR_RG row groups; every thread loads its RPT values of
// one column ONCE (all loads issued before any arithmetic), so the statistics, the
// normalisation and the backward's two sums cost one HBM latency instead of B / 16 serial
// dependent loads per pass.  Numerics equal the looped kernels (two-pass mean / variance).
constexpr int BNR_COLS = 8, BNR_RG = 64;     // 8 columns: twice the workgroups of 16 (C = 512: 64 CUs)

TTMI_DEV float bnr_colsum(float v, float (*red)[BNR_COLS], int rg, int cl) {
  __syncthreads();
  red[rg][cl] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < BNR_RG; ++k) s += red[k][cl];
  return s;
}

template <typename T, int RPT>
__global__ __launch_bounds__(512) void bnr_fwd_kernel(int B, int C, const float* __restrict__ z,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ b, float eps,
                                                      float momentum, float* running_mean,
                                                      float* running_var, int64_t* nbt, int relu,
                                                      DropParams dp, T* __restrict__ y,
                                                      float* __restrict__ mean,
                                                      float* __restrict__ rstd) {
  __shared__ float red[BNR_RG][BNR_COLS];
  const int cl = threadIdx.x % BNR_COLS, rg = threadIdx.x / BNR_COLS;
  const int c = blockIdx.x * BNR_COLS + cl;
  const int cc = min(c, C - 1);
  float v[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) v[j] = z[(int64_t)min(rg + BNR_RG * j, B - 1) * C + cc];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < RPT; ++j) s += rg + BNR_RG * j < B ? v[j] : 0.f;
  const float mu = bnr_colsum(s, red, rg, cl) / (float)B;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const float d = v[j] - mu;
    q += rg + BNR_RG * j < B ? d * d : 0.f;
  }
  const float var = bnr_colsum(q, red, rg, cl) / (float)B;
  const float rs = 1.f / sqrtf(var + eps);
  if (c >= C) return;
  const DropKeys dk = resolve_drop(dp);
  const float wc = w[c], bc = b[c];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int r = rg + BNR_RG * j;
    if (r < B) {
      float o = (v[j] - mu) * rs * wc + bc;
      if (relu) o = fmaxf(o, 0.f);
      if (dk.on) o = drop_apply(dk, (uint32_t)((int64_t)r * C + c), o);
      stf<T>(y, (int64_t)r * C + c, o);
    }
  }
  if (rg == 0) {
    if (mean) mean[c] = mu;
    if (rstd) rstd[c] = rs;
    if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mu;
    if (running_var)
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * var * ((float)B / (float)(B - 1));
  }
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
}

template <typename T, int RPT>
__global__ __launch_bounds__(512) void bnr_bwd_kernel(int B, int C, const float* __restrict__ dy,
                                                      const float* __restrict__ z,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ rstd,
                                                      const T* __restrict__ y, float gate_scale,
                                                      int gated, float* __restrict__ dz,
                                                      float* __restrict__ dw, float* __restrict__ db,
                                                      bf16_t* __restrict__ dz16) {
  __shared__ float red[BNR_RG][BNR_COLS];
  const int cl = threadIdx.x % BNR_COLS, rg = threadIdx.x / BNR_COLS;
  const int c = blockIdx.x * BNR_COLS + cl;
  const int cc = min(c, C - 1);
  float d[RPT], xh[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int64_t o = (int64_t)min(rg + BNR_RG * j, B - 1) * C + cc;
    d[j] = dy[o];
    xh[j] = z[o];
    if (gated) d[j] = ldf<T>(y, o) > 0.f ? d[j] * gate_scale : 0.f;
  }
  const float mu = mean[cc], rs = rstd[cc], wc = w[cc];
  float s1 = 0.f, s2 = 0.f;   // Σ dy', Σ dy'·x̂
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    xh[j] = (xh[j] - mu) * rs;
    if (rg + BNR_RG * j < B) {
      s1 += d[j];
      s2 += d[j] * xh[j];
    }
  }
  const float S1 = bnr_colsum(s1, red, rg, cl);
  const float S2 = bnr_colsum(s2, red, rg, cl);
  if (c >= C) return;
  const float invB = 1.f / (float)B;
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int r = rg + BNR_RG * j;
    if (r < B) {
      const float v = wc * rs * (d[j] - S1 * invB - xh[j] * S2 * invB);
      dz[(int64_t)r * C + c] = v;
      if (dz16) dz16[(int64_t)r * C + c] = f2bf(v);   // the next GEMM's bf16 operand
    }
  }
  if (rg == 0) {
    if (dw) atomicAdd(dw + c, S2);
    if (db) atomicAdd(db + c, S1);
  }
}

// rows-per-thread class of the register kernels for batch B (0: use the looped kernels)
int bnr_rpt(int B) { return B <= 4 * BNR_RG ? 4 : B <= 8 * BNR_RG ? 8 : B <= 16 * BNR_RG ? 16 : 0; }

// 4 rows (waves) per 256-thread block, one row per wave up to 2^20 blocks (grid-stride beyond):
// a row is a dependent load -> two wave reductions -> store chain, so rows in flight set the
// time (the round-2 cap of 2,048 blocks made each wave walk ~3 rows serially at M = 25,600)
int rows_grid(int64_t rows) {
  return (int)std::min<int64_t>(std::max<int64_t>((rows + 3) / 4, 1), (int64_t)1 << 20);
}

}  // namespace

extern "C" int ttmi_layernorm_fwd(int64_t M, int D, const float* x, int64_t ldx, const float* w,
                                  const float* b, float eps, int relu, float drop_p,
                                  const uint64_t* drop_seed, void* y, int y_dtype, int64_t ldy,
                                  float* mean, float* rstd, hipStream_t s) {
  TTMI_REQUIRE(M >= 0 && D > 0 && D <= 64 * MAXV, "ttmi_layernorm_fwd: need 0 < D <= %d", 64 * MAXV);
  TTMI_REQUIRE(x && w && b && y && ldx >= D && ldy >= D, "ttmi_layernorm_fwd: bad args");
  TTMI_REQUIRE(y_dtype == TTMI_F32 || y_dtype == TTMI_BF16, "ttmi_layernorm_fwd: bad dtype");
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "ttmi_layernorm_fwd: drop_p out of [0,1)");
  if (M == 0) return TTMI_OK;
  DropParams dp = make_drop(drop_p, drop_seed);
  TTMI_NV_DISPATCH(D, {
    if (y_dtype == TTMI_BF16)
      hipLaunchKernelGGL((ln_fwd_kernel<bf16_t, NV>), dim3(rows_grid(M)), dim3(256), 0, s, M, D, x, ldx,
                         w, b, eps, relu, dp, (bf16_t*)y, ldy, mean, rstd);
    else
      hipLaunchKernelGGL((ln_fwd_kernel<float, NV>), dim3(rows_grid(M)), dim3(256), 0, s, M, D, x, ldx,
                         w, b, eps, relu, dp, (float*)y, ldy, mean, rstd);
  });
  return ttmi_check_launch("ttmi_layernorm_fwd");
}

extern "C" int64_t ttmi_layernorm_bwd_workspace(int D) {
  return (int64_t)LN_REPL * 2 * D * (int64_t)sizeof(int64_t);
}

extern "C" int ttmi_layernorm_bwd_folds(int D, void* ws, float* dw, float* db, ttmi_fold_desc* out) {
  TTMI_REQUIRE(D > 0 && D % 4 == 0 && ws && out, "ttmi_layernorm_bwd_folds: bad arguments");
  int n = 0;
  float* dst[2] = {dw, db};
  for (int j = 0; j < 2; ++j) {
    if (!dst[j]) continue;
    ttmi_fold_desc& f = out[n++];
    f.part = static_cast<int64_t*>(ws) + (int64_t)j * D;
    f.S = LN_REPL; f.s_stride = 2 * (int64_t)D; f.M = 1; f.N = D;
    f.C = dst[j]; f.ldc = D; f.accumulate = 3; f.fx_shift = TTMI_FX_GRAD;
  }
  return TTMI_OK;
}

extern "C" int ttmi_layernorm_bwd(int64_t M, int D, const float* dy, int64_t lddy, const float* x,
                                  int64_t ldx, const float* mean, const float* rstd,
                                  const float* w, const void* gate, int gate_dtype, int64_t ldg,
                                  float gate_scale, const float* res, float* dx, int64_t lddx,
                                  float* dw, float* db, void* ws, void* dx16, int64_t ld16,
                                  float drop_p, const uint64_t* drop_seed, int defer, hipStream_t s) {
  TTMI_REQUIRE(M >= 0 && D > 0 && D <= 64 * MAXV, "ttmi_layernorm_bwd: need 0 < D <= %d", 64 * MAXV);
  TTMI_REQUIRE(dy && x && mean && rstd && w && dx, "ttmi_layernorm_bwd: null argument");
  TTMI_REQUIRE(lddy >= D && ldx >= D && lddx >= D && (!gate || ldg >= D), "ttmi_layernorm_bwd: bad ld");
  TTMI_REQUIRE(!(dw || db) || ws, "ttmi_layernorm_bwd: dw/db need the workspace");
  TTMI_REQUIRE(!dx16 || ld16 >= D, "ttmi_layernorm_bwd: ld16 < D");
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || (dx16 && drop_seed)),
               "ttmi_layernorm_bwd: dropout applies to dx16 and needs a seed");
  const DropParams dp16 = make_drop(drop_p, drop_seed);
  if (M == 0) return TTMI_OK;
  const bool sums = dw || db;
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!sums && !gate && D % 256 == 0 && D <= 1024 && lddy % 4 == 0 && ldx % 4 == 0 &&
      lddx % 4 == 0 && al16(dy) && al16(x) && al16(w) && al16(dx) && (!res || al16(res)) &&
      (!dx16 || (((uintptr_t)dx16 & 7) == 0 && ld16 % 4 == 0))) {
    const dim3 vg((unsigned)((M + 3) / 4));
    switch (D / 256) {
      case 1: hipLaunchKernelGGL(ln_bwd_vec_kernel<1>, vg, dim3(256), 0, s, M, D, dy, lddy, x, ldx, mean, rstd, w, res, dx, lddx, (bf16_t*)dx16, ld16, dp16); break;
      case 2: hipLaunchKernelGGL(ln_bwd_vec_kernel<2>, vg, dim3(256), 0, s, M, D, dy, lddy, x, ldx, mean, rstd, w, res, dx, lddx, (bf16_t*)dx16, ld16, dp16); break;
      case 3: hipLaunchKernelGGL(ln_bwd_vec_kernel<3>, vg, dim3(256), 0, s, M, D, dy, lddy, x, ldx, mean, rstd, w, res, dx, lddx, (bf16_t*)dx16, ld16, dp16); break;
      default: hipLaunchKernelGGL(ln_bwd_vec_kernel<4>, vg, dim3(256), 0, s, M, D, dy, lddy, x, ldx, mean, rstd, w, res, dx, lddx, (bf16_t*)dx16, ld16, dp16); break;
    }
    return ttmi_check_launch("ttmi_layernorm_bwd");
  }
  // one row per wave when there are no column sums (the frozen text-encoder LayerNorms:
  // a wave walking 16 rows serially ran the stream at ~2.9 TB/s); with sums, 1024 blocks
  // bound the replicas' adders.  The column sums go to LN_REPL int64 fixed-point replica
  // rows (ws [LN_REPL][2][D]; order-independent) folded once: deterministic.
  int grid = (int)std::min<int64_t>((M + 3) / 4, sums ? 1024 : 16384);
  int64_t* cw = sums ? static_cast<int64_t*>(ws) : nullptr;
  int64_t* cb = sums ? static_cast<int64_t*>(ws) + D : nullptr;
  TTMI_NV_DISPATCH(D, hipLaunchKernelGGL((ln_bwd_kernel<NV>), dim3(grid), dim3(256), 0, s, M, D, dy,
                                         lddy, x, ldx, mean, rstd, w, gate, gate_dtype == TTMI_F32,
                                         ldg, gate_scale, res, dx, lddx, cw, cb, LN_REPL, 2 * (int64_t)D,
                                         (bf16_t*)dx16, ld16, dp16));
  int rc = ttmi_check_launch("ttmi_layernorm_bwd");
  if (rc || !sums || defer) return rc;      // defer: the caller folds (ttmi_layernorm_bwd_folds)
  hipLaunchKernelGGL(colsum_fold_kernel, dim3((2 * D + 255) / 256), dim3(256), 0, s, 2 * D, D,
                     LN_REPL, static_cast<int64_t*>(ws), dw, db);
  return ttmi_check_launch("ttmi_layernorm_bwd/fold");
}

extern "C" int ttmi_seq_embed_fwd(int B, int L, int D, const int64_t* ids, const float* E, int64_t V,
                                  const float* P, const float* w, const float* b, float eps,
                                  float drop_p, const uint64_t* drop_seed, float* x, float* mean,
                                  float* rstd, const float* w1, const float* b1, float eps1, void* y1,
                                  float* mean1, float* rstd1, int32_t* id_err, hipStream_t s) {
  TTMI_REQUIRE(B >= 0 && L > 0 && D > 0 && D <= 64 * MAXV, "ttmi_seq_embed_fwd: bad sizes");
  TTMI_REQUIRE(ids && E && P && w && b && x && mean && rstd, "ttmi_seq_embed_fwd: null argument");
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "ttmi_seq_embed_fwd: drop_p out of [0,1)");
  const bool ln2 = y1 != nullptr;
  TTMI_REQUIRE(!ln2 || (w1 && b1 && mean1 && rstd1), "ttmi_seq_embed_fwd: norm1 needs w1, b1, mean1, rstd1");
  if (B == 0) return TTMI_OK;
  const DropParams dp = make_drop(drop_p, drop_seed);
  // one row per wave (rows_grid): a row is a dependent chain ids -> E[id] -> two wave
  // reductions -> stores.  TTMI_SEQ_GRID=cap caps the grid (A/B runs only; 2048 = round 2)
  static const int64_t cap = [] {
    const char* e = getenv("TTMI_SEQ_GRID");
    return e ? (int64_t)atoll(e) : (int64_t)1 << 20;
  }();
  const int64_t M = (int64_t)B * L;
  static const int vec = [] {                        // TTMI_SEQ_VEC=0: the row-per-wave kernel (A/B)
    const char* e = getenv("TTMI_SEQ_VEC");
    return e ? atoi(e) : 1;
  }();
  const bool al = (((uintptr_t)E | (uintptr_t)P | (uintptr_t)w | (uintptr_t)b | (uintptr_t)x |
                    (uintptr_t)(ln2 ? w1 : w) | (uintptr_t)(ln2 ? b1 : b)) & 15) == 0 &&
                  (!ln2 || ((uintptr_t)y1 & 7) == 0);
  if (vec && al && (D == 128 || D == 256)) {
#ifndef TTMI_SEQ_U
#define TTMI_SEQ_U 2
#endif
    constexpr int U = TTMI_SEQ_U;                    // row groups in flight per wave
    const int rpw = D == 128 ? 2 : 1;
    const int64_t waves = (M + U * rpw - 1) / (U * rpw);
    const dim3 g((unsigned)std::min<int64_t>((waves + 3) / 4, cap));
#define TTMI_SEQV(DD, LN) hipLaunchKernelGGL((seq_embed_fwd_vec_kernel<DD, LN, U>), g, dim3(256), 0, s, B, L, ids, E, V, P, \
                                             w, b, eps, dp, x, mean, rstd, w1, b1, eps1, (bf16_t*)y1, mean1, rstd1, id_err)
    if (D == 128) { if (ln2) TTMI_SEQV(128, true); else TTMI_SEQV(128, false); }
    else { if (ln2) TTMI_SEQV(256, true); else TTMI_SEQV(256, false); }
#undef TTMI_SEQV
    return ttmi_check_launch("ttmi_seq_embed_fwd");
  }
  const dim3 grid((unsigned)std::min<int64_t>(rows_grid(M), cap));
  TTMI_NV_DISPATCH(D, {
    if (ln2)
      hipLaunchKernelGGL((seq_embed_fwd_kernel<NV, true>), grid, dim3(256), 0, s, B, L, D, ids, E, V, P,
                         w, b, eps, dp, x, mean, rstd, w1, b1, eps1, (bf16_t*)y1, mean1, rstd1, id_err);
    else
      hipLaunchKernelGGL((seq_embed_fwd_kernel<NV, false>), grid, dim3(256), 0, s, B, L, D, ids, E, V, P,
                         w, b, eps, dp, x, mean, rstd, nullptr, nullptr, 0.f, nullptr, nullptr, nullptr, id_err);
  });
  return ttmi_check_launch("ttmi_seq_embed_fwd");
}

extern "C" int64_t ttmi_seq_embed_bwd_workspace(int64_t V, int L, int D) {
  if (V <= 0 || L <= 0 || D <= 0) return 0;
  return ((int64_t)V * D + 3 * (int64_t)L * D) * (int64_t)sizeof(int64_t);
}

extern "C" int ttmi_seq_embed_bwd_folds(int64_t V, int L, int D, void* ws, float* dE, float* dP,
                                        float* dw, float* db, ttmi_fold_desc* out) {
  TTMI_REQUIRE(V > 0 && L > 0 && D > 0 && D % 4 == 0 && ws && dE && dP && dw && db && out,
               "ttmi_seq_embed_bwd_folds: bad arguments (D %% 4 == 0)");
  int64_t* accE = static_cast<int64_t*>(ws);
  int64_t* accL = accE + V * D;
  const int64_t LD = (int64_t)L * D;
  auto set = [&](ttmi_fold_desc& f, const int64_t* part, int64_t S, int64_t ss, int64_t M, float* C) {
    f.part = part; f.S = S; f.s_stride = ss; f.M = M; f.N = D; f.C = C; f.ldc = D;
    f.accumulate = 3; f.fx_shift = TTMI_FX_GRAD;      // add, and leave the accumulators zero
  };
  set(out[0], accE, 1, V * D, V, dE);
  set(out[1], accL, 1, LD, L, dP);
  set(out[2], accL + LD, L, D, 1, dw);
  set(out[3], accL + 2 * LD, L, D, 1, db);
  return TTMI_OK;
}

extern "C" int ttmi_seq_embed_bwd(int B, int L, int D, int64_t V, const int64_t* ids, const float* E,
                                  const float* P, const float* w, const float* mean,
                                  const float* rstd, float drop_p, const uint64_t* drop_seed,
                                  const float* dx, float* dE, float* dP, float* dw, float* db,
                                  int64_t padding_idx, void* ws, int defer, hipStream_t s) {
  TTMI_REQUIRE(B >= 0 && L > 0 && D > 0 && D <= 64 * MAXV && D % 4 == 0 && V > 0,
               "ttmi_seq_embed_bwd: bad sizes (D %% 4 == 0)");
  TTMI_REQUIRE(ids && E && P && w && mean && rstd && dx && dE && dP && dw && db && ws,
               "ttmi_seq_embed_bwd: null argument");
  TTMI_REQUIRE(((uintptr_t)ws & 15) == 0, "ttmi_seq_embed_bwd: ws must be 16-byte aligned");
  if (B > 0) {
    // SEB_R passes of two rows per wave (SEB_R = 4: 800 blocks at B = 512, L = 50)
    const int bpc = 2 * SEB_R * SEB_W;
    dim3 grid(L, (B + bpc - 1) / bpc);
    int64_t* accE = static_cast<int64_t*>(ws);
    TTMI_NV_DISPATCH(D, hipLaunchKernelGGL((seq_embed_bwd_kernel<NV>), grid, dim3(64 * SEB_W), 0, s, B, L, D, ids,
                                           E, P, w, mean, rstd, make_drop(drop_p, drop_seed), dx, accE,
                                           accE + V * D, padding_idx, V, bpc));
    const int rc = ttmi_check_launch("ttmi_seq_embed_bwd");
    if (rc) return rc;
  }
  if (defer) return TTMI_OK;            // the caller folds (ttmi_seq_embed_bwd_folds)
  ttmi_fold_desc f[4];
  int rc = ttmi_seq_embed_bwd_folds(V, L, D, ws, dE, dP, dw, db, f);
  if (rc) return rc;
  return ttmi_wgrad_fold(0, nullptr, 4, f, s);
}

extern "C" int ttmi_user_concat_fwd(int dtype, int B, int L, int D, const float* x,
                                    const int64_t* len_src, const int64_t* gender, const float* G,
                                    int dg, const int64_t* country, const float* C, int dc,
                                    void* comb, int32_t* rows, int n_genders, int n_countries,
                                    int32_t* id_err, hipStream_t s) {
  TTMI_REQUIRE(dtype == TTMI_F32 || dtype == TTMI_BF16, "ttmi_user_concat_fwd: bad dtype");
  TTMI_REQUIRE(B >= 0 && L > 0 && D > 0 && dg >= 0 && dc >= 0 && n_genders > 0 && n_countries > 0,
               "ttmi_user_concat_fwd: bad sizes");
  TTMI_REQUIRE(x && gender && country && comb && rows && (dg == 0 || G) && (dc == 0 || C),
               "ttmi_user_concat_fwd: null argument");
  TTMI_REQUIRE(len_src || L == 1, "ttmi_user_concat_fwd: len_src == NULL needs L == 1");
  if (B == 0) return TTMI_OK;
  dim3 grid((B + 3) / 4);
  if (dtype == TTMI_BF16)
    hipLaunchKernelGGL(user_concat_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, B, L, D, x, len_src,
                       gender, G, dg, country, C, dc, (bf16_t*)comb, rows, n_genders, n_countries, id_err);
  else
    hipLaunchKernelGGL(user_concat_fwd_kernel<float>, grid, dim3(256), 0, s, B, L, D, x, len_src,
                       gender, G, dg, country, C, dc, (float*)comb, rows, n_genders, n_countries, id_err);
  return ttmi_check_launch("ttmi_user_concat_fwd");
}

extern "C" int ttmi_user_concat_bwd(int B, int D, const float* dcomb, const int32_t* rows,
                                    const int64_t* gender, int dg, const int64_t* country, int dc,
                                    float* dx, int64_t* dG, int64_t* dC, int accumulate,
                                    int n_genders, int n_countries, hipStream_t s) {
  TTMI_REQUIRE(B >= 0 && D > 0 && dg >= 0 && dc >= 0 && n_genders > 0 && n_countries > 0,
               "ttmi_user_concat_bwd: bad sizes");
  TTMI_REQUIRE(dcomb && rows && gender && country && dx, "ttmi_user_concat_bwd: null argument");
  if (B == 0) return TTMI_OK;
  hipLaunchKernelGGL(user_concat_bwd_kernel, dim3((B + 3) / 4), dim3(256), 0, s, B, D, dcomb, rows,
                     gender, dg, country, dc, dx, dG, dC, accumulate, n_genders, n_countries);
  return ttmi_check_launch("ttmi_user_concat_bwd");
}

extern "C" int ttmi_batchnorm_fwd(int dtype, int B, int C, const float* z, const float* w,
                                  const float* b, float eps, float momentum, float* running_mean,
                                  float* running_var, int64_t* num_batches_tracked, int training,
                                  int relu, float drop_p, const uint64_t* drop_seed, void* y,
                                  float* mean, float* rstd, hipStream_t s) {
  TTMI_REQUIRE(dtype == TTMI_F32 || dtype == TTMI_BF16, "ttmi_batchnorm_fwd: bad dtype");
  TTMI_REQUIRE(C > 0 && B >= 0, "ttmi_batchnorm_fwd: bad sizes");
  TTMI_REQUIRE(!training || B > 1,
               "ttmi_batchnorm_fwd: expected more than 1 value per channel when training");
  TTMI_REQUIRE(training || (running_mean && running_var), "ttmi_batchnorm_fwd: eval needs running stats");
  TTMI_REQUIRE(z && w && b && y, "ttmi_batchnorm_fwd: null argument");
  if (B == 0) return TTMI_OK;
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "ttmi_batchnorm_fwd: drop_p out of [0,1)");
  DropParams dp = make_drop(drop_p, drop_seed);
  const int rpt = training ? bnr_rpt(B) : 0;
  if (rpt) {
    const dim3 g((C + BNR_COLS - 1) / BNR_COLS);
#define TTMI_BNR_FWD(T, R)                                                                          \
  hipLaunchKernelGGL((bnr_fwd_kernel<T, R>), g, dim3(512), 0, s, B, C, z, w, b, eps, momentum,      \
                     running_mean, running_var, num_batches_tracked, relu, dp, (T*)y, mean, rstd)
    if (dtype == TTMI_BF16) {
      if (rpt == 4) TTMI_BNR_FWD(bf16_t, 4); else if (rpt == 8) TTMI_BNR_FWD(bf16_t, 8); else TTMI_BNR_FWD(bf16_t, 16);
    } else {
      if (rpt == 4) TTMI_BNR_FWD(float, 4); else if (rpt == 8) TTMI_BNR_FWD(float, 8); else TTMI_BNR_FWD(float, 16);
    }
#undef TTMI_BNR_FWD
    return ttmi_check_launch("ttmi_batchnorm_fwd");
  }
  dim3 grid((C + BN_COLS - 1) / BN_COLS);
  if (dtype == TTMI_BF16)
    hipLaunchKernelGGL(bn_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, B, C, z, w, b, eps, momentum,
                       running_mean, running_var, num_batches_tracked, training, relu, dp, (bf16_t*)y, mean, rstd);
  else
    hipLaunchKernelGGL(bn_fwd_kernel<float>, grid, dim3(256), 0, s, B, C, z, w, b, eps, momentum,
                       running_mean, running_var, num_batches_tracked, training, relu, dp, (float*)y, mean, rstd);
  return ttmi_check_launch("ttmi_batchnorm_fwd");
}

extern "C" int ttmi_batchnorm_bwd(int dtype, int B, int C, const float* dy, const float* z,
                                  const float* w, const float* mean, const float* rstd,
                                  const void* y, float gate_scale, int gated, float* dz, float* dw,
                                  float* db, void* dz16, hipStream_t s) {
  TTMI_REQUIRE(dtype == TTMI_F32 || dtype == TTMI_BF16, "ttmi_batchnorm_bwd: bad dtype");
  TTMI_REQUIRE(B > 1 && C > 0, "ttmi_batchnorm_bwd: bad sizes");
  TTMI_REQUIRE(dy && z && w && mean && rstd && dz && (!gated || y), "ttmi_batchnorm_bwd: null argument");
  TTMI_REQUIRE(!dz16 || bnr_rpt(B), "ttmi_batchnorm_bwd: the bf16 copy needs B <= %d", 16 * BNR_RG);
  if (const int rpt = bnr_rpt(B)) {
    const dim3 g((C + BNR_COLS - 1) / BNR_COLS);
#define TTMI_BNR_BWD(T, R)                                                                          \
  hipLaunchKernelGGL((bnr_bwd_kernel<T, R>), g, dim3(512), 0, s, B, C, dy, z, w, mean, rstd,        \
                     (const T*)y, gate_scale, gated, dz, dw, db, (bf16_t*)dz16)
    if (dtype == TTMI_BF16) {
      if (rpt == 4) TTMI_BNR_BWD(bf16_t, 4); else if (rpt == 8) TTMI_BNR_BWD(bf16_t, 8); else TTMI_BNR_BWD(bf16_t, 16);
    } else {
      if (rpt == 4) TTMI_BNR_BWD(float, 4); else if (rpt == 8) TTMI_BNR_BWD(float, 8); else TTMI_BNR_BWD(float, 16);
    }
#undef TTMI_BNR_BWD
    return ttmi_check_launch("ttmi_batchnorm_bwd");
  }
  dim3 grid((C + BN_COLS - 1) / BN_COLS);
  if (dtype == TTMI_BF16)
    hipLaunchKernelGGL(bn_bwd_kernel<bf16_t>, grid, dim3(256), 0, s, B, C, dy, z, w, mean, rstd,
                       (const bf16_t*)y, gate_scale, gated, dz, dw, db);
  else
    hipLaunchKernelGGL(bn_bwd_kernel<float>, grid, dim3(256), 0, s, B, C, dy, z, w, mean, rstd,
                       (const float*)y, gate_scale, gated, dz, dw, db);
  return ttmi_check_launch("ttmi_batchnorm_bwd");
}

TTMI_STAMP_DUMP(norm)
