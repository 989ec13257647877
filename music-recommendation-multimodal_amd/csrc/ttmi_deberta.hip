// ttmi_deberta.hip — the mDeBERTa-v3 text encoder of the cfg-4 item tower (reference
// src/models/item_tower.py:41-83: DebertaV2Model + peft LoRA + masked mean-pool).
//
//   deb_embed_fwd   word-embedding gather + LayerNorm + mask + dropout (DebertaV2Embeddings)
//   deb_ln_fwd      post-LayerNorm of the residual sum, fp32 copy (next residual) + bf16 operand
//   (the disentangled self-attention itself lives in ttmi_disattn.hip)
//   deb_pool_fwd/bwd masked mean-pool (item_tower.py:73-80, clamp 1e-9).
#include "ttmi_common.h"

namespace {

// ---------------------------------------------------------------- embeddings + LayerNorm
// One wave per token row: y = LN(E[id]) · mask (· dropout); fp32 copy (residual) and bf16
// copy (GEMM operand, row stride ld16).  H % 64 == 0, H <= 1024.
__global__ __launch_bounds__(256) void deb_embed_kernel(int64_t M, int H, const int64_t* __restrict__ ids,
                                                        const bf16_t* __restrict__ table,
                                                        const float* __restrict__ lw,
                                                        const float* __restrict__ lb, float eps,
                                                        const int64_t* __restrict__ mask,
                                                        DropParams drop, float* __restrict__ y32,
                                                        bf16_t* __restrict__ y16, int64_t ld16,
                                                        int64_t V, int32_t* __restrict__ id_err) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const DropKeys dk = resolve_drop(drop);
  const int per = H / 64;                                  // <= 16 values per lane
  float v[16];
  const bf16_t* src = table + clamp_id(ids[row], V, id_err, TTMI_IDERR_TEXT) * (int64_t)H;
  float s = 0.f;
  for (int e = 0; e < per; ++e) { v[e] = bf2f(src[e * 64 + lane]); s += v[e]; }
  for (int off = 32; off; off >>= 1) s += __shfl_xor(s, off, 64);
  const float mu = s / H;
  float q = 0.f;
  for (int e = 0; e < per; ++e) { const float d = v[e] - mu; q += d * d; }
  for (int off = 32; off; off >>= 1) q += __shfl_xor(q, off, 64);
  const float rs = rsqrtf(q / H + eps);
  const float mk = mask ? (mask[row] != 0 ? 1.f : 0.f) : 1.f;
  for (int e = 0; e < per; ++e) {
    const int c = e * 64 + lane;
    float o = ((v[e] - mu) * rs * lw[c] + lb[c]) * mk;
    o = drop_apply(dk, (uint32_t)(row * H + c), o);
    if (y32) y32[row * H + c] = o;
    y16[row * ld16 + c] = f2bf(o);
  }
}

// Post-LayerNorm: y = LN(z) -> y32 (fp32, may be NULL) and y16 (bf16, stride ld16); saves
// mean / rstd for the backward.
__global__ __launch_bounds__(256) void deb_ln_kernel(int64_t M, int H, const float* __restrict__ z,
                                                     const float* __restrict__ lw,
                                                     const float* __restrict__ lb, float eps,
                                                     float* __restrict__ y32, bf16_t* __restrict__ y16,
                                                     int64_t ld16, float* __restrict__ mean,
                                                     float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int per = H / 64;
  float v[16];
  float s = 0.f;
  for (int e = 0; e < per; ++e) { v[e] = z[row * H + e * 64 + lane]; s += v[e]; }
  for (int off = 32; off; off >>= 1) s += __shfl_xor(s, off, 64);
  const float mu = s / H;
  float q = 0.f;
  for (int e = 0; e < per; ++e) { const float d = v[e] - mu; q += d * d; }
  for (int off = 32; off; off >>= 1) q += __shfl_xor(q, off, 64);
  const float rs = rsqrtf(q / H + eps);
  for (int e = 0; e < per; ++e) {
    const int c = e * 64 + lane;
    const float o = (v[e] - mu) * rs * lw[c] + lb[c];
    if (y32) y32[row * H + c] = o;
    if (y16) y16[row * ld16 + c] = f2bf(o);
  }
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
}

// The same for H % 256 == 0 (H = 768): each lane owns 4 consecutive columns per 16-byte
// access, Q4 = H/256 of them (the 4-byte-per-lane form above streams at ~3.3 TB/s).
template <int Q4>
__global__ __launch_bounds__(256) void deb_ln_vec_kernel(int64_t M, int H, const float* __restrict__ z,
                                                         const float* __restrict__ lw,
                                                         const float* __restrict__ lb, float eps,
                                                         float* __restrict__ y32, bf16_t* __restrict__ y16,
                                                         int64_t ld16, float* __restrict__ mean,
                                                         float* __restrict__ rstd,
                                                         bf16_t* __restrict__ yq, bf16_t* __restrict__ yv,
                                                         DropParams dq, DropParams dv) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const DropKeys kq = resolve_drop(dq), kv = resolve_drop(dv);
  float4 v[Q4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < Q4; ++i) {
    v[i] = *reinterpret_cast<const float4*>(z + row * H + (lane + 64 * i) * 4);
    s += v[i].x + v[i].y + v[i].z + v[i].w;
  }
  const float mu = wave_sum(s) / H;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < Q4; ++i) {
    const float a = v[i].x - mu, b = v[i].y - mu, c = v[i].z - mu, d = v[i].w - mu;
    q += a * a + b * b + c * c + d * d;
  }
  const float rs = rsqrtf(wave_sum(q) / H + eps);
#pragma unroll
  for (int i = 0; i < Q4; ++i) {
    const int c = (lane + 64 * i) * 4;
    const float4 w = *reinterpret_cast<const float4*>(lw + c), b = *reinterpret_cast<const float4*>(lb + c);
    const float4 o = make_float4((v[i].x - mu) * rs * w.x + b.x, (v[i].y - mu) * rs * w.y + b.y,
                                 (v[i].z - mu) * rs * w.z + b.z, (v[i].w - mu) * rs * w.w + b.w);
    if (y32) *reinterpret_cast<float4*>(y32 + row * H + c) = o;
    if (y16) {
      ushort4 h;
      h.x = f2bf(o.x); h.y = f2bf(o.y); h.z = f2bf(o.z); h.w = f2bf(o.w);
      *reinterpret_cast<ushort4*>(y16 + row * ld16 + c) = h;
    }
    // the next layer's LoRA inputs bf16(drop_q(y)), bf16(drop_v(y)) (keep index row*H + c, as
    // ttmi_dropout_bwd's): two more outputs of the row already in registers
    if (yq) {
      float4 a = o;
      drop_apply_vec<4>(kq, (uint32_t)(row * H + c), &a.x);
      ushort4 h;
      h.x = f2bf(a.x); h.y = f2bf(a.y); h.z = f2bf(a.z); h.w = f2bf(a.w);
      *reinterpret_cast<ushort4*>(yq + row * H + c) = h;
    }
    if (yv) {
      float4 a = o;
      drop_apply_vec<4>(kv, (uint32_t)(row * H + c), &a.x);
      ushort4 h;
      h.x = f2bf(a.x); h.y = f2bf(a.y); h.z = f2bf(a.z); h.w = f2bf(a.w);
      *reinterpret_cast<ushort4*>(yv + row * H + c) = h;
    }
  }
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
}

// ---------------------------------------------------------------- masked mean-pool
// Valid-token count of sequence b (block-wide; every thread gets it).
TTMI_DEV float pool_count(int S, const int64_t* __restrict__ mrow) {
  int n = 0;
  for (int s0 = 0; s0 < S; s0 += blockDim.x) {
    const int s = s0 + threadIdx.x;
    n += __syncthreads_count(s < S && mrow[s] != 0);
  }
  return (float)n;
}

// out[b, :] = Σ_{s: mask} x[b, s, :] / count.  Block (b, 256-column chunk): 64 lanes x 4
// columns (float4) x 4 row groups; every row load of a thread is independent (no serial
// dependent chain over S: the one-thread-per-column version took 341 µs at B=256, S=256),
// and the 4 partials meet in LDS.
constexpr int POOL_MAXS = 4096;
__global__ __launch_bounds__(256) void deb_pool_fwd_kernel(int S, int H, const float* __restrict__ x,
                                                           const int64_t* __restrict__ mask,
                                                           float* __restrict__ out) {
  __shared__ unsigned char smk[POOL_MAXS];
  __shared__ float4 red[4][64];
  const int b = blockIdx.x, lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int64_t* mrow = mask + (int64_t)b * S;
  for (int s = threadIdx.x; s < S; s += blockDim.x) smk[s] = mrow[s] != 0;
  const float inv = 1.f / fmaxf(pool_count(S, mrow), 1e-9f);   // (its barriers publish smk)
  const int c = (blockIdx.y * 64 + lane) * 4;
  const bool cok = c < H;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (cok) {
    const float* xb = x + (int64_t)b * S * H + c;
    for (int s = rg; s < S; s += 4)
      if (smk[s]) {
        const float4 v = *reinterpret_cast<const float4*>(xb + (int64_t)s * H);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
  }
  red[rg][lane] = acc;
  __syncthreads();
  if (rg != 0 || !cok) return;
  float4 t = red[0][lane];
#pragma unroll
  for (int g = 1; g < 4; ++g) {
    const float4 u = red[g][lane];
    t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
  }
  *reinterpret_cast<float4*>(out + (int64_t)b * H + c) = make_float4(t.x * inv, t.y * inv, t.z * inv, t.w * inv);
}

// dx[b, s, :] = mask ? dout[b, :] / count : 0.  Block (b, 16 rows), float4 stores (the
// one-block-per-row version recounted the mask serially per row: 633 µs).
constexpr int POOL_BWD_ROWS = 16;
__global__ __launch_bounds__(256) void deb_pool_bwd_kernel(int S, int H, const float* __restrict__ dout,
                                                           const int64_t* __restrict__ mask,
                                                           float* __restrict__ dx) {
  const int b = blockIdx.x;
  const int64_t* mrow = mask + (int64_t)b * S;
  const float inv = 1.f / fmaxf(pool_count(S, mrow), 1e-9f);
  const int s0 = blockIdx.y * POOL_BWD_ROWS, H4 = H / 4;
  for (int i = threadIdx.x; i < POOL_BWD_ROWS * H4; i += blockDim.x) {
    const int s = s0 + i / H4, c = (i % H4) * 4;
    if (s >= S) break;
    const float m = mrow[s] != 0 ? inv : 0.f;
    const float4 d = *reinterpret_cast<const float4*>(dout + (int64_t)b * H + c);
    *reinterpret_cast<float4*>(dx + ((int64_t)b * S + s) * H + c) = make_float4(d.x * m, d.y * m, d.z * m, d.w * m);
  }
}

// h = GELU(pre), bf16 -> bf16, 8 elements per thread (DebertaV2Intermediate activation; the
// pre-activation is kept for the backward's GELU' epilogue).
__global__ __launch_bounds__(256) void deb_gelu_kernel(int64_t n8, const bf16_t* __restrict__ x,
                                                       bf16_t* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float v[8];
    unpack8(reinterpret_cast<const uint4*>(x)[i], v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
    reinterpret_cast<uint4*>(y)[i] = pack8(v);
  }
}

// ---------------------------------------------------------------- rank-8 LoRA gradients
// Skinny weight gradient (the LoRA A/B gradients of the cfg-4 text encoder, item_tower.py:
// 51-59 under peft): C(m, c) += alpha · Σ_r W[r, m] · S[r, soff(m) + c] for m < Mw, c < 8,
// r < R, where W (bf16, row stride ldw) is the wide operand (768 columns) and S (bf16 or
// fp32, row stride lds) the rank-8 one; soff(m) = (m / group) · sgs selects a per-head slice
// (group = 64, sgs = 8 for the relative-path Bq contraction; group = Mw for plain dB/dA).
// C element (m, c) sits at m·ldc_m + c·ldc_c.  R is long (B·S = 65,536) and the output tiny
// (768 x 8), so this is an HBM stream of W: each thread owns 8 consecutive W columns (16-byte
// loads, 64 fp32 accumulators) over a strided row set; RG row groups of Mw/8 threads per block
// (768 threads at Mw 768) are added in turn into one LDS tile and every block adds its 24 KB
// partial with contiguous int64 fixed-point atomics (deterministic), converted into C by a
// second tiny launch.  One block per CU: the per-thread row walk is the latency chain, the
// atomics (blocks x 48 KB at ~1.3 TB/s) the other cost.  The generic tile path
// spent ~260 us per call here padding the rank-8 side to 64.
template <typename TS, int U>
__global__ __launch_bounds__(1024) void skinny_wgrad_kernel(int64_t R, int Mw, const bf16_t* __restrict__ W,
                                                            int64_t ldw, const TS* __restrict__ S,
                                                            int64_t lds, int group, int sgs, float alpha,
                                                            int64_t* __restrict__ cacc, int64_t ldc_m,
                                                            int64_t ldc_c, int64_t rows_per_block) {
  extern __shared__ float red[];                       // [Mw·8], the row groups added in turn
  const int ncol8 = Mw / 8, RG = blockDim.x / ncol8;   // blockDim.x = RG·ncol8
  const int t = threadIdx.x, rg = t / ncol8, c8 = t % ncol8;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(R, r0 + rows_per_block);
  float acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[i][c] = 0.f;
  {
    const int soff = (c8 * 8 / group) * sgs;
    // U rows per step: all loads issued before the FMAs (the loop is load-latency bound)
    for (int64_t rb = r0 + rg; rb < r1; rb += U * RG) {
      uint4 wq[U], sq[U], sq2[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int64_t r = min(rb + k * RG, r1 - 1);
        wq[k] = *reinterpret_cast<const uint4*>(W + r * ldw + c8 * 8);
        sq[k] = *reinterpret_cast<const uint4*>(S + r * lds + soff);
        if constexpr (sizeof(TS) == 4) sq2[k] = *reinterpret_cast<const uint4*>(S + r * lds + soff + 4);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (rb + k * RG >= r1) break;
        float w[8], s[8];
        unpack8(wq[k], w);
        if constexpr (sizeof(TS) == 2) {
          unpack8(sq[k], s);
        } else {
          s[0] = __uint_as_float(sq[k].x); s[1] = __uint_as_float(sq[k].y);
          s[2] = __uint_as_float(sq[k].z); s[3] = __uint_as_float(sq[k].w);
          s[4] = __uint_as_float(sq2[k].x); s[5] = __uint_as_float(sq2[k].y);
          s[6] = __uint_as_float(sq2[k].z); s[7] = __uint_as_float(sq2[k].w);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int c = 0; c < 8; ++c) acc[i][c] += w[i] * s[c];
      }
    }
  }
  float* dst = red + c8 * 64;
  for (int g = 0; g < RG; ++g) {                       // fixed order: deterministic per block
    if (rg == g) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int c = 0; c < 8; c += 4) {
          float4* p = reinterpret_cast<float4*>(dst + i * 8 + c);
          float4 v = make_float4(acc[i][c], acc[i][c + 1], acc[i][c + 2], acc[i][c + 3]);
          if (g > 0) {
            const float4 o = *p;
            v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
          }
          *p = v;
        }
    }
    __syncthreads();
  }
  // contiguous in C's layout: walk (m fastest) when ldc_m == 1, else (c fastest); int64
  // fixed-point adds (ABI 16): the blocks' partials sum to the same bits in any order
  const int n = Mw * 8;
  for (int o = t; o < n; o += blockDim.x) {
    int m, c;
    if (ldc_m == 1) { c = o / Mw; m = o % Mw; } else { m = o / 8; c = o % 8; }
    fx_add(cacc + m * ldc_m + c * ldc_c, alpha * red[m * 8 + c], TTMI_FX_GRAD);
  }
}

// C(m, c) += acc(m, c) converted; acc cleared (the skinny gradient's accumulator, C's layout).
__global__ __launch_bounds__(256) void skinny_fx_out_kernel(int Mw, int64_t* __restrict__ acc,
                                                            float* __restrict__ C, int64_t ldc_m,
                                                            int64_t ldc_c) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= Mw * 8) return;
  int m, c;
  if (ldc_m == 1) { c = o / Mw; m = o % Mw; } else { m = o / 8; c = o % 8; }
  const int64_t i = m * ldc_m + c * ldc_c;
  C[i] += fx_to_f(acc[i], TTMI_FX_GRAD);
  acc[i] = 0;
}

struct SkinnyCfg { int rg, u, blocks; };
SkinnyCfg skinny_cfg() {                               // TTMI_SKINNY="RG,U,BLOCKS": tuning runs
  static const SkinnyCfg cfg = [] {
    SkinnyCfg c{8, 4, 256};   // tools/skinny_sweep.py (R 65,536, Mw 768): 69 -> 44 us vs {2, 8, 512}
    if (const char* e = getenv("TTMI_SKINNY")) {
      int rg = 0, u = 0, bl = 0;
      if (sscanf(e, "%d,%d,%d", &rg, &u, &bl) == 3 && rg > 0 && (u == 4 || u == 8) && bl > 0) c = SkinnyCfg{rg, u, bl};
    }
    return c;
  }();
  return cfg;
}

// dx[m, n] += s · Σ_{p in {q, v}} drop_p(dL_p[m, :] · A_p[:, n])  (the LoRA input gradient of
// query_proj / value_proj; drop_p regenerates the forward LoRA-dropout mask at m·ld_drop + n).
// dL [M, 16] bf16 = [dL_q | dL_v], A_q/A_v [8, H] bf16.  One thread per 8 columns; HBM-bound on
// the fp32 read-modify-write of dx (replaces two K=8 accumulate GEMMs with atomics).
// A thread owns 8 columns of LDX_ROWS consecutive rows: the 16 A fragments (8 ranks x q/v) it
// needs are loaded once per LDX_ROWS rows, and every row's dL / dx loads are issued before
// the arithmetic.
constexpr int LDX_ROWS = 4;
__global__ __launch_bounds__(256) void lora_dx_kernel(int64_t M, int H, const bf16_t* __restrict__ dL,
                                                      int64_t ld_dl, const bf16_t* __restrict__ aq,
                                                      const bf16_t* __restrict__ av, float s,
                                                      DropParams dq, DropParams dv, int64_t ld_drop,
                                                      float* __restrict__ dx, int64_t ld_dx) {
  const int ncol8 = H / 8;
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t mblocks = (M + LDX_ROWS - 1) / LDX_ROWS;
  if (id >= mblocks * ncol8) return;
  const int64_t m0 = (id / ncol8) * LDX_ROWS;
  const int n = (int)(id % ncol8) * 8;
  const DropKeys kq = resolve_drop(dq), kv = resolve_drop(dv);
  uint4 lqv[LDX_ROWS][2];
  float4 xr[LDX_ROWS][2];
#pragma unroll
  for (int j = 0; j < LDX_ROWS; ++j) {
    const int64_t m = min(m0 + j, M - 1);
    lqv[j][0] = *reinterpret_cast<const uint4*>(dL + m * ld_dl);
    lqv[j][1] = *reinterpret_cast<const uint4*>(dL + m * ld_dl + 8);
    xr[j][0] = *reinterpret_cast<const float4*>(dx + m * ld_dx + n);
    xr[j][1] = *reinterpret_cast<const float4*>(dx + m * ld_dx + n + 4);
  }
  uint4 ap[8], bp[8];                     // packed bf16, unpacked per use (register budget)
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    ap[r] = *reinterpret_cast<const uint4*>(aq + r * H + n);
    bp[r] = *reinterpret_cast<const uint4*>(av + r * H + n);
  }
#pragma unroll
  for (int j = 0; j < LDX_ROWS; ++j) {
    const int64_t m = m0 + j;
    if (m >= M) break;
    float lq[8], lv[8];
    unpack8(lqv[j][0], lq);
    unpack8(lqv[j][1], lv);
    float yq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, yv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      float a[8], b[8];
      unpack8(ap[r], a);
      unpack8(bp[r], b);
#pragma unroll
      for (int e = 0; e < 8; ++e) { yq[e] += lq[r] * a[e]; yv[e] += lv[r] * b[e]; }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) { yq[e] *= s; yv[e] *= s; }
    drop_apply_vec<8>(kq, (uint32_t)(m * ld_drop + n), yq);
    drop_apply_vec<8>(kv, (uint32_t)(m * ld_drop + n), yv);
    float4 x0 = xr[j][0], x1 = xr[j][1];
    x0.x += yq[0] + yv[0]; x0.y += yq[1] + yv[1]; x0.z += yq[2] + yv[2]; x0.w += yq[3] + yv[3];
    x1.x += yq[4] + yv[4]; x1.y += yq[5] + yv[5]; x1.z += yq[6] + yv[6]; x1.w += yq[7] + yv[7];
    float* p = dx + m * ld_dx + n;
    *reinterpret_cast<float4*>(p) = x0;
    *reinterpret_cast<float4*>(p + 4) = x1;
  }
}

}  // namespace

// ---------------------------------------------------------------- C ABI
extern "C" int ttmi_deb_gelu(int64_t n, const uint16_t* x, uint16_t* y, hipStream_t s) {
  TTMI_REQUIRE(n > 0 && n % 8 == 0 && x && y, "ttmi_deb_gelu: need n %% 8 == 0");
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(deb_gelu_kernel, dim3((unsigned)std::min<int64_t>((n8 + 255) / 256, 8192)), dim3(256), 0, s,
                     n8, (const bf16_t*)x, (bf16_t*)y);
  return ttmi_check_launch("ttmi_deb_gelu");
}

extern "C" int ttmi_deb_embed_fwd(int64_t M, int H, const int64_t* ids, const uint16_t* table,
                                  const float* ln_w, const float* ln_b, float eps,
                                  const int64_t* mask, float drop_p, const uint64_t* drop_seed,
                                  float* y32, uint16_t* y16, int64_t ld16, int64_t V, int32_t* id_err,
                                  hipStream_t s) {
  TTMI_REQUIRE(M > 0 && H % 64 == 0 && H <= 1024 && ld16 >= H && V > 0,
               "ttmi_deb_embed_fwd: need H %% 64 == 0, H <= 1024, V > 0");
  TTMI_REQUIRE(ids && table && ln_w && ln_b && y16, "ttmi_deb_embed_fwd: null argument");
  TTMI_REQUIRE(drop_p == 0.f || drop_seed, "ttmi_deb_embed_fwd: dropout needs a seed");
  hipLaunchKernelGGL(deb_embed_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, s, M, H, ids,
                     (const bf16_t*)table, ln_w, ln_b, eps, mask, make_drop(drop_p, drop_seed), y32,
                     (bf16_t*)y16, ld16, V, id_err);
  return ttmi_check_launch("ttmi_deb_embed_fwd");
}

extern "C" int ttmi_deb_ln_fwd(int64_t M, int H, const float* z, const float* ln_w, const float* ln_b,
                               float eps, float* y32, uint16_t* y16, int64_t ld16, float* mean,
                               float* rstd, uint16_t* yq, uint16_t* yv, float drop_p,
                               const uint64_t* seed_q, const uint64_t* seed_v, hipStream_t s) {
  TTMI_REQUIRE(M > 0 && H % 64 == 0 && H <= 1024, "ttmi_deb_ln_fwd: need H %% 64 == 0, H <= 1024");
  TTMI_REQUIRE(z && ln_w && ln_b && mean && rstd && (y32 || y16), "ttmi_deb_ln_fwd: null argument");
  TTMI_REQUIRE(!y16 || ld16 >= H, "ttmi_deb_ln_fwd: ld16 < H");
  auto al = [](const void* p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; };
  const bool vec = H % 256 == 0 && al(z, 16) && al(ln_w, 16) && al(ln_b, 16) && (!y32 || al(y32, 16)) &&
                   (!y16 || (al(y16, 8) && ld16 % 4 == 0)) && (!yq || al(yq, 8)) && (!yv || al(yv, 8));
  TTMI_REQUIRE(!(yq || yv) || vec, "ttmi_deb_ln_fwd: the LoRA-dropout outputs need H %% 256 == 0, aligned");
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || (seed_q && seed_v)),
               "ttmi_deb_ln_fwd: bad LoRA dropout");
  if (vec) {
    const dim3 g((unsigned)((M + 3) / 4));
    const DropParams dq = make_drop(drop_p, seed_q), dv = make_drop(drop_p, seed_v);
#define TTMI_DEBLN(Q)                                                                                   \
  hipLaunchKernelGGL(deb_ln_vec_kernel<Q>, g, dim3(256), 0, s, M, H, z, ln_w, ln_b, eps, y32,            \
                     (bf16_t*)y16, ld16, mean, rstd, (bf16_t*)yq, (bf16_t*)yv, dq, dv)
    switch (H / 256) {
      case 1: TTMI_DEBLN(1); break;
      case 2: TTMI_DEBLN(2); break;
      case 3: TTMI_DEBLN(3); break;
      default: TTMI_DEBLN(4); break;
    }
#undef TTMI_DEBLN
    return ttmi_check_launch("ttmi_deb_ln_fwd");
  }
  hipLaunchKernelGGL(deb_ln_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, s, M, H, z, ln_w, ln_b,
                     eps, y32, (bf16_t*)y16, ld16, mean, rstd);
  return ttmi_check_launch("ttmi_deb_ln_fwd");
}

extern "C" int ttmi_deb_pool_fwd(int B, int S, int H, const float* x, const int64_t* mask, float* out,
                                 hipStream_t s) {
  TTMI_REQUIRE(B > 0 && S > 0 && S <= POOL_MAXS && H > 0 && H % 4 == 0 && x && mask && out,
               "ttmi_deb_pool_fwd: need S <= %d, H %% 4 == 0", POOL_MAXS);
  TTMI_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0, "ttmi_deb_pool_fwd: x/out need 16-byte alignment");
  hipLaunchKernelGGL(deb_pool_fwd_kernel, dim3((unsigned)B, (unsigned)((H / 4 + 63) / 64)), dim3(256), 0, s, S, H,
                     x, mask, out);
  return ttmi_check_launch("ttmi_deb_pool_fwd");
}

extern "C" int ttmi_deb_pool_bwd(int B, int S, int H, const float* dout, const int64_t* mask, float* dx,
                                 hipStream_t s) {
  TTMI_REQUIRE(B > 0 && S > 0 && H > 0 && H % 4 == 0 && dout && mask && dx,
               "ttmi_deb_pool_bwd: need H %% 4 == 0");
  TTMI_REQUIRE(((uintptr_t)dout & 15) == 0 && ((uintptr_t)dx & 15) == 0, "ttmi_deb_pool_bwd: dout/dx need 16-byte alignment");
  hipLaunchKernelGGL(deb_pool_bwd_kernel, dim3((unsigned)B, (unsigned)((S + POOL_BWD_ROWS - 1) / POOL_BWD_ROWS)),
                     dim3(256), 0, s, S, H, dout, mask, dx);
  return ttmi_check_launch("ttmi_deb_pool_bwd");
}

extern "C" int ttmi_skinny_wgrad(int64_t R, int Mw, const uint16_t* W, int64_t ldw, const void* S,
                                 int s_f32, int64_t lds, int group, int sgs, float alpha, float* C,
                                 int64_t ldc_m, int64_t ldc_c, int64_t* acc, hipStream_t s) {
  TTMI_REQUIRE(R > 0 && Mw > 0 && Mw % 8 == 0 && Mw / 8 <= 256 && W && S && C && acc,
               "ttmi_skinny_wgrad: need Mw %% 8 == 0, Mw <= 2048, and the accumulator");
  TTMI_REQUIRE(group > 0 && group % 8 == 0 && ldw % 8 == 0 && (uintptr_t)W % 16 == 0 &&
               (uintptr_t)S % 16 == 0 && lds % (s_f32 ? 4 : 8) == 0,
               "ttmi_skinny_wgrad: W/S need 16-byte rows, group %% 8 == 0");
  TTMI_REQUIRE((int64_t)((Mw - 1) / group) * sgs + 8 <= lds, "ttmi_skinny_wgrad: S slice past its row");
  const SkinnyCfg cfg = skinny_cfg();
  const int ncol8 = Mw / 8;
  const int RG = std::max(1, std::min(cfg.rg, 1024 / ncol8));
  const size_t shm = (size_t)Mw * 8 * sizeof(float);
  TTMI_REQUIRE(shm <= 64 * 1024, "ttmi_skinny_wgrad: reduction tile exceeds 64 KB");
  const int64_t blocks = std::min<int64_t>(cfg.blocks, std::max<int64_t>(1, R / (4 * RG)));
  const int64_t rpb = (R + blocks - 1) / blocks;
  const dim3 grid((unsigned)blocks), blk((unsigned)(RG * ncol8));
#define TTMI_SKINNY_LAUNCH(TS_, U_)                                                              \
  hipLaunchKernelGGL((skinny_wgrad_kernel<TS_, U_>), grid, blk, shm, s, R, Mw, (const bf16_t*)W, ldw, \
                     (const TS_*)S, lds, group, sgs, alpha, acc, ldc_m, ldc_c, rpb)
  if (s_f32) {
    if (cfg.u == 4) TTMI_SKINNY_LAUNCH(float, 4); else TTMI_SKINNY_LAUNCH(float, 8);
  } else {
    if (cfg.u == 4) TTMI_SKINNY_LAUNCH(bf16_t, 4); else TTMI_SKINNY_LAUNCH(bf16_t, 8);
  }
#undef TTMI_SKINNY_LAUNCH
  const int rc = ttmi_check_launch("ttmi_skinny_wgrad");
  if (rc) return rc;
  hipLaunchKernelGGL(skinny_fx_out_kernel, dim3((unsigned)((Mw * 8 + 255) / 256)), dim3(256), 0, s, Mw, acc,
                     C, ldc_m, ldc_c);
  return ttmi_check_launch("ttmi_skinny_wgrad/out");
}

extern "C" int ttmi_lora_dx(int64_t M, int H, const uint16_t* dL, int64_t ld_dl, const uint16_t* aq,
                            const uint16_t* av, float scale, float drop_p, const uint64_t* seed_q,
                            const uint64_t* seed_v, int64_t ld_drop, float* dx, int64_t ld_dx,
                            hipStream_t s) {
  TTMI_REQUIRE(M > 0 && H > 0 && H % 8 == 0 && dL && aq && av && dx, "ttmi_lora_dx: bad argument");
  TTMI_REQUIRE(ld_dl % 8 == 0 && ld_dl >= 16 && ld_dx % 4 == 0 && (uintptr_t)dL % 16 == 0 &&
               (uintptr_t)aq % 16 == 0 && (uintptr_t)av % 16 == 0 && (uintptr_t)dx % 16 == 0,
               "ttmi_lora_dx: operands need 16-byte rows");
  TTMI_REQUIRE(drop_p == 0.f || (seed_q && seed_v), "ttmi_lora_dx: dropout needs both seeds");
  const int64_t n = (M + LDX_ROWS - 1) / LDX_ROWS * (H / 8);
  hipLaunchKernelGGL(lora_dx_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, M, H,
                     (const bf16_t*)dL, ld_dl, (const bf16_t*)aq, (const bf16_t*)av, scale,
                     make_drop(drop_p, seed_q), make_drop(drop_p, seed_v), ld_drop, dx, ld_dx);
  return ttmi_check_launch("ttmi_lora_dx");
}
