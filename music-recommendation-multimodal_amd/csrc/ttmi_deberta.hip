// ttmi_deberta.hip — the mDeBERTa-v3 text encoder of the cfg-4 item tower (reference
// src/models/item_tower.py:41-83: DebertaV2Model + peft LoRA + masked mean-pool).
//
//   deb_embed_fwd   word-embedding gather + LayerNorm + mask + dropout (DebertaV2Embeddings)
//   deb_ln_fwd      post-LayerNorm of the residual sum, fp32 copy (next residual) + bf16 operand
//   dis_attn_fwd    fused disentangled self-attention (DisentangledSelfAttention with
//                   share_att_key, c2p|p2c, position buckets): per (64 query rows, head, batch)
//                   stream 64-key blocks; for each block pair the c2p / p2c terms come from two
//                   128-row windows of the projected relative table (posK / posQ), computed with
//                   MFMA into LDS and gathered by delta(i - j); online softmax, probs dropout,
//                   P·V on MFMA; writes ctx (bf16) and the row log-sum-exp.
//   dis_attn_bwd    one workgroup per (head, batch), key blocks outer / query blocks inner:
//                   recomputes the scores, dV += Pdᵀ·dO, dK += dSᵀ·Q + H·posQ_win,
//                   dQ += dS·K + G·posK_win (G, H = dS binned by delta into the windows), plus
//                   the rank-8 contractions that carry the query_proj LoRA gradient through the
//                   relative path (posQ = query_proj(rel)): HU[j] = Σ_i dS_ij·u[δ_ij] and
//                   PB[δ] = Σ dS_ij·(K_j·Bq_h).  posK needs no gradient (key_proj and the
//                   relative table are frozen), so the [B, H, S, 2·span] relative-score
//                   gradient is never materialised.
//   deb_pool_fwd/bwd masked mean-pool (item_tower.py:73-80, clamp 1e-9).
// d_head = 64, S <= 256 (the backward keeps dQ of all query blocks in registers).
#include "ttmi_common.h"

namespace {

constexpr int DH = 64;                 // head width
constexpr int TP = 144;                // LDS pitch (bytes) of a [64][64] bf16 tile
constexpr int WIN = 128;               // relative-table rows per block pair (>= 127 deltas)
constexpr int GP = 132;                // fp32 window pitch (floats)
constexpr float FMIN = -3.4028234663852886e38f;   // torch.finfo(torch.float32).min
constexpr int MAXS = 256;

typedef __attribute__((ext_vector_type(4))) short s16x4d_t;

TTMI_DEV uint2 lds8(const char* p) { return *reinterpret_cast<const uint2*>(p); }
TTMI_DEV uint2 lds_tr8(const char* p) {
  const s16x4d_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4d_t*)(p));
  return __builtin_bit_cast(uint2, v);
}
// MFMA operand fragment (16 rows x 32 k; lane group g holds k = 4g..4g+3, 16+4g..16+4g+3)
// from a [row][k] bf16 tile ...
template <int P>
TTMI_DEV uint4 fk(const char* s, int row0, int c, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const char* p = s + (row0 + i) * P + c * 64 + g * 8;
  const uint2 lo = lds8(p), hi = lds8(p + 32);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}
// ... from a [k][row] bf16 tile (transposing LDS read) ...
template <int P>
TTMI_DEV uint4 ft(const char* s, int row0, int c, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int q = i >> 2, pp = i & 3;
  const char* p = s + (c * 32 + 4 * g + q) * P + (row0 + 4 * pp) * 2;
  const uint2 lo = lds_tr8(p), hi = lds_tr8(p + 16 * P);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}
TTMI_DEV uint32_t pk2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }
// ... from a [row][k] fp32 tile (rounded to bf16) ...
TTMI_DEV uint4 fk32(const float* s, int row0, int c, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const float* p = s + (row0 + i) * GP + c * 32 + g * 4;
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 16);
  return make_uint4(pk2(a.x, a.y), pk2(a.z, a.w), pk2(b.x, b.y), pk2(b.z, b.w));
}
// ... and from score-layout registers (tile t holds cols 16t + 4·lg + e of row lane & 15).
TTMI_DEV uint4 freg(const f32x4_t& lo, const f32x4_t& hi) {
  return make_uint4(pk2(lo[0], lo[1]), pk2(lo[2], lo[3]), pk2(hi[0], hi[1]), pk2(hi[2], hi[3]));
}

// rows [r0, r0 + R) x 64 bf16 of src (row stride ld elements) -> LDS tile; rows >= nrows zero.
// Loads are unconditional from a clamped row (then zeroed by a select): a guarded load would
// compile to a branch + vmcnt(0) and serialise the whole group.
template <int R>
TTMI_DEV void load_rows(char* dst, const bf16_t* src, int64_t ld, int r0, int nrows, int tid) {
  constexpr int C = R * 8 / 256;
  uint4 v[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int idx = tid + 256 * c, r = idx >> 3, ch = idx & 7;
    const int rr = min(r0 + r, nrows - 1);
    v[c] = *reinterpret_cast<const uint4*>(src + (int64_t)rr * ld + ch * 8);
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int idx = tid + 256 * c, r = idx >> 3, ch = idx & 7;
    const bool ok = r0 + r < nrows;
    const uint4 z = make_uint4(ok ? v[c].x : 0u, ok ? v[c].y : 0u, ok ? v[c].z : 0u, ok ? v[c].w : 0u);
    *reinterpret_cast<uint4*>(dst + r * TP + ch * 16) = z;
  }
}
TTMI_DEV void load_tile(char* dst, const bf16_t* src, int64_t ld, int r0, int nrows, int tid) {
  load_rows<64>(dst, src, ld, r0, nrows, tid);
}
TTMI_DEV void load_win(char* dst, const bf16_t* src, int64_t ld, int r0, int nrows, int tid) {
  load_rows<WIN>(dst, src, ld, r0, nrows, tid);
}

struct DisArgs {
  int B, S, nh, npos;               // npos = 2·position_buckets rows of posq/posk
  const bf16_t* q; const bf16_t* k; const bf16_t* v; int64_t ldqkv;   // head h at column h·64
  const bf16_t* posq; const bf16_t* posk; int64_t ldpos;
  const int64_t* mask;              // [B, S] attention_mask
  const int16_t* delta;             // [2S-1]: δ(rel = i - j) (index rel + S - 1)
  float inv_scale;                  // 1/sqrt(3·d_head)
  DropParams drop;                  // attention-probs dropout, idx ((b·nh + h)·S + i)·S + j
  bf16_t* ctx; int64_t ldctx;       // forward output (head h at column h·64)
  float* lse;                       // [B, nh, S]
  // backward
  const bf16_t* dctx; int64_t lddctx;
  bf16_t* dq; bf16_t* dk; bf16_t* dv; int64_t lddqkv;
  const float* u;                   // [npos, 8] rel-path LoRA down projection, or NULL
  const float* bq;                  // [nh·64, 8] LoRA B of query_proj
  float* hu;                        // [B·S, nh, 8]
  float* pb;                        // [B·nh, npos, 8]
  float* dq32;                      // [B·S, nh·64] fp32 scratch (dQ accumulation)
};

// Scores of a 64x64 block pair for wave w's 16 query rows (fwd and bwd share this):
// sc[t][e] = Q_i·K_j + Q_i·posK[δ_ij] + K_j·posQ[δ_ij] (unscaled) for j = 16t + 4·lg + e.
TTMI_DEV void block_scores(const char* sQ, const char* sK, const char* sPK, const char* sPQ,
                           float* sW, const int16_t* sDelta, int i0, int j0, int dlo, int S,
                           int w, int lane, f32x4_t sc[4]) {
  const int li = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int t = 0; t < 4; ++t) sc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  f32x4_t win[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) win[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const uint4 af = fk<TP>(sQ, 16 * w, c, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t) Mma<bf16_t>::run(sc[t], fk<TP>(sK, 16 * t, c, lane), af);
#pragma unroll
    for (int t = 0; t < 8; ++t) Mma<bf16_t>::run(win[t], fk<TP>(sPK, 16 * t, c, lane), af);
  }
  // c2p window (own rows) -> LDS -> gather
#pragma unroll
  for (int t = 0; t < 8; ++t)
    *reinterpret_cast<f32x4_t*>(sW + (16 * w + li) * GP + 16 * t + 4 * lg) = win[t];
  __syncthreads();
  const int i = i0 + 16 * w + li;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int rel = min(max(i - (j0 + 16 * t + 4 * lg + e), -(S - 1)), S - 1);
      const int wi = min(max((int)sDelta[rel + S - 1] - dlo, 0), WIN - 1);
      sc[t][e] += sW[(16 * w + li) * GP + wi];
    }
  __syncthreads();
  // p2c window: keys 16w..16w+15 against posQ rows
#pragma unroll
  for (int t = 0; t < 8; ++t) win[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const uint4 af = fk<TP>(sK, 16 * w, c, lane);
#pragma unroll
    for (int t = 0; t < 8; ++t) Mma<bf16_t>::run(win[t], fk<TP>(sPQ, 16 * t, c, lane), af);
  }
#pragma unroll
  for (int t = 0; t < 8; ++t)
    *reinterpret_cast<f32x4_t*>(sW + (16 * w + li) * GP + 16 * t + 4 * lg) = win[t];
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int jl = 16 * t + 4 * lg + e;
      const int rel = min(max(i - (j0 + jl), -(S - 1)), S - 1);
      const int wi = min(max((int)sDelta[rel + S - 1] - dlo, 0), WIN - 1);
      sc[t][e] += sW[jl * GP + wi];
    }
  __syncthreads();
}

TTMI_DEV int block_dlo(const int16_t* sDelta, int i0, int j0, int S) {
  const int rel = min(max(i0 - j0 - 63, -(S - 1)), S - 1);
  return sDelta[rel + S - 1];
}

__global__ __launch_bounds__(256) void dis_attn_fwd_kernel(DisArgs a) {
  __shared__ __attribute__((aligned(16))) char sQ[64 * TP];
  __shared__ __attribute__((aligned(16))) char sK[64 * TP];
  __shared__ __attribute__((aligned(16))) char sV[64 * TP];
  __shared__ __attribute__((aligned(16))) char sPK[WIN * TP];
  __shared__ __attribute__((aligned(16))) char sPQ[WIN * TP];
  __shared__ __attribute__((aligned(16))) float sW[64 * GP];
  __shared__ int16_t sDelta[2 * MAXS];
  __shared__ float sMk[64];
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int S = a.S, i0 = qb * 64;
  const DropKeys dk = resolve_drop(a.drop);
  for (int r = tid; r < 2 * S - 1; r += 256) sDelta[r] = a.delta[r];
  const int64_t rowb = (int64_t)b * S;
  load_tile(sQ, a.q + rowb * a.ldqkv + h * DH, a.ldqkv, i0, S, tid);
  const int i = i0 + 16 * w + li;
  const bool irow = i < S;
  const bool qvalid = irow && a.mask[rowb + i] != 0;
  float m_run = -INFINITY, l_run = 0.f;
  f32x4_t o[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) o[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  for (int j0 = 0; j0 < S; j0 += 64) {
    const int dlo = block_dlo(sDelta, i0, j0, S);
    load_tile(sK, a.k + rowb * a.ldqkv + h * DH, a.ldqkv, j0, S, tid);
    load_tile(sV, a.v + rowb * a.ldqkv + h * DH, a.ldqkv, j0, S, tid);
    load_win(sPK, a.posk + h * DH, a.ldpos, dlo, a.npos, tid);
    load_win(sPQ, a.posq + h * DH, a.ldpos, dlo, a.npos, tid);
    if (tid < 64) {
      const int j = j0 + tid;
      sMk[tid] = j < S ? (a.mask[rowb + j] != 0 ? 1.f : 0.f) : -1.f;
    }
    __syncthreads();
    f32x4_t sc[4];
    block_scores(sQ, sK, sPK, sPQ, sW, sDelta, i0, j0, dlo, S, w, lane, sc);
    float rmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float mk = sMk[16 * t + 4 * lg + e];
        const float s = sc[t][e] * a.inv_scale;
        sc[t][e] = mk < 0.f ? -INFINITY : ((qvalid && mk > 0.f) ? s : FMIN);
        rmax = fmaxf(rmax, sc[t][e]);
      }
    rmax = fmaxf(rmax, __shfl_xor(rmax, 16, 64));
    rmax = fmaxf(rmax, __shfl_xor(rmax, 32, 64));
    const float m_new = fmaxf(m_run, rmax);
    const float corr = __expf(m_run - m_new);
    float rsum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float p = __expf(sc[t][e] - m_new);
        rsum += p;
        const uint32_t idx = (uint32_t)((((int64_t)b * a.nh + h) * S + i) * S + j0 + 16 * t + 4 * lg + e);
        sc[t][e] = dk.on ? (drop_keep(dk, idx) ? p * dk.scale : 0.f) : p;
      }
    rsum += __shfl_xor(rsum, 16, 64);
    rsum += __shfl_xor(rsum, 32, 64);
    l_run = l_run * corr + rsum;
    m_run = m_new;
#pragma unroll
    for (int u = 0; u < 4; ++u) o[u] *= corr;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint4 af = freg(sc[2 * c], sc[2 * c + 1]);
#pragma unroll
      for (int u = 0; u < 4; ++u) Mma<bf16_t>::run(o[u], ft<TP>(sV, 16 * u, c, lane), af);
    }
    __syncthreads();
  }
  if (!irow) return;
  const float inv = 1.f / l_run;
  bf16_t* dst = a.ctx + (rowb + i) * a.ldctx + h * DH;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    ushort4 q;
    q.x = f2bf(o[u][0] * inv); q.y = f2bf(o[u][1] * inv); q.z = f2bf(o[u][2] * inv); q.w = f2bf(o[u][3] * inv);
    *reinterpret_cast<ushort4*>(dst + 16 * u + 4 * lg) = q;
  }
  if (lg == 0) a.lse[((int64_t)b * a.nh + h) * S + i] = m_run + __logf(l_run);
}

__global__ __launch_bounds__(256) void dis_attn_bwd_kernel(DisArgs a) {
  __shared__ __attribute__((aligned(16))) char sQ[64 * TP];
  __shared__ __attribute__((aligned(16))) char sK[64 * TP];
  __shared__ __attribute__((aligned(16))) char sV[64 * TP];
  __shared__ __attribute__((aligned(16))) char sdO[64 * TP];
  __shared__ __attribute__((aligned(16))) char sP[64 * TP];
  __shared__ __attribute__((aligned(16))) char sdS[64 * TP];
  __shared__ __attribute__((aligned(16))) char sPK[WIN * TP];
  __shared__ __attribute__((aligned(16))) char sPQ[WIN * TP];
  __shared__ __attribute__((aligned(16))) float sW[64 * GP];
  __shared__ int16_t sDelta[2 * MAXS];
  __shared__ float sLse[MAXS], sD[MAXS], sMq[MAXS];
  __shared__ float sMk[64];
  __shared__ __attribute__((aligned(16))) float sKB[64 * 8];
  __shared__ float sHU[64 * 8];
  __shared__ __attribute__((aligned(16))) float sUw[WIN * 8];
  const int h = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int S = a.S, nqb = (S + 63) / 64;
  const bool lora = a.u != nullptr;
  const DropKeys dk = resolve_drop(a.drop);
  const int64_t rowb = (int64_t)b * S;
  for (int r = tid; r < 2 * S - 1; r += 256) sDelta[r] = a.delta[r];
  float* pbw = lora ? a.pb + ((int64_t)b * a.nh + h) * a.npos * 8 : nullptr;   // owned slice
  if (lora)
    for (int r = tid; r < a.npos * 8; r += 256) pbw[r] = 0.f;
  // per-row D_i = dO_i · O_i, lse, mask
  for (int r = tid; r < S; r += 256) {
    const bf16_t* o = a.ctx + (rowb + r) * a.ldctx + h * DH;
    const bf16_t* go = a.dctx + (rowb + r) * a.lddctx + h * DH;
    float d = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float x[8], y[8];
      unpack8(*reinterpret_cast<const uint4*>(o + 8 * c), x);
      unpack8(*reinterpret_cast<const uint4*>(go + 8 * c), y);
#pragma unroll
      for (int e = 0; e < 8; ++e) d += x[e] * y[e];
    }
    sD[r] = d;
    sLse[r] = a.lse[((int64_t)b * a.nh + h) * S + r];
    sMq[r] = a.mask[rowb + r] != 0 ? 1.f : 0.f;
  }
  __syncthreads();

  for (int j0 = 0; j0 < S; j0 += 64) {
    load_tile(sK, a.k + rowb * a.ldqkv + h * DH, a.ldqkv, j0, S, tid);
    load_tile(sV, a.v + rowb * a.ldqkv + h * DH, a.ldqkv, j0, S, tid);
    if (tid < 64) {
      const int j = j0 + tid;
      sMk[tid] = j < S ? (a.mask[rowb + j] != 0 ? 1.f : 0.f) : -1.f;
    }
    for (int r = tid; r < 64 * 8; r += 256) sHU[r] = 0.f;
    __syncthreads();
    if (lora) {                                   // KB[j][c] = K_j · Bq[h·64 + :, c]
      for (int r = tid; r < 64 * 8; r += 256) {
        const int jl = r >> 3, c = r & 7;
        float acc = 0.f;
        for (int d = 0; d < DH; d += 8) {
          float kv[8];
          unpack8(*reinterpret_cast<const uint4*>(sK + jl * TP + d * 2), kv);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc += kv[e] * a.bq[(h * DH + d + e) * 8 + c];
        }
        sKB[r] = acc;
      }
    }
    f32x4_t dkacc[4], dvacc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) dkacc[u] = dvacc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int qq = 0; qq < nqb; ++qq) {
      const int i0 = qq * 64;
      const int dlo = block_dlo(sDelta, i0, j0, S);
      __syncthreads();
      load_tile(sQ, a.q + rowb * a.ldqkv + h * DH, a.ldqkv, i0, S, tid);
      load_tile(sdO, a.dctx + rowb * a.lddctx + h * DH, a.lddctx, i0, S, tid);
      load_win(sPK, a.posk + h * DH, a.ldpos, dlo, a.npos, tid);
      load_win(sPQ, a.posq + h * DH, a.ldpos, dlo, a.npos, tid);
      if (lora) {
        float uv[WIN * 8 / 256];
#pragma unroll
        for (int c = 0; c < WIN * 8 / 256; ++c) {
          const int r = tid + 256 * c;
          uv[c] = a.u[(int64_t)min(dlo + (r >> 3), a.npos - 1) * 8 + (r & 7)];
        }
#pragma unroll
        for (int c = 0; c < WIN * 8 / 256; ++c) {
          const int r = tid + 256 * c;
          sUw[r] = dlo + (r >> 3) < a.npos ? uv[c] : 0.f;
        }
      }
      __syncthreads();
      f32x4_t sc[4];
      block_scores(sQ, sK, sPK, sPQ, sW, sDelta, i0, j0, dlo, S, w, lane, sc);
      const int i = i0 + 16 * w + li;
      const bool irow = i < S;
      const float qv = irow ? sMq[i] : 0.f;
      const float lse = irow ? sLse[i] : 0.f, Di = irow ? sD[i] : 0.f;
      // dP = dO_i · V_j
      f32x4_t dp[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) dp[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const uint4 af = fk<TP>(sdO, 16 * w, c, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t) Mma<bf16_t>::run(dp[t], fk<TP>(sV, 16 * t, c, lane), af);
      }
      f32x4_t pd[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float mk = sMk[16 * t + 4 * lg + e];
          const float s = mk < 0.f ? -INFINITY : ((qv > 0.f && mk > 0.f) ? sc[t][e] * a.inv_scale : FMIN);
          // a fully padded query row attends uniformly to the S keys (finfo.min everywhere);
          // its masked_fill'ed scores are constants, so they receive no gradient
          const float p = !irow ? 0.f : (qv > 0.f ? __expf(s - lse) : (mk >= 0.f ? 1.f / (float)S : 0.f));
          const uint32_t idx = (uint32_t)((((int64_t)b * a.nh + h) * S + i) * S + j0 + 16 * t + 4 * lg + e);
          const float keep = dk.on ? (drop_keep(dk, idx) ? dk.scale : 0.f) : 1.f;
          pd[t][e] = p * keep;
          const float ds = qv > 0.f ? p * (dp[t][e] * keep - Di) : 0.f;   // grad of the scaled score
          sc[t][e] = ds * a.inv_scale;                          // -> raw c2c / c2p / p2c terms
        }
      // dQ (this block pair) = dS·K + G·posK_win, added to the fp32 scratch below
      f32x4_t dqp[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) dqp[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const uint4 af = freg(sc[2 * c], sc[2 * c + 1]);
#pragma unroll
        for (int u = 0; u < 4; ++u) Mma<bf16_t>::run(dqp[u], ft<TP>(sK, 16 * u, c, lane), af);
      }
      // stash Pd and dS (bf16) for the key-side products; zero the window for G
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        uint2 pv, sv;
        pv.x = pk2(pd[t][0], pd[t][1]); pv.y = pk2(pd[t][2], pd[t][3]);
        sv.x = pk2(sc[t][0], sc[t][1]); sv.y = pk2(sc[t][2], sc[t][3]);
        *reinterpret_cast<uint2*>(sP + (16 * w + li) * TP + (16 * t + 4 * lg) * 2) = pv;
        *reinterpret_cast<uint2*>(sdS + (16 * w + li) * TP + (16 * t + 4 * lg) * 2) = sv;
      }
      // G[i][w] / H[j][w] = dS binned by w = δ(i - j) - dlo (fp32, LDS atomics: log buckets
      // share w); then dQ += G·posK_win and dK += H·posQ_win
      auto add_dq = [&]() {
        if (irow) {           // each lane owns the same dQ elements in every block pair
          float* d = a.dq32 + (rowb + i) * (int64_t)(a.nh * DH) + h * DH + 4 * lg;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            f32x4_t* pd4 = reinterpret_cast<f32x4_t*>(d + 16 * u);
            *pd4 = j0 == 0 ? dqp[u] : *pd4 + dqp[u];
          }
        }
      };
      {
        for (int r = tid; r < 64 * GP; r += 256) sW[r] = 0.f;
        __syncthreads();
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int rel = min(max(i - (j0 + 16 * t + 4 * lg + e), -(S - 1)), S - 1);
            const int wi = min(max((int)sDelta[rel + S - 1] - dlo, 0), WIN - 1);
            atomicAdd(&sW[(16 * w + li) * GP + wi], sc[t][e]);
          }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint4 af = fk32(sW, 16 * w, c, lane);
#pragma unroll
          for (int u = 0; u < 4; ++u) Mma<bf16_t>::run(dqp[u], ft<TP>(sPK, 16 * u, c, lane), af);
        }
        add_dq();
        __syncthreads();
        for (int r = tid; r < 64 * GP; r += 256) sW[r] = 0.f;
        __syncthreads();
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int jl = 16 * t + 4 * lg + e;
            const int rel = min(max(i - (j0 + jl), -(S - 1)), S - 1);
            const int wi = min(max((int)sDelta[rel + S - 1] - dlo, 0), WIN - 1);
            atomicAdd(&sW[jl * GP + wi], sc[t][e]);
          }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint4 af = fk32(sW, 16 * w, c, lane);
#pragma unroll
          for (int u = 0; u < 4; ++u) Mma<bf16_t>::run(dkacc[u], ft<TP>(sPQ, 16 * u, c, lane), af);
        }
      }
      if (lora) {
        auto hval = [&](int jl, int x) { return sW[jl * GP + x]; };
        // HU[j][c] += Σ_w H[j][w]·u[dlo + w][c]
        for (int r = tid; r < 64 * 8; r += 256) {
          const int jl = r >> 3, c = r & 7;
          float acc = 0.f;
          for (int x = 0; x < WIN; ++x) acc += hval(jl, x) * sUw[x * 8 + c];
          sHU[r] += acc;
        }
        // PB[dlo + w][c] += Σ_j H[j][w]·KB[j][c]
        {
          const int x = tid >> 1, c0 = (tid & 1) * 4;
          float acc[4] = {0.f, 0.f, 0.f, 0.f};
          for (int jl = 0; jl < 64; ++jl) {
            const float hv = hval(jl, x);
            const float4 kb = *reinterpret_cast<const float4*>(sKB + jl * 8 + c0);
            acc[0] += hv * kb.x; acc[1] += hv * kb.y; acc[2] += hv * kb.z; acc[3] += hv * kb.w;
          }
          const int row = dlo + x;
          if (row < a.npos)
#pragma unroll
            for (int e = 0; e < 4; ++e) pbw[row * 8 + c0 + e] += acc[e];
        }
      }
      // dK_j += dSᵀ·Q, dV_j += Pdᵀ·dO (rows j = 16w.. of this key block)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const uint4 aS = ft<TP>(sdS, 16 * w, c, lane), aP = ft<TP>(sP, 16 * w, c, lane);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          Mma<bf16_t>::run(dkacc[u], ft<TP>(sQ, 16 * u, c, lane), aS);
          Mma<bf16_t>::run(dvacc[u], ft<TP>(sdO, 16 * u, c, lane), aP);
        }
      }
    }
    // key-block outputs
    const int j = j0 + 16 * w + li;
    if (j < S) {
      bf16_t* pk = a.dk + (rowb + j) * a.lddqkv + h * DH;
      bf16_t* pv = a.dv + (rowb + j) * a.lddqkv + h * DH;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        uint2 x, y;
        x.x = pk2(dkacc[u][0], dkacc[u][1]); x.y = pk2(dkacc[u][2], dkacc[u][3]);
        y.x = pk2(dvacc[u][0], dvacc[u][1]); y.y = pk2(dvacc[u][2], dvacc[u][3]);
        *reinterpret_cast<uint2*>(pk + 16 * u + 4 * lg) = x;
        *reinterpret_cast<uint2*>(pv + 16 * u + 4 * lg) = y;
      }
    }
    __syncthreads();
    if (lora)
      for (int r = tid; r < 64 * 8; r += 256) {
        const int jj = j0 + (r >> 3);
        if (jj < S) a.hu[((rowb + jj) * a.nh + h) * 8 + (r & 7)] = sHU[r];
      }
  }
  // dQ of every query block: fp32 scratch -> bf16 (same lane ownership as the accumulation)
  for (int qq = 0; qq < nqb; ++qq) {
    const int i = qq * 64 + 16 * w + li;
    if (i < S) {
      const float* d = a.dq32 + (rowb + i) * (int64_t)(a.nh * DH) + h * DH + 4 * lg;
      bf16_t* pq = a.dq + (rowb + i) * a.lddqkv + h * DH;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4_t v4 = *reinterpret_cast<const f32x4_t*>(d + 16 * u);
        uint2 x;
        x.x = pk2(v4[0], v4[1]); x.y = pk2(v4[2], v4[3]);
        *reinterpret_cast<uint2*>(pq + 16 * u + 4 * lg) = x;
      }
    }
  }
}

// ---------------------------------------------------------------- embeddings + LayerNorm
// One wave per token row: y = LN(E[id]) · mask (· dropout); fp32 copy (residual) and bf16
// copy (GEMM operand, row stride ld16).  H % 64 == 0, H <= 1024.
__global__ __launch_bounds__(256) void deb_embed_kernel(int64_t M, int H, const int64_t* __restrict__ ids,
                                                        const bf16_t* __restrict__ table,
                                                        const float* __restrict__ lw,
                                                        const float* __restrict__ lb, float eps,
                                                        const int64_t* __restrict__ mask,
                                                        DropParams drop, float* __restrict__ y32,
                                                        bf16_t* __restrict__ y16, int64_t ld16) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const DropKeys dk = resolve_drop(drop);
  const int per = H / 64;                                  // <= 16 values per lane
  float v[16];
  const bf16_t* src = table + ids[row] * (int64_t)H;
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

// ---------------------------------------------------------------- masked mean-pool
__global__ __launch_bounds__(256) void deb_pool_fwd_kernel(int S, int H, const float* __restrict__ x,
                                                           const int64_t* __restrict__ mask,
                                                           float* __restrict__ out) {
  const int b = blockIdx.x;
  float den = 0.f;
  for (int s = 0; s < S; ++s) den += mask[(int64_t)b * S + s] != 0 ? 1.f : 0.f;
  const float inv = 1.f / fmaxf(den, 1e-9f);
  for (int c = threadIdx.x; c < H; c += blockDim.x) {
    float acc = 0.f;
    for (int s = 0; s < S; ++s)
      if (mask[(int64_t)b * S + s] != 0) acc += x[((int64_t)b * S + s) * H + c];
    out[(int64_t)b * H + c] = acc * inv;
  }
}
__global__ __launch_bounds__(256) void deb_pool_bwd_kernel(int S, int H, const float* __restrict__ dout,
                                                           const int64_t* __restrict__ mask,
                                                           float* __restrict__ dx) {
  const int64_t row = blockIdx.x;                          // b·S + s
  const int b = (int)(row / S);
  __shared__ float sinv;
  if (threadIdx.x == 0) {
    float den = 0.f;
    for (int s = 0; s < S; ++s) den += mask[(int64_t)b * S + s] != 0 ? 1.f : 0.f;
    sinv = 1.f / fmaxf(den, 1e-9f);
  }
  __syncthreads();
  const float m = mask[row] != 0 ? sinv : 0.f;
  for (int c = threadIdx.x; c < H; c += blockDim.x) dx[row * H + c] = dout[(int64_t)b * H + c] * m;
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
// loads, 64 fp32 accumulators) over a strided row set; the block's row groups are summed in
// LDS and every block adds its 6 KB partial with contiguous atomics.  The generic tile path
// spent ~260 us per call here padding the rank-8 side to 64.
template <typename TS>
__global__ __launch_bounds__(256) void skinny_wgrad_kernel(int64_t R, int Mw, const bf16_t* __restrict__ W,
                                                           int64_t ldw, const TS* __restrict__ S,
                                                           int64_t lds, int group, int sgs, float alpha,
                                                           float* __restrict__ C, int64_t ldc_m,
                                                           int64_t ldc_c, int64_t rows_per_block) {
  extern __shared__ float red[];                       // [RG][Mw·8]
  const int ncol8 = Mw / 8, RG = 256 / ncol8;
  const int t = threadIdx.x, rg = t / ncol8, c8 = t % ncol8;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(R, r0 + rows_per_block);
  float acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[i][c] = 0.f;
  if (rg < RG) {
    const int soff = (c8 * 8 / group) * sgs;
    for (int64_t r = r0 + rg; r < r1; r += RG) {
      float w[8], s[8];
      unpack8(*reinterpret_cast<const uint4*>(W + r * ldw + c8 * 8), w);
      if constexpr (sizeof(TS) == 2) {
        unpack8(*reinterpret_cast<const uint4*>(S + r * lds + soff), s);
      } else {
        const float4 a = *reinterpret_cast<const float4*>(S + r * lds + soff);
        const float4 b = *reinterpret_cast<const float4*>(S + r * lds + soff + 4);
        s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w; s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[i][c] += w[i] * s[c];
    }
    float* dst = red + (int64_t)rg * Mw * 8 + c8 * 64;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int c = 0; c < 8; c += 4)
        *reinterpret_cast<float4*>(dst + i * 8 + c) = make_float4(acc[i][c], acc[i][c + 1], acc[i][c + 2], acc[i][c + 3]);
  }
  __syncthreads();
  // contiguous in C: walk (m fastest) when ldc_m == 1, else (c fastest)
  const int n = Mw * 8;
  for (int o = t; o < n; o += 256) {
    int m, c;
    if (ldc_m == 1) { c = o / Mw; m = o % Mw; } else { m = o / 8; c = o % 8; }
    float v = 0.f;
    for (int g = 0; g < RG; ++g) v += red[(int64_t)g * n + m * 8 + c];
    atomicAdd(C + m * ldc_m + c * ldc_c, alpha * v);
  }
}

// dx[m, n] += s · Σ_{p in {q, v}} drop_p(dL_p[m, :] · A_p[:, n])  (the LoRA input gradient of
// query_proj / value_proj; drop_p regenerates the forward LoRA-dropout mask at m·ld_drop + n).
// dL [M, 16] bf16 = [dL_q | dL_v], A_q/A_v [8, H] bf16.  One thread per 8 columns; HBM-bound on
// the fp32 read-modify-write of dx (replaces two K=8 accumulate GEMMs with atomics).
__global__ __launch_bounds__(256) void lora_dx_kernel(int64_t M, int H, const bf16_t* __restrict__ dL,
                                                      int64_t ld_dl, const bf16_t* __restrict__ aq,
                                                      const bf16_t* __restrict__ av, float s,
                                                      DropParams dq, DropParams dv, int64_t ld_drop,
                                                      float* __restrict__ dx, int64_t ld_dx) {
  const int ncol8 = H / 8;
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= M * ncol8) return;
  const int64_t m = id / ncol8;
  const int n = (int)(id % ncol8) * 8;
  const DropKeys kq = resolve_drop(dq), kv = resolve_drop(dv);
  float lq[8], lv[8];
  unpack8(*reinterpret_cast<const uint4*>(dL + m * ld_dl), lq);
  unpack8(*reinterpret_cast<const uint4*>(dL + m * ld_dl + 8), lv);
  float yq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, yv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    float a[8], b[8];
    unpack8(*reinterpret_cast<const uint4*>(aq + r * H + n), a);
    unpack8(*reinterpret_cast<const uint4*>(av + r * H + n), b);
#pragma unroll
    for (int e = 0; e < 8; ++e) { yq[e] += lq[r] * a[e]; yv[e] += lv[r] * b[e]; }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { yq[e] *= s; yv[e] *= s; }
  drop_apply_vec<8>(kq, (uint32_t)(m * ld_drop + n), yq);
  drop_apply_vec<8>(kv, (uint32_t)(m * ld_drop + n), yv);
  float* p = dx + m * ld_dx + n;
  float4 x0 = *reinterpret_cast<float4*>(p), x1 = *reinterpret_cast<float4*>(p + 4);
  x0.x += yq[0] + yv[0]; x0.y += yq[1] + yv[1]; x0.z += yq[2] + yv[2]; x0.w += yq[3] + yv[3];
  x1.x += yq[4] + yv[4]; x1.y += yq[5] + yv[5]; x1.z += yq[6] + yv[6]; x1.w += yq[7] + yv[7];
  *reinterpret_cast<float4*>(p) = x0;
  *reinterpret_cast<float4*>(p + 4) = x1;
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
                                  float* y32, uint16_t* y16, int64_t ld16, hipStream_t s) {
  TTMI_REQUIRE(M > 0 && H % 64 == 0 && H <= 1024 && ld16 >= H, "ttmi_deb_embed_fwd: need H %% 64 == 0, H <= 1024");
  TTMI_REQUIRE(ids && table && ln_w && ln_b && y16, "ttmi_deb_embed_fwd: null argument");
  TTMI_REQUIRE(drop_p == 0.f || drop_seed, "ttmi_deb_embed_fwd: dropout needs a seed");
  hipLaunchKernelGGL(deb_embed_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, s, M, H, ids,
                     (const bf16_t*)table, ln_w, ln_b, eps, mask, make_drop(drop_p, drop_seed), y32,
                     (bf16_t*)y16, ld16);
  return ttmi_check_launch("ttmi_deb_embed_fwd");
}

extern "C" int ttmi_deb_ln_fwd(int64_t M, int H, const float* z, const float* ln_w, const float* ln_b,
                               float eps, float* y32, uint16_t* y16, int64_t ld16, float* mean,
                               float* rstd, hipStream_t s) {
  TTMI_REQUIRE(M > 0 && H % 64 == 0 && H <= 1024, "ttmi_deb_ln_fwd: need H %% 64 == 0, H <= 1024");
  TTMI_REQUIRE(z && ln_w && ln_b && mean && rstd && (y32 || y16), "ttmi_deb_ln_fwd: null argument");
  TTMI_REQUIRE(!y16 || ld16 >= H, "ttmi_deb_ln_fwd: ld16 < H");
  hipLaunchKernelGGL(deb_ln_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, s, M, H, z, ln_w, ln_b,
                     eps, y32, (bf16_t*)y16, ld16, mean, rstd);
  return ttmi_check_launch("ttmi_deb_ln_fwd");
}

static int dis_check(const ttmi_dis_attn_desc* d) {
  TTMI_REQUIRE(d != nullptr, "ttmi_dis_attn: null descriptor");
  TTMI_REQUIRE(d->B > 0 && d->S > 0 && d->S <= MAXS && d->nh > 0, "ttmi_dis_attn: need 0 < S <= %d", MAXS);
  TTMI_REQUIRE(d->d_head == DH, "ttmi_dis_attn: d_head must be 64");
  TTMI_REQUIRE(d->npos > 0 && d->npos <= 512, "ttmi_dis_attn: npos must be in (0, 512]");
  TTMI_REQUIRE(d->q && d->k && d->v && d->posq && d->posk && d->mask && d->delta && d->ctx && d->lse,
               "ttmi_dis_attn: null argument");
  TTMI_REQUIRE(d->ldqkv % 8 == 0 && d->ldpos % 8 == 0 && d->ldctx % 8 == 0,
               "ttmi_dis_attn: leading dimensions must be multiples of 8");
  TTMI_REQUIRE(d->drop_p == 0.f || d->drop_seed, "ttmi_dis_attn: dropout needs a seed");
  TTMI_REQUIRE((int64_t)d->B * d->nh * d->S * d->S < (1ll << 32), "ttmi_dis_attn: dropout index overflow");
  return TTMI_OK;
}

static DisArgs dis_args(const ttmi_dis_attn_desc* d) {
  DisArgs a{};
  a.B = d->B; a.S = d->S; a.nh = d->nh; a.npos = d->npos;
  a.q = (const bf16_t*)d->q; a.k = (const bf16_t*)d->k; a.v = (const bf16_t*)d->v; a.ldqkv = d->ldqkv;
  a.posq = (const bf16_t*)d->posq; a.posk = (const bf16_t*)d->posk; a.ldpos = d->ldpos;
  a.mask = d->mask; a.delta = d->delta; a.inv_scale = d->inv_scale;
  a.drop = make_drop(d->drop_p, d->drop_seed);
  a.ctx = (bf16_t*)d->ctx; a.ldctx = d->ldctx; a.lse = d->lse;
  a.dctx = (const bf16_t*)d->dctx; a.lddctx = d->lddctx;
  a.dq = (bf16_t*)d->dq; a.dk = (bf16_t*)d->dk; a.dv = (bf16_t*)d->dv; a.lddqkv = d->lddqkv;
  a.u = d->lora_u; a.bq = d->lora_bq; a.hu = d->lora_hu; a.pb = d->lora_pb;
  a.dq32 = d->dq_scratch;
  return a;
}

extern "C" int ttmi_dis_attn_fwd(const ttmi_dis_attn_desc* d, hipStream_t s) {
  int rc = dis_check(d);
  if (rc) return rc;
  const DisArgs a = dis_args(d);
  hipLaunchKernelGGL(dis_attn_fwd_kernel, dim3((unsigned)((d->S + 63) / 64), (unsigned)d->nh, (unsigned)d->B),
                     dim3(256), 0, s, a);
  return ttmi_check_launch("ttmi_dis_attn_fwd");
}

extern "C" int ttmi_dis_attn_bwd(const ttmi_dis_attn_desc* d, hipStream_t s) {
  int rc = dis_check(d);
  if (rc) return rc;
  TTMI_REQUIRE(d->dctx && d->dq && d->dk && d->dv && d->dq_scratch,
               "ttmi_dis_attn_bwd: null gradient argument (dq_scratch: fp32 [B·S, nh·64])");
  TTMI_REQUIRE(d->lddctx % 8 == 0 && d->lddqkv % 4 == 0, "ttmi_dis_attn_bwd: bad leading dimension");
  TTMI_REQUIRE(!d->lora_u || (d->lora_bq && d->lora_hu && d->lora_pb),
               "ttmi_dis_attn_bwd: LoRA outputs need u, bq, hu and pb together");
  const DisArgs a = dis_args(d);
  hipLaunchKernelGGL(dis_attn_bwd_kernel, dim3((unsigned)d->nh, (unsigned)d->B), dim3(256), 0, s, a);
  return ttmi_check_launch("ttmi_dis_attn_bwd");
}

extern "C" int ttmi_deb_pool_fwd(int B, int S, int H, const float* x, const int64_t* mask, float* out,
                                 hipStream_t s) {
  TTMI_REQUIRE(B > 0 && S > 0 && H > 0 && x && mask && out, "ttmi_deb_pool_fwd: bad argument");
  hipLaunchKernelGGL(deb_pool_fwd_kernel, dim3((unsigned)B), dim3(256), 0, s, S, H, x, mask, out);
  return ttmi_check_launch("ttmi_deb_pool_fwd");
}

extern "C" int ttmi_deb_pool_bwd(int B, int S, int H, const float* dout, const int64_t* mask, float* dx,
                                 hipStream_t s) {
  TTMI_REQUIRE(B > 0 && S > 0 && H > 0 && dout && mask && dx, "ttmi_deb_pool_bwd: bad argument");
  hipLaunchKernelGGL(deb_pool_bwd_kernel, dim3((unsigned)((int64_t)B * S)), dim3(256), 0, s, S, H, dout,
                     mask, dx);
  return ttmi_check_launch("ttmi_deb_pool_bwd");
}

extern "C" int ttmi_skinny_wgrad(int64_t R, int Mw, const uint16_t* W, int64_t ldw, const void* S,
                                 int s_f32, int64_t lds, int group, int sgs, float alpha, float* C,
                                 int64_t ldc_m, int64_t ldc_c, hipStream_t s) {
  TTMI_REQUIRE(R > 0 && Mw > 0 && Mw % 8 == 0 && Mw / 8 <= 256 && W && S && C,
               "ttmi_skinny_wgrad: need Mw %% 8 == 0, Mw <= 2048");
  TTMI_REQUIRE(group > 0 && group % 8 == 0 && ldw % 8 == 0 && (uintptr_t)W % 16 == 0 &&
               (uintptr_t)S % 16 == 0 && lds % (s_f32 ? 4 : 8) == 0,
               "ttmi_skinny_wgrad: W/S need 16-byte rows, group %% 8 == 0");
  TTMI_REQUIRE((int64_t)((Mw - 1) / group) * sgs + 8 <= lds, "ttmi_skinny_wgrad: S slice past its row");
  const int RG = 256 / (Mw / 8);
  const size_t shm = (size_t)RG * Mw * 8 * sizeof(float);
  TTMI_REQUIRE(shm <= 64 * 1024, "ttmi_skinny_wgrad: reduction tile exceeds 64 KB");
  const int64_t blocks = std::min<int64_t>(256, std::max<int64_t>(1, R / (4 * RG)));
  const int64_t rpb = (R + blocks - 1) / blocks;
  if (s_f32)
    hipLaunchKernelGGL(skinny_wgrad_kernel<float>, dim3((unsigned)blocks), dim3(256), shm, s, R, Mw,
                       (const bf16_t*)W, ldw, (const float*)S, lds, group, sgs, alpha, C, ldc_m, ldc_c, rpb);
  else
    hipLaunchKernelGGL(skinny_wgrad_kernel<bf16_t>, dim3((unsigned)blocks), dim3(256), shm, s, R, Mw,
                       (const bf16_t*)W, ldw, (const bf16_t*)S, lds, group, sgs, alpha, C, ldc_m, ldc_c, rpb);
  return ttmi_check_launch("ttmi_skinny_wgrad");
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
  const int64_t n = M * (H / 8);
  hipLaunchKernelGGL(lora_dx_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, M, H,
                     (const bf16_t*)dL, ld_dl, (const bf16_t*)aq, (const bf16_t*)av, scale,
                     make_drop(drop_p, seed_q), make_drop(drop_p, seed_v), ld_drop, dx, ld_dx);
  return ttmi_check_launch("ttmi_lora_dx");
}
