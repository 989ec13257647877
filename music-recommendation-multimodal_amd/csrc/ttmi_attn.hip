// ttmi_attn.hip — SASRec causal self-attention core (SDPA inside nn.MultiheadAttention,
// reference user_tower.py:111-116), forward and backward.
//
// One 64-lane wave owns one (sequence b, head h).  A whole sequence (L <= 64 keys) fits
// in LDS, so there is no online softmax: S = Q·Kᵀ is built in MFMA accumulators (4x4 tiles
// of 16x16; the six tiles above the diagonal are fully masked and skipped), softmax runs
// in registers (row = 16 lanes x 4 column tiles -> group16 shuffles), P goes back to LDS
// as the A operand of O = P·V.  The backward recomputes P from the forward's per-row LSE
// and produces dQ, dK, dV with five MFMA products, overlaying the transposed P/dS images
// on the row-major Q/K/V/dO images once they are consumed.
//
// Tiles are padded: keys/queries to 64 rows, the head dim to DHP (32 or 64) with zeros.
#include "ttmi_common.h"

#include <cstdlib>

namespace {

constexpr int LP = 64;   // padded sequence length

template <typename T, int DHP>
struct AttnGeom {
  static constexpr int ES = (int)sizeof(T);
  static constexpr int E = 16 / ES;                 // elements per 16-byte chunk
  static constexpr int RQ = DHP * ES + 16;          // row pitch of [64][DHP] images
  static constexpr int RP = LP * ES + 16;           // row pitch of [*][64] images
  static constexpr int CQ = DHP * ES / 64;          // 64-byte k-chunks along DHP
  static constexpr int CP = LP * ES / 64;           // 64-byte k-chunks along 64 keys
  static constexpr int TD = DHP / 16;               // 16-wide tiles along DHP
  static constexpr int ROW_IMG = LP * RQ;           // bytes of one [64][DHP] image
  static constexpr int SQ_IMG = LP * RP;            // bytes of one [64][64] image
  static constexpr int T_IMG = DHP * RP;            // bytes of one [DHP][64] image
};

// Load a head slice [L][Dh] (row stride ld elements) into a row-major [64][DHP] image and/or
// a transposed [DHP][64] image, zero-padded.
template <typename T, int DHP>
TTMI_DEV void load_head(const T* __restrict__ src, int64_t ld, int L, int Dh, char* rowimg,
                        char* trimg, int lane) {
  using G = AttnGeom<T, DHP>;
  constexpr int CPR = DHP / G::E;                   // 16-byte chunks per row
  for (int idx = lane; idx < LP * CPR; idx += 64) {
    const int r = idx / CPR, ch = idx % CPR;
    const int d0 = ch * G::E;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < L && d0 < Dh) v = *reinterpret_cast<const uint4*>(src + (int64_t)r * ld + d0);
    if (rowimg) *reinterpret_cast<uint4*>(rowimg + r * G::RQ + ch * 16) = v;
    if (trimg) {
      const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
      for (int k = 0; k < G::E; ++k)
        *reinterpret_cast<T*>(trimg + (d0 + k) * G::RP + r * G::ES) = e[k];
    }
  }
}

// acc[ti][tj] (tj <= ti) = Σ_k A[ti rows][k] · B[tj rows][k] over NCH 64-byte chunks.
template <typename T, int NCH, int PITCH>
TTMI_DEV void mma_lower(f32x4_t (&acc)[4][4], const char* A, const char* Bm, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int r = lane & 15, kq = (lane >> 4) * 16;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    uint4 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i] = lds16(A + (i * 16 + r) * PITCH + c * 64 + kq);
      b[i] = lds16(Bm + (i * 16 + r) * PITCH + c * 64 + kq);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j <= i; ++j) Mma<T>::run(acc[i][j], a[i], b[j]);
  }
}

// out[ti][td] = Σ_k A[ti rows][k] · B[td rows][k]; A pitch RP (k = 64 keys), B [DHP][64].
template <typename T, int DHP>
TTMI_DEV void mma_pv(f32x4_t (&acc)[4][DHP / 16], const char* A, const char* Bm, int lane) {
  using G = AttnGeom<T, DHP>;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < G::TD; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int r = lane & 15, kq = (lane >> 4) * 16;
#pragma unroll
  for (int c = 0; c < G::CP; ++c) {
    uint4 a[4], b[G::TD];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = lds16(A + (i * 16 + r) * G::RP + c * 64 + kq);
#pragma unroll
    for (int j = 0; j < G::TD; ++j) b[j] = lds16(Bm + (j * 16 + r) * G::RP + c * 64 + kq);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < G::TD; ++j) Mma<T>::run(acc[i][j], a[i], b[j]);
  }
}

template <typename T, int DHP>
TTMI_DEV void store_head(T* __restrict__ dst, int64_t ld, int L, int Dh,
                         const f32x4_t (&acc)[4][DHP / 16], int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < DHP / 16; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = i * 16 + (lane >> 4) * 4 + e, d = j * 16 + (lane & 15);
        if (r < L && d < Dh) stf<T>(dst, (int64_t)r * ld + d, acc[i][j][e]);
      }
}

template <typename T, int DHP>
__global__ __launch_bounds__(64) void mha_fwd_kernel(int B, int L, int H, int Dh,
                                                     const T* __restrict__ qkv,
                                                     const int64_t* __restrict__ kvalid,
                                                     DropParams dp, T* __restrict__ ctx,
                                                     float* __restrict__ lse, float scale) {
  using G = AttnGeom<T, DHP>;
  __shared__ __attribute__((aligned(16))) char smem[2 * G::ROW_IMG + G::T_IMG + G::SQ_IMG];
  char* sQ = smem;
  char* sK = sQ + G::ROW_IMG;
  char* sVt = sK + G::ROW_IMG;
  char* sP = sVt + G::T_IMG;
  const int lane = threadIdx.x;
  const int bh = blockIdx.x;
  const int b = bh / H, h = bh % H;
  const int D = H * Dh;
  const int64_t ld = 3LL * D;
  const T* base = qkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  load_head<T, DHP>(base, ld, L, Dh, sQ, nullptr, lane);
  load_head<T, DHP>(base + D, ld, L, Dh, sK, nullptr, lane);
  load_head<T, DHP>(base + 2 * D, ld, L, Dh, nullptr, sVt, lane);
  bool kv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = j * 16 + (lane & 15);
    kv[j] = c < L && kvalid[(int64_t)b * L + c] != 0;
  }
  __syncthreads();

  f32x4_t s[4][4];
  mma_lower<T, G::CQ, G::RQ>(s, sQ, sK, lane);
  const DropKeys dk = resolve_drop(dp);

  const int q4 = (lane >> 4) * 4;
  const int cl = lane & 15;
  const uint32_t pbase = (uint32_t)((int64_t)bh * L * L);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = i * 16 + q4 + e;
      float m = -INFINITY;
#pragma unroll
      for (int j = 0; j <= i; ++j) {
        const int c = j * 16 + cl;
        const bool ok = kv[j] && c <= r && r < L;
        const float v = ok ? s[i][j][e] * scale : -INFINITY;
        s[i][j][e] = v;
        m = fmaxf(m, v);
      }
      m = group16_max(m);
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j <= i; ++j) {
        const float p = m == -INFINITY ? 0.f : expf(s[i][j][e] - m);
        s[i][j][e] = p;
        sum += p;
      }
      sum = group16_sum(sum);
      const float inv = sum > 0.f ? 1.f / sum : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = j * 16 + cl;
        float p = 0.f;
        if (j <= i) {
          p = s[i][j][e] * inv;
          if (dk.on && r < L && c < L) p = drop_apply(dk, pbase + (uint32_t)(r * L + c), p);
        }
        stf<T>(reinterpret_cast<T*>(sP + r * G::RP), c, p);
      }
      if (cl == 0 && r < L) lse[(int64_t)bh * L + r] = m == -INFINITY ? INFINITY : m + logf(sum);
    }
  }
  __syncthreads();
  f32x4_t o[4][G::TD];
  mma_pv<T, DHP>(o, sP, sVt, lane);
  store_head<T, DHP>(ctx + (int64_t)b * L * D + (int64_t)h * Dh, D, L, Dh, o, lane);
}

template <typename T, int DHP>
__global__ __launch_bounds__(64) void mha_bwd_kernel(int B, int L, int H, int Dh,
                                                     const T* __restrict__ qkv,
                                                     const int64_t* __restrict__ kvalid,
                                                     const float* __restrict__ lse,
                                                     const T* __restrict__ dctx, DropParams dp,
                                                     T* __restrict__ dqkv, float scale) {
  using G = AttnGeom<T, DHP>;
  constexpr int R1 = (4 * G::ROW_IMG > 3 * G::SQ_IMG) ? 4 * G::ROW_IMG : 3 * G::SQ_IMG;
  __shared__ __attribute__((aligned(16))) char smem[R1 + 3 * G::T_IMG];
  char* sQ = smem;                   // phase 1: row-major images
  char* sK = sQ + G::ROW_IMG;
  char* sV = sK + G::ROW_IMG;
  char* sdO = sV + G::ROW_IMG;
  char* sPt = smem;                  // phase 2: overlays region 1
  char* sdS = sPt + G::SQ_IMG;
  char* sdSt = sdS + G::SQ_IMG;
  char* sQt = smem + R1;             // transposed images (both phases)
  char* sKt = sQt + G::T_IMG;
  char* sdOt = sKt + G::T_IMG;
  const int lane = threadIdx.x;
  const int bh = blockIdx.x;
  const int b = bh / H, h = bh % H;
  const int D = H * Dh;
  const int64_t ld = 3LL * D;
  const T* base = qkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  const T* dob = dctx + (int64_t)b * L * D + (int64_t)h * Dh;
  load_head<T, DHP>(base, ld, L, Dh, sQ, sQt, lane);
  load_head<T, DHP>(base + D, ld, L, Dh, sK, sKt, lane);
  load_head<T, DHP>(base + 2 * D, ld, L, Dh, sV, nullptr, lane);
  load_head<T, DHP>(dob, D, L, Dh, sdO, sdOt, lane);
  bool kv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = j * 16 + (lane & 15);
    kv[j] = c < L && kvalid[(int64_t)b * L + c] != 0;
  }
  __syncthreads();

  f32x4_t s[4][4], dpd[4][4];
  mma_lower<T, G::CQ, G::RQ>(s, sQ, sK, lane);      // S  = Q Kᵀ
  mma_lower<T, G::CQ, G::RQ>(dpd, sdO, sV, lane);   // dPd = dO Vᵀ (grad of dropped probs)

  const int q4 = (lane >> 4) * 4;
  const int cl = lane & 15;
  const uint32_t pbase = (uint32_t)((int64_t)bh * L * L);
  const DropKeys dk = resolve_drop(dp);
  __syncthreads();   // region 1 is rewritten below
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = i * 16 + q4 + e;
      const float lr = r < L ? lse[(int64_t)bh * L + r] : INFINITY;
      // pass A: p = softmax prob (pre-dropout), dP = dPd * keep/(1-p); row sum Σ p·dP
      float dsum = 0.f;
#pragma unroll
      for (int j = 0; j <= i; ++j) {
        const int c = j * 16 + cl;
        const bool ok = kv[j] && c <= r && r < L;
        const float p = ok ? expf(s[i][j][e] * scale - lr) : 0.f;
        float dP = 0.f;
        if (ok) {
          dP = dpd[i][j][e];
          if (dk.on) dP = drop_keep(dk, pbase + (uint32_t)(r * L + c)) ? dP * dk.scale : 0.f;
        }
        s[i][j][e] = p;
        dpd[i][j][e] = dP;
        dsum += p * dP;
      }
      dsum = group16_sum(dsum);
      // pass B: dS = p (dP - Σ) · scale;  Pd = p·keep/(1-p); scatter to the LDS images
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = j * 16 + cl;
        float pd = 0.f, ds = 0.f;
        if (j <= i) {
          const float p = s[i][j][e];
          ds = p * (dpd[i][j][e] - dsum) * scale;
          pd = p;
          if (dk.on && p != 0.f) pd = drop_keep(dk, pbase + (uint32_t)(r * L + c)) ? p * dk.scale : 0.f;
        }
        stf<T>(reinterpret_cast<T*>(sPt + c * G::RP), r, pd);
        stf<T>(reinterpret_cast<T*>(sdS + r * G::RP), c, ds);
        stf<T>(reinterpret_cast<T*>(sdSt + c * G::RP), r, ds);
      }
    }
  }
  __syncthreads();

  T* gq = dqkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  f32x4_t o[4][G::TD];
  mma_pv<T, DHP>(o, sPt, sdOt, lane);                // dV = Pdᵀ dO
  store_head<T, DHP>(gq + 2 * D, ld, L, Dh, o, lane);
  mma_pv<T, DHP>(o, sdS, sKt, lane);                 // dQ = dS K
  store_head<T, DHP>(gq, ld, L, Dh, o, lane);
  mma_pv<T, DHP>(o, sdSt, sQt, lane);                // dK = dSᵀ Q
  store_head<T, DHP>(gq + D, ld, L, Dh, o, lane);
}

template <typename T, int DHP>
void launch_fwd(int B, int L, int H, int Dh, const void* qkv, const int64_t* kv, DropParams dp,
                void* ctx, float* lse, hipStream_t s) {
  hipLaunchKernelGGL((mha_fwd_kernel<T, DHP>), dim3(B * H), dim3(64), 0, s, B, L, H, Dh,
                     (const T*)qkv, kv, dp, (T*)ctx, lse, 1.f / sqrtf((float)Dh));
}
template <typename T, int DHP>
void launch_bwd(int B, int L, int H, int Dh, const void* qkv, const int64_t* kv, const float* lse,
                const void* dctx, DropParams dp, void* dqkv, hipStream_t s) {
  hipLaunchKernelGGL((mha_bwd_kernel<T, DHP>), dim3(B * H), dim3(64), 0, s, B, L, H, Dh,
                     (const T*)qkv, kv, lse, (const T*)dctx, dp, (T*)dqkv, 1.f / sqrtf((float)Dh));
}

// ============================================================================================
// bf16 path v2 (the cfg-2 step): same math, one wave per (sequence, head), laid out so every
// global access is a full 16-byte vector and no operand is transposed on its way into LDS:
//   * Q/K/V/dO head slices are staged with unconditional (row-clamped) 16-byte loads, all
//     issued before the first LDS write, into row-major [64][DH] images;
//   * scores are built as Sᵀ-tiles (MFMA row operand = K), so a lane holds 4 consecutive keys
//     of one query row: the softmax reduces over 4 lanes, P·V takes P straight from registers
//     and V through the transposing LDS read (ds_read_b64_tr_b16), and the output lane holds
//     4 consecutive head columns -> 8-byte stores;
//   * the backward writes dS / Pd once as packed 8-byte rows and reads them transposed for
//     dK = dSᵀ·Q and dV = Pdᵀ·dO.

typedef __attribute__((ext_vector_type(4))) short s16x4a_t;
TTMI_DEV uint2 a_lds8(const char* p) { return *reinterpret_cast<const uint2*>(p); }
TTMI_DEV uint2 a_tr8(const char* p) {
  const s16x4a_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4a_t*)(p));
  return __builtin_bit_cast(uint2, v);
}
// fragment (16 rows x 32 k) of a [row][k] bf16 image; k-chunk c
template <int P>
TTMI_DEV uint4 a_fk(const char* s, int row0, int c, int lane) {
  const char* p = s + (row0 + (lane & 15)) * P + c * 64 + (lane >> 4) * 8;
  const uint2 lo = a_lds8(p), hi = a_lds8(p + 32);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}
// fragment (16 rows x 32 k) of a [k][row] bf16 image (transposing read)
template <int P>
TTMI_DEV uint4 a_ft(const char* s, int row0, int c, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const char* p = s + (c * 32 + 4 * g + (i >> 2)) * P + (row0 + 4 * (i & 3)) * 2;
  const uint2 lo = a_tr8(p), hi = a_tr8(p + 16 * P);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}
TTMI_DEV uint32_t a_pk2(float a, float b) { return pk_bf2(a, b); }
TTMI_DEV uint4 a_freg(const f32x4_t& lo, const f32x4_t& hi) {
  return make_uint4(a_pk2(lo[0], lo[1]), a_pk2(lo[2], lo[3]), a_pk2(hi[0], hi[1]), a_pk2(hi[2], hi[3]));
}
TTMI_DEV void a_st4(void* p, const f32x4_t& v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(a_pk2(v[0], v[1]), a_pk2(v[2], v[3]));
}

template <int DH>
struct Img2 {
  static constexpr int P = DH * 2 + 16;          // [64][DH] image pitch
  static constexpr int BYTES = 64 * P;
  static constexpr int SP = 64 * 2 + 16;         // [64][64] image pitch
  static constexpr int CPR = DH / 8;             // 16-byte chunks per row
};

// [L rows][DH] slice (row stride ld) -> [64][DH] image; rows >= L zero.  256 threads.
template <int DH, int NOP>
TTMI_DEV void stage_heads(char* const (&dst)[NOP], const bf16_t* const (&src)[NOP], int64_t ld,
                          int L, int lane) {
  using G = Img2<DH>;
  constexpr int NT = 256;
  static_assert((64 * G::CPR) % NT == 0, "head slice must split evenly over the workgroup");
  constexpr int PER = 64 * G::CPR / NT;
  uint4 v[NOP][PER];
#pragma unroll
  for (int o = 0; o < NOP; ++o)
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int idx = lane + NT * c, r = idx / G::CPR, ch = idx % G::CPR;
      v[o][c] = *reinterpret_cast<const uint4*>(src[o] + (int64_t)min(r, L - 1) * ld + ch * 8);
    }
#pragma unroll
  for (int o = 0; o < NOP; ++o)
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int idx = lane + NT * c, r = idx / G::CPR, ch = idx % G::CPR;
      *reinterpret_cast<uint4*>(dst[o] + r * G::P + ch * 16) = r < L ? v[o][c] : make_uint4(0u, 0u, 0u, 0u);
    }
}

// stage_heads in two halves (per-operand row strides): every operand's loads are issued, the
// caller issues its other loads, then the LDS images are written — one memory round trip for
// the whole prologue instead of one per operand group and per dependent small load
template <int DH, int NOP>
struct HeadStage {
  static constexpr int PER = 64 * Img2<DH>::CPR / 256;
  uint4 v[NOP][PER];
  TTMI_DEV void load(const bf16_t* const (&src)[NOP], const int64_t (&ld)[NOP], int L, int tid) {
#pragma unroll
    for (int o = 0; o < NOP; ++o)
#pragma unroll
      for (int c = 0; c < PER; ++c) {
        const int idx = tid + 256 * c, r = idx / Img2<DH>::CPR, ch = idx % Img2<DH>::CPR;
        v[o][c] = *reinterpret_cast<const uint4*>(src[o] + (int64_t)min(r, L - 1) * ld[o] + ch * 8);
      }
  }
  TTMI_DEV void store(char* const (&dst)[NOP], int L, int tid) const {
#pragma unroll
    for (int o = 0; o < NOP; ++o)
#pragma unroll
      for (int c = 0; c < PER; ++c) {
        const int idx = tid + 256 * c, r = idx / Img2<DH>::CPR, ch = idx % Img2<DH>::CPR;
        *reinterpret_cast<uint4*>(dst[o] + r * Img2<DH>::P + ch * 16) = r < L ? v[o][c] : make_uint4(0u, 0u, 0u, 0u);
      }
  }
};

// One wave's share of one (sequence, head): query tile i (rows 16i..16i+15) against the
// causal keys of the [64][DH] Q, K, V images at sQ / sK / sV (row pitch P bytes; rows >= L
// finite — they are masked keys / unstored queries).  kvm: the sequence's key-validity bits.
// ctx points at the sequence's first row of this head (row stride D), lse at the head's
// first query.  Shared by mha2_fwd_kernel and the fused projection + attention kernel.
template <int DH, int P>
TTMI_DEV void attn_tile_fwd(const char* sQ, const char* sK, const char* sV, uint64_t kvm, int i,
                            int L, int lane, const DropKeys& dk, uint32_t pbase, float scale,
                            bf16_t* ctx, int D, float* lse, f32x4_t* o_out = nullptr) {
  if (16 * i >= L) return;
  // The per-score work is VALU-issue bound (the softmax, the mask and the dropout hash over 16
  // scores a lane): key tiles above the diagonal (t > i, wave-uniform) are skipped outright, the
  // mask is one bit test per score, the scale rides in the exp2 argument and the dropout scale
  // in the row's 1/sum.
  const int li = lane & 15, lg = lane >> 4;
  const int q = 16 * i + li;
  // keys this query may attend: valid, causal (k <= q), and none for padded query rows
  const uint64_t causal = q >= 63 ? ~0ull : ((2ull << q) - 1ull);
  const uint64_t allow = q < L ? (kvm & causal) : 0ull;
  constexpr int NC = DH / 32;                      // 32-wide k chunks of the head dim
  uint4 qf[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) qf[c] = a_fk<P>(sQ, 16 * i, c, lane);
  f32x4_t s[4];
  float m = -INFINITY;                             // row max of the raw scores
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    s[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (t > i) continue;                           // wave-uniform
#pragma unroll
    for (int c = 0; c < NC; ++c) Mma<bf16_t>::run(s[t], a_fk<P>(sK, 16 * t, c, lane), qf[c]);
    const uint32_t nib = (uint32_t)(allow >> (16 * t + 4 * lg));
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s[t][e] = (nib >> e) & 1u ? s[t][e] : -INFINITY;
      m = fmaxf(m, s[t][e]);
    }
  }
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  const float sl2 = scale * 1.4426950408889634f;   // exp(scale (s - m)) = exp2(sl2 (s - m))
  const float mo = m == -INFINITY ? 0.f : m;       // fully masked row: every exp2(-inf) = 0
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (t > i) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float p = __builtin_amdgcn_exp2f((s[t][e] - mo) * sl2);   // v_exp_f32 (no range fix-up)
      s[t][e] = p;
      sum += p;
    }
  }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  const float inv = sum > 0.f ? (dk.on ? dk.scale : 1.f) / sum : 0.f;
  if (dk.on) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t > i) continue;
      // (the pair hash when L is even; identical to drop_keep per index)
      bool kp[4];
      drop_keep4(dk, pbase + (uint32_t)(q * L + 16 * t + 4 * lg), kp);
#pragma unroll
      for (int e = 0; e < 4; ++e) s[t][e] = kp[e] ? s[t][e] * inv : 0.f;
    }
  } else {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) s[t][e] *= inv;
  }
  f32x4_t o[DH / 16];
#pragma unroll
  for (int u = 0; u < DH / 16; ++u) o[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 2; ++c) {                  // 32-key chunks
    if (32 * c > 16 * i + 15) break;
    const uint4 pf = a_freg(s[2 * c], s[2 * c + 1]);
#pragma unroll
    for (int u = 0; u < DH / 16; ++u) Mma<bf16_t>::run(o[u], a_ft<P>(sV, 16 * u, c, lane), pf);
  }
  if (o_out != nullptr) {
#pragma unroll
    for (int u = 0; u < DH / 16; ++u) o_out[u] = o[u];
  }
  if (q < L) {
    bf16_t* dst = ctx + (int64_t)q * D + 4 * lg;
#pragma unroll
    for (int u = 0; u < DH / 16; ++u) a_st4(dst + 16 * u, o[u]);
    if (lg == 0) lse[q] = m == -INFINITY ? INFINITY : m * scale + __logf(sum);
  }
}

template <int DH>
__global__ __launch_bounds__(256) void mha2_fwd_kernel(int L, int H, const bf16_t* __restrict__ qkv,
                                                      const int64_t* __restrict__ kvalid, DropParams dp,
                                                      bf16_t* __restrict__ ctx, float* __restrict__ lse,
                                                      float scale) {
  using G = Img2<DH>;
  __shared__ __attribute__((aligned(16))) char smem[3 * G::BYTES];
  char* sQ = smem;
  char* sK = sQ + G::BYTES;
  char* sV = sK + G::BYTES;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // the H heads of one sequence read the same QKV rows: keep them on one XCD
  const int bh = xcd_contiguous(blockIdx.x, gridDim.x), b = bh / H, h = bh % H;
  const int D = H * DH;
  const int64_t ld = 3LL * D;
  const bf16_t* base = qkv + (int64_t)b * L * ld + (int64_t)h * DH;
  // key validity as one 64-bit ballot of wave 0 (one 8-byte load per lane, not 16); its load
  // and the head slices' are all in flight before the first LDS write
  const int64_t kvl = kvalid[(int64_t)b * L + min(lane, L - 1)];
  {
    HeadStage<DH, 3> st;
    const bf16_t* const src[3] = {base, base + D, base + 2 * D};
    const int64_t lds3[3] = {ld, ld, ld};
    st.load(src, lds3, L, threadIdx.x);
    char* const dst[3] = {sQ, sK, sV};
    st.store(dst, L, threadIdx.x);
  }
  __shared__ uint64_t s_kv;
  if (wave == 0) {
    const uint64_t bal = __ballot(lane < L && kvl != 0);
    if (lane == 0) s_kv = bal;
  }
  __syncthreads();
  const DropKeys dk = resolve_drop(dp);
  // wave w owns query tile w
  attn_tile_fwd<DH, G::P>(sQ, sK, sV, s_kv, wave, L, lane, dk, (uint32_t)((int64_t)bh * L * L), scale,
                          ctx + (int64_t)b * L * D + (int64_t)h * DH, D, lse + (int64_t)bh * L);
}

// DY: dO is not read from dctx but computed here from the out-projection's output gradient,
// dO = dy·W_o (the head's 32 columns; dy [B·L, 128] bf16, wot = W_oᵀ's k-major mirror), with
// the row-panel kernel's fragment order, MFMA order and bf16 rounding: the separate input-grad
// launch and its dctx round trip are gone, the values are the ones it would have written
// (DH = 32, D = 128 only; ABI 21, ttmi_mha_bwd_dy).
template <int DH, bool DY = false>
__global__ __launch_bounds__(256) void mha2_bwd_kernel(int L, int H, const bf16_t* __restrict__ qkv,
                                                      const int64_t* __restrict__ kvalid,
                                                      const float* __restrict__ lse,
                                                      const bf16_t* __restrict__ dctx, DropParams dp,
                                                      bf16_t* __restrict__ dqkv, float scale,
                                                      const bf16_t* __restrict__ dy = nullptr,
                                                      const bf16_t* __restrict__ wot = nullptr) {
  static_assert(!DY || DH == 32, "dO from dy: d_model 128, 4 heads of 32");
  using G = Img2<DH>;
  __shared__ __attribute__((aligned(16))) char smem[4 * G::BYTES + 2 * 64 * G::SP];
  char* sQ = smem;
  char* sK = sQ + G::BYTES;
  char* sV = sK + G::BYTES;
  char* sdO = sV + G::BYTES;
  char* sdS = sdO + G::BYTES;                      // [q][k] bf16 (raw-score gradient · scale)
  char* sPd = sdS + 64 * G::SP;                    // [q][k] bf16 (dropped probabilities)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, lg = lane >> 4;
  // the H heads of one sequence read the same QKV rows: keep them on one XCD
  const int bh = xcd_contiguous(blockIdx.x, gridDim.x), b = bh / H, h = bh % H;
  const int D = H * DH;
  const int64_t ld = 3LL * D;
  const bf16_t* base = qkv + (int64_t)b * L * ld + (int64_t)h * DH;
  // every global load of the prologue in flight at once (the head slices, the key validity,
  // this lane's query row's log-sum-exp), then the LDS images: one memory round trip
  const int64_t kvl = kvalid[(int64_t)b * L + min(lane, L - 1)];
  const int qrow = 16 * wave + li;
  const float lr0 = lse[(int64_t)bh * L + min(qrow, L - 1)];
  uint4 daf[DY ? 4 : 1], dwf[DY ? 2 : 1][DY ? 4 : 1];
  if constexpr (DY) {
    // this wave's 16 rows of dy (k = 32 lg + 8 c) and the head's 32 rows of W_oᵀ, column-paired
    // as the panel pairs them (tile t rows 4 t + 8 (li >> 2) + (li & 3) of the head's 32)
    const char* ap = reinterpret_cast<const char*>(dy + ((int64_t)b * L + min(qrow, L - 1)) * 128 + lg * 32);
#pragma unroll
    for (int c = 0; c < 4; ++c) daf[c] = *reinterpret_cast<const uint4*>(ap + 16 * c);
    const int wrow = 8 * (li >> 2) + (li & 3);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const char* wp = reinterpret_cast<const char*>(wot + (int64_t)(32 * h + 4 * t + wrow) * 128 + lg * 32);
#pragma unroll
      for (int c = 0; c < 4; ++c) dwf[t][c] = *reinterpret_cast<const uint4*>(wp + 16 * c);
    }
    HeadStage<DH, 3> st;
    const bf16_t* const src[3] = {base, base + D, base + 2 * D};
    const int64_t lds3[3] = {ld, ld, ld};
    st.load(src, lds3, L, threadIdx.x);
    char* const dst[3] = {sQ, sK, sV};
    st.store(dst, L, threadIdx.x);
  } else {
    HeadStage<DH, 4> st;
    const bf16_t* const src[4] = {base, base + D, base + 2 * D, dctx + (int64_t)b * L * D + (int64_t)h * DH};
    const int64_t lds4[4] = {ld, ld, ld, (int64_t)D};
    st.load(src, lds4, L, threadIdx.x);
    char* const dst[4] = {sQ, sK, sV, sdO};
    st.store(dst, L, threadIdx.x);
  }
  if constexpr (DY) {   // dO rows of this wave's tile (rows >= L zero, as the staging writes them)
    f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int t = 0; t < 2; ++t) Mma<bf16_t>::run(acc[t], dwf[t][c], daf[c]);
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = acc[0][e] + 0.f; v[4 + e] = acc[1][e] + 0.f; }
    const bool live = qrow < L;
    *reinterpret_cast<uint4*>(sdO + qrow * G::P + lg * 16) =
        live ? make_uint4(a_pk2(v[0], v[1]), a_pk2(v[2], v[3]), a_pk2(v[4], v[5]), a_pk2(v[6], v[7]))
             : make_uint4(0u, 0u, 0u, 0u);
  }
  __shared__ uint64_t s_kv;
  if (wave == 0) {
    const uint64_t bal = __ballot(lane < L && kvl != 0);
    if (lane == 0) s_kv = bal;
  }
  __syncthreads();
  const uint64_t kvm = s_kv;
  const DropKeys dk = resolve_drop(dp);
  const float dsc = dk.on ? dk.scale : 1.f;
  const uint32_t pbase = (uint32_t)((int64_t)bh * L * L);
  constexpr int NC = DH / 32;
  bf16_t* gq = dqkv + (int64_t)b * L * ld + (int64_t)h * DH;
#pragma unroll
  for (int i = wave; i < 4; i += 4) {      // wave w owns query tile w
    const int q = 16 * i + li;
    uint4 qf[NC], of[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      qf[c] = a_fk<G::P>(sQ, 16 * i, c, lane);
      of[c] = a_fk<G::P>(sdO, 16 * i, c, lane);
    }
    // the recomputed P is VALU-issue bound like the forward's softmax (attn_tile_fwd): key
    // tiles above the diagonal are skipped, the mask is a bit test, exp(s·scale - lse) one exp2
    const uint64_t causal = q >= 63 ? ~0ull : ((2ull << q) - 1ull);
    const uint64_t allow = q < L ? (kvm & causal) : 0ull;
    const float sl2 = scale * 1.4426950408889634f, lr2 = lr0 * 1.4426950408889634f;
    f32x4_t s[4], dpv[4];
    uint32_t keep[4];                              // dropout keep bits, one hash pass
    float dsum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = dpv[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      keep[t] = 0xFu;
      if (t > i) continue;                         // wave-uniform
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        Mma<bf16_t>::run(s[t], a_fk<G::P>(sK, 16 * t, c, lane), qf[c]);
        Mma<bf16_t>::run(dpv[t], a_fk<G::P>(sV, 16 * t, c, lane), of[c]);
      }
      if (dk.on) {
        bool kp[4];
        drop_keep4(dk, pbase + (uint32_t)(q * L + 16 * t + 4 * lg), kp);
        keep[t] = (kp[0] ? 1u : 0u) | (kp[1] ? 2u : 0u) | (kp[2] ? 4u : 0u) | (kp[3] ? 8u : 0u);
      }
      const uint32_t nib = (uint32_t)(allow >> (16 * t + 4 * lg));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = (nib >> e) & 1u;
        const float p = ok ? __builtin_amdgcn_exp2f(fmaf(s[t][e], sl2, -lr2)) : 0.f;
        const float dP = ok && ((keep[t] >> e) & 1u) ? dpv[t][e] * dsc : 0.f;
        s[t][e] = p;
        dpv[t][e] = dP;
        dsum += p * dP;
      }
    }
    dsum += __shfl_xor(dsum, 16, 64);
    dsum += __shfl_xor(dsum, 32, 64);
    f32x4_t ds[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x4_t pd;
      if (t > i) {                                 // zeros: the dK / dV pass reads these rows
        ds[t] = pd = f32x4_t{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float p = s[t][e];
          ds[t][e] = p * (dpv[t][e] - dsum) * scale;
          pd[e] = ((keep[t] >> e) & 1u) ? p * dsc : 0.f;
        }
      }
      a_st4(sdS + q * G::SP + (16 * t + 4 * lg) * 2, ds[t]);
      a_st4(sPd + q * G::SP + (16 * t + 4 * lg) * 2, pd);
    }
    // dQ rows of this tile = dS·K (K through the transposing read)
    f32x4_t dq[DH / 16];
#pragma unroll
    for (int u = 0; u < DH / 16; ++u) dq[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      if (32 * c > 16 * i + 15) break;
      const uint4 af = a_freg(ds[2 * c], ds[2 * c + 1]);
#pragma unroll
      for (int u = 0; u < DH / 16; ++u) Mma<bf16_t>::run(dq[u], a_ft<G::P>(sK, 16 * u, c, lane), af);
    }
    if (q < L) {
      bf16_t* dst = gq + (int64_t)q * ld + 4 * lg;
#pragma unroll
      for (int u = 0; u < DH / 16; ++u) a_st4(dst + 16 * u, dq[u]);
    }
  }
  __syncthreads();
  // dK = dSᵀ·Q and dV = Pdᵀ·dO per key tile t (query rows >= 16t only: causal)
#pragma unroll
  for (int t = wave; t < 4; t += 4) {      // wave w owns key tile w
    if (16 * t >= L) break;
    f32x4_t dkv[DH / 16], dvv[DH / 16];
#pragma unroll
    for (int u = 0; u < DH / 16; ++u) dkv[u] = dvv[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 2; ++c) {                  // 32-query chunks
      if (32 * c + 31 < 16 * t) continue;
      const uint4 as = a_ft<G::SP>(sdS, 16 * t, c, lane), ap = a_ft<G::SP>(sPd, 16 * t, c, lane);
#pragma unroll
      for (int u = 0; u < DH / 16; ++u) {
        Mma<bf16_t>::run(dkv[u], a_ft<G::P>(sQ, 16 * u, c, lane), as);
        Mma<bf16_t>::run(dvv[u], a_ft<G::P>(sdO, 16 * u, c, lane), ap);
      }
    }
    const int k = 16 * t + li;
    if (k < L) {
      bf16_t* dst = gq + (int64_t)k * ld + 4 * lg;
#pragma unroll
      for (int u = 0; u < DH / 16; ++u) {
        a_st4(dst + D + 16 * u, dkv[u]);
        a_st4(dst + 2 * D + 16 * u, dvv[u]);
      }
    }
  }
}

// ---------------------------------------------------------------- in_proj + attention (forward)
// nn.MultiheadAttention's input projection and its SDPA core in one launch (reference
// user_tower.py:111-116) for d_model 128, 4 heads of 32.  A workgroup owns whole sequences
// (2 at L = 50: 100 rows, 7 row tiles of 16), so the attention reads Q, K, V straight from the
// LDS images of the projection it has just computed — the separate attention launch, its
// dispatch ramp and its qkv re-read are gone.  qkv still goes to HBM (the backward reads it),
// copied out of the images with coalesced stores under the attention.
//
// Every operand arrives by LDS-DMA, all of it issued up front (the A rows, the bias, the three
// 128-column groups of W_in: one memory round trip), so no compiler-counted load sits in the
// vmcnt queue ahead of a manual wait.  LDS: W0 | W1 | W2 | A (later the Q image) | bias.  The
// K image overlays W0 once group 0 is consumed, V overlays W1.  The projection's MFMA order,
// bias add and bf16 rounding are the panel kernel's (ttmi_gemm.hip), the attention is
// attn_tile_fwd: bit-identical to ttmi_linear (from M = 2048 rows, where the panel serves it)
// + ttmi_mha_fwd.
constexpr int QA_D = 128;                         // d_model (= in_proj K)
constexpr int QA_P = 2 * QA_D + 16;               // row pitch (bytes) of every image (W, A, Q, K, V)
constexpr int QA_CPR = QA_D / 8 + 1;              // 16-byte chunks per image row (incl. the pad)
constexpr int QA_WBUF = 128 * QA_P;               // one W column group's image
constexpr int QA_ROWS = 114;                      // Q / K / V image rows (the last key tile of the
                                                  // last sequence reads up to row (spw-1)L + 63)
constexpr int QA_IMG = QA_ROWS * QA_P;
constexpr int QA_AI = (112 * QA_CPR + 63) / 64;   // A DMA wave-instructions (7 row tiles)
constexpr int QA_BI = 2;                          // bias DMA wave-instructions (384 fp32)
constexpr int QA_WI = 128 * QA_CPR / 64;          // one W group's DMA wave-instructions
constexpr int QA_I0 = QA_AI + QA_BI + QA_WI;      // the first wait's instructions (A, bias, W0)
constexpr int QA_NW = 16;                         // waves per workgroup
constexpr int QA_MAXSEQ = 8;
static_assert(QA_AI * 1024 <= QA_IMG, "A staging fits the Q image");
static_assert((128 * QA_CPR) % 64 == 0, "whole W DMA instructions");

struct QaArgs {
  const bf16_t* a;          // [B*L, 128] normed input
  const bf16_t* w;          // [384, 128] in_proj weight
  const float* bias;        // [384]
  const int64_t* kvalid;    // [B, L]
  bf16_t* qkv;              // [B*L, 384]
  bf16_t* ctx;              // [B*L, 128]
  float* lse;               // [B*4*L]
  DropParams dp;
  float scale;
  int B, L, spw;
  // OP (ABI 21, ttmi_attn_block_fwd): the out-projection, residual, dropout 1 and norm2 too
  const bf16_t* wo; const float* bo; const float* res; const float* n2w; const float* n2b;
  float eps; DropParams dp1;
  float* x1; bf16_t* a2; float* m2; float* r2;
};

// s_waitcnt vmcnt(N) for a wave-dependent N in {lo, hi}
template <int HI, int LO>
TTMI_DEV void qa_wait(bool hi) {
  if (hi) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(HI) : "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LO) : "memory");
}

// OP: the attention's out-projection, residual (+ dropout 1) and norm2 in the same launch
// (user_tower.py:37-45, norm_first: x1 = x + drop1(ctx·W_oᵀ + b_o), a2 = norm2(x1)).  W_o is
// DMA'd into the consumed W2 image under the attention, the context rows stay in registers
// until the attention's last read of the Q / K / V images, then become an LDS image over K's.
// Each wave computes one row tile's half (64 columns); norm2's row statistics meet across the
// two halves through LDS.  Two rounds of (sequence, head) pairs at most (spw <= 2).
constexpr int QA_PI = 3;                          // OP: b_o, norm2 weight / bias, 1 KB slot each
template <bool OP>
__global__ __launch_bounds__(1024) void qkv_attn_fwd_kernel(QaArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[3 * QA_WBUF + QA_IMG + QA_BI * 1024 + (OP ? QA_PI * 1024 : 0)];
  __shared__ uint64_t s_kv[QA_MAXSEQ];
  __shared__ float s_red[OP ? 2 : 1][8][2][16];  // OP: norm2's per-half row sums (mean, variance)
  char* const sq = smem + 3 * QA_WBUF;            // A staging, then the Q image
  const float* const sbias = reinterpret_cast<const float*>(sq + QA_IMG);
  const float* const sbo = sbias + QA_BI * 256;   // OP: b_o, n2w, n2b at 1 KB strides
  const float* const sn2w = sbo + 256;
  const float* const sn2b = sbo + 512;
  TTMI_TSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int L = g.L, b0 = blockIdx.x * g.spw, nseq = min(g.spw, g.B - b0), R = nseq * L;
  const int64_t r0 = (int64_t)b0 * L;
  const int ntiles = (R + 15) >> 4;               // <= 7 (host: spw * L <= 112)
  const int64_t kvl = wave < nseq ? g.kvalid[r0 + (int64_t)wave * L + min(lane, L - 1)] : 0;
  // ---- every DMA up front; wave w issues wave-instructions w, w + 16, ... of each batch
  {
    // (the row pad chunks read at each buffer's end: out of range, zeros)
    const uint32_t abytes = (uint32_t)R * QA_D * 2, wbytes = 3 * QA_D * QA_D * 2;
    const i32x4_t ra = make_rsrc(g.a + r0 * QA_D, abytes);          // rows >= R: zeros
    const i32x4_t rb = make_rsrc(g.bias, 3 * QA_D * 4);
    const i32x4_t rw = make_rsrc(g.w, wbytes);
    const uint32_t lw = lds_addr(smem), la = lds_addr(sq), lb = lds_addr(sq + QA_IMG);
    if constexpr (OP) {      // (batch 0: older than the W1 / W2 batches the waits below count)
      if (wave >= QA_NW - QA_PI) {
        const int k = wave - (QA_NW - QA_PI);
        const float* src = k == 0 ? g.bo : (k == 1 ? g.n2w : g.n2b);
        dma16(make_rsrc(src, QA_D * 4), (uint32_t)(lane * 16), lb + (QA_BI + k) * 1024);
      }
    }
#pragma unroll
    for (int t = 0; t < (QA_I0 + QA_NW - 1) / QA_NW; ++t) {
      const int ii = wave + QA_NW * t;            // wave-uniform branches
      if (ii >= QA_I0) break;
      if (ii < QA_AI) {
        const int q = ii * 64 + lane, r = q / QA_CPR, c = q % QA_CPR;
        dma16(ra, c == QA_CPR - 1 ? abytes : (uint32_t)((r * QA_D + 8 * c) * 2), la + ii * 1024);
      } else if (ii < QA_AI + QA_BI) {
        const int j = ii - QA_AI;
        dma16(rb, (uint32_t)((j * 64 + lane) * 16), lb + j * 1024);
      } else {
        const int j = ii - QA_AI - QA_BI, q = j * 64 + lane, n = q / QA_CPR, c = q % QA_CPR;
        dma16(rw, c == QA_CPR - 1 ? wbytes : (uint32_t)((n * QA_D + 8 * c) * 2), lw + j * 1024);
      }
    }
#pragma unroll
    for (int cg = 1; cg < 3; ++cg)
#pragma unroll
      for (int t = 0; t < (QA_WI + QA_NW - 1) / QA_NW; ++t) {
        const int j = wave + QA_NW * t;
        if (j >= QA_WI) break;
        const int q = j * 64 + lane, n = q / QA_CPR, c = q % QA_CPR;
        dma16(rw, c == QA_CPR - 1 ? wbytes : (uint32_t)(((cg * 128 + n) * QA_D + 8 * c) * 2),
              lw + cg * QA_WBUF + j * 1024);
      }
  }
  // per-wave DMA counts of the W1 and W2 batches: the waits below leave exactly those in flight
  constexpr int C_HI = (QA_WI + QA_NW - 1) / QA_NW;             // waves below QA_WI % 16
  static_assert(QA_WI % QA_NW != 0 && C_HI - 1 == QA_WI / QA_NW, "two per-wave counts");
  const bool hi = wave < QA_WI % QA_NW;
  // the Q image's rows past the A staging are read as masked keys: zero
  for (int i = QA_AI * 64 + tid; i < QA_ROWS * QA_CPR; i += 64 * QA_NW)
    *reinterpret_cast<uint4*>(sq + 16 * i) = make_uint4(0u, 0u, 0u, 0u);
  // ---- projection: 16 waves, wave w computes row tile w & 7, column half w >> 3 (4 of the 8
  // column tiles of each group)
  const int rt = wave & 7, half = wave >> 3;
  const int wrow = 8 * (li >> 2) + (li & 3);      // column-paired W rows (panel layout)
  const int row = 16 * rt + li;
  const bool mine = rt < ntiles;
  uint4 af[4];
#pragma unroll 1
  for (int cg = 0; cg < 3; ++cg) {
    if (cg == 0) qa_wait<2 * C_HI, 2 * (C_HI - 1)>(hi);
    else if (cg == 1) qa_wait<C_HI, C_HI - 1>(hi);
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                              // every wave's DMAs of this batch landed
    if (cg == 0) {
      TTMI_TSTAMP(1);
#pragma unroll
      for (int c = 0; c < 4; ++c) af[c] = lds16(sq + row * QA_P + lg * 64 + 16 * c);
    } else {
      // group cg - 1's W image is consumed: it becomes the K (cg 1) / V (cg 2) image, whose
      // rows past the last tile must read as zeros
      char* img = smem + (cg - 1) * QA_WBUF;
      for (int i = 16 * ntiles * QA_CPR + tid; i < QA_ROWS * QA_CPR; i += 64 * QA_NW)
        *reinterpret_cast<uint4*>(img + 16 * i) = make_uint4(0u, 0u, 0u, 0u);
    }
    f32x4_t acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (mine) {
      const char* wb = smem + cg * QA_WBUF + (64 * half + wrow) * QA_P + lg * (QA_D / 2);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          Mma<bf16_t>::run(acc[t], lds16(wb + (32 * (t >> 1) + 4 * (t & 1)) * QA_P + 16 * c), af[c]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (cg == 0) __syncthreads();                 // every wave's A rows read: Q overwrites them
    if (mine) {
      char* lrow = (cg == 0 ? sq : smem + (cg - 1) * QA_WBUF) + row * QA_P;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int nl = 64 * half + 32 * p + 8 * lg;   // column within the group
        const float* bp = sbias + cg * 128 + nl;
        const float4 b_lo = *reinterpret_cast<const float4*>(bp);
        const float4 b_hi = *reinterpret_cast<const float4*>(bp + 4);
        const float v[8] = {acc[2 * p][0] + b_lo.x, acc[2 * p][1] + b_lo.y, acc[2 * p][2] + b_lo.z,
                            acc[2 * p][3] + b_lo.w, acc[2 * p + 1][0] + b_hi.x, acc[2 * p + 1][1] + b_hi.y,
                            acc[2 * p + 1][2] + b_hi.z, acc[2 * p + 1][3] + b_hi.w};
        *reinterpret_cast<uint4*>(lrow + 2 * nl) =
            make_uint4(a_pk2(v[0], v[1]), a_pk2(v[2], v[3]), a_pk2(v[4], v[5]), a_pk2(v[6], v[7]));
      }
    }
  }
  if (wave < nseq) {
    const uint64_t bal = __ballot(lane < L && kvl != 0);
    if (lane == 0) s_kv[wave] = bal;
  }
  __syncthreads();
  TTMI_TSTAMP(2);
  // the dropout seeds and (OP) the residual values are loaded BEFORE W_o's DMAs: a compiler-
  // counted wait for them then never includes the DMAs behind it (vmcnt retires in order)
  const DropKeys dk = resolve_drop(g.dp);
  const DropKeys dk1 = OP ? resolve_drop(g.dp1) : dk;
  float4 rpre[OP ? 4 : 1];
  if constexpr (OP) {
    const float* rp = g.res + (r0 + min(row, R - 1)) * QA_D + 64 * half + 8 * lg;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      rpre[2 * p] = *reinterpret_cast<const float4*>(rp + 32 * p);
      rpre[2 * p + 1] = *reinterpret_cast<const float4*>(rp + 32 * p + 4);
    }
    // W_o into the consumed W2 image (lands under the attention)
    const i32x4_t ro = make_rsrc(g.wo, QA_D * QA_D * 2);
    const uint32_t lo = lds_addr(smem + 2 * QA_WBUF);
#pragma unroll
    for (int t = 0; t < (QA_WI + QA_NW - 1) / QA_NW; ++t) {
      const int j = wave + QA_NW * t;
      if (j >= QA_WI) break;
      const int q = j * 64 + lane, n = q / QA_CPR, c = q % QA_CPR;
      dma16(ro, c == QA_CPR - 1 ? (uint32_t)(QA_D * QA_D * 2) : (uint32_t)((n * QA_D + 8 * c) * 2), lo + j * 1024);
    }
  }
  // ---- qkv to HBM from the images (coalesced 16-byte stores, in flight under the attention)
  for (int i = tid; i < R * 48; i += 64 * QA_NW) {
    const int r = i / 48, c = i % 48, m = c >> 4;  // m: Q (A region), K (W0), V (W1)
    const char* src = (m == 0 ? sq : smem + (m - 1) * QA_WBUF) + r * QA_P + 16 * (c & 15);
    *reinterpret_cast<uint4*>(g.qkv + (r0 + r) * (3 * QA_D) + 8 * c) = lds16(src);
  }
  // ---- attention: round s handles sequence s, wave w its head w >> 2 and query tile w & 3 on
  // even rounds, 3 - (w & 3) on odd ones (tile i costs i + 1 key tiles: pairing i with 3 - i
  // evens the waves' work, the workgroup ends with its slowest wave)
  f32x4_t oc[OP ? 2 : 1][2];
  if constexpr (OP) {
#pragma unroll
    for (int s = 0; s < 2; ++s) oc[s][0] = oc[s][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  for (int s = 0; s < nseq; ++s) {
    const int h = wave >> 2, qt = (s & 1) ? 3 - (wave & 3) : (wave & 3);
    const int64_t bh = (int64_t)(b0 + s) * 4 + h;
    const int off = s * L * QA_P + h * 64;
    attn_tile_fwd<32, QA_P>(sq + off, smem + off, smem + QA_WBUF + off, s_kv[s], qt, L, lane, dk,
                            (uint32_t)(bh * L * L), g.scale, g.ctx + (r0 + (int64_t)s * L) * QA_D + h * 32,
                            QA_D, g.lse + bh * L, OP ? oc[s & 1] : nullptr);
  }
  TTMI_TSTAMP(3);
  if constexpr (OP) {
    __syncthreads();                              // every wave is past its Q / K / V reads
    char* const sctx = smem;                      // the context image over K's
    {
      const int h = wave >> 2;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (s >= nseq) break;
        const int qt = (s & 1) ? 3 - (wave & 3) : (wave & 3), q = 16 * qt + li;
        if (q < L) {
          char* dst = sctx + (s * L + q) * QA_P + (h * 32 + 4 * lg) * 2;
          a_st4(dst, oc[s][0]);
          a_st4(dst + 32, oc[s][1]);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // W_o landed (this wave's DMAs)
    __syncthreads();
    // ---- x1 = res + drop1(ctx·W_oᵀ + b_o) for this wave's row tile, 64 columns
    f32x4_t acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (mine) {
      uint4 cf[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) cf[c] = lds16(sctx + row * QA_P + lg * 64 + 16 * c);
      const char* wb = smem + 2 * QA_WBUF + (64 * half + wrow) * QA_P + lg * (QA_D / 2);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          Mma<bf16_t>::run(acc[t], lds16(wb + (32 * (t >> 1) + 4 * (t & 1)) * QA_P + 16 * c), cf[c]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    const int64_t m = r0 + row;
    const bool mok = mine && row < R;
    float vr[16];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int n = 64 * half + 32 * p + 8 * lg;
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[2 * p][e] + sbo[n + e];
        v[4 + e] = acc[2 * p + 1][e] + sbo[n + 4 + e];
      }
      drop_apply_vec<8>(dk1, (uint32_t)(m * QA_D + n), v);
      const float4 q0 = rpre[2 * p], q1 = rpre[2 * p + 1];
      v[0] += q0.x; v[1] += q0.y; v[2] += q0.z; v[3] += q0.w;
      v[4] += q1.x; v[5] += q1.y; v[6] += q1.z; v[7] += q1.w;
      if (mok) {
        float* xp = g.x1 + m * QA_D + n;
        *reinterpret_cast<float4*>(xp) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(xp + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) vr[8 * p + e] = v[e];
    }
    // ---- a2 = norm2(x1): the row's 128 columns over two waves (mean, then variance)
    float s1 = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) s1 += vr[e];
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    if (lg == 0) s_red[0][rt][half][li] = s1;
    __syncthreads();
    const float mu = (s_red[0][rt][0][li] + s_red[0][rt][1][li]) * (1.f / QA_D);
    float s2 = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) s2 += (vr[e] - mu) * (vr[e] - mu);
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (lg == 0) s_red[1][rt][half][li] = s2;
    __syncthreads();
    const float rs = 1.f / sqrtf((s_red[1][rt][0][li] + s_red[1][rt][1][li]) * (1.f / QA_D) + g.eps);
    if (mok) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int n = 64 * half + 32 * p + 8 * lg;
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (vr[8 * p + e] - mu) * rs * sn2w[n + e] + sn2b[n + e];
        *reinterpret_cast<uint4*>(g.a2 + m * QA_D + n) =
            make_uint4(a_pk2(o[0], o[1]), a_pk2(o[2], o[3]), a_pk2(o[4], o[5]), a_pk2(o[6], o[7]));
      }
      if (half == 0 && lg == 0) {
        g.m2[m] = mu;
        g.r2[m] = rs;
      }
    }
  }
}


// sequences per workgroup for the fused kernel: the most whose rows fit the 7 row tiles and
// whose last key tile stays inside the image; 0 = shape not served
int qa_spw(int L) {
  if (L <= 0 || L > 64) return 0;
  for (int s = QA_MAXSEQ; s >= 1; --s)
    if (s * L <= 112 && (s - 1) * L + 64 <= QA_ROWS) return s;
  return 0;
}

int check_mha(const char* fn, int dtype, int B, int L, int H, int Dh, const void* qkv,
              const int64_t* kv, float drop_p) {
  TTMI_REQUIRE(dtype == TTMI_F32 || dtype == TTMI_BF16, "%s: bad dtype", fn);
  TTMI_REQUIRE(B >= 0 && L > 0 && L <= TTMI_ATTN_LMAX && H > 0, "%s: need 0 < L <= %d (got L=%d)", fn,
               TTMI_ATTN_LMAX, L);
  TTMI_REQUIRE(Dh > 0 && Dh <= 64 && Dh % 8 == 0, "%s: need Dh %% 8 == 0 and Dh <= 64 (got %d)", fn, Dh);
  TTMI_REQUIRE(qkv && kv, "%s: null argument", fn);
  TTMI_REQUIRE(((uintptr_t)qkv & 15) == 0, "%s: qkv must be 16-byte aligned", fn);
  // the attention-dropout mask index (b·H + h)·L² + i·L + j is 32-bit: bounded only when
  // dropout is on (eval and inference encoding of any batch size pass)
  TTMI_REQUIRE(drop_p == 0.f || (int64_t)B * H * L * L < (1LL << 32),
               "%s: with dropout on, B*H*L*L must stay below 2^32 (32-bit mask index); split the batch", fn);
  return TTMI_OK;
}

}  // namespace

extern "C" int ttmi_mha_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                            const int64_t* key_valid, float drop_p, const uint64_t* drop_seed, void* ctx,
                            float* lse, hipStream_t s) {
  int rc = check_mha("ttmi_mha_fwd", dtype, B, L, H, Dh, qkv, key_valid, drop_p);
  if (rc) return rc;
  TTMI_REQUIRE(ctx && lse, "ttmi_mha_fwd: null output");
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "ttmi_mha_fwd: drop_p out of [0,1)");
  if (B == 0) return TTMI_OK;
  DropParams dp = make_drop(drop_p, drop_seed);
  if (L > LP) return attn_long_fwd(dtype, B, L, H, Dh, qkv, key_valid, dp, ctx, lse, s);
  if (dtype == TTMI_BF16 && (Dh == 32 || Dh == 64) && !getenv("TTMI_MHA_V1")) {
    TTMI_REQUIRE(((uintptr_t)ctx & 7) == 0, "ttmi_mha_fwd: ctx must be 8-byte aligned");
    const float sc = 1.f / sqrtf((float)Dh);
    if (Dh == 32)
      hipLaunchKernelGGL(mha2_fwd_kernel<32>, dim3(B * H), dim3(256), 0, s, L, H, (const bf16_t*)qkv,
                         key_valid, dp, (bf16_t*)ctx, lse, sc);
    else
      hipLaunchKernelGGL(mha2_fwd_kernel<64>, dim3(B * H), dim3(256), 0, s, L, H, (const bf16_t*)qkv,
                         key_valid, dp, (bf16_t*)ctx, lse, sc);
  } else if (dtype == TTMI_BF16) {
    if (Dh <= 32) launch_fwd<bf16_t, 32>(B, L, H, Dh, qkv, key_valid, dp, ctx, lse, s);
    else launch_fwd<bf16_t, 64>(B, L, H, Dh, qkv, key_valid, dp, ctx, lse, s);
  } else {
    if (Dh <= 32) launch_fwd<float, 32>(B, L, H, Dh, qkv, key_valid, dp, ctx, lse, s);
    else launch_fwd<float, 64>(B, L, H, Dh, qkv, key_valid, dp, ctx, lse, s);
  }
  return ttmi_check_launch("ttmi_mha_fwd");
}

extern "C" int ttmi_qkv_attn_supported(int dtype, int L, int H, int Dh) {
  return dtype == TTMI_BF16 && H * Dh == QA_D && Dh == 32 && qa_spw(L) > 0;
}

extern "C" int ttmi_qkv_attn_fwd(int dtype, int B, int L, int H, int Dh, const void* a, const void* w_in,
                                 const float* b_in, const int64_t* key_valid, float drop_p,
                                 const uint64_t* drop_seed, void* qkv, void* ctx, float* lse, hipStream_t s) {
  static const char* fn = "ttmi_qkv_attn_fwd";
  int rc = check_mha(fn, dtype, B, L, H, Dh, qkv, key_valid, drop_p);
  if (rc) return rc;
  TTMI_REQUIRE(ttmi_qkv_attn_supported(dtype, L, H, Dh),
               "%s: serves bf16, H*Dh = 128 with Dh = 32, L <= 64 (got L=%d H=%d Dh=%d); use ttmi_linear + "
               "ttmi_mha_fwd", fn, L, H, Dh);
  TTMI_REQUIRE(a && w_in && b_in && ctx && lse, "%s: null argument", fn);
  TTMI_REQUIRE((((uintptr_t)a | (uintptr_t)w_in | (uintptr_t)b_in | (uintptr_t)ctx) & 15) == 0,
               "%s: a, w_in, b_in, ctx must be 16-byte aligned", fn);
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "%s: drop_p out of [0,1)", fn);
  if (B == 0) return TTMI_OK;
  QaArgs g{(const bf16_t*)a, (const bf16_t*)w_in, b_in, key_valid, (bf16_t*)qkv, (bf16_t*)ctx, lse,
           make_drop(drop_p, drop_seed), 1.f / sqrtf((float)Dh), B, L, qa_spw(L)};
  hipLaunchKernelGGL(qkv_attn_fwd_kernel<false>, dim3((B + g.spw - 1) / g.spw), dim3(1024), 0, s, g);
  return ttmi_check_launch(fn);
}

extern "C" int ttmi_attn_block_fwd(const ttmi_attn_block_desc* d, hipStream_t s) {
  static const char* fn = "ttmi_attn_block_fwd";
  TTMI_REQUIRE(d != nullptr, "%s: null descriptor", fn);
  int rc = check_mha(fn, TTMI_BF16, d->B, d->L, d->H, d->Dh, d->qkv, d->key_valid, d->drop_p);
  if (rc) return rc;
  const int spw = qa_spw(d->L);
  TTMI_REQUIRE(d->H * d->Dh == QA_D && d->Dh == 32 && spw > 0 && spw <= 2,
               "%s: serves bf16, H*Dh = 128 with Dh = 32 and 38 <= L <= 64 (got L=%d)", fn, d->L);
  TTMI_REQUIRE(d->a && d->w_in && d->b_in && d->ctx && d->lse && d->wo && d->bo && d->res && d->n2w && d->n2b &&
                   d->x1 && d->a2 && d->m2 && d->r2, "%s: null argument", fn);
  TTMI_REQUIRE((((uintptr_t)d->a | (uintptr_t)d->w_in | (uintptr_t)d->b_in | (uintptr_t)d->ctx | (uintptr_t)d->wo |
                 (uintptr_t)d->bo | (uintptr_t)d->res | (uintptr_t)d->n2w | (uintptr_t)d->n2b | (uintptr_t)d->x1 |
                 (uintptr_t)d->a2) & 15) == 0, "%s: operands must be 16-byte aligned", fn);
  TTMI_REQUIRE(d->drop_p >= 0.f && d->drop_p < 1.f && d->drop1_p >= 0.f && d->drop1_p < 1.f,
               "%s: dropout out of [0,1)", fn);
  if (d->B == 0) return TTMI_OK;
  QaArgs g{};
  g.a = (const bf16_t*)d->a; g.w = (const bf16_t*)d->w_in; g.bias = d->b_in; g.kvalid = d->key_valid;
  g.qkv = (bf16_t*)d->qkv; g.ctx = (bf16_t*)d->ctx; g.lse = d->lse;
  g.dp = make_drop(d->drop_p, d->drop_seed); g.scale = 1.f / sqrtf((float)d->Dh);
  g.B = d->B; g.L = d->L; g.spw = spw;
  g.wo = (const bf16_t*)d->wo; g.bo = d->bo; g.res = d->res; g.n2w = d->n2w; g.n2b = d->n2b; g.eps = d->eps;
  g.dp1 = make_drop(d->drop1_p, d->drop1_seed);
  g.x1 = d->x1; g.a2 = (bf16_t*)d->a2; g.m2 = d->m2; g.r2 = d->r2;
  hipLaunchKernelGGL(qkv_attn_fwd_kernel<true>, dim3((d->B + spw - 1) / spw), dim3(1024), 0, s, g);
  return ttmi_check_launch(fn);
}

extern "C" int ttmi_mha_bwd_dy(int B, int L, int H, int Dh, const void* qkv, const int64_t* key_valid,
                               const float* lse, const void* dy, const void* wot, float drop_p,
                               const uint64_t* drop_seed, void* dqkv, hipStream_t s) {
  static const char* fn = "ttmi_mha_bwd_dy";
  int rc = check_mha(fn, TTMI_BF16, B, L, H, Dh, qkv, key_valid, drop_p);
  if (rc) return rc;
  TTMI_REQUIRE(Dh == 32 && H * Dh == 128 && L <= LP, "%s: serves bf16, H*Dh = 128 with Dh = 32, L <= 64", fn);
  TTMI_REQUIRE(lse && dy && wot && dqkv, "%s: null argument", fn);
  TTMI_REQUIRE((((uintptr_t)dy | (uintptr_t)wot) & 15) == 0 && ((uintptr_t)dqkv & 7) == 0,
               "%s: dy / wot must be 16-byte, dqkv 8-byte aligned", fn);
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "%s: drop_p out of [0,1)", fn);
  if (B == 0) return TTMI_OK;
  hipLaunchKernelGGL((mha2_bwd_kernel<32, true>), dim3(B * H), dim3(256), 0, s, L, H, (const bf16_t*)qkv,
                     key_valid, lse, nullptr, make_drop(drop_p, drop_seed), (bf16_t*)dqkv, 1.f / sqrtf(32.f),
                     (const bf16_t*)dy, (const bf16_t*)wot);
  return ttmi_check_launch(fn);
}

extern "C" int ttmi_mha_bwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                            const int64_t* key_valid, const float* lse, const void* dctx,
                            float drop_p, const uint64_t* drop_seed, void* dqkv, hipStream_t s) {
  int rc = check_mha("ttmi_mha_bwd", dtype, B, L, H, Dh, qkv, key_valid, drop_p);
  if (rc) return rc;
  TTMI_REQUIRE(lse && dctx && dqkv, "ttmi_mha_bwd: null argument");
  TTMI_REQUIRE(((uintptr_t)dctx & 15) == 0, "ttmi_mha_bwd: dctx must be 16-byte aligned");
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "ttmi_mha_bwd: drop_p out of [0,1)");
  if (B == 0) return TTMI_OK;
  DropParams dp = make_drop(drop_p, drop_seed);
  if (L > LP) return attn_long_bwd(dtype, B, L, H, Dh, qkv, key_valid, lse, dctx, dp, dqkv, s);
  if (dtype == TTMI_BF16 && (Dh == 32 || Dh == 64) && !getenv("TTMI_MHA_V1")) {
    TTMI_REQUIRE(((uintptr_t)dqkv & 7) == 0, "ttmi_mha_bwd: dqkv must be 8-byte aligned");
    const float sc = 1.f / sqrtf((float)Dh);
    if (Dh == 32)
      hipLaunchKernelGGL(mha2_bwd_kernel<32>, dim3(B * H), dim3(256), 0, s, L, H, (const bf16_t*)qkv,
                         key_valid, lse, (const bf16_t*)dctx, dp, (bf16_t*)dqkv, sc);
    else
      hipLaunchKernelGGL(mha2_bwd_kernel<64>, dim3(B * H), dim3(256), 0, s, L, H, (const bf16_t*)qkv,
                         key_valid, lse, (const bf16_t*)dctx, dp, (bf16_t*)dqkv, sc);
  } else if (dtype == TTMI_BF16) {
    if (Dh <= 32) launch_bwd<bf16_t, 32>(B, L, H, Dh, qkv, key_valid, lse, dctx, dp, dqkv, s);
    else launch_bwd<bf16_t, 64>(B, L, H, Dh, qkv, key_valid, lse, dctx, dp, dqkv, s);
  } else {
    if (Dh <= 32) launch_bwd<float, 32>(B, L, H, Dh, qkv, key_valid, lse, dctx, dp, dqkv, s);
    else launch_bwd<float, 64>(B, L, H, Dh, qkv, key_valid, lse, dctx, dp, dqkv, s);
  }
  return ttmi_check_launch("ttmi_mha_bwd");
}

TTMI_STAMP_DUMP(attn)
