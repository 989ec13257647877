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
TTMI_DEV uint32_t a_pk2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }
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
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, lg = lane >> 4;
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
  const uint64_t kvm = s_kv;
  bool kv[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) kv[t][e] = (kvm >> (16 * t + 4 * lg + e)) & 1ull;
  const DropKeys dk = resolve_drop(dp);
  const uint32_t pbase = (uint32_t)((int64_t)bh * L * L);
  constexpr int NC = DH / 32;                      // 32-wide k chunks of the head dim
#pragma unroll
  for (int i = wave; i < 4; i += 4) {      // wave w owns query tile w
    if (16 * i >= L) break;
    const int q = 16 * i + li;
    uint4 qf[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) qf[c] = a_fk<G::P>(sQ, 16 * i, c, lane);
    f32x4_t s[4];
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      if (t <= i) {
#pragma unroll
        for (int c = 0; c < NC; ++c) Mma<bf16_t>::run(s[t], a_fk<G::P>(sK, 16 * t, c, lane), qf[c]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 16 * t + 4 * lg + e;
        const bool ok = t <= i && kv[t][e] && k <= q && q < L;
        s[t][e] = ok ? s[t][e] * scale : -INFINITY;
        m = fmaxf(m, s[t][e]);
      }
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float p = m == -INFINITY ? 0.f : __expf(s[t][e] - m);
        s[t][e] = p;
        sum += p;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      // masked scores are 0 already, so the mask applies without a range check (the pair
      // hash when L is even; identical to drop_keep per index)
      bool kp[4] = {true, true, true, true};
      if (dk.on) drop_keep4(dk, pbase + (uint32_t)(q * L + 16 * t + 4 * lg), kp);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float p = s[t][e] * inv;
        s[t][e] = kp[e] ? (dk.on ? p * dk.scale : p) : 0.f;
      }
    }
    f32x4_t o[DH / 16];
#pragma unroll
    for (int u = 0; u < DH / 16; ++u) o[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 2; ++c) {                  // 32-key chunks
      if (32 * c > 16 * i + 15) break;
      const uint4 pf = a_freg(s[2 * c], s[2 * c + 1]);
#pragma unroll
      for (int u = 0; u < DH / 16; ++u) Mma<bf16_t>::run(o[u], a_ft<G::P>(sV, 16 * u, c, lane), pf);
    }
    if (q < L) {
      bf16_t* dst = ctx + ((int64_t)b * L + q) * D + (int64_t)h * DH + 4 * lg;
#pragma unroll
      for (int u = 0; u < DH / 16; ++u) a_st4(dst + 16 * u, o[u]);
      if (lg == 0) lse[(int64_t)bh * L + q] = m == -INFINITY ? INFINITY : m + __logf(sum);
    }
  }
}

template <int DH>
__global__ __launch_bounds__(256) void mha2_bwd_kernel(int L, int H, const bf16_t* __restrict__ qkv,
                                                      const int64_t* __restrict__ kvalid,
                                                      const float* __restrict__ lse,
                                                      const bf16_t* __restrict__ dctx, DropParams dp,
                                                      bf16_t* __restrict__ dqkv, float scale) {
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
  {
    HeadStage<DH, 4> st;
    const bf16_t* const src[4] = {base, base + D, base + 2 * D, dctx + (int64_t)b * L * D + (int64_t)h * DH};
    const int64_t lds4[4] = {ld, ld, ld, (int64_t)D};
    st.load(src, lds4, L, threadIdx.x);
    char* const dst[4] = {sQ, sK, sV, sdO};
    st.store(dst, L, threadIdx.x);
  }
  __shared__ uint64_t s_kv;
  if (wave == 0) {
    const uint64_t bal = __ballot(lane < L && kvl != 0);
    if (lane == 0) s_kv = bal;
  }
  __syncthreads();
  const uint64_t kvm = s_kv;
  bool kv[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) kv[t][e] = (kvm >> (16 * t + 4 * lg + e)) & 1ull;
  const DropKeys dk = resolve_drop(dp);
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
    const float lr = q < L ? lr0 : INFINITY;      // (q = qrow: wave w owns query tile w)
    f32x4_t s[4], dpv[4];
    uint32_t keep[4];                              // dropout keep bits, one hash pass
    float dsum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = dpv[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      if (t <= i) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          Mma<bf16_t>::run(s[t], a_fk<G::P>(sK, 16 * t, c, lane), qf[c]);
          Mma<bf16_t>::run(dpv[t], a_fk<G::P>(sV, 16 * t, c, lane), of[c]);
        }
      }
      bool kp[4] = {true, true, true, true};
      if (dk.on) drop_keep4(dk, pbase + (uint32_t)(q * L + 16 * t + 4 * lg), kp);
      keep[t] = (kp[0] ? 1u : 0u) | (kp[1] ? 2u : 0u) | (kp[2] ? 4u : 0u) | (kp[3] ? 8u : 0u);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 16 * t + 4 * lg + e;
        const bool ok = t <= i && kv[t][e] && k <= q && q < L;
        const float p = ok ? __expf(s[t][e] * scale - lr) : 0.f;
        float dP = 0.f;
        if (ok) {
          dP = dpv[t][e];
          if (dk.on) dP = kp[e] ? dP * dk.scale : 0.f;
        }
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
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float p = s[t][e];
        ds[t][e] = p * (dpv[t][e] - dsum) * scale;
        pd[e] = dk.on ? (((keep[t] >> e) & 1u) ? p * dk.scale : 0.f) : p;
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

