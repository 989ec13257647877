// ttmi_head.hip — the user tower's head in one launch (reference user_tower.py:37-57 and
// :131-144): on the gathered last-valid rows of the pruned last encoder layer,
//   x1 = res + drop1(ctx·Woᵀ + bo);  a2 = LN2(x1);  h = dropf(relu(a2·W1ᵀ + b1));
//   x2 = x1 + drop2(h·W2ᵀ + b2);  comb = [x2, G[gender], C[country]];
//   z = comb·Wf0ᵀ + bf0;  az = relu(LN(z));  u = az·Wf3ᵀ + bf3.
// These eight steps were eight launches of a few microseconds of work each on B = 512 rows;
// in a captured step each launch costs ~4.8 us however small it is.  Here a workgroup takes
// 16 rows through the whole chain with its activations in LDS (the row-local chain has no
// cross-row dependency): four waves split each Linear's output columns, A fragments come from
// LDS, weight fragments straight from L2, LayerNorm reduces across the waves through LDS.
// Every value the backward reads is written out as the unfused ops did (x1, a2, m2, r2, h,
// comb, rows, z, az, mz, rz) and the dropout masks are the same hash at the same indices
// (drop_rows[m]·N + n).
#include "ttmi_q1.h"

#include <cstdlib>

namespace {

constexpr int HR = 16;                 // rows per workgroup (one MFMA row tile)
constexpr int HD = 128;                // d_model
constexpr int FMAX = 512;              // FFN width
constexpr int WPAD = 192;              // concat width D + 16 + 32 = 176, padded to 32
constexpr int PD = (HD + 8) * 2;       // LDS pitches (bytes) of the bf16 row images
constexpr int PF = (FMAX + 8) * 2;
constexpr int PW = (WPAD + 8) * 2;

constexpr int IK = 512;                // modal width (4 x 128) = Linear 0 fan-in
constexpr int IN1 = 512;               // Linear 0 width (BatchNorm channels)
constexpr int PI = (IK + 8) * 2;       // LDS pitch of a bf16 row of 512

struct ItemArgs {
  int B;
  int D;                       // output width (fusion_layer.4 rows): 128 or 256 (ABI 21)
  const float* modal; const bf16_t* w0; const float* b0;
  const bf16_t* y1; const bf16_t* w4; const float* b4; const float* lnw; const float* lnb; float ln_eps;
  bf16_t* m16; float* z; float* y2; float* out; float* m5; float* r5;
  float* ohat; float* onrm;    // optional: out / max(||out||, eps) and ||out|| (InfoNCE's l2norm)
  // fused BatchNorm (ABI 15; bncnt NULL: the separate bnr_fwd launch): stage A leaves per-block
  // column (mean, M2) in bnpart, the last row block of a column quarter merges them into the
  // batch statistics; stage C applies BN + ReLU + dropout while staging z rows
  const float* bnw; const float* bnb; float bn_eps, bn_mom;
  float* rmean; float* rvar; int64_t* nbt; float* bmean; float* brstd; bf16_t* y1w;
  DropParams bd;
  float* bnpart; int* bncnt;
  // ABI 18, ttmi_user_item_head_fwd_ac: stages A and C in ONE launch (beside the user head).
  // Stage A stores z, bmean, brstd write-through (sc1) and its quarter mergers count on
  // bncnt[IN1/64]; the C workgroups poll that count, then read them with sc1 loads.
  int fin;
  int32_t* err;                // the user head's id_err flags: [TTMI_IDERR_HEAD_POLL] on a poll timeout
};

struct ItemLdsA {
  char sA[HR * PI];
  int s_last;
};

// Item head backward's row-local part (ttmi_item_head_bwd_c): the LayerNorm backward of
// fusion_layer.5 and the input gradient of fusion_layer.4 on 16 rows per workgroup.
struct ItemBwdArgs {
  int B;
  int D;
  const float* dout; const float* y2; const float* m5; const float* r5; const float* lnw;
  const bf16_t* w4t;
  bf16_t* dy2; float* dy1; float* ws;
};

struct HeadArgs {
  int B, F, dg, dc;
  float eps;
  const bf16_t* ctx; const float* res; const int32_t* drows;
  const bf16_t* wo; const float* bo; const float* n2w; const float* n2b;
  const bf16_t* w1; const float* b1; const bf16_t* w2; const float* b2;
  const int64_t* gender; const float* G; const int64_t* country; const float* C;
  const bf16_t* wf0; const float* bf0; const float* lnw; const float* lnb;
  const bf16_t* wf3; const float* bf3;
  DropParams d1, dff, d2;
  float* x1; bf16_t* a2; float* m2; float* r2; bf16_t* h; bf16_t* comb; int32_t* rows;
  float* z; bf16_t* az; float* mz; float* rz; float* u;
  float* uhat; float* unrm;    // optional: u / max(||u||, eps) and ||u|| (InfoNCE's l2norm)
  // co-launched item head stage A (ttmi_user_item_head_fwd): workgroups >= nbu run
  // item_a_body on row block (l % it_nblk), column quarter (l / it_nblk)
  ItemArgs it; int nbu, it_nblk;
  int it_stage;                // 0: item stage A (it_nblk x 8 workgroups), 2: item stage C (it_nblk),
                               // 3: both, A's then C's (C waits for A's statistics in-launch)
  int ng, nc; int32_t* id_err; // table rows of G / C; ids outside are clamped and flagged (ABI 20)
  float* ffn_part; int* ffn_cnt;   // ABI 21: the FFN split's exchange slots and arrival counts
};

struct HeadLds {
  char sA[HR * PD];        // ctx, then a2, then az
  char sH[HR * PF];        // h
  char sC[HR * PW];        // comb (zero-padded to WPAD)
  float sX1[HR][HD + 4];   // x1 (fp32 residual of the FFN)
  float red[4][HR];        // LayerNorm cross-wave partials
};

// MFMA k order.  Both operands of every product here use the same k permutation, so the sum
// is the same: lane group g holds the 8 CONTIGUOUS k = 8g .. 8g+7 of a 32-wide chunk (one
// 16-byte access per fragment, and each weight row segment is fetched once, by one lane).
// A fragment (rows li, k chunk c) of an LDS row image.
template <int P>
TTMI_DEV uint4 afrag(const char* s, int c, int lane) {
  return *reinterpret_cast<const uint4*>(s + (lane & 15) * P + c * 64 + (lane >> 4) * 16);
}
// Weight fragment: output column n (a row of the [N, K] k-major weight), k chunk c; k past
// Kreal (Kreal % 8 == 0) reads as zero.  The load is unconditional from a clamped address (a
// guarded load is a branch + vmcnt(0), which would serialise the stage's loads).
TTMI_DEV uint4 wfrag(const bf16_t* W, int64_t ldw, int n, int c, int lane, int Kreal) {
  const int k0 = c * 32 + (lane >> 4) * 8;
  const uint4 q = *reinterpret_cast<const uint4*>(W + (int64_t)n * ldw + min(k0, Kreal - 8));
  return k0 < Kreal ? q : make_uint4(0u, 0u, 0u, 0u);
}
// Weight fragments of one Linear stage for this wave (NT column tiles x K/32 chunks), all
// loads issued at once: each stage is one L2 round trip, not K/32 of them.
template <int NT, int K>
struct WFrags {
  uint4 f[K / 32][NT];
  TTMI_DEV void load(const bf16_t* W, int64_t ldw, int n0, int lane, int Kreal) {
#pragma unroll
    for (int c = 0; c < K / 32; ++c)
#pragma unroll
      for (int t = 0; t < NT; ++t) f[c][t] = wfrag(W, ldw, n0 + 16 * t + (lane & 15), c, lane, Kreal);
  }
};
// acc[t] (lane: row li, columns n0 + 16t + 4g .. +3) = A[16 x K] · W[n0 + 16t .., :]ᵀ
template <int NT, int K, int P>
TTMI_DEV void head_gemm(const char* sA, const WFrags<NT, K>& wf, f32x4_t (&acc)[NT], int lane) {
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < K / 32; ++c) {
    const uint4 a = afrag<P>(sA, c, lane);
#pragma unroll
    for (int t = 0; t < NT; ++t) Mma<bf16_t>::run(acc[t], wf.f[c][t], a);
  }
}

TTMI_DEV void st4_bf(char* p, const float* v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pk_bf2(v[0], v[1]),
                                            pk_bf2(v[2], v[3]));
}

// Row sum over the 128 columns held as v[t][e] by the 4 lanes of row li in each of 4 waves.
template <class LDS>
TTMI_DEV float row_sum(float s, LDS& L, int w, int lane) {
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  if (lane < 16) L.red[w][lane] = s;
  __syncthreads();
  const int li = lane & 15;
  const float tot = L.red[0][li] + L.red[1][li] + L.red[2][li] + L.red[3][li];
  __syncthreads();
  return tot;
}
// F.normalize of the row values x (2 tiles x 4 per lane, columns n0 + 16t + 4g + e) as
// ttmi_infonce_fwd's l2norm writes it (eps 1e-12): xhat rows and the norms.  Every thread
// calls it (row_sum barriers); no-op outputs when xhat is NULL.
template <class LDS>
TTMI_DEV void row_l2norm(const float (&x)[2][4], float* xhat, float* nrm, int m, bool mrow, int n0,
                         LDS& L, int w, int lane) {
  if (xhat == nullptr) return;                     // uniform: a kernel argument
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) s += x[t][e] * x[t][e];
  const float nr = sqrtf(row_sum(s, L, w, lane));
  const float inv = 1.f / fmaxf(nr, 1e-12f);
  const int g = lane >> 4;
  if (mrow) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
      *reinterpret_cast<float4*>(xhat + (int64_t)m * HD + n0 + 16 * t + 4 * g) =
          make_float4(x[t][0] * inv, x[t][1] * inv, x[t][2] * inv, x[t][3] * inv);
    if (lane < 16 && w == 0) nrm[m] = nr;
  }
}

// LayerNorm of the row values v (2 tiles x 4 per lane); returns mean / rstd.
template <class LDS>
TTMI_DEV void row_ln(f32x4_t (&v)[2], const float* w_, const float* b_, float eps, bool relu,
                     int n0, LDS& L, int w, int lane, float& mu, float& rs) {
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) s += v[t][e];
  mu = row_sum(s, L, w, lane) * (1.f / HD);
  float q = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[t][e] - mu;
      q += d * d;
    }
  rs = 1.f / sqrtf(row_sum(q, L, w, lane) * (1.f / HD) + eps);
  const int g = lane >> 4;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = n0 + 16 * t + 4 * g + e;
      float o = (v[t][e] - mu) * rs * w_[n] + b_[n];
      v[t][e] = relu ? fmaxf(o, 0.f) : o;
    }
}

// Per-column parameters staged in LDS once (bias / LayerNorm vectors: the epilogues read
// them without a global round trip).
struct HeadParams {
  float bo[HD], n2w[HD], n2b[HD], b1[FMAX], b2[HD], bf0[HD], lnw[HD], lnb[HD], bf3[HD];
};
// Every thread loads (clamped index: no branch, so no vmcnt(0) that would serialise the
// staging loads) and stores; duplicate stores write the same value.
template <int N>
TTMI_DEV float4 vec_ld(const float* src, int tid) {
  return reinterpret_cast<const float4*>(src)[tid & (N / 4 - 1)];
}
template <int N>
TTMI_DEV void vec_st(float* dst, const float4& v, int tid) {
  reinterpret_cast<float4*>(dst)[tid & (N / 4 - 1)] = v;
}

constexpr int BN_MAXBLK = 32;          // fused BatchNorm statistics: B <= 512
TTMI_DEV void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
TTMI_DEV float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte write-through (sc1) store / load for data handed to another workgroup inside a launch
// (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms row 1).  The buffer resource is
// built from a workgroup-uniform base (it lives in SGPRs) and each lane passes its byte offset:
// a per-lane base makes hipcc wrap every access in a readfirstlane loop over the 64 lanes, which
// cost this launch ~70 us (a 64-way serialised load per access).
TTMI_DEV void st16_wt(float* base, uint32_t off, float4 v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7FFFFFFF, 0x00020000);
  const i32x4_t q = {(int)__float_as_uint(v.x), (int)__float_as_uint(v.y), (int)__float_as_uint(v.z),
                     (int)__float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(q, r, off, 0, 16);
}
TTMI_DEV float4 ld16_wt(const float* base, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7FFFFFFF, 0x00020000);
  const i32x4_t q = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
  return make_float4(__int_as_float(q.x), __int_as_float(q.y), __int_as_float(q.z), __int_as_float(q.w));
}
constexpr int BN_DONE = IN1 / 64, BN_CDONE = IN1 / 64 + 1;   // bncnt slots past the quarters'

// Item head stage A on row block bx, column quarter q (item_head_a_kernel, or the workgroups
// of ttmi_user_item_head_fwd past the user head's).
TTMI_DEV void item_a_body(const ItemArgs& a, int bx, int q, ItemLdsA& L) {
  TTMI_TSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, g = lane >> 4;
  const int r0 = bx * HR;
  const int n0 = 64 * q + 16 * w;                    // this wave's 16 of the 512 columns
  WFrags<1, IK> wf;
  wf.load(a.w0, IK, n0, lane, IK);
  const float4 bias = *reinterpret_cast<const float4*>(a.b0 + n0 + 4 * g);
  // 16 rows x 128 float4 of modal -> bf16: every load issued before the first store (the m16
  // copy's global store may alias modal for all hipcc knows, so a load after it waited for the
  // loads before it: eight serial round trips)
  float4 mv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int idx = tid + 256 * k, r = idx >> 7, c4 = idx & 127;
    const int rr = min(r0 + r, a.B - 1);
    mv[k] = *reinterpret_cast<const float4*>(a.modal + (int64_t)rr * IK + 4 * c4);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int idx = tid + 256 * k, r = idx >> 7, c4 = idx & 127;
    const float x[4] = {mv[k].x, mv[k].y, mv[k].z, mv[k].w};
    st4_bf(L.sA + r * PI + c4 * 8, x);
    if (q == 0 && r0 + r < a.B) st4_bf(reinterpret_cast<char*>(a.m16 + (int64_t)(r0 + r) * IK + 4 * c4), x);
  }
  __syncthreads();
  f32x4_t v[1];
  head_gemm<1, IK, PI>(L.sA, wf, v, lane);
  const int m = r0 + li;
  if (m < a.B) {
    const float4 zo = make_float4(v[0][0] + bias.x, v[0][1] + bias.y, v[0][2] + bias.z, v[0][3] + bias.w);
    if (a.fin) st16_wt(a.z, (uint32_t)(((int64_t)m * IN1 + n0 + 4 * g) * 4), zo);   // read by this launch's C
    else *reinterpret_cast<float4*>(a.z + (int64_t)m * IN1 + n0 + 4 * g) = zo;
  }
  TTMI_TSTAMP(1);
  if (a.bncnt == nullptr) return;
  // ---- fused BatchNorm statistics: this block's (mean, M2) of its 4 x 16 columns over its
  // valid rows (the 16 lanes of a lane group share the columns), exchanged through agent-scope
  // relaxed atomics (cross-XCD, no cache-writeback fence); the last of the column quarter's
  // row blocks merges them in block order (Chan et al.'s pairwise update: deterministic).
  const int nv = min(HR, a.B - r0);
  const float bv[4] = {bias.x, bias.y, bias.z, bias.w};
  float bm[4], b2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float x = m < a.B ? v[0][e] + bv[e] : 0.f;
    float s = x;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) s += __shfl_xor(s, off, 64);
    bm[e] = s / (float)nv;
    const float d = m < a.B ? x - bm[e] : 0.f;
    float q2 = d * d;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) q2 += __shfl_xor(q2, off, 64);
    b2[e] = q2;
  }
  if (li == 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      st_agent(a.bnpart + (int64_t)(2 * bx) * IN1 + n0 + 4 * g + e, bm[e]);
      st_agent(a.bnpart + (int64_t)(2 * bx + 1) * IN1 + n0 + 4 * g + e, b2[e]);
    }
  }
  const int nblk = (a.B + HR - 1) / HR;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  TTMI_TSTAMP(3);
  if (tid == 0)
    L.s_last = __hip_atomic_fetch_add(a.bncnt + q, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1;
  __syncthreads();
  TTMI_TSTAMP(4);
  if (!L.s_last || tid >= 64) return;
  const int c = 64 * q + tid;
  // every load in flight first, the running statistics' read-modify-writes included (three
  // dependent round trips at the end of the merge otherwise)
  const float rm0 = a.rmean ? a.rmean[c] : 0.f, rv0 = a.rvar ? a.rvar[c] : 0.f;
  const bool nbt_lane = q == 0 && tid == 0 && a.nbt;
  const int64_t nbt0 = nbt_lane ? a.nbt[0] : 0;
  float pm[BN_MAXBLK], p2[BN_MAXBLK], pn[BN_MAXBLK];
#pragma unroll
  for (int b = 0; b < BN_MAXBLK; ++b) {
    const int bb = min(b, nblk - 1);
    pm[b] = ld_agent(a.bnpart + (int64_t)(2 * bb) * IN1 + c);
    p2[b] = ld_agent(a.bnpart + (int64_t)(2 * bb + 1) * IN1 + c);
    pn[b] = b < nblk ? (float)min(HR, a.B - HR * b) : 0.f;
  }
  TTMI_TSTAMP_VAL(5, TTMI_TNOW() + (uint64_t)(pm[0] == 1234.5f) + (uint64_t)(p2[BN_MAXBLK - 1] == 1234.5f));
  // Chan's pairwise update in a fixed tree order (blocks b and b + w, w = 1, 2, 4, ...): five
  // dependent levels instead of a 32-step chain (2.7 us of the launch, phase stamps); the
  // order is fixed, so the statistics are the same bits on every run
#pragma unroll
  for (int w = 1; w < BN_MAXBLK; w <<= 1)
#pragma unroll
    for (int b = 0; b + w < BN_MAXBLK; b += 2 * w) {
      const float na = pn[b], nb = pn[b + w];
      if (nb > 0.f) {
        const float tot = na + nb, f = nb / tot, delta = pm[b + w] - pm[b];
        pm[b] += delta * f;
        p2[b] += p2[b + w] + delta * delta * (na * f);
        pn[b] = tot;
      }
    }
  const float mean = pm[0], M2 = p2[0];
  const float var = M2 / (float)a.B;
  TTMI_TSTAMP_VAL(6, TTMI_TNOW() + (uint64_t)(var == 1234.5f));
  if (a.fin) {                                       // read by this launch's C workgroups
    st_agent(a.bmean + c, mean);
    st_agent(a.brstd + c, 1.f / sqrtf(var + a.bn_eps));
  } else {
    a.bmean[c] = mean;
    a.brstd[c] = 1.f / sqrtf(var + a.bn_eps);
  }
  if (a.rmean) a.rmean[c] = (1.f - a.bn_mom) * rm0 + a.bn_mom * mean;
  if (a.rvar) a.rvar[c] = (1.f - a.bn_mom) * rv0 + a.bn_mom * var * ((float)a.B / (float)(a.B - 1));
  if (nbt_lane) a.nbt[0] = nbt0 + 1;
  if (tid == 0) __hip_atomic_store(a.bncnt + q, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.fin) {      // this (single) storing wave drained, then one lane signals the quarter done
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) __hip_atomic_fetch_add(a.bncnt + BN_DONE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  TTMI_TSTAMP(2);
}

// ---- per-width geometry and row reductions of the D-templated head kernels (D = 128 / 256)
template <int D_>
struct SplitGeo {
  static constexpr int NW = D_ / 32;                 // waves
  static constexpr int PD = (D_ + 8) * 2;            // LDS pitches (bytes)
  static constexpr int PH = (128 + 8) * 2;           // the split's 128 hidden units
  static constexpr int WPAD = (D_ + 48 + 31) / 32 * 32;
  static constexpr int PW = (WPAD + 8) * 2;
  static constexpr int TH = 128 / 16 / NW;           // hidden 16-column tiles per wave
};
// Row sum over the D columns held by the 4 lanes of row li in each of NW waves (in wave order).
template <int NW>
TTMI_DEV float split_row_sum(float s, float (*red)[HR], int w, int lane) {
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  if (lane < 16) red[w][lane] = s;
  __syncthreads();
  const int li = lane & 15;
  float tot = red[0][li];
#pragma unroll
  for (int k = 1; k < NW; ++k) tot += red[k][li];
  __syncthreads();
  return tot;
}
template <int D_>
TTMI_DEV void split_row_ln(f32x4_t (&v)[2], const float* w_, const float* b_, float eps, bool relu, int n0,
                           float (*red)[HR], int w, int lane, float& mu, float& rs) {
  constexpr int NW = SplitGeo<D_>::NW;
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) s += v[t][e];
  mu = split_row_sum<NW>(s, red, w, lane) * (1.f / D_);
  float q = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[t][e] - mu;
      q += d * d;
    }
  rs = 1.f / sqrtf(split_row_sum<NW>(q, red, w, lane) * (1.f / D_) + eps);
  const int g = lane >> 4;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = n0 + 16 * t + 4 * g + e;
      float o = (v[t][e] - mu) * rs * w_[n] + b_[n];
      v[t][e] = relu ? fmaxf(o, 0.f) : o;
    }
}
template <int D_>
TTMI_DEV void split_row_l2norm(const float (&x)[2][4], float* xhat, float* nrm, int m, bool mrow, int n0,
                               float (*red)[HR], int w, int lane) {
  if (xhat == nullptr) return;                       // uniform: a kernel argument
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) s += x[t][e] * x[t][e];
  const float nr = sqrtf(split_row_sum<SplitGeo<D_>::NW>(s, red, w, lane));
  const float inv = 1.f / fmaxf(nr, 1e-12f);
  const int g = lane >> 4;
  if (mrow) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
      *reinterpret_cast<float4*>(xhat + (int64_t)m * D_ + n0 + 16 * t + 4 * g) =
          make_float4(x[t][0] * inv, x[t][1] * inv, x[t][2] * inv, x[t][3] * inv);
    if (lane < 16 && w == 0) nrm[m] = nr;
  }
}

template <int D_>
struct ItemLdsCT {
  char sY[HR * PI];
  float red[D_ / 32][HR];
};
using ItemLdsC = ItemLdsCT<HD>;

// Item head stage C on row block bx (item_head_c_kernel, or the workgroups of
// ttmi_user_item_head_fwd_c past the user head's).
// D_ = 128 (4 waves) or 256 (8 waves): a wave owns 32 of the D_ output columns.
template <bool FIN, int D_ = HD>
TTMI_DEV void item_c_body(const ItemArgs& a, int bx, ItemLdsCT<D_>& L) {
  constexpr int NW = D_ / 32, NT = NW * 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, g = lane >> 4;
  const int r0 = bx * HR;
  const int n0 = 32 * w;                             // this wave's 32 of the D_ output columns
  TTMI_TSTAMP(0);
  if constexpr (FIN) {
    // stage A runs in this launch: wait until the IN1/64 column-quarter mergers have published
    // the batch statistics (one lane polls the count, sc1 loads with s_sleep; bounded: on a
    // timeout the error word bncnt[BN_CDONE + 1] is set instead of hanging the GPU)
    if (tid == 0) {
      int spins = 0;
      while (__hip_atomic_load(a.bncnt + BN_DONE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < IN1 / 64) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1 << 22)) {
          __hip_atomic_store(a.bncnt + BN_CDONE + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          raise_id_err(a.err, TTMI_IDERR_HEAD_POLL);      // the host raises (ops.check_id_errors)
          break;
        }
      }
      // the last C workgroup past the poll resets both counts for the next launch
      const int nb = (a.B + HR - 1) / HR;
      if (__hip_atomic_fetch_add(a.bncnt + BN_CDONE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nb - 1) {
        __hip_atomic_store(a.bncnt + BN_DONE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.bncnt + BN_CDONE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
  }
  TTMI_TSTAMP(3);
  // the weight fragments first: their loads then overlap the staging below, instead of
  // waiting behind its y1 stores
  WFrags<2, IN1> wf;
  wf.load(a.w4, IN1, n0, lane, IN1);
  if (a.bncnt != nullptr) {      // fused BatchNorm: y1 = drop(relu(BN(z))) staged from z rows
    constexpr int ZK = HR * IN1 / 4 / NT;            // float4 of z per thread
    float4 zv[ZK];
#pragma unroll
    for (int k = 0; k < ZK; ++k) {
      const int idx = tid + NT * k, r = idx >> 7, c4 = idx & 127;
      const int64_t zo = (int64_t)min(r0 + r, a.B - 1) * IN1 + 4 * c4;
      if constexpr (FIN) zv[k] = ld16_wt(a.z, (uint32_t)(zo * 4));
      else zv[k] = *reinterpret_cast<const float4*>(a.z + zo);
    }
    const DropKeys dk = resolve_drop(a.bd);
    // a thread's column quad is the same for all 8 rows it stages (idx & 127 = tid & 127): its
    // BatchNorm parameters are loaded once, with the z rows, before any store (a load after
    // the y1 store would wait for it: hipcc cannot tell the buffers apart)
    const int c4 = tid & 127;
    const float4 mu = FIN ? ld16_wt(a.bmean, 16u * c4) : *reinterpret_cast<const float4*>(a.bmean + 4 * c4);
    const float4 rs = FIN ? ld16_wt(a.brstd, 16u * c4) : *reinterpret_cast<const float4*>(a.brstd + 4 * c4);
    const float4 ww = *reinterpret_cast<const float4*>(a.bnw + 4 * c4);
    const float4 bb = *reinterpret_cast<const float4*>(a.bnb + 4 * c4);
#pragma unroll
    for (int k = 0; k < ZK; ++k) {
      const int idx = tid + NT * k, r = idx >> 7;
      float x[4] = {fmaxf((zv[k].x - mu.x) * rs.x * ww.x + bb.x, 0.f), fmaxf((zv[k].y - mu.y) * rs.y * ww.y + bb.y, 0.f),
                    fmaxf((zv[k].z - mu.z) * rs.z * ww.z + bb.z, 0.f), fmaxf((zv[k].w - mu.w) * rs.w * ww.w + bb.w, 0.f)};
      drop_apply_vec<4>(dk, (uint32_t)((int64_t)(r0 + r) * IN1 + 4 * c4), x);
      st4_bf(L.sY + r * PI + c4 * 8, x);
      if (r0 + r < a.B) st4_bf(reinterpret_cast<char*>(a.y1w + (int64_t)(r0 + r) * IN1 + 4 * c4), x);
    }
  } else {                                           // y1 rows: 16 x 64 chunks of 16 bytes
#pragma unroll
    for (int k = 0; k < HR * IN1 / 8 / NT; ++k) {
      const int idx = tid + NT * k, r = idx >> 6, ch = idx & 63;
      *reinterpret_cast<uint4*>(L.sY + r * PI + ch * 16) =
          *reinterpret_cast<const uint4*>(a.y1 + (int64_t)min(r0 + r, a.B - 1) * IN1 + ch * 8);
    }
  }
  float b4[2][4], lw[2][4], lb[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
    const float4 b = *reinterpret_cast<const float4*>(a.b4 + n);
    const float4 x = *reinterpret_cast<const float4*>(a.lnw + n);
    const float4 y = *reinterpret_cast<const float4*>(a.lnb + n);
    b4[t][0] = b.x; b4[t][1] = b.y; b4[t][2] = b.z; b4[t][3] = b.w;
    lw[t][0] = x.x; lw[t][1] = x.y; lw[t][2] = x.z; lw[t][3] = x.w;
    lb[t][0] = y.x; lb[t][1] = y.y; lb[t][2] = y.z; lb[t][3] = y.w;
  }
  __syncthreads();
  f32x4_t v[2];
  head_gemm<2, IN1, PI>(L.sY, wf, v, lane);
  const int m = r0 + li;
  const bool mrow = m < a.B;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[t][e] += b4[t][e];
    if (mrow) *reinterpret_cast<float4*>(a.y2 + (int64_t)m * D_ + n) = make_float4(v[t][0], v[t][1], v[t][2], v[t][3]);
  }
  // LayerNorm over the D_ columns (the waves' 32 each), two-pass like ttmi_layernorm_fwd
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) s += v[t][e];
  const float mu = split_row_sum<NW>(s, L.red, w, lane) * (1.f / D_);
  float qv = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[t][e] - mu;
      qv += d * d;
    }
  const float rs = 1.f / sqrtf(split_row_sum<NW>(qv, L.red, w, lane) * (1.f / D_) + a.ln_eps);
  float oo[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
    float* o = oo[t];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (v[t][e] - mu) * rs * lw[t][e] + lb[t][e];
    if (mrow) *reinterpret_cast<float4*>(a.out + (int64_t)m * D_ + n) = make_float4(o[0], o[1], o[2], o[3]);
  }
  if (mrow && lane < 16 && w == 0) { a.m5[m] = mu; a.r5[m] = rs; }
  split_row_l2norm<D_>(oo, a.ohat, a.onrm, m, mrow, n0, L.red, w, lane);
  TTMI_TSTAMP(4);
}

template <int D_>
__global__ __launch_bounds__(D_ * 2) void item_head_c_kernel(ItemArgs a) {
  __shared__ __attribute__((aligned(16))) ItemLdsCT<D_> L;
  item_c_body<false, D_>(a, blockIdx.x, L);
}

// phase stamps of the diagnostic build (ttmi_common.h TTMI_TSTAMP; tools/stamp_build.sh)
#define STAMP(i) TTMI_TSTAMP(i)

// Each stage's weight fragments are loaded one stage ahead.  (Loading every stage's weights
// at the start, with the whole register file, measured slower: the ~360 KB of weights a
// workgroup streams take ~25k cycles through one CU's vector memory path whatever the order,
// and vmcnt retires in order, so the first stage then waited for all of them.)
template <int F>
__global__ __launch_bounds__(256) void user_head_fwd_kernel(HeadArgs a) {
  STAMP(0);
  __shared__ __attribute__((aligned(16))) HeadLds L;
  __shared__ __attribute__((aligned(16))) HeadParams Q;
  static_assert(sizeof(HeadLds) >= sizeof(ItemLdsA), "item stage A reuses the head's LDS");
  static_assert(sizeof(HeadLds) >= sizeof(ItemLdsC), "item stage C reuses the head's LDS");
  // block order: stages 0 / 2, the user head's row blocks first, then the item blocks; stage 3,
  // the item stage-A blocks first (one per CU as the grid is dispatched: the slowest of them
  // sets when stage C can start), then the user head's, then stage C's
  int ub = (int)blockIdx.x;
  if (a.it_stage == 3) {
    const int na = a.it_nblk * (IN1 / 64);
    if (ub < na) {
      item_a_body(a.it, ub % a.it_nblk, ub / a.it_nblk, *reinterpret_cast<ItemLdsA*>(&L));
      return;
    }
    ub -= na;
    if (ub >= a.nbu) {
      item_c_body<true>(a.it, ub - a.nbu, *reinterpret_cast<ItemLdsC*>(&L));
      return;
    }
  } else if (ub >= a.nbu) {                          // co-launched item head stage A or C
    const int l = ub - a.nbu;
    if (a.it_stage == 0) item_a_body(a.it, l % a.it_nblk, l / a.it_nblk, *reinterpret_cast<ItemLdsA*>(&L));
    else item_c_body<false>(a.it, l, *reinterpret_cast<ItemLdsC*>(&L));
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, g = lane >> 4;
  const int r0 = ub * HR, m = r0 + li;
  const bool mrow = m < a.B;
  const int W = HD + a.dg + a.dc;
  const int n0 = w * 32;                             // this wave's 32 of the 128 columns
  const int nf0 = w * (F / 4);                       // ... and its F / 4 FFN columns
  // every stage's weights are loaded one stage ahead (first: now, beside the staging below)
  // Prologue: the first stage's weights first (the longest wait), then the row staging
  WFrags<2, HD> wo;
  wo.load(a.wo, HD, n0, lane, HD);
  {                                                  // ctx: 16 rows x 16 chunks of 16 bytes
    const int r = tid >> 4, ch = tid & 15;
    *reinterpret_cast<uint4*>(L.sA + r * PD + ch * 16) =
        *reinterpret_cast<const uint4*>(a.ctx + (int64_t)min(r0 + r, a.B - 1) * HD + ch * 8);
#pragma unroll
    for (int q = 0; q < 2; ++q) {                     // residual: 16 rows x 32 float4
      const int idx = tid + 256 * q;
      *reinterpret_cast<float4*>(&L.sX1[idx >> 5][(idx & 31) * 4]) =
          *reinterpret_cast<const float4*>(a.res + (int64_t)min(r0 + (idx >> 5), a.B - 1) * HD + (idx & 31) * 4);
    }
  }
  {
    const float4 p0 = vec_ld<HD>(a.bo, tid), p1 = vec_ld<HD>(a.n2w, tid), p2 = vec_ld<HD>(a.n2b, tid);
    const float4 p3 = vec_ld<F>(a.b1, tid), p4 = vec_ld<HD>(a.b2, tid), p5 = vec_ld<HD>(a.bf0, tid);
    const float4 p6 = vec_ld<HD>(a.lnw, tid), p7 = vec_ld<HD>(a.lnb, tid), p8 = vec_ld<HD>(a.bf3, tid);
    vec_st<HD>(Q.bo, p0, tid); vec_st<HD>(Q.n2w, p1, tid); vec_st<HD>(Q.n2b, p2, tid);
    vec_st<F>(Q.b1, p3, tid); vec_st<HD>(Q.b2, p4, tid); vec_st<HD>(Q.bf0, p5, tid);
    vec_st<HD>(Q.lnw, p6, tid); vec_st<HD>(Q.lnb, p7, tid); vec_st<HD>(Q.bf3, p8, tid);
  }
  {   // demographics: a thread owns 4 of a row's 64 trailing columns (one index load, then
      // both tables read at clamped addresses and the value selected: no conditional load)
    const int r = tid >> 4, k0 = HD + 4 * (tid & 15), rr = min(r0 + r, a.B - 1);
    const int64_t gi = clamp_id(a.gender[rr], a.ng, a.id_err, TTMI_IDERR_GENDER);
    const int64_t ci = clamp_id(a.country[rr], a.nc, a.id_err, TTMI_IDERR_COUNTRY);
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int kk = k0 + e;
      float gv = a.G[gi * a.dg + min(kk - HD, a.dg - 1)];
      float cv = a.C[ci * a.dc + min(max(kk - HD - a.dg, 0), a.dc - 1)];
      asm volatile("" : "+v"(gv), "+v"(cv));
      v[e] = kk < HD + a.dg ? gv : (kk < W ? cv : 0.f);
    }
    st4_bf(L.sC + r * PW + k0 * 2, v);
    if (k0 < W && r0 + r < a.B) st4_bf(reinterpret_cast<char*>(a.comb + (int64_t)(r0 + r) * W + k0), v);
  }
  if (tid < HR && r0 + tid < a.B) a.rows[r0 + tid] = r0 + tid;
  const int drow = a.drows[min(m, a.B - 1)];
  // the three sites' keys, read once (the launcher points an unused seed at valid memory)
  const uint64_t s1 = *a.d1.seed, sf = *a.dff.seed, s2 = *a.d2.seed;
  const DropKeys dk1{(uint32_t)s1, (uint32_t)(s1 >> 32), a.d1.thresh, a.d1.scale, a.d1.on};
  const DropKeys dkf{(uint32_t)sf, (uint32_t)(sf >> 32), a.dff.thresh, a.dff.scale, a.dff.on};
  const DropKeys dk2{(uint32_t)s2, (uint32_t)(s2 >> 32), a.d2.thresh, a.d2.scale, a.d2.on};
  __syncthreads();
  STAMP(1);
  // ---- x1 = res + drop1(ctx·Woᵀ + bo); a2 = LN2(x1)
  f32x4_t v[2];
  head_gemm<2, HD, PD>(L.sA, wo, v, lane);
  WFrags<4, HD> w1a;
  w1a.load(a.w1, HD, nf0, lane, HD);
  {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
      float x[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = v[t][e] + Q.bo[n + e];
      drop_apply_vec<4>(dk1, (uint32_t)(drow * HD + n), x);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[e] += L.sX1[li][n + e];
        v[t][e] = x[e];
      }
      if (mrow) *reinterpret_cast<float4*>(a.x1 + (int64_t)m * HD + n) = make_float4(x[0], x[1], x[2], x[3]);
    }
    __syncthreads();                                 // every wave is done reading ctx and res
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) L.sX1[li][n0 + 16 * t + 4 * g + e] = v[t][e];
    float mu, rs;
    row_ln(v, Q.n2w, Q.n2b, a.eps, false, n0, L, w, lane, mu, rs);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
      const float x[4] = {v[t][0], v[t][1], v[t][2], v[t][3]};
      st4_bf(L.sA + li * PD + n * 2, x);
      if (mrow) st4_bf(reinterpret_cast<char*>(a.a2 + (int64_t)m * HD + n), x);
    }
    if (mrow && lane < 16 && w == 0) { a.m2[m] = mu; a.r2[m] = rs; }
  }
  __syncthreads();
  STAMP(2);
  // ---- h = dropf(relu(a2·W1ᵀ + b1)), 64 columns of the wave's F / 4 at a time
  WFrags<2, F> w2;
  {
    WFrags<4, HD> w1n;
#pragma unroll
    for (int nb = 0; nb < F / 4; nb += 64) {
      f32x4_t hv[4];
      head_gemm<4, HD, PD>(L.sA, nb == 0 ? w1a : w1n, hv, lane);
      if (nb + 64 < F / 4) w1n.load(a.w1, HD, nf0 + nb + 64, lane, HD);
      else w2.load(a.w2, F, n0, lane, F);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int n = nf0 + nb + 16 * t + 4 * g;
        float x[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = fmaxf(hv[t][e] + Q.b1[n + e], 0.f);
        drop_apply_vec<4>(dkf, (uint32_t)(drow * F + n), x);
        st4_bf(L.sH + li * PF + n * 2, x);
        if (mrow) st4_bf(reinterpret_cast<char*>(a.h + (int64_t)m * F + n), x);
      }
    }
  }
  __syncthreads();
  STAMP(3);
  // ---- x2 = x1 + drop2(h·W2ᵀ + b2) -> comb[:, :128]
  head_gemm<2, F, PF>(L.sH, w2, v, lane);
  WFrags<2, WPAD> wf0;
  wf0.load(a.wf0, W, n0, lane, W);
  {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
      float x[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = v[t][e] + Q.b2[n + e];
      drop_apply_vec<4>(dk2, (uint32_t)(drow * HD + n), x);
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] += L.sX1[li][n + e];
      st4_bf(L.sC + li * PW + n * 2, x);
      if (mrow) st4_bf(reinterpret_cast<char*>(a.comb + (int64_t)m * W + n), x);
    }
  }
  __syncthreads();
  STAMP(4);
  // ---- z = comb·Wf0ᵀ + bf0; az = relu(LN(z))
  head_gemm<2, WPAD, PW>(L.sC, wf0, v, lane);
  WFrags<2, HD> wf3;
  wf3.load(a.wf3, HD, n0, lane, HD);
  {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[t][e] += Q.bf0[n + e];
      if (mrow) *reinterpret_cast<float4*>(a.z + (int64_t)m * HD + n) = make_float4(v[t][0], v[t][1], v[t][2], v[t][3]);
    }
    float mu, rs;
    row_ln(v, Q.lnw, Q.lnb, a.eps, true, n0, L, w, lane, mu, rs);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
      const float x[4] = {v[t][0], v[t][1], v[t][2], v[t][3]};
      st4_bf(L.sA + li * PD + n * 2, x);
      if (mrow) st4_bf(reinterpret_cast<char*>(a.az + (int64_t)m * HD + n), x);
    }
    if (mrow && lane < 16 && w == 0) { a.mz[m] = mu; a.rz[m] = rs; }
  }
  __syncthreads();
  STAMP(5);
  // ---- u = az·Wf3ᵀ + bf3
  head_gemm<2, HD, PD>(L.sA, wf3, v, lane);
  float uo[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
#pragma unroll
    for (int e = 0; e < 4; ++e) uo[t][e] = v[t][e] + Q.bf3[n + e];
    if (mrow)
      *reinterpret_cast<float4*>(a.u + (int64_t)m * HD + n) = make_float4(uo[t][0], uo[t][1], uo[t][2], uo[t][3]);
  }
  row_l2norm(uo, a.uhat, a.unrm, m, mrow, n0, L, w, lane);
  STAMP(6);
}

// ---- the FFN split over its hidden units (ABI 21, ttmi_user_head_desc::ffn_ws)
// The kernel above runs 32 row blocks: 7 of 8 CUs idle, and each workgroup streams all 368 KB
// of the head's weights through its one CU (~36 GB/s a CU: that stream is the kernel's time).
// Here row block rb runs on NS = F / 128 workgroups j.  Each computes out-proj + LN2 for the
// block's rows (the out-proj weights, redundantly), the hidden units [128 j, 128 j + 128) of
// FFN1 and their partial FFN2 product, and hands the fp32 partial [16 x D] over through
// write-through stores and an agent-scope arrival count (the item head's handoff pattern
// above).  The last of the NS to arrive sums the partials in split order — the same bits
// whichever arrives last — then runs the residual, the concat and the fusion MLP.  Weight bytes
// through a CU at D = 128: 96 KB (176 KB for the last arriver) instead of 368.
// D = 128 (4 waves) or 256 (8 waves, F = 1024: the reference's default width, ABI 21); each
// wave owns 32 of the D columns of every D-wide stage.
template <int D_, int F>
struct SplitLds {
  using G = SplitGeo<D_>;
  char sA[HR * G::PD];      // ctx, then a2, then az
  char sH[HR * G::PH];      // the split's h columns
  char sC[HR * G::PW];      // comb (zero-padded to WPAD)
  float sX1[HR][D_ + 4];    // x1 (fp32 residual of the FFN)
  float red[G::NW][HR];     // LayerNorm cross-wave partials
  float bo[D_], n2w[D_], n2b[D_], b1[F], b2[D_], bf0[D_], lnw[D_], lnb[D_], bf3[D_];
};
template <int D_, int F>
__global__ __launch_bounds__(D_ * 2) void user_head_fwd_split_kernel(HeadArgs a) {
  using G = SplitGeo<D_>;
  constexpr int NS = F / 128, NW = G::NW, NT = NW * 64, TH = G::TH;
  STAMP(0);
  __shared__ __attribute__((aligned(16))) union {
    SplitLds<D_, F> s;
    ItemLdsA ia;
    ItemLdsCT<D_> ic;
  } U;
  SplitLds<D_, F>& L = U.s;
  __shared__ int s_last;
  const int nsplit = a.nbu * NS;
  int ub = (int)blockIdx.x;
  if (a.it_stage == 3) {                             // co-launched item head stages
    const int na = a.it_nblk * (IN1 / 64);
    if (ub < na) {
      item_a_body(a.it, ub % a.it_nblk, ub / a.it_nblk, U.ia);
      return;
    }
    ub -= na;
    if (ub >= nsplit) {
      item_c_body<true, D_>(a.it, ub - nsplit, U.ic);
      return;
    }
  } else if (ub >= nsplit) {
    const int l = ub - nsplit;
    if (a.it_stage == 0) item_a_body(a.it, l % a.it_nblk, l / a.it_nblk, U.ia);
    else item_c_body<false, D_>(a.it, l, U.ic);
    return;
  }
  const int rb = ub / NS, j = ub % NS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, g = lane >> 4;
  const int r0 = rb * HR, m = r0 + li;
  const bool mrow = m < a.B;
  const bool lead = j == 0;                          // writes what every split computes alike
  const int W = D_ + a.dg + a.dc;
  const int n0 = w * 32;                             // this wave's 32 of the D columns
  const int nh = 128 * j + 16 * TH * w;              // ... and its hidden units of the split
  WFrags<2, D_> wo;
  wo.load(a.wo, D_, n0, lane, D_);
  {                                                  // ctx: 16 rows x D/8 chunks of 16 bytes
    const int r = tid / (D_ / 8), ch = tid % (D_ / 8);
    *reinterpret_cast<uint4*>(L.sA + r * G::PD + ch * 16) =
        *reinterpret_cast<const uint4*>(a.ctx + (int64_t)min(r0 + r, a.B - 1) * D_ + ch * 8);
#pragma unroll
    for (int q = 0; q < 2; ++q) {                     // residual: 16 rows x D/4 float4
      const int idx = tid + NT * q, rr = idx / (D_ / 4), c4 = idx % (D_ / 4);
      *reinterpret_cast<float4*>(&L.sX1[rr][c4 * 4]) =
          *reinterpret_cast<const float4*>(a.res + (int64_t)min(r0 + rr, a.B - 1) * D_ + c4 * 4);
    }
  }
  {
    const float4 p0 = vec_ld<D_>(a.bo, tid), p1 = vec_ld<D_>(a.n2w, tid), p2 = vec_ld<D_>(a.n2b, tid);
    const float4 p3 = vec_ld<F>(a.b1, tid), p4 = vec_ld<D_>(a.b2, tid), p5 = vec_ld<D_>(a.bf0, tid);
    const float4 p6 = vec_ld<D_>(a.lnw, tid), p7 = vec_ld<D_>(a.lnb, tid), p8 = vec_ld<D_>(a.bf3, tid);
    vec_st<D_>(L.bo, p0, tid); vec_st<D_>(L.n2w, p1, tid); vec_st<D_>(L.n2b, p2, tid);
    vec_st<F>(L.b1, p3, tid); vec_st<D_>(L.b2, p4, tid); vec_st<D_>(L.bf0, p5, tid);
    vec_st<D_>(L.lnw, p6, tid); vec_st<D_>(L.lnb, p7, tid); vec_st<D_>(L.bf3, p8, tid);
  }
  if (tid < 256) {   // demographics (as user_head_fwd_kernel); the lead writes comb's trailing columns
    const int r = tid >> 4, k0 = D_ + 4 * (tid & 15), rr = min(r0 + r, a.B - 1);
    const int64_t gi = clamp_id(a.gender[rr], a.ng, a.id_err, TTMI_IDERR_GENDER);
    const int64_t ci = clamp_id(a.country[rr], a.nc, a.id_err, TTMI_IDERR_COUNTRY);
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int kk = k0 + e;
      float gv = a.G[gi * a.dg + min(kk - D_, a.dg - 1)];
      float cv = a.C[ci * a.dc + min(max(kk - D_ - a.dg, 0), a.dc - 1)];
      asm volatile("" : "+v"(gv), "+v"(cv));
      v[e] = kk < D_ + a.dg ? gv : (kk < W ? cv : 0.f);
    }
    st4_bf(L.sC + r * G::PW + k0 * 2, v);
    if (lead && k0 < W && r0 + r < a.B) st4_bf(reinterpret_cast<char*>(a.comb + (int64_t)(r0 + r) * W + k0), v);
  }
  if (lead && tid < HR && r0 + tid < a.B) a.rows[r0 + tid] = r0 + tid;
  const int drow = a.drows[min(m, a.B - 1)];
  const uint64_t s1 = *a.d1.seed, sf = *a.dff.seed, s2 = *a.d2.seed;
  const DropKeys dk1{(uint32_t)s1, (uint32_t)(s1 >> 32), a.d1.thresh, a.d1.scale, a.d1.on};
  const DropKeys dkf{(uint32_t)sf, (uint32_t)(sf >> 32), a.dff.thresh, a.dff.scale, a.dff.on};
  const DropKeys dk2{(uint32_t)s2, (uint32_t)(s2 >> 32), a.d2.thresh, a.d2.scale, a.d2.on};
  __syncthreads();
  STAMP(1);
  // ---- x1 = res + drop1(ctx·Woᵀ + bo); a2 = LN2(x1)   (every split; the lead stores them)
  f32x4_t v[2];
  head_gemm<2, D_, G::PD>(L.sA, wo, v, lane);
  WFrags<TH, D_> w1s;
  w1s.load(a.w1, D_, nh, lane, D_);
  {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
      float x[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = v[t][e] + L.bo[n + e];
      drop_apply_vec<4>(dk1, (uint32_t)(drow * D_ + n), x);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[e] += L.sX1[li][n + e];
        v[t][e] = x[e];
      }
      if (lead && mrow) *reinterpret_cast<float4*>(a.x1 + (int64_t)m * D_ + n) = make_float4(x[0], x[1], x[2], x[3]);
    }
    __syncthreads();                                 // every wave is done reading ctx and res
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) L.sX1[li][n0 + 16 * t + 4 * g + e] = v[t][e];
    float mu, rs;
    split_row_ln<D_>(v, L.n2w, L.n2b, a.eps, false, n0, L.red, w, lane, mu, rs);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
      const float x[4] = {v[t][0], v[t][1], v[t][2], v[t][3]};
      st4_bf(L.sA + li * G::PD + n * 2, x);
      if (lead && mrow) st4_bf(reinterpret_cast<char*>(a.a2 + (int64_t)m * D_ + n), x);
    }
    if (lead && mrow && lane < 16 && w == 0) { a.m2[m] = mu; a.r2[m] = rs; }
  }
  __syncthreads();
  STAMP(2);
  // ---- h[:, 128j ..) = dropf(relu(a2·W1ᵀ + b1)): the wave's hidden units
  WFrags<2, 128> w2s;                                // W2[:, 128j .. 128j + 128): k window
  {
    f32x4_t hv[TH];
    head_gemm<TH, D_, G::PD>(L.sA, w1s, hv, lane);
    w2s.load(a.w2 + 128 * j, F, n0, lane, 128);
#pragma unroll
    for (int t = 0; t < TH; ++t) {
      const int n = nh + 16 * t + 4 * g;
      float x[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = fmaxf(hv[t][e] + L.b1[n + e], 0.f);
      drop_apply_vec<4>(dkf, (uint32_t)(drow * F + n), x);
      st4_bf(L.sH + li * G::PH + (n - 128 * j) * 2, x);
      if (mrow) st4_bf(reinterpret_cast<char*>(a.h + (int64_t)m * F + n), x);
    }
  }
  __syncthreads();
  STAMP(3);
  // ---- this split's FFN2 partial -> exchange slot (rb, j); the last arriver goes on
  head_gemm<2, 128, G::PH>(L.sH, w2s, v, lane);
  STAMP(4);
  // fusion_layer.0's fragments before the handoff (every split: their L2 round trip then
  // overlaps the exchange's instead of following it)
  WFrags<2, G::WPAD> wf0;
  wf0.load(a.wf0, W, n0, lane, W);
  float* const part = a.ffn_part + (int64_t)rb * NS * HR * D_;      // [NS][HR][D]
#pragma unroll
  for (int t = 0; t < 2; ++t)
    st16_wt(part, (uint32_t)(((j * HR + li) * D_ + n0 + 16 * t + 4 * g) * 4),
            make_float4(v[t][0], v[t][1], v[t][2], v[t][3]));
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (tid == 0)
    s_last = __hip_atomic_fetch_add(a.ffn_cnt + rb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == NS - 1;
  __syncthreads();
  if (!s_last) return;
  if (tid == 0) __hip_atomic_store(a.ffn_cnt + rb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  STAMP(5);
  {
    // x2 = x1 + drop2(Σ_j partial_j + b2), summed in split order -> comb[:, :D]
    float4 pp[NS][2];
#pragma unroll
    for (int jj = 0; jj < NS; ++jj)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        pp[jj][t] = ld16_wt(part, (uint32_t)(((jj * HR + li) * D_ + n0 + 16 * t + 4 * g) * 4));
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
      float x[4] = {pp[0][t].x, pp[0][t].y, pp[0][t].z, pp[0][t].w};
#pragma unroll
      for (int jj = 1; jj < NS; ++jj) {
        x[0] += pp[jj][t].x; x[1] += pp[jj][t].y; x[2] += pp[jj][t].z; x[3] += pp[jj][t].w;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] += L.b2[n + e];
      drop_apply_vec<4>(dk2, (uint32_t)(drow * D_ + n), x);
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] += L.sX1[li][n + e];
      st4_bf(L.sC + li * G::PW + n * 2, x);
      if (mrow) st4_bf(reinterpret_cast<char*>(a.comb + (int64_t)m * W + n), x);
    }
  }
  __syncthreads();
  STAMP(6);
  // ---- z = comb·Wf0ᵀ + bf0; az = relu(LN(z))
  head_gemm<2, G::WPAD, G::PW>(L.sC, wf0, v, lane);
  WFrags<2, D_> wf3;
  wf3.load(a.wf3, D_, n0, lane, D_);
  {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[t][e] += L.bf0[n + e];
      if (mrow) *reinterpret_cast<float4*>(a.z + (int64_t)m * D_ + n) = make_float4(v[t][0], v[t][1], v[t][2], v[t][3]);
    }
    float mu, rs;
    split_row_ln<D_>(v, L.lnw, L.lnb, a.eps, true, n0, L.red, w, lane, mu, rs);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
      const float x[4] = {v[t][0], v[t][1], v[t][2], v[t][3]};
      st4_bf(L.sA + li * G::PD + n * 2, x);
      if (mrow) st4_bf(reinterpret_cast<char*>(a.az + (int64_t)m * D_ + n), x);
    }
    if (mrow && lane < 16 && w == 0) { a.mz[m] = mu; a.rz[m] = rs; }
  }
  __syncthreads();
  // ---- u = az·Wf3ᵀ + bf3
  head_gemm<2, D_, G::PD>(L.sA, wf3, v, lane);
  float uo[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
#pragma unroll
    for (int e = 0; e < 4; ++e) uo[t][e] = v[t][e] + L.bf3[n + e];
    if (mrow)
      *reinterpret_cast<float4*>(a.u + (int64_t)m * D_ + n) = make_float4(uo[t][0], uo[t][1], uo[t][2], uo[t][3]);
  }
  split_row_l2norm<D_>(uo, a.uhat, a.unrm, m, mrow, n0, L.red, w, lane);
  STAMP(7);
}

// ------------------------------------------------------------------------------ backward
// The head's backward, one launch (the unfused sequence: linear_dx of fusion_layer.3, the
// ReLU-gated LayerNorm backward, linear_dx of fusion_layer.0, the concat backward, the
// dropout-2 backward, the ReLU/dropout-gated linear2 input grad, linear1's input grad with
// LN2's backward, the residual and the dropout-1 backward, and out_proj's input grad):
//   daz = du·Wf3;  dz = LNᵀ(daz ⊙ [az > 0]);  dcomb = dz·Wf0;  dx2 = dcomb[:, :D] (dG, dC by
//   fixed-point int64 atomics: order-independent, folded into the fp32 grads by the caller);  dy2 = drop2ᵀ(dx2);  dz1 = (dy2·W2) ⊙ [h > 0]·sf;
//   dx1 = LN2ᵀ(dz1·W1) + dx2;  dy1 = drop1ᵀ(dx1);  dctx = dy1·Wo.
// Weights are the transposed k-major mirrors.  The LayerNorm weight / bias gradients leave as
// per-workgroup column sums (ws [nwg][4][D]: dlnw, dlnb, dn2w, dn2b), folded in workgroup order
// with the step's weight gradients.
struct HeadBwdArgs {
  int B, F, dg, dc;
  float sf;                                 // FFN dropout scale 1 / (1 - p)
  const bf16_t* du; const bf16_t* az; const float* z; const float* mz; const float* rz;
  const bf16_t* h; const float* x1; const float* m2; const float* r2;
  const int32_t* drows; const int64_t* gender; const int64_t* country;
  const bf16_t* wf3t; const bf16_t* wf0t; const bf16_t* w2t; const bf16_t* w1t; const bf16_t* wot;
  const float* lnw; const float* n2w;
  DropParams d1, d2;
  int64_t* dG; int64_t* dC;          // TTMI_FX_GRAD fixed-point accumulators
  bf16_t* dz16; bf16_t* dy2; bf16_t* dz1; float* dx1; bf16_t* dy1; bf16_t* dctx; float* ws;
  ItemBwdArgs it; int nbu;     // co-launched item head backward: workgroups >= nbu
  int ng, nc;                  // table rows of G / C (ids clamped as in the forward)
  float* ffn_part; int* ffn_cnt;   // ABI 21: the FFN split's exchange slots and arrival counts
};

struct HeadBwdLds {
  char sA[HR * PD];         // du, then dz, then dy2, then dy1
  char sH[HR * PF];         // dz1
  float sX[HR][HD + 4];     // dx2 (fp32 residual of dx1)
  float sW[HR][HD + 4];     // LayerNorm weight-gradient terms dy·x̂ (column sums)
  float sB[HR][HD + 4];     // ... and dy
  float sDem[HR][48];       // dcomb's demographic columns (dG, dC rows), added at the end
  int sGi[HR], sCi[HR];     // the rows' gender / country indices
  float red[4][HR];
};

TTMI_DEV float bwd_row_sum(float s, HeadBwdLds& L, int w, int lane) {
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  if (lane < 16) L.red[w][lane] = s;
  __syncthreads();
  const int li = lane & 15;
  const float tot = L.red[0][li] + L.red[1][li] + L.red[2][li] + L.red[3][li];
  __syncthreads();
  return tot;
}
// LayerNorm backward of the row values dy (2 tiles x 4 per lane, columns n0 + 16t + 4g + e);
// xs / wv: the lane's LN-input values and LN weights, preloaded: dx = rs·(g − mean g − x̂·mean(g·x̂)), g = dy·w.
// The weight / bias gradient terms are summed over the block's 16 rows through LDS and
// written to ws (wsw / wsb rows).
TTMI_DEV void ln_bwd16(f32x4_t (&dy)[2], const float (&xs)[2][4], float mu, float rs, const float (&wv)[2][4],
                       int n0, bool mrow, HeadBwdLds& L, int w, int lane, float* wsw, float* wsb,
                       bool sums = true) {
  const int g = lane >> 4, li = lane & 15;
  float xh[2][4], gg[2][4];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = mrow ? dy[t][e] : 0.f;
      xh[t][e] = (xs[t][e] - mu) * rs;
      L.sW[li][n + e] = d * xh[t][e];
      L.sB[li][n + e] = d;
      gg[t][e] = d * wv[t][e];
      s1 += gg[t][e];
      s2 += gg[t][e] * xh[t][e];
    }
  }
  const float c1 = bwd_row_sum(s1, L, w, lane) * (1.f / HD);   // (its barriers publish sW, sB)
  const float c2 = bwd_row_sum(s2, L, w, lane) * (1.f / HD);
  if (sums && threadIdx.x < HD) {                    // one column per thread, rows in order
    const int c = threadIdx.x;
    float cw = 0.f, cb = 0.f;
#pragma unroll
    for (int r = 0; r < HR; ++r) { cw += L.sW[r][c]; cb += L.sB[r][c]; }
    wsw[c] = cw;
    wsb[c] = cb;
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) dy[t][e] = rs * (gg[t][e] - c1 - xh[t][e] * c2);
}

template <int D_>
struct SplitBwdLds {
  static constexpr int NW = D_ / 32;
  char sA[HR * SplitGeo<D_>::PD];   // du, then dz, then dy2, then dy1
  char sH[HR * SplitGeo<D_>::PH];   // the split's dz1 columns
  float sX[HR][D_ + 4];             // dx2 (fp32 residual of dx1)
  float sW[HR][D_ + 4];             // LayerNorm weight-gradient terms dy·x̂ (column sums)
  float sB[HR][D_ + 4];             // ... and dy
  float sDem[HR][48];               // dcomb's demographic columns (dG, dC rows)
  int sGi[HR], sCi[HR];
  float red[NW][HR];
};
// ln_bwd16 over D_ columns and NW waves (same arithmetic and order at D = 128).
template <int D_>
TTMI_DEV void split_ln_bwd(f32x4_t (&dy)[2], const float (&xs)[2][4], float mu, float rs, const float (&wv)[2][4],
                           int n0, bool mrow, SplitBwdLds<D_>& L, int w, int lane, float* wsw, float* wsb,
                           bool sums) {
  constexpr int NW = D_ / 32;
  const int g = lane >> 4, li = lane & 15;
  float xh[2][4], gg[2][4];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = mrow ? dy[t][e] : 0.f;
      xh[t][e] = (xs[t][e] - mu) * rs;
      L.sW[li][n + e] = d * xh[t][e];
      L.sB[li][n + e] = d;
      gg[t][e] = d * wv[t][e];
      s1 += gg[t][e];
      s2 += gg[t][e] * xh[t][e];
    }
  }
  const float c1 = split_row_sum<NW>(s1, L.red, w, lane) * (1.f / D_);   // (its barriers publish sW, sB)
  const float c2 = split_row_sum<NW>(s2, L.red, w, lane) * (1.f / D_);
  if (sums && threadIdx.x < D_) {                    // one column per thread, rows in order
    const int c = threadIdx.x;
    float cw = 0.f, cb = 0.f;
#pragma unroll
    for (int r = 0; r < HR; ++r) { cw += L.sW[r][c]; cb += L.sB[r][c]; }
    wsw[c] = cw;
    wsb[c] = cb;
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) dy[t][e] = rs * (gg[t][e] - c1 - xh[t][e] * c2);
}

// Item head backward, row-local part (ABI 15; reference item_tower.py:122-129 under autograd),
// on 16 rows: dy2 = backward of LayerNorm fusion_layer.5 (stored mean / rstd), written bf16
// (the fusion_layer.4 weight-gradient operand) and kept in LDS; dy1 = dy2·W4 (fp32, the
// BatchNorm backward's input) from W4ᵀ fragments.  The LN weight / bias gradient terms leave
// as this block's column sums (ws rows 2·bx, 2·bx + 1), folded later in block order.
template <int D_ = HD>
TTMI_DEV void item_c_bwd_body(const ItemBwdArgs& a, int bx, SplitBwdLds<D_>& L) {
  constexpr int NW = D_ / 32, TD = IN1 / NW / 16;    // dy1: a wave's IN1 / NW columns, TD tiles
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, g = lane >> 4;
  const int r0 = bx * HR, m = r0 + li, mc = min(m, a.B - 1);
  const bool mrow = m < a.B;
  const int n0 = 32 * w;                             // LN: this wave's 32 of the D_ columns
  const int nn0 = (IN1 / NW) * w;                    // dy1: this wave's columns of the 512
  float xs[2][4], wv[2][4];
  f32x4_t dy[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
    const float4 d = *reinterpret_cast<const float4*>(a.dout + (int64_t)mc * D_ + n);
    const float4 x = *reinterpret_cast<const float4*>(a.y2 + (int64_t)mc * D_ + n);
    const float4 v = *reinterpret_cast<const float4*>(a.lnw + n);
    dy[t] = f32x4_t{d.x, d.y, d.z, d.w};
    xs[t][0] = x.x; xs[t][1] = x.y; xs[t][2] = x.z; xs[t][3] = x.w;
    wv[t][0] = v.x; wv[t][1] = v.y; wv[t][2] = v.z; wv[t][3] = v.w;
  }
  const float mu = a.m5[mc], rs = a.r5[mc];
  WFrags<TD, D_> wf;                                 // W4ᵀ [512, D_]: the wave's column tiles
  wf.load(a.w4t, D_, nn0, lane, D_);
  float* wsr = a.ws + (int64_t)bx * 2 * D_;
  split_ln_bwd<D_>(dy, xs, mu, rs, wv, n0, mrow, L, w, lane, wsr, wsr + D_, true);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
    const float o[4] = {dy[t][0], dy[t][1], dy[t][2], dy[t][3]};
    st4_bf(L.sA + li * SplitGeo<D_>::PD + n * 2, o);
    if (mrow) st4_bf(reinterpret_cast<char*>(a.dy2 + (int64_t)m * D_ + n), o);
  }
  __syncthreads();
  f32x4_t acc[TD];
  head_gemm<TD, D_, SplitGeo<D_>::PD>(L.sA, wf, acc, lane);
  if (mrow) {
#pragma unroll
    for (int t = 0; t < TD; ++t)
      *reinterpret_cast<float4*>(a.dy1 + (int64_t)m * IN1 + nn0 + 16 * t + 4 * g) =
          make_float4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
  }
}

template <int D_>
__global__ __launch_bounds__(D_ * 2) void item_head_bwd_c_kernel(ItemBwdArgs a) {
  __shared__ __attribute__((aligned(16))) SplitBwdLds<D_> L;
  item_c_bwd_body<D_>(a, blockIdx.x, L);
}


template <int F>
__global__ __launch_bounds__(256) void user_head_bwd_kernel(HeadBwdArgs a) {
  STAMP(0);
  __shared__ __attribute__((aligned(16))) union {
    HeadBwdLds h;
    SplitBwdLds<HD> ic;
  } U;
  HeadBwdLds& L = U.h;
  if ((int)blockIdx.x >= a.nbu) {                   // co-launched item head backward (rows)
    item_c_bwd_body<HD>(a.it, (int)blockIdx.x - a.nbu, U.ic);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, g = lane >> 4;
  const int r0 = blockIdx.x * HR, m = r0 + li, mc = min(m, a.B - 1);
  const bool mrow = m < a.B;
  const int W = HD + a.dg + a.dc;
  const int n0 = w * 32, nf0 = w * (F / 4);
  float* wsb = a.ws + (int64_t)blockIdx.x * 4 * HD;   // this workgroup's four sum rows
  WFrags<2, HD> wf3;
  wf3.load(a.wf3t, HD, n0, lane, HD);
  {                                                  // du rows -> LDS
    const int r = tid >> 4, ch = tid & 15;
    *reinterpret_cast<uint4*>(L.sA + r * PD + ch * 16) =
        *reinterpret_cast<const uint4*>(a.du + (int64_t)min(r0 + r, a.B - 1) * HD + ch * 8);
  }
  const int drow = a.drows[mc];
  const float mzr = a.mz[mc], rzr = a.rz[mc], m2r = a.m2[mc], r2r = a.r2[mc];
  const uint64_t s1 = *a.d1.seed, s2 = *a.d2.seed;
  const DropKeys dk1{(uint32_t)s1, (uint32_t)(s1 >> 32), a.d1.thresh, a.d1.scale, a.d1.on};
  const DropKeys dk2{(uint32_t)s2, (uint32_t)(s2 >> 32), a.d2.thresh, a.d2.scale, a.d2.on};
  if (tid < HR) {
    L.sGi[tid] = (int)clamp_id(a.gender[min(r0 + tid, a.B - 1)], a.ng, nullptr, 0);
    L.sCi[tid] = (int)clamp_id(a.country[min(r0 + tid, a.B - 1)], a.nc, nullptr, 0);
  }
  // every per-row operand of the chain now, before any weight prefetch: vmcnt retires in
  // order, so a late small load would also wait for the weights issued before it
  uint2 azq[2];
  float zs[2][4], x1s[2][4], lnw[2][4], n2w[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
    const float4 lw = *reinterpret_cast<const float4*>(a.lnw + n);
    const float4 nw = *reinterpret_cast<const float4*>(a.n2w + n);
    lnw[t][0] = lw.x; lnw[t][1] = lw.y; lnw[t][2] = lw.z; lnw[t][3] = lw.w;
    n2w[t][0] = nw.x; n2w[t][1] = nw.y; n2w[t][2] = nw.z; n2w[t][3] = nw.w;
    azq[t] = *reinterpret_cast<const uint2*>(a.az + (int64_t)mc * HD + n);
    const float4 zv = *reinterpret_cast<const float4*>(a.z + (int64_t)mc * HD + n);
    const float4 xv = *reinterpret_cast<const float4*>(a.x1 + (int64_t)mc * HD + n);
    zs[t][0] = zv.x; zs[t][1] = zv.y; zs[t][2] = zv.z; zs[t][3] = zv.w;
    x1s[t][0] = xv.x; x1s[t][1] = xv.y; x1s[t][2] = xv.z; x1s[t][3] = xv.w;
  }
  uint2 hq[F / 64];                                  // the wave's F / 4 gate columns, 4 per lane
#pragma unroll
  for (int q = 0; q < F / 64; ++q)
    hq[q] = *reinterpret_cast<const uint2*>(a.h + (int64_t)mc * F + nf0 + 16 * q + 4 * g);
  __syncthreads();
  STAMP(1);
  // ---- daz = du·Wf3; dz = LNᵀ(daz ⊙ [az > 0])
  f32x4_t v[2];
  head_gemm<2, HD, PD>(L.sA, wf3, v, lane);
  WFrags<3, HD> wf0;                                 // dcomb's 11 column tiles: w, w+4, w+8
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int tj = min(w + 4 * j, W / 16 - 1);
#pragma unroll
    for (int c = 0; c < HD / 32; ++c) wf0.f[c][j] = wfrag(a.wf0t, HD, 16 * tj + li, c, lane, HD);
  }
  {
#pragma unroll
    for (int t = 0; t < 2; ++t) {                    // ReLU gate of the forward's az
      const uint2 q = azq[t];
      const float gz[4] = {__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xFFFF0000u),
                           __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xFFFF0000u)};
#pragma unroll
      for (int e = 0; e < 4; ++e) v[t][e] = gz[e] > 0.f ? v[t][e] : 0.f;
    }
    __syncthreads();                                 // every wave is done reading du
    ln_bwd16(v, zs, mzr, rzr, lnw, n0, mrow, L, w, lane, wsb, wsb + HD);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
      const float x[4] = {v[t][0], v[t][1], v[t][2], v[t][3]};
      st4_bf(L.sA + li * PD + n * 2, x);
      if (mrow) st4_bf(reinterpret_cast<char*>(a.dz16 + (int64_t)m * HD + n), x);
    }
  }
  __syncthreads();
  STAMP(2);
  // ---- dcomb = dz·Wf0: columns < D -> dx2 (LDS), the demographic ones -> dG / dC
  WFrags<4, HD> w2a;
  {
    f32x4_t dc[3];
    head_gemm<3, HD, PD>(L.sA, wf0, dc, lane);
    w2a.load(a.w2t, HD, nf0, lane, HD);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int tj = w + 4 * j;
      if (tj >= W / 16) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 16 * tj + 4 * g + e;
        const float val = dc[j][e];
        if (k < HD) L.sX[li][k] = mrow ? val : 0.f;
        else L.sDem[li][k - HD] = val;
      }
    }
  }
  __syncthreads();
  STAMP(3);
  // ---- dy2 = drop2ᵀ(dx2) -> LDS (A of the next product) and HBM
  {
    const int n = n0 + 4 * g;                        // two 16-column tiles per wave
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float x[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = L.sX[li][n + 16 * t + e];
      drop_apply_vec<4>(dk2, (uint32_t)(drow * HD + n + 16 * t), x);
      st4_bf(L.sA + li * PD + (n + 16 * t) * 2, x);
      if (mrow) st4_bf(reinterpret_cast<char*>(a.dy2 + (int64_t)m * HD + n + 16 * t), x);
    }
  }
  __syncthreads();
  STAMP(4);
  // ---- dz1 = (dy2·W2) ⊙ [h > 0]·sf
  WFrags<2, F> w1;
  {
    WFrags<4, HD> w2n;
#pragma unroll
    for (int nb = 0; nb < F / 4; nb += 64) {
      f32x4_t hv[4];
      head_gemm<4, HD, PD>(L.sA, nb == 0 ? w2a : w2n, hv, lane);
      if (nb + 64 < F / 4) w2n.load(a.w2t, HD, nf0 + nb + 64, lane, HD);
      else w1.load(a.w1t, F, n0, lane, F);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int n = nf0 + nb + 16 * t + 4 * g;
        const uint2 q = hq[nb / 16 + t];
        const float hg[4] = {__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xFFFF0000u),
                             __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xFFFF0000u)};
        float x[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = hg[e] > 0.f ? hv[t][e] * a.sf : 0.f;
        st4_bf(L.sH + li * PF + n * 2, x);
        if (mrow) st4_bf(reinterpret_cast<char*>(a.dz1 + (int64_t)m * F + n), x);
      }
    }
  }
  __syncthreads();
  STAMP(5);
  // ---- dx1 = LN2ᵀ(dz1·W1) + dx2; dy1 = drop1ᵀ(dx1)
  head_gemm<2, F, PF>(L.sH, w1, v, lane);
  WFrags<2, HD> wo;
  wo.load(a.wot, HD, n0, lane, HD);
  ln_bwd16(v, x1s, m2r, r2r, n2w, n0, mrow, L, w, lane, wsb + 2 * HD, wsb + 3 * HD);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
    float x[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = v[t][e] + L.sX[li][n + e];
    if (mrow) *reinterpret_cast<float4*>(a.dx1 + (int64_t)m * HD + n) = make_float4(x[0], x[1], x[2], x[3]);
    drop_apply_vec<4>(dk1, (uint32_t)(drow * HD + n), x);
    st4_bf(L.sA + li * PD + n * 2, x);               // every wave is past its dy2 reads
    if (mrow) st4_bf(reinterpret_cast<char*>(a.dy1 + (int64_t)m * HD + n), x);
  }
  __syncthreads();
  STAMP(6);
  // ---- dctx = dy1·Wo
  head_gemm<2, HD, PD>(L.sA, wo, v, lane);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
    const float x[4] = {v[t][0], v[t][1], v[t][2], v[t][3]};
    if (mrow) st4_bf(reinterpret_cast<char*>(a.dctx + (int64_t)m * HD + n), x);
  }
  // ---- dG / dC last (nothing later waits on the atomics).  Rows sharing an index are summed
  // here first (in row order): one fixed-point atomic per (distinct index, column) per
  // workgroup, a row's 48 columns in one coalesced instruction (lanes 0-15 gender, 16-47
  // country).  Integer adds: the accumulated bits do not depend on the workgroups' order.
  if (lane < 48) {
    const bool isg = lane < 16;
    const int k = isg ? lane : lane - 16;
    const int nr = min(HR, a.B - r0);
    int key[HR];
    float val[HR];
#pragma unroll
    for (int j = 0; j < HR; ++j) {                   // all LDS reads at once, then registers
      key[j] = isg ? L.sGi[j] : L.sCi[j];
      val[j] = L.sDem[j][lane];
    }
#pragma unroll
    for (int r = 0; r < HR; ++r) {                   // wave w issues rows r % 4 == w
      if ((r & 3) != w || r >= nr) continue;
      bool first = true;
#pragma unroll
      for (int j = 0; j < r; ++j) first &= key[j] != key[r];
      if (!first) continue;
      float sum = 0.f;
#pragma unroll
      for (int j = r; j < HR; ++j) sum += (j < nr && key[j] == key[r]) ? val[j] : 0.f;
      fx_add(isg ? a.dG + (int64_t)key[r] * a.dg + k : a.dC + (int64_t)key[r] * a.dc + k, sum, TTMI_FX_GRAD);
    }
  }
  STAMP(7);
}

// ---- the FFN split over its hidden units (ABI 21, ttmi_user_head_bwd_desc::ffn_ws), as the
// forward's: row block rb on NS = F / 128 workgroups j.  Each runs the fusion MLP's backward
// (daz, the ReLU-gated LayerNorm backward, dcomb, dy2: 76 KB of weights at D = 128, redundantly;
// the lead split stores what they all compute alike), the hidden units [128 j, 128 j + 128) of
// dz1 = (dy2·W2) ⊙ gate and their partial dz1·W1, handed over like the forward's partial; the
// last to arrive sums the partials in split order, then runs LN2's backward, the residual,
// drop1, dctx = dy1·Wo and the dG / dC adds.  D = 128 (4 waves) or 256 (8 waves, F = 1024).
template <int D_, int F>
__global__ __launch_bounds__(D_ * 2) void user_head_bwd_split_kernel(HeadBwdArgs a) {
  using G = SplitGeo<D_>;
  constexpr int NS = F / 128, NW = G::NW, TH = G::TH;
  STAMP(0);
  __shared__ __attribute__((aligned(16))) SplitBwdLds<D_> L;
  __shared__ int s_last;
  const int nsplit = a.nbu * NS;
  if ((int)blockIdx.x >= nsplit) {                  // co-launched item head backward (rows)
    item_c_bwd_body<D_>(a.it, (int)blockIdx.x - nsplit, L);
    return;
  }
  const int rb = (int)blockIdx.x / NS, j = (int)blockIdx.x % NS;
  const bool lead = j == 0;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, g = lane >> 4;
  const int r0 = rb * HR, m = r0 + li, mc = min(m, a.B - 1);
  const bool mrow = m < a.B;
  const int W = D_ + a.dg + a.dc;
  const int n0 = w * 32;
  const int nh = 128 * j + 16 * TH * w;              // this wave's hidden units of the split
  float* wsb = a.ws + (int64_t)rb * 4 * D_;          // the row block's four sum rows
  WFrags<2, D_> wf3;
  wf3.load(a.wf3t, D_, n0, lane, D_);
  {                                                  // du rows -> LDS
    const int r = tid / (D_ / 8), ch = tid % (D_ / 8);
    *reinterpret_cast<uint4*>(L.sA + r * G::PD + ch * 16) =
        *reinterpret_cast<const uint4*>(a.du + (int64_t)min(r0 + r, a.B - 1) * D_ + ch * 8);
  }
  const int drow = a.drows[mc];
  const float mzr = a.mz[mc], rzr = a.rz[mc], m2r = a.m2[mc], r2r = a.r2[mc];
  const uint64_t s1 = *a.d1.seed, s2 = *a.d2.seed;
  const DropKeys dk1{(uint32_t)s1, (uint32_t)(s1 >> 32), a.d1.thresh, a.d1.scale, a.d1.on};
  const DropKeys dk2{(uint32_t)s2, (uint32_t)(s2 >> 32), a.d2.thresh, a.d2.scale, a.d2.on};
  if (tid < HR) {
    L.sGi[tid] = (int)clamp_id(a.gender[min(r0 + tid, a.B - 1)], a.ng, nullptr, 0);
    L.sCi[tid] = (int)clamp_id(a.country[min(r0 + tid, a.B - 1)], a.nc, nullptr, 0);
  }
  uint2 azq[2];
  float zs[2][4], x1s[2][4], lnw[2][4], n2w[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
    const float4 lw = *reinterpret_cast<const float4*>(a.lnw + n);
    const float4 nw = *reinterpret_cast<const float4*>(a.n2w + n);
    lnw[t][0] = lw.x; lnw[t][1] = lw.y; lnw[t][2] = lw.z; lnw[t][3] = lw.w;
    n2w[t][0] = nw.x; n2w[t][1] = nw.y; n2w[t][2] = nw.z; n2w[t][3] = nw.w;
    azq[t] = *reinterpret_cast<const uint2*>(a.az + (int64_t)mc * D_ + n);
    const float4 zv = *reinterpret_cast<const float4*>(a.z + (int64_t)mc * D_ + n);
    const float4 xv = *reinterpret_cast<const float4*>(a.x1 + (int64_t)mc * D_ + n);
    zs[t][0] = zv.x; zs[t][1] = zv.y; zs[t][2] = zv.z; zs[t][3] = zv.w;
    x1s[t][0] = xv.x; x1s[t][1] = xv.y; x1s[t][2] = xv.z; x1s[t][3] = xv.w;
  }
  uint2 hq[TH];                                      // the wave's gate columns, 4 per lane
#pragma unroll
  for (int q = 0; q < TH; ++q)
    hq[q] = *reinterpret_cast<const uint2*>(a.h + (int64_t)mc * F + nh + 16 * q + 4 * g);
  __syncthreads();
  STAMP(1);
  // ---- daz = du·Wf3; dz = LNᵀ(daz ⊙ [az > 0])
  f32x4_t v[2];
  head_gemm<2, D_, G::PD>(L.sA, wf3, v, lane);
  WFrags<3, D_> wf0;                                 // dcomb's W / 16 column tiles: w, w+NW, w+2NW
#pragma unroll
  for (int jj = 0; jj < 3; ++jj) {
    const int tj = min(w + NW * jj, W / 16 - 1);
#pragma unroll
    for (int c = 0; c < D_ / 32; ++c) wf0.f[c][jj] = wfrag(a.wf0t, D_, 16 * tj + li, c, lane, D_);
  }
  {
#pragma unroll
    for (int t = 0; t < 2; ++t) {                    // ReLU gate of the forward's az
      const uint2 q = azq[t];
      const float gz[4] = {__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xFFFF0000u),
                           __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xFFFF0000u)};
#pragma unroll
      for (int e = 0; e < 4; ++e) v[t][e] = gz[e] > 0.f ? v[t][e] : 0.f;
    }
    __syncthreads();                                 // every wave is done reading du
    split_ln_bwd<D_>(v, zs, mzr, rzr, lnw, n0, mrow, L, w, lane, wsb, wsb + D_, lead);   // (the lead's sums)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + 16 * t + 4 * g;
      const float x[4] = {v[t][0], v[t][1], v[t][2], v[t][3]};
      st4_bf(L.sA + li * G::PD + n * 2, x);
      if (lead && mrow) st4_bf(reinterpret_cast<char*>(a.dz16 + (int64_t)m * D_ + n), x);
    }
  }
  __syncthreads();
  STAMP(2);
  // ---- dcomb = dz·Wf0: columns < D -> dx2 (LDS), the demographic ones -> sDem
  WFrags<TH, D_> w2s;                                // W2ᵀ rows of the wave's hidden units
  {
    f32x4_t dc[3];
    head_gemm<3, D_, G::PD>(L.sA, wf0, dc, lane);
    w2s.load(a.w2t, D_, nh, lane, D_);
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      const int tj = w + NW * jj;
      if (tj >= W / 16) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 16 * tj + 4 * g + e;
        const float val = dc[jj][e];
        if (k < D_) L.sX[li][k] = mrow ? val : 0.f;
        else L.sDem[li][k - D_] = val;
      }
    }
  }
  __syncthreads();
  STAMP(3);
  // ---- dy2 = drop2ᵀ(dx2) -> LDS (A of the next product); the lead stores it
  {
    const int n = n0 + 4 * g;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float x[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = L.sX[li][n + 16 * t + e];
      drop_apply_vec<4>(dk2, (uint32_t)(drow * D_ + n + 16 * t), x);
      st4_bf(L.sA + li * G::PD + (n + 16 * t) * 2, x);
      if (lead && mrow) st4_bf(reinterpret_cast<char*>(a.dy2 + (int64_t)m * D_ + n + 16 * t), x);
    }
  }
  __syncthreads();
  STAMP(4);
  // ---- dz1[:, 128j ..) = (dy2·W2) ⊙ [h > 0]·sf
  WFrags<2, 128> w1s;                                // W1ᵀ[:, 128j .. 128j + 128): k window
  {
    f32x4_t hv[TH];
    head_gemm<TH, D_, G::PD>(L.sA, w2s, hv, lane);
    w1s.load(a.w1t + 128 * j, F, n0, lane, 128);
#pragma unroll
    for (int t = 0; t < TH; ++t) {
      const int n = nh + 16 * t + 4 * g;
      const uint2 q = hq[t];
      const float hg[4] = {__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xFFFF0000u),
                           __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xFFFF0000u)};
      float x[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = hg[e] > 0.f ? hv[t][e] * a.sf : 0.f;
      st4_bf(L.sH + li * G::PH + (n - 128 * j) * 2, x);
      if (mrow) st4_bf(reinterpret_cast<char*>(a.dz1 + (int64_t)m * F + n), x);
    }
  }
  __syncthreads();
  STAMP(5);
  // ---- this split's partial dz1·W1 -> exchange slot (rb, j); the last arriver goes on
  head_gemm<2, 128, G::PH>(L.sH, w1s, v, lane);
  WFrags<2, D_> wo;                                  // (before the handoff, as the forward's wf0)
  wo.load(a.wot, D_, n0, lane, D_);
  float* const part = a.ffn_part + (int64_t)rb * NS * HR * D_;      // [NS][HR][D]
#pragma unroll
  for (int t = 0; t < 2; ++t)
    st16_wt(part, (uint32_t)(((j * HR + li) * D_ + n0 + 16 * t + 4 * g) * 4),
            make_float4(v[t][0], v[t][1], v[t][2], v[t][3]));
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (tid == 0)
    s_last = __hip_atomic_fetch_add(a.ffn_cnt + rb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == NS - 1;
  __syncthreads();
  if (!s_last) return;
  if (tid == 0) __hip_atomic_store(a.ffn_cnt + rb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  STAMP(6);
  // ---- dx1 = LN2ᵀ(Σ_j partial_j) + dx2; dy1 = drop1ᵀ(dx1)
  {
    float4 pp[NS][2];
#pragma unroll
    for (int jj = 0; jj < NS; ++jj)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        pp[jj][t] = ld16_wt(part, (uint32_t)(((jj * HR + li) * D_ + n0 + 16 * t + 4 * g) * 4));
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      v[t] = f32x4_t{pp[0][t].x, pp[0][t].y, pp[0][t].z, pp[0][t].w};
#pragma unroll
      for (int jj = 1; jj < NS; ++jj) {
        v[t][0] += pp[jj][t].x; v[t][1] += pp[jj][t].y; v[t][2] += pp[jj][t].z; v[t][3] += pp[jj][t].w;
      }
    }
  }
  split_ln_bwd<D_>(v, x1s, m2r, r2r, n2w, n0, mrow, L, w, lane, wsb + 2 * D_, wsb + 3 * D_, true);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
    float x[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = v[t][e] + L.sX[li][n + e];
    if (mrow) *reinterpret_cast<float4*>(a.dx1 + (int64_t)m * D_ + n) = make_float4(x[0], x[1], x[2], x[3]);
    drop_apply_vec<4>(dk1, (uint32_t)(drow * D_ + n), x);
    st4_bf(L.sA + li * G::PD + n * 2, x);            // every wave is past its dy2 reads
    if (mrow) st4_bf(reinterpret_cast<char*>(a.dy1 + (int64_t)m * D_ + n), x);
  }
  __syncthreads();
  // ---- dctx = dy1·Wo
  head_gemm<2, D_, G::PD>(L.sA, wo, v, lane);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 16 * t + 4 * g;
    const float x[4] = {v[t][0], v[t][1], v[t][2], v[t][3]};
    if (mrow) st4_bf(reinterpret_cast<char*>(a.dctx + (int64_t)m * D_ + n), x);
  }
  // ---- dG / dC (as user_head_bwd_kernel; lanes < 48 of waves 0-3 issue the rows)
  if (lane < 48 && w < 4) {
    const bool isg = lane < 16;
    const int k = isg ? lane : lane - 16;
    const int nr = min(HR, a.B - r0);
    int key[HR];
    float val[HR];
#pragma unroll
    for (int jj = 0; jj < HR; ++jj) {
      key[jj] = isg ? L.sGi[jj] : L.sCi[jj];
      val[jj] = L.sDem[jj][lane];
    }
#pragma unroll
    for (int r = 0; r < HR; ++r) {
      if ((r & 3) != w || r >= nr) continue;
      bool first = true;
#pragma unroll
      for (int jj = 0; jj < r; ++jj) first &= key[jj] != key[r];
      if (!first) continue;
      float sum = 0.f;
#pragma unroll
      for (int jj = r; jj < HR; ++jj) sum += (jj < nr && key[jj] == key[r]) ? val[jj] : 0.f;
      fx_add(isg ? a.dG + (int64_t)key[r] * a.dg + k : a.dC + (int64_t)key[r] * a.dc + k, sum, TTMI_FX_GRAD);
    }
  }
  STAMP(7);
}

// ------------------------------------------------------------------------------ item head
// The item tower's late-fusion MLP (reference item_tower.py:122-129) in three launches instead
// of five (cast, Linear, BatchNorm+ReLU+dropout, Linear, LayerNorm):
//   A: m = bf16(modal); z = m·W0ᵀ + b0 (16 rows x 64 columns per workgroup);
//   BatchNorm + ReLU + dropout: bnr_fwd_kernel (ttmi_norm.hip), unchanged — the batch
//      statistics are a reduction over all rows, column-blocked;
//   C: y2 = y1·W4ᵀ + b4; out = LN(y2) (16 rows per workgroup, y1 rows in LDS).
// Saved for the backward exactly as the unfused ops wrote them: m, z, BN mean / rstd, y1, y2,
// the LayerNorm mean / rstd.
__global__ __launch_bounds__(256) void item_head_a_kernel(ItemArgs a) {
  __shared__ __attribute__((aligned(16))) ItemLdsA L;
  item_a_body(a, blockIdx.x, blockIdx.y, L);
}

// The pruned layer's one-query attention (with the last-valid gather) and item stage A on one
// grid (ttmi_mha_q1_gather_item_fwd): workgroups [0, nit) run item_a_body (they take longest,
// so they are dispatched first), the rest one (sequence, head) per wave (ttmi_q1.h).
template <typename T>
__global__ __launch_bounds__(256) void q1_item_fwd_kernel(Q1Args q, ItemArgs it, int it_nblk, int nit) {
  __shared__ __attribute__((aligned(16))) union U {
    ItemLdsA ia;
    Q1Lds q[4];
  } S;
  if ((int)blockIdx.x < nit) {
    item_a_body(it, (int)blockIdx.x % it_nblk, (int)blockIdx.x / it_nblk, S.ia);
    return;
  }
  const int w = threadIdx.x >> 6, bh = ((int)blockIdx.x - nit) * 4 + w;
  if (bh >= q.B * q.H) return;
  q1_fwd_wave<T, true>(q, bh, S.q[w]);
}

}  // namespace

namespace {
int item_fwd_check(const ttmi_item_head_desc* d) {
  TTMI_REQUIRE(d != nullptr, "ttmi_item_head_fwd: null descriptor");
  TTMI_REQUIRE(d->B > 1 && d->K == IK && d->N1 == IN1 && (d->D == HD || d->D == 2 * HD),
               "ttmi_item_head_fwd: needs B > 1 (training BatchNorm), K == N1 == %d, D in {%d, %d}", IK, HD,
               2 * HD);
  TTMI_REQUIRE(d->modal && d->w0 && d->b0 && d->bn_w && d->bn_b && d->w4 && d->b4 && d->ln_w && d->ln_b &&
               d->modal16 && d->z && d->bn_mean && d->bn_rstd && d->y1 && d->y2 && d->out && d->m5 &&
               d->r5 && (!d->out_hat || d->out_norm), "ttmi_item_head_fwd: null argument");
  return TTMI_OK;
}
ItemArgs item_args(const ttmi_item_head_desc* d) {
  ItemArgs a{};
  a.B = d->B;
  a.D = d->D;
  a.modal = d->modal; a.w0 = (const bf16_t*)d->w0; a.b0 = d->b0;
  a.y1 = (const bf16_t*)d->y1; a.w4 = (const bf16_t*)d->w4; a.b4 = d->b4;
  a.lnw = d->ln_w; a.lnb = d->ln_b; a.ln_eps = d->ln_eps;
  a.m16 = (bf16_t*)d->modal16; a.z = d->z; a.y2 = d->y2; a.out = d->out; a.m5 = d->m5; a.r5 = d->r5;
  a.ohat = d->out_hat; a.onrm = d->out_hat ? d->out_norm : nullptr;
  a.bnw = d->bn_w; a.bnb = d->bn_b; a.bn_eps = d->bn_eps; a.bn_mom = d->momentum;
  a.rmean = d->running_mean; a.rvar = d->running_var; a.nbt = d->num_batches_tracked;
  a.bmean = d->bn_mean; a.brstd = d->bn_rstd; a.y1w = (bf16_t*)d->y1;
  a.bd = make_drop(d->drop_p, d->drop_seed ? d->drop_seed : reinterpret_cast<const uint64_t*>(d->b0));
  const bool fuse = d->bn_part && d->bn_cnt && d->B <= BN_MAXBLK * HR;
  a.bnpart = fuse ? d->bn_part : nullptr;
  a.bncnt = fuse ? d->bn_cnt : nullptr;
  return a;
}
int item_bwd_check(const ttmi_item_head_bwd_desc* d) {
  TTMI_REQUIRE(d != nullptr, "ttmi_item_head_bwd_c: null descriptor");
  TTMI_REQUIRE(d->B > 0 && (d->D == HD || d->D == 2 * HD) && d->N1 == IN1,
               "ttmi_item_head_bwd_c: needs D in {%d, %d}, N1 == %d", HD, 2 * HD, IN1);
  TTMI_REQUIRE(d->dout && d->y2 && d->m5 && d->r5 && d->ln_w && d->w4t && d->dy2 && d->dy1 && d->ws,
               "ttmi_item_head_bwd_c: null argument");
  TTMI_REQUIRE(((uintptr_t)d->dout & 15) == 0 && ((uintptr_t)d->y2 & 15) == 0 && ((uintptr_t)d->dy1 & 15) == 0 &&
               ((uintptr_t)d->w4t & 15) == 0 && ((uintptr_t)d->dy2 & 7) == 0,
               "ttmi_item_head_bwd_c: dout / y2 / dy1 / w4t need 16-byte, dy2 8-byte alignment");
  return TTMI_OK;
}
ItemBwdArgs item_bwd_args(const ttmi_item_head_bwd_desc* d) {
  ItemBwdArgs a{};
  a.B = d->B; a.D = d->D; a.dout = d->dout; a.y2 = d->y2; a.m5 = d->m5; a.r5 = d->r5; a.lnw = d->ln_w;
  a.w4t = (const bf16_t*)d->w4t; a.dy2 = (bf16_t*)d->dy2; a.dy1 = d->dy1; a.ws = d->ws;
  return a;
}
}  // namespace

extern "C" int ttmi_item_head_fwd_stages(const ttmi_item_head_desc* d, int stages, hipStream_t s) {
  int rc = item_fwd_check(d);
  if (rc != TTMI_OK) return rc;
  TTMI_REQUIRE(stages > 0 && stages < 8, "ttmi_item_head_fwd_stages: stages is a mask of 1 (A), 2 (BN), 4 (C)");
  const ItemArgs a = item_args(d);
  const unsigned nblk = (unsigned)((d->B + HR - 1) / HR);
  if (stages & 1) {
    hipLaunchKernelGGL(item_head_a_kernel, dim3(nblk, IN1 / 64), dim3(256), 0, s, a);
    rc = ttmi_check_launch("ttmi_item_head_fwd");
    if (rc != TTMI_OK) return rc;
  }
  if ((stages & 2) && a.bncnt == nullptr) {          // fused: statistics in A, applied in C
    rc = ttmi_batchnorm_fwd(TTMI_BF16, d->B, IN1, d->z, d->bn_w, d->bn_b, d->bn_eps, d->momentum,
                            d->running_mean, d->running_var, d->num_batches_tracked, 1, 1, d->drop_p,
                            d->drop_seed, d->y1, d->bn_mean, d->bn_rstd, s);
    if (rc != TTMI_OK) return rc;
  }
  if (stages & 4) {
    if (d->D == 2 * HD) hipLaunchKernelGGL(item_head_c_kernel<2 * HD>, dim3(nblk), dim3(4 * HD), 0, s, a);
    else hipLaunchKernelGGL(item_head_c_kernel<HD>, dim3(nblk), dim3(2 * HD), 0, s, a);
    return ttmi_check_launch("ttmi_item_head_fwd");
  }
  return TTMI_OK;
}

extern "C" int ttmi_item_head_fwd(const ttmi_item_head_desc* d, hipStream_t s) {
  return ttmi_item_head_fwd_stages(d, 7, s);
}

extern "C" int64_t ttmi_item_head_bn_part_floats(int B) { return (int64_t)((B + HR - 1) / HR) * 2 * IN1; }
// the column quarters' arrival counts, then (ABI 18) stage A's done count, stage C's count and an
// error word (a C workgroup's poll timed out)
extern "C" int64_t ttmi_item_head_bn_counter_bytes(int B) { (void)B; return (IN1 / 64 + 3) * 4; }

// [nblk][2][D] column sums, sized for D = 256 (ABI 21)
extern "C" int64_t ttmi_item_head_bwd_ws_floats(int B) { return (int64_t)((B + HR - 1) / HR) * 2 * 2 * HD; }

extern "C" int ttmi_item_head_bwd_c(const ttmi_item_head_bwd_desc* d, hipStream_t s) {
  const int rc = item_bwd_check(d);
  if (rc != TTMI_OK) return rc;
  if (d->D == 2 * HD)
    hipLaunchKernelGGL(item_head_bwd_c_kernel<2 * HD>, dim3((unsigned)((d->B + HR - 1) / HR)), dim3(4 * HD), 0, s,
                       item_bwd_args(d));
  else
    hipLaunchKernelGGL(item_head_bwd_c_kernel<HD>, dim3((unsigned)((d->B + HR - 1) / HR)), dim3(2 * HD), 0, s,
                       item_bwd_args(d));
  return ttmi_check_launch("ttmi_item_head_bwd_c");
}

namespace {
// the FFN split's workspace: arrival counts (one int per row block, 256-byte padded), then the
// exchange slots [nbu][F / 128][HR][HD] fp32
int64_t ffn_cnt_bytes(int B) { return ((int64_t)((B + HR - 1) / HR) * 4 + 255) / 256 * 256; }

int user_item_head_fwd_impl(const ttmi_user_head_desc* d, const ttmi_item_head_desc* it, int stage,
                            hipStream_t s) {
  TTMI_REQUIRE(d != nullptr, "ttmi_user_head_fwd: null descriptor");
  // D = 128 with F in {256, 512}; D = 256 with F = 1024 on the split kernel only (the
  // reference's default width), without item head co-launches
  const bool d256 = d->D == 2 * HD && d->F == 4 * 2 * HD;
  TTMI_REQUIRE(d->B > 0 && (d->D == HD || d256), "ttmi_user_head_fwd: needs D == %d, or D == %d with F == %d",
               HD, 2 * HD, 8 * HD);
  TTMI_REQUIRE(d256 || (d->F > 0 && d->F <= FMAX && d->F % 256 == 0),
               "ttmi_user_head_fwd: needs F %% 256 == 0, F <= %d", FMAX);
  TTMI_REQUIRE(!d256 || (d->ffn_ws && !getenv("TTMI_HEAD_NOSPLIT")),
               "ttmi_user_head_fwd: D == 256 runs the FFN split only (ffn_ws)");
  TTMI_REQUIRE(!it || it->D == d->D, "ttmi_user_item_head_fwd: the item head's width must be the user head's");
  TTMI_REQUIRE(d->dg == 16 && d->dc == 32, "ttmi_user_head_fwd: demographic widths must be 16 and 32");
  TTMI_REQUIRE(d->n_genders > 0 && d->n_countries > 0, "ttmi_user_head_fwd: n_genders / n_countries must be > 0");
  TTMI_REQUIRE(d->ctx && d->res && d->drop_rows && d->wo && d->bo && d->n2w && d->n2b && d->w1 && d->b1 && d->w2 &&
               d->b2 && d->gender && d->G && d->country && d->C && d->wf0 && d->bf0 && d->lnw &&
               d->lnb && d->wf3 && d->bf3 && d->x1 && d->a2 && d->m2 && d->r2 && d->h && d->comb &&
               d->rows && d->z && d->az && d->mz && d->rz && d->u, "ttmi_user_head_fwd: null argument");
  TTMI_REQUIRE((d->d1_p == 0.f || d->d1_seed) && (d->dff_p == 0.f || d->dff_seed) && (d->d2_p == 0.f || d->d2_seed),
               "ttmi_user_head_fwd: dropout needs a seed");
  HeadArgs a{};
  a.B = d->B; a.F = d->F; a.dg = d->dg; a.dc = d->dc; a.eps = d->eps;
  a.ctx = (const bf16_t*)d->ctx; a.res = d->res; a.drows = d->drop_rows;
  a.wo = (const bf16_t*)d->wo; a.bo = d->bo; a.n2w = d->n2w; a.n2b = d->n2b;
  a.w1 = (const bf16_t*)d->w1; a.b1 = d->b1; a.w2 = (const bf16_t*)d->w2; a.b2 = d->b2;
  a.gender = d->gender; a.G = d->G; a.country = d->country; a.C = d->C;
  a.ng = d->n_genders; a.nc = d->n_countries; a.id_err = d->id_err;
  a.wf0 = (const bf16_t*)d->wf0; a.bf0 = d->bf0; a.lnw = d->lnw; a.lnb = d->lnb;
  a.wf3 = (const bf16_t*)d->wf3; a.bf3 = d->bf3;
  const uint64_t* any = reinterpret_cast<const uint64_t*>(d->bo);   // read, never used when off
  a.d1 = make_drop(d->d1_p, d->d1_seed ? d->d1_seed : any);
  a.dff = make_drop(d->dff_p, d->dff_seed ? d->dff_seed : any);
  a.d2 = make_drop(d->d2_p, d->d2_seed ? d->d2_seed : any);
  a.x1 = d->x1; a.a2 = (bf16_t*)d->a2; a.m2 = d->m2; a.r2 = d->r2; a.h = (bf16_t*)d->h;
  a.comb = (bf16_t*)d->comb; a.rows = d->rows; a.z = d->z; a.az = (bf16_t*)d->az;
  a.mz = d->mz; a.rz = d->rz; a.u = d->u;
  a.uhat = d->u_hat; a.unrm = d->u_hat ? d->u_norm : nullptr;
  TTMI_REQUIRE(!d->u_hat || d->u_norm, "ttmi_user_head_fwd: u_hat needs u_norm");
  a.nbu = (d->B + HR - 1) / HR;
  a.it_nblk = 1;
  a.it_stage = stage;
  int extra = 0;
  if (it) {                                          // item stage A or C on the idle CUs
    const int rc = item_fwd_check(it);
    if (rc != TTMI_OK) return rc;
    a.it = item_args(it);
    TTMI_REQUIRE(stage == 0 || a.it.bncnt != nullptr,
                 "ttmi_user_item_head_fwd_c: stage C here needs the BatchNorm statistics of stage A "
                 "(bn_part / bn_cnt, B <= %d)", BN_MAXBLK * HR);
    a.it_nblk = (it->B + HR - 1) / HR;
    a.it.fin = stage == 3;
    a.it.err = d->id_err;
    extra = stage == 0 ? a.it_nblk * (IN1 / 64) : stage == 2 ? a.it_nblk : a.it_nblk * (IN1 / 64 + 1);
  }
  if (d->ffn_ws && !getenv("TTMI_HEAD_NOSPLIT")) {   // the FFN split over its hidden units
    TTMI_REQUIRE(((uintptr_t)d->ffn_ws & 255) == 0, "ttmi_user_head_fwd: ffn_ws must be 256-byte aligned");
    a.ffn_cnt = static_cast<int*>(d->ffn_ws);
    a.ffn_part = reinterpret_cast<float*>(static_cast<char*>(d->ffn_ws) + ffn_cnt_bytes(d->B));
    const dim3 grid((unsigned)(a.nbu * (d->F / 128) + extra));
    if (d->D == 256) hipLaunchKernelGGL((user_head_fwd_split_kernel<256, 1024>), grid, dim3(512), 0, s, a);
    else if (d->F == 512) hipLaunchKernelGGL((user_head_fwd_split_kernel<128, 512>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((user_head_fwd_split_kernel<128, 256>), grid, dim3(256), 0, s, a);
    return ttmi_check_launch("ttmi_user_head_fwd");
  }
  const dim3 grid((unsigned)(a.nbu + extra));
  if (d->F == 512) hipLaunchKernelGGL(user_head_fwd_kernel<512>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(user_head_fwd_kernel<256>, grid, dim3(256), 0, s, a);
  return ttmi_check_launch("ttmi_user_head_fwd");
}
}  // namespace

extern "C" int ttmi_user_item_head_fwd(const ttmi_user_head_desc* d, const ttmi_item_head_desc* it,
                                       hipStream_t s) {
  return user_item_head_fwd_impl(d, it, 0, s);
}

extern "C" int ttmi_user_item_head_fwd_c(const ttmi_user_head_desc* d, const ttmi_item_head_desc* it,
                                         hipStream_t s) {
  TTMI_REQUIRE(it != nullptr, "ttmi_user_item_head_fwd_c: null item descriptor");
  return user_item_head_fwd_impl(d, it, 2, s);
}

extern "C" int ttmi_user_item_head_fwd_ac(const ttmi_user_head_desc* d, const ttmi_item_head_desc* it,
                                          hipStream_t s) {
  TTMI_REQUIRE(it != nullptr, "ttmi_user_item_head_fwd_ac: null item descriptor");
  return user_item_head_fwd_impl(d, it, 3, s);
}

extern "C" int ttmi_mha_q1_gather_item_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                                           const int64_t* key_valid, const float* x, int32_t* rows,
                                           float* x_rows, float drop_p, const uint64_t* drop_seed,
                                           void* ctx, float* lse, const ttmi_item_head_desc* it,
                                           hipStream_t s) {
  if (it == nullptr || L > 64 || B == 0) {          // separate launches
    if (it) {
      const int rc = ttmi_item_head_fwd_stages(it, 1, s);
      if (rc) return rc;
    }
    return ttmi_mha_q1_gather_fwd(dtype, B, L, H, Dh, qkv, key_valid, x, rows, x_rows, drop_p, drop_seed, ctx,
                                  lse, s);
  }
  int rc = q1_validate("ttmi_mha_q1_gather_item_fwd", dtype, B, L, H, Dh, qkv, drop_p, drop_seed);
  if (rc) return rc;
  TTMI_REQUIRE(qkv && key_valid && x && rows && x_rows && ctx && lse, "ttmi_mha_q1_gather_item_fwd: null argument");
  rc = item_fwd_check(it);
  if (rc) return rc;
  Q1Args q{};
  q.B = B; q.L = L; q.H = H; q.Dh = Dh; q.scale = 1.f / sqrtf((float)Dh);
  q.qkv = qkv; q.kvalid = key_valid; q.rows = rows; q.x = x; q.x_rows = x_rows;
  q.dp = make_drop(drop_p, drop_seed); q.ctx = ctx; q.lse = lse;
  const ItemArgs ia = item_args(it);
  const int it_nblk = (it->B + HR - 1) / HR, nit = it_nblk * (IN1 / 64);
  const dim3 grid((unsigned)(nit + (B * H + 3) / 4));
  if (dtype == TTMI_BF16) hipLaunchKernelGGL(q1_item_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, q, ia, it_nblk, nit);
  else hipLaunchKernelGGL(q1_item_fwd_kernel<float>, grid, dim3(256), 0, s, q, ia, it_nblk, nit);
  return ttmi_check_launch("ttmi_mha_q1_gather_item_fwd");
}

extern "C" int64_t ttmi_user_head_ffn_ws_bytes(int B, int F) {
  if (B <= 0 || F <= 0 || F % 128) return 0;
  return ffn_cnt_bytes(B) + (int64_t)((B + HR - 1) / HR) * (F / 128) * HR * 2 * HD * 4;   // D <= 256
}

extern "C" int ttmi_mha_q1_proj_gather_fwd(int B, int L, int H, int Dh, void* qkv, const int64_t* key_valid,
                                           const void* a_in, const void* wq, const float* bq, const float* x,
                                           int32_t* rows, float* x_rows, float drop_p, const uint64_t* drop_seed,
                                           void* ctx, float* lse, const ttmi_item_head_desc* it, hipStream_t s) {
  static const char* fn = "ttmi_mha_q1_proj_gather_fwd";
  int rc = q1_validate(fn, TTMI_BF16, B, L, H, Dh, qkv, drop_p, drop_seed);
  if (rc) return rc;
  TTMI_REQUIRE(H * Dh == HD && Dh == 32 && L <= 64, "%s: serves bf16, H*Dh = %d with Dh = 32, L <= 64", fn, HD);
  TTMI_REQUIRE(qkv && key_valid && a_in && wq && bq && x && rows && x_rows && ctx && lse, "%s: null argument", fn);
  TTMI_REQUIRE((((uintptr_t)a_in | (uintptr_t)wq) & 15) == 0, "%s: a_in and wq must be 16-byte aligned", fn);
  if (B == 0) return TTMI_OK;
  if (it) {
    rc = item_fwd_check(it);
    if (rc) return rc;
  }
  Q1Args q{};
  q.B = B; q.L = L; q.H = H; q.Dh = Dh; q.scale = 1.f / sqrtf((float)Dh);
  q.qkv = qkv; q.kvalid = key_valid; q.rows = rows; q.x = x; q.x_rows = x_rows;
  q.dp = make_drop(drop_p, drop_seed); q.ctx = ctx; q.lse = lse;
  q.qa = (const bf16_t*)a_in; q.wq = (const bf16_t*)wq; q.bq = bq;
  const ItemArgs ia = it ? item_args(it) : ItemArgs{};
  const int it_nblk = it ? (it->B + HR - 1) / HR : 1, nit = it ? it_nblk * (IN1 / 64) : 0;
  const dim3 grid((unsigned)(nit + (B * H + 3) / 4));
  hipLaunchKernelGGL(q1_item_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, q, ia, it_nblk, nit);
  return ttmi_check_launch(fn);
}

extern "C" int ttmi_user_head_fwd(const ttmi_user_head_desc* d, hipStream_t s) {
  return ttmi_user_item_head_fwd(d, nullptr, s);
}

// (sized for D = 256: the D = 128 layout uses its first half)
extern "C" int64_t ttmi_user_head_bwd_ws_floats(int B) { return (int64_t)((B + HR - 1) / HR) * 4 * 2 * HD; }

extern "C" int ttmi_user_item_head_bwd(const ttmi_user_head_bwd_desc* d, const ttmi_item_head_bwd_desc* it,
                                       hipStream_t s) {
  TTMI_REQUIRE(d != nullptr, "ttmi_user_head_bwd: null descriptor");
  const bool d256 = d->D == 2 * HD && d->F == 8 * HD;
  TTMI_REQUIRE(d->B > 0 && ((d->D == HD && (d->F == 256 || d->F == 512)) || d256) && d->dg == 16 && d->dc == 32,
               "ttmi_user_head_bwd: needs D == %d with F in {256, 512} (or D == %d with F == %d), dg == 16, dc == 32",
               HD, 2 * HD, 8 * HD);
  TTMI_REQUIRE(!d256 || (d->ffn_ws && !getenv("TTMI_HEAD_NOSPLIT")),
               "ttmi_user_head_bwd: D == 256 runs the FFN split only (ffn_ws)");
  TTMI_REQUIRE(!it || it->D == d->D, "ttmi_user_item_head_bwd: the item head's width must be the user head's");
  TTMI_REQUIRE(d->n_genders > 0 && d->n_countries > 0, "ttmi_user_head_bwd: n_genders / n_countries must be > 0");
  TTMI_REQUIRE(d->du && d->az && d->z && d->mz && d->rz && d->h && d->x1 && d->m2 && d->r2 &&
               d->drop_rows && d->gender && d->country && d->wf3t && d->wf0t && d->w2t && d->w1t &&
               d->wot && d->lnw && d->n2w && d->dG && d->dC && d->dz16 && d->dy2 && d->dz1 &&
               d->dx1 && d->dy1 && d->dctx && d->ws, "ttmi_user_head_bwd: null argument");
  HeadBwdArgs a{};
  a.B = d->B; a.F = d->F; a.dg = d->dg; a.dc = d->dc; a.sf = d->ffn_scale;
  a.du = (const bf16_t*)d->du; a.az = (const bf16_t*)d->az; a.z = d->z; a.mz = d->mz; a.rz = d->rz;
  a.h = (const bf16_t*)d->h; a.x1 = d->x1; a.m2 = d->m2; a.r2 = d->r2;
  a.drows = d->drop_rows; a.gender = d->gender; a.country = d->country;
  a.ng = d->n_genders; a.nc = d->n_countries;
  a.wf3t = (const bf16_t*)d->wf3t; a.wf0t = (const bf16_t*)d->wf0t; a.w2t = (const bf16_t*)d->w2t;
  a.w1t = (const bf16_t*)d->w1t; a.wot = (const bf16_t*)d->wot; a.lnw = d->lnw; a.n2w = d->n2w;
  const uint64_t* any = reinterpret_cast<const uint64_t*>(d->lnw);   // read, never used when off
  a.d1 = make_drop(d->d1_p, d->d1_seed ? d->d1_seed : any);
  a.d2 = make_drop(d->d2_p, d->d2_seed ? d->d2_seed : any);
  a.dG = d->dG; a.dC = d->dC;
  a.dz16 = (bf16_t*)d->dz16; a.dy2 = (bf16_t*)d->dy2; a.dz1 = (bf16_t*)d->dz1; a.dx1 = d->dx1;
  a.dy1 = (bf16_t*)d->dy1; a.dctx = (bf16_t*)d->dctx; a.ws = d->ws;
  a.nbu = (d->B + HR - 1) / HR;
  int extra = 0;
  if (it) {                                          // item head rows on the idle CUs
    const int rc = item_bwd_check(it);
    if (rc != TTMI_OK) return rc;
    a.it = item_bwd_args(it);
    extra = (it->B + HR - 1) / HR;
  }
  if (d->ffn_ws && !getenv("TTMI_HEAD_NOSPLIT")) {   // the FFN split over its hidden units
    TTMI_REQUIRE(((uintptr_t)d->ffn_ws & 255) == 0, "ttmi_user_head_bwd: ffn_ws must be 256-byte aligned");
    a.ffn_cnt = static_cast<int*>(d->ffn_ws);
    a.ffn_part = reinterpret_cast<float*>(static_cast<char*>(d->ffn_ws) + ffn_cnt_bytes(d->B));
    const dim3 grid((unsigned)(a.nbu * (d->F / 128) + extra));
    if (d256) hipLaunchKernelGGL((user_head_bwd_split_kernel<256, 1024>), grid, dim3(512), 0, s, a);
    else if (d->F == 512) hipLaunchKernelGGL((user_head_bwd_split_kernel<128, 512>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((user_head_bwd_split_kernel<128, 256>), grid, dim3(256), 0, s, a);
    return ttmi_check_launch("ttmi_user_head_bwd");
  }
  const dim3 grid((unsigned)(a.nbu + extra));
  if (d->F == 512) hipLaunchKernelGGL(user_head_bwd_kernel<512>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(user_head_bwd_kernel<256>, grid, dim3(256), 0, s, a);
  return ttmi_check_launch("ttmi_user_head_bwd");
}

extern "C" int ttmi_user_head_bwd(const ttmi_user_head_bwd_desc* d, hipStream_t s) {
  return ttmi_user_item_head_bwd(d, nullptr, s);
}

TTMI_STAMP_DUMP(head)
