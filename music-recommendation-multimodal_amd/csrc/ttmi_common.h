// ttmi_common.h — shared device helpers for the MI355X (gfx950) two-tower kernels.
//
// * bf16 stored as uint16_t; f32->bf16 is round-to-nearest-even via the __bf16 cast
//   (hipcc emits v_cvt_pk_bf16_f32, which keeps NaN a NaN).
// * Dropout uses a stateless counter hash (restated in oracle/two_tower_ref.py:hash_keep)
//   so forward and backward regenerate the same mask from (seed, flat index).
// * MFMA operands: every kernel stages tiles in LDS as [row][k] with k contiguous and
//   reads 16 bytes per lane at (row = lane&15, byte 16*(lane>>4)) of a 64-byte k-chunk.
//   For bf16 that is exactly the v_mfma_f32_16x16x32_bf16 A/B fragment; for f32 the four
//   floats feed four v_mfma_f32_16x16x4_f32 (k permuted identically on A and B, so the
//   sum is unchanged).  C/D layout (both): col = lane&15, row = 4*(lane>>4) + reg.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <climits>

#include "../../include/ttmi.h"

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

#define TTMI_DEV __device__ __forceinline__

TTMI_DEV float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
TTMI_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
// Two floats to a bf16 pair (a in the low half): the same RNE rounding as f2bf, one
// v_cvt_pk_bf16_f32 (two scalar conversions pack through a shift and an or).
typedef __bf16 ttmi_bf16x2_t __attribute__((ext_vector_type(2)));
typedef float ttmi_f32x2_t __attribute__((ext_vector_type(2)));
TTMI_DEV uint32_t pk_bf2(float a, float b) {
  const ttmi_f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, ttmi_bf16x2_t));
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  static TTMI_DEV float ld(const float* p, int64_t i) { return p[i]; }
  static TTMI_DEV void st(float* p, int64_t i, float v) { p[i] = v; }
};
template <> struct Elem<bf16_t> {
  static TTMI_DEV float ld(const bf16_t* p, int64_t i) { return bf2f(p[i]); }
  static TTMI_DEV void st(bf16_t* p, int64_t i, float v) { p[i] = f2bf(v); }
};
template <typename T> TTMI_DEV float ldf(const T* p, int64_t i) { return Elem<T>::ld(p, i); }
template <typename T> TTMI_DEV void stf(T* p, int64_t i, float v) { Elem<T>::st(p, i, v); }
TTMI_DEV float ld_dyn(const void* p, int64_t i, bool f32) {
  return f32 ? ((const float*)p)[i] : bf2f(((const bf16_t*)p)[i]);
}
TTMI_DEV void st_dyn(void* p, int64_t i, float v, bool f32) {
  if (f32) ((float*)p)[i] = v; else ((bf16_t*)p)[i] = f2bf(v);
}

// ---------------------------------------------------------------- dropout hash
// keep(i) = u16(i) >= thresh16, where one 32-bit hash serves an element pair:
//   h = lowbias32(((i >> 1) + k0) ^ k1),  u16(i) = (i & 1) ? h >> 16 : h & 0xFFFF,
//   thresh16 = floor(p * 65536)  (p resolved to 1/65536).
// Restated in oracle/two_tower_ref.py:hash_keep.  One mixer round per two elements keeps
// the mask off the VALU critical path of the GEMM epilogues it is fused into.
TTMI_DEV uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}
// Host-built descriptor; the 64-bit seed lives in device memory so a captured hipGraph
// replays with fresh masks (the train step rewrites its seed table every step).
struct DropParams {
  const uint64_t* seed;
  uint32_t thresh;   // 16-bit threshold
  float scale;       // 1/(1-p)
  int on;            // p > 0
};
// Device-resolved keys (read the seed once at kernel entry).
struct DropKeys {
  uint32_t k0, k1, thresh;
  float scale;
  int on;
};
TTMI_DEV DropKeys resolve_drop(const DropParams& d) {
  DropKeys k;
  k.on = d.on;
  k.thresh = d.thresh;
  k.scale = d.scale;
  const uint64_t s = d.on ? *d.seed : 0ull;
  k.k0 = (uint32_t)(s & 0xFFFFFFFFull);
  k.k1 = (uint32_t)(s >> 32);
  return k;
}
TTMI_DEV uint32_t drop_hash(const DropKeys& d, uint32_t pair) {
  return lowbias32((pair + d.k0) ^ d.k1);
}
TTMI_DEV bool drop_keep(const DropKeys& d, uint32_t idx) {
  const uint32_t h = drop_hash(d, idx >> 1);
  return ((idx & 1) ? (h >> 16) : (h & 0xFFFFu)) >= d.thresh;
}
TTMI_DEV float drop_apply(const DropKeys& d, uint32_t idx, float v) {
  if (!d.on) return v;
  return drop_keep(d, idx) ? v * d.scale : 0.f;
}
// keep bits of the 4 consecutive indices idx0 .. idx0+3: two pair hashes when idx0 is even
// (identical to drop_keep per index), else one hash per index.
TTMI_DEV void drop_keep4(const DropKeys& d, uint32_t idx0, bool (&kp)[4]) {
  if ((idx0 & 1) == 0) {
    const uint32_t h0 = drop_hash(d, idx0 >> 1), h1 = drop_hash(d, (idx0 >> 1) + 1);
    kp[0] = (h0 & 0xFFFFu) >= d.thresh;
    kp[1] = (h0 >> 16) >= d.thresh;
    kp[2] = (h1 & 0xFFFFu) >= d.thresh;
    kp[3] = (h1 >> 16) >= d.thresh;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) kp[e] = drop_keep(d, idx0 + e);
  }
}
// v[0..NV) at consecutive indices idx0.. (one hash per aligned pair).
template <int NV>
TTMI_DEV void drop_apply_vec(const DropKeys& d, uint32_t idx0, float* v) {
  if (!d.on) return;
  if ((idx0 & 1) == 0) {
#pragma unroll
    for (int e = 0; e < NV; e += 2) {
      const uint32_t h = drop_hash(d, (idx0 + e) >> 1);
      v[e] = (h & 0xFFFFu) >= d.thresh ? v[e] * d.scale : 0.f;
      if (e + 1 < NV) v[e + 1] = (h >> 16) >= d.thresh ? v[e + 1] * d.scale : 0.f;
    }
  } else {
#pragma unroll
    for (int e = 0; e < NV; ++e) v[e] = drop_apply(d, idx0 + e, v[e]);
  }
}
static inline DropParams make_drop(float p, const uint64_t* seed) {
  DropParams d;
  d.seed = seed;
  const double t = (double)p * 65536.0;
  d.thresh = t >= 65535.0 ? 65535u : (uint32_t)t;
  d.on = p > 0.f;
  d.scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  return d;
}

// ---------------------------------------------------------------- long-sequence attention
// ttmi_attn_long.hip: the attention entry points' path for 64 < L <= TTMI_ATTN_LMAX.
int attn_long_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv, const int64_t* kv, DropParams dp,
                  void* ctx, float* lse, hipStream_t s);
int attn_long_bwd(int dtype, int B, int L, int H, int Dh, const void* qkv, const int64_t* kv, const float* lse,
                  const void* dctx, DropParams dp, void* dqkv, hipStream_t s);
int attn_long_q1_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv, const int64_t* kv, int32_t* rows,
                     const float* x, float* x_rows, bool gather, DropParams dp, void* ctx, float* lse,
                     hipStream_t s);
int attn_long_q1_bwd(int dtype, int B, int L, int H, int Dh, const void* qkv, const int64_t* kv,
                     const int32_t* rows, const float* lse, const void* dctx, DropParams dp, void* dqkv,
                     hipStream_t s);

// ---------------------------------------------------------------- deterministic scatter-add
// Sums whose adders arrive in no fixed order (embedding-row scatters, column statistics over
// many workgroups) accumulate in int64 fixed point: integer addition is associative, so the
// total is the same bit pattern whatever the arrival order, and graph replays equal eager
// runs bit for bit.  v is rounded to the nearest multiple of 2^-shift once per adder:
//   TTMI_FX_GRAD (gradient scatters)        2^-36 ≈ 1.5e-11 resolution, |sum| < 2^27 ≈ 1.3e8
//   TTMI_FX_STAT (BatchNorm Σy, Σy²)        2^-24 ≈ 6.0e-8  resolution, |sum| < 2^39 ≈ 5.5e11
// Consumers convert with fx_to_f (through double; exact for |sum| < 2^53 units).
constexpr int TTMI_FX_GRAD = TTMI_FX_GRAD_SHIFT;   // 36 (include/ttmi.h)
constexpr int TTMI_FX_STAT = TTMI_FX_STAT_SHIFT;   // 24
TTMI_DEV long long fx_of(float v, int shift) {
  const float s = __builtin_ldexpf(v, shift);
  return __builtin_llrintf(fminf(fmaxf(s, -9.0e18f), 9.0e18f));
}
TTMI_DEV void fx_add(int64_t* p, float v, int shift) {
  atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)fx_of(v, shift));
}
TTMI_DEV double fx_to_d(int64_t q, int shift) { return __builtin_ldexp((double)q, -shift); }
TTMI_DEV float fx_to_f(int64_t q, int shift) { return (float)fx_to_d(q, shift); }

// ---------------------------------------------------------------- AdamW (torch.optim.AdamW)
// Non-amsgrad, maximize=False.  The scalar terms in double, as torch computes them on the host
// (then used as f32 scalars); shared by adamw_kernel and the fold-fused AdamW (ttmi_gemm.hip) so
// both run the same arithmetic.  hyper = {lr, beta1, beta2, eps, weight_decay}, step = t.
struct AdamScalars { float step_size, bc2_sqrt, decay, b1c, b2, b2c, eps; };
TTMI_DEV AdamScalars adam_scalars(const double* hyper, const int32_t* step) {
  const double lr = hyper[0], b1d = hyper[1], b2d = hyper[2], wd = hyper[4];
  const double tt = (double)step[0];
  AdamScalars a;
  a.step_size = (float)(lr / (1.0 - pow(b1d, tt)));
  a.bc2_sqrt = (float)sqrt(1.0 - pow(b2d, tt));
  a.decay = (float)(1.0 - lr * wd);
  a.b1c = (float)(1.0 - b1d);
  a.b2 = (float)b2d;
  a.b2c = (float)(1.0 - b2d);
  a.eps = (float)hyper[3];
  return a;
}
// Contraction off, fma spelled out: hipcc may contract a*b + c differently in two kernels, and
// adamw_kernel / adamw_fold_kernel (one-process fold-in-update vs the data-parallel plain
// update) must produce the same bits from the same gradient.
TTMI_DEV void adam_upd(const AdamScalars& a, float& P, float G, float& Mv, float& Vv) {
#pragma clang fp contract(off)
  P = P * a.decay;
  Mv = fmaf(a.b1c, G - Mv, Mv);                   // exp_avg.lerp_(grad, 1-beta1)
  Vv = fmaf(Vv, a.b2, a.b2c * (G * G));           // exp_avg_sq.mul_(b2).addcmul_(g,g,1-b2)
  const float denom = sqrtf(Vv) / a.bc2_sqrt + a.eps;
  P = fmaf(-a.step_size, Mv / denom, P);
}

// ---------------------------------------------------------------- XCD-aware block order
// Workgroups are dispatched round-robin over the 8 XCDs (blockIdx % 8).  This bijection of
// [0, n) gives each XCD a contiguous run of logical ids, so neighbouring logical blocks that
// read the same rows share one L2.
TTMI_DEV int xcd_contiguous(int bid, int n) {
  const int xcd = bid & 7, q = n >> 3, rem = n & 7;
  return (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
}

// ---------------------------------------------------------------- wave reductions
TTMI_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// The same sum through the device library's DPP reduction (row shifts within 16 lanes, a row
// mirror, two lane reads): a few cycles a step instead of an LDS-permute round trip.  A
// different (fixed) order than wave_sum: use it where no other kernel must match bit for bit.
extern "C" __device__ float __ockl_wfred_add_f32(float);
TTMI_DEV float wave_sum_dpp(float v) { return __ockl_wfred_add_f32(v); }
TTMI_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// reduce across the 16 lanes that share (lane >> 4) — one MFMA C-row group
TTMI_DEV float group16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
TTMI_DEV float group16_max(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------- MFMA on 16-byte fragments
// acc(16x16 f32) += A_frag · B_frag over one 64-byte k-chunk (32 bf16 or 16 f32).
template <typename T> struct Mma;
template <> struct Mma<bf16_t> {
  static TTMI_DEV void run(f32x4_t& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                  __builtin_bit_cast(bf16x8_t, b), acc, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  static TTMI_DEV void run(f32x4_t& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
  }
};
TTMI_DEV uint4 lds16(const char* p) { return *reinterpret_cast<const uint4*>(p); }

// ---------------------------------------------------------------- LDS-DMA (buffer_load ... lds)
typedef int i32x4_t __attribute__((ext_vector_type(4)));

// Raw buffer descriptor over [base, base + bytes): loads past the end return zero.
TTMI_DEV i32x4_t make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  i32x4_t r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xFFFFu));
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}

// One 16-byte-per-lane LDS-DMA (buffer_load_dwordx4 ... lds): lane l's bytes land at
// lds + 16*l.  Issued from asm so hipcc's waitcnt pass does not see an LDS write it would
// drain with vmcnt(0) before every ds_read; callers count vmcnt themselves.
TTMI_DEV void dma16(const i32x4_t& rs, uint32_t voff, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rs), "s"(__builtin_amdgcn_readfirstlane((int)lds))
               : "memory");
}

TTMI_DEV uint32_t lds_addr(const void* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p);
}


// ---------------------------------------------------------------- phase stamps (diagnostic builds)
// Built with -DTTMI_STAMP (tools/stamp_build.sh; never the shipped library): lane 0 of each
// wave records s_memrealtime (100 MHz) at named phases of an instrumented kernel into
// ttmi_stamps[block][wave][phase]; ttmi_dbg_stamps() copies them out.
constexpr int TTMI_STAMP_BLOCKS = 512, TTMI_STAMP_WAVES = 16, TTMI_STAMP_PHASES = 8;
#ifdef TTMI_STAMP
// one array per translation unit (no relocatable device code); TTMI_STAMP_DUMP(tu) defines
// that unit's host copy-out, extern "C" ttmi_dbg_stamps_<tu>(uint64_t* host, int64_t n)
static __device__ uint64_t ttmi_stamps[TTMI_STAMP_BLOCKS * TTMI_STAMP_WAVES * TTMI_STAMP_PHASES];
#define TTMI_STAMP_DUMP(tu)                                                                    \
  extern "C" int ttmi_dbg_stamps_##tu(uint64_t* host, int64_t n) {                             \
    const int64_t tot = (int64_t)TTMI_STAMP_BLOCKS * TTMI_STAMP_WAVES * TTMI_STAMP_PHASES;      \
    if (!host || n < tot) return TTMI_ERR_ARG;                                                 \
    if (hipDeviceSynchronize() != hipSuccess) return TTMI_ERR_LAUNCH;                           \
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(ttmi_stamps), tot * 8) != hipSuccess) return TTMI_ERR_LAUNCH; \
    static uint64_t zero[TTMI_STAMP_BLOCKS * TTMI_STAMP_WAVES * TTMI_STAMP_PHASES];            \
    return hipMemcpyToSymbol(HIP_SYMBOL(ttmi_stamps), zero, tot * 8) == hipSuccess ? TTMI_OK : TTMI_ERR_LAUNCH; \
  }
#define TTMI_TSTAMP(ph)                                                                        \
  do {                                                                                         \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < TTMI_STAMP_BLOCKS)                             \
      ttmi_stamps[((int)blockIdx.x * TTMI_STAMP_WAVES + (int)(threadIdx.x >> 6)) * TTMI_STAMP_PHASES + (ph)] = \
          __builtin_amdgcn_s_memrealtime();                                                   \
  } while (0)
// an arbitrary per-wave value in the phase slot (e.g. cycles accumulated inside a loop)
#define TTMI_TSTAMP_VAL(ph, v)                                                                 \
  do {                                                                                         \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < TTMI_STAMP_BLOCKS)                             \
      ttmi_stamps[((int)blockIdx.x * TTMI_STAMP_WAVES + (int)(threadIdx.x >> 6)) * TTMI_STAMP_PHASES + (ph)] = \
          (uint64_t)(v);                                                                       \
  } while (0)
#define TTMI_TNOW() __builtin_amdgcn_s_memrealtime()
#else
#define TTMI_TSTAMP(ph) do {} while (0)
#define TTMI_TSTAMP_VAL(ph, v) do {} while (0)
#define TTMI_TNOW() 0ull
#define TTMI_STAMP_DUMP(tu)
#endif

// ---------------------------------------------------------------- embedding-id range (ABI 22)
// nn.Embedding raises on an id outside its table; the device lookups clamp it into [0, n)
// (no out-of-bounds access) and raise flag k of the caller's id_err block (include/ttmi.h
// TTMI_IDERR_*) with plain vector stores: every writer stores the same value, so no atomic is
// needed.  The block is int32 flags[8] in device memory (what AdamW's skip_if reads) followed, at
// byte 32, by an optional pointer to the host-mapped int32[8] the host polls; both get the flag.
// The device flag is stored as the bit pattern of 1.0f (TTMI_IDERR_RAISED): a data-parallel step
// can then sum every rank's flags in its fp32 gradient all-reduce and skip on all ranks at once.
#define TTMI_IDERR_RAISED 0x3F800000
TTMI_DEV void raise_id_err(int32_t* id_err, int k) {
  if (!id_err) return;
  id_err[k] = TTMI_IDERR_RAISED;
  int32_t* host = *reinterpret_cast<int32_t* const*>(id_err + 8);
  if (host) host[k] = 1;
}
TTMI_DEV int64_t clamp_id(int64_t id, int64_t n, int32_t* id_err, int k) {
  const bool bad = (uint64_t)id >= (uint64_t)n;
  if (bad) raise_id_err(id_err, k);
  return bad ? (id < 0 ? 0 : n - 1) : id;
}
// AdamW's bad-step skip (ABI 22): any raised flag of the block's device half.
TTMI_DEV bool id_err_raised(const int32_t* skip_if) {
  if (!skip_if) return false;
  const int4 a = reinterpret_cast<const int4*>(skip_if)[0];
  const int4 b = reinterpret_cast<const int4*>(skip_if)[1];
  return ((a.x | a.y | a.z | a.w) | (b.x | b.y | b.z | b.w)) != 0;
}

// ---------------------------------------------------------------- host-side error plumbing
void ttmi_set_error(const char* fmt, ...);
#define TTMI_REQUIRE(cond, ...)                      \
  do {                                               \
    if (!(cond)) {                                   \
      ttmi_set_error(__VA_ARGS__);                   \
      return TTMI_ERR_ARG;                           \
    }                                                \
  } while (0)
int ttmi_check_launch(const char* what);

// GELU, erf form (torch.nn.functional.gelu default; DeBERTa-v2 hidden_act "gelu"), and its
// derivative GELU'(x) = Phi(x) + x·phi(x).  Phi through erf by Abramowitz-Stegun 7.1.26
// (|error| <= 1.5e-7): erfc(z) = poly(t)·exp(-z²), t = 1 / (1 + p·z), z = |x|/√2, and exp(-z²)
// is also the exponential phi needs — one exp and one rcp per element (libm erff was ~3x the
// VALU in the GEMM epilogues).  Phi = 1 - erfc/2 for x >= 0 and erfc/2 below, so the negative
// tail keeps its relative precision (no 1 - (1 - small)).
TTMI_DEV float gelu_phi_e(float x, float& e) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * z);
  e = __expf(-0.5f * x * x);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f +
                     t * (-1.453152027f + t * 1.061405429f))));
  const float half_erfc = 0.5f * poly * e;
  return x >= 0.f ? 1.f - half_erfc : half_erfc;
}
TTMI_DEV float gelu_erf(float x) {
  float e;
  return x * gelu_phi_e(x, e);
}
TTMI_DEV float gelu_erf_grad(float x) {
  float e;
  const float phi_cdf = gelu_phi_e(x, e);
  return phi_cdf + x * 0.39894228040143268f * e;
}

// 8 bf16 <-> 8 floats (one 16-byte chunk)
TTMI_DEV void unpack8(const uint4& q, float* v) {
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
  }
}
TTMI_DEV uint4 pack8(const float* v) {
  uint4 q;
  q.x = pk_bf2(v[0], v[1]);
  q.y = pk_bf2(v[2], v[3]);
  q.z = pk_bf2(v[4], v[5]);
  q.w = pk_bf2(v[6], v[7]);
  return q;
}

