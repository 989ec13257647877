// ttmi_attn_generic.hip — SASRec self-attention for the shapes the tuned kernels do not serve
// (ABI 22): head widths above 64 or not a multiple of 8, histories longer than TTMI_ATTN_LMAX.
//
// Reference: nn.MultiheadAttention inside TransformerEncoderLayer(norm_first=True), the merged
// causal + key-padding mask, a query row with no allowed key yielding 0 (user_tower.py:37-45,
// 100-116; torch's math SDPA _safe_softmax), dropout on the probabilities at the flat index
// ((b·H + h)·L + i)·L + j (the mask ttmi_mha_fwd draws).  Correctness-first: one wave per query
// row (forward, query-side backward) or key row (key-side backward), the head width spread over
// the lanes (Dh <= 64·NV), every dot product a wave reduction, nothing staged in LDS, so any L
// and any Dh up to 512 run.  The tuned kernels (ttmi_attn.hip, ttmi_attn_long.hip) cover the
// reference's configurations; this path exists so a model the reference accepts is not refused.
//
//   forward:   ctx_i = Σ_j P_ij·κ_ij·V_j,  P_ij = softmax_j(q_i·k_j / √Dh),  lse_i = m + ln Σ e^(s-m)
//   backward:  D_i = dO_i·O_i (O the stored ctx rows), dS_ij = P_ij (κ_ij dO_i·V_j − D_i),
//              dQ_i = Σ_j dS_ij K_j / √Dh,  dK_j = Σ_i dS_ij Q_i / √Dh,  dV_j = Σ_i P_ij κ_ij dO_i
// with κ the dropout keep factor (0 or 1/(1-p)).  dQ and dK / dV come from separate launches (a
// query row, then a key row, per wave), so every sum runs in one fixed order: deterministic.
#include "ttmi_common.h"

namespace {

struct GaArgs {
  int B, L, H, Dh;
  const void* qkv; const int64_t* kv;
  float scale;
  DropParams drop;
  void* ctx; float* lse;
  const void* dctx; float* dsum; void* dqkv;
};

TTMI_DEV float ga_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// the row's Dh values held as lane + 64 k (k < NV), zero past Dh
template <typename T, int NV>
TTMI_DEV void ga_load(const T* row, int Dh, int lane, float (&v)[NV]) {
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int d = lane + 64 * k;
    v[k] = d < Dh ? ldf<T>(row, d) : 0.f;
  }
}
template <typename T, int NV>
TTMI_DEV float ga_dot(const T* row, int Dh, int lane, const float (&v)[NV]) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int d = lane + 64 * k;
    if (d < Dh) s += v[k] * ldf<T>(row, d);
  }
  return ga_wave_sum(s);
}
TTMI_DEV float ga_keep(const DropKeys& dk, uint32_t idx) {
  return dk.on ? (drop_keep(dk, idx) ? dk.scale : 0.f) : 1.f;
}

// One wave per (b, h, i).
template <typename T, int NV>
__global__ __launch_bounds__(256) void ga_fwd_kernel(GaArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= (int64_t)a.B * a.H * a.L) return;
  const int L = a.L, H = a.H, Dh = a.Dh, D = H * Dh;
  const int i = (int)(w % L);
  const int64_t bh = w / L;
  const int h = (int)(bh % H), b = (int)(bh / H);
  const int64_t ld = 3 * (int64_t)D;
  const T* qkv = static_cast<const T*>(a.qkv);
  const T* base = qkv + (int64_t)b * L * ld + h * Dh;
  const int64_t* kv = a.kv + (int64_t)b * L;
  const DropKeys dk = resolve_drop(a.drop);
  float q[NV];
  ga_load<T, NV>(base + (int64_t)i * ld, Dh, lane, q);
  float m = -INFINITY, l = 0.f;
  for (int j = 0; j <= i; ++j) {
    if (kv[j] == 0) continue;                            // (wave-uniform)
    const float s = ga_dot<T, NV>(base + (int64_t)j * ld + D, Dh, lane, q) * a.scale;
    if (s > m) { l = l * expf(m - s) + 1.f; m = s; }
    else l += expf(s - m);
  }
  T* out = static_cast<T*>(a.ctx) + ((int64_t)b * L + i) * D + h * Dh;
  float acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.f;
  if (m != -INFINITY) {
    const float inv = 1.f / l;
    const uint32_t row0 = (uint32_t)w * (uint32_t)L;     // dropout index of (b, h, i, 0)
    for (int j = 0; j <= i; ++j) {
      if (kv[j] == 0) continue;
      const float s = ga_dot<T, NV>(base + (int64_t)j * ld + D, Dh, lane, q) * a.scale;
      const float p = expf(s - m) * inv * ga_keep(dk, row0 + (uint32_t)j);
      const T* vr = base + (int64_t)j * ld + 2 * D;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int d = lane + 64 * k;
        if (d < Dh) acc[k] += p * ldf<T>(vr, d);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int d = lane + 64 * k;
    if (d < Dh) stf<T>(out, d, acc[k]);
  }
  // a row with no allowed key: output 0, lse +inf (its probabilities read as 0 in the backward)
  if (lane == 0) a.lse[w] = m == -INFINITY ? INFINITY : m + logf(l);
}

// Query side of the backward, one wave per (b, h, i): D_i, then dQ_i.
template <typename T, int NV>
__global__ __launch_bounds__(256) void ga_bwd_q_kernel(GaArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= (int64_t)a.B * a.H * a.L) return;
  const int L = a.L, H = a.H, Dh = a.Dh, D = H * Dh;
  const int i = (int)(w % L);
  const int64_t bh = w / L;
  const int h = (int)(bh % H), b = (int)(bh / H);
  const int64_t ld = 3 * (int64_t)D;
  const T* base = static_cast<const T*>(a.qkv) + (int64_t)b * L * ld + h * Dh;
  const int64_t* kv = a.kv + (int64_t)b * L;
  const int64_t orow = ((int64_t)b * L + i) * D + h * Dh;
  const DropKeys dk = resolve_drop(a.drop);
  float q[NV], dO[NV], o[NV];
  ga_load<T, NV>(base + (int64_t)i * ld, Dh, lane, q);
  ga_load<T, NV>(static_cast<const T*>(a.dctx) + orow, Dh, lane, dO);
  ga_load<T, NV>(static_cast<const T*>(a.ctx) + orow, Dh, lane, o);
  float dsum = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) dsum += dO[k] * o[k];
  dsum = ga_wave_sum(dsum);
  const float lse = a.lse[w];
  float dq[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) dq[k] = 0.f;
  if (lse != INFINITY) {
    const uint32_t row0 = (uint32_t)w * (uint32_t)L;
    for (int j = 0; j <= i; ++j) {
      if (kv[j] == 0) continue;
      const T* kr = base + (int64_t)j * ld + D;
      const float s = ga_dot<T, NV>(kr, Dh, lane, q) * a.scale;
      const float dp = ga_dot<T, NV>(base + (int64_t)j * ld + 2 * D, Dh, lane, dO);
      const float p = expf(s - lse);
      const float ds = p * (ga_keep(dk, row0 + (uint32_t)j) * dp - dsum);
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int d = lane + 64 * k;
        if (d < Dh) dq[k] += ds * ldf<T>(kr, d);
      }
    }
  }
  T* dst = static_cast<T*>(a.dqkv) + ((int64_t)b * L + i) * ld + h * Dh;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int d = lane + 64 * k;
    if (d < Dh) stf<T>(dst, d, dq[k] * a.scale);
  }
  if (lane == 0) a.dsum[w] = lse != INFINITY ? dsum : 0.f;
}

// Key side of the backward, one wave per (b, h, j): dK_j, dV_j over the queries i >= j.
template <typename T, int NV>
__global__ __launch_bounds__(256) void ga_bwd_kv_kernel(GaArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= (int64_t)a.B * a.H * a.L) return;
  const int L = a.L, H = a.H, Dh = a.Dh, D = H * Dh;
  const int j = (int)(w % L);
  const int64_t bh = w / L;
  const int h = (int)(bh % H), b = (int)(bh / H);
  const int64_t ld = 3 * (int64_t)D;
  const T* base = static_cast<const T*>(a.qkv) + (int64_t)b * L * ld + h * Dh;
  const T* dctx = static_cast<const T*>(a.dctx) + (int64_t)b * L * D + h * Dh;
  const DropKeys dk = resolve_drop(a.drop);
  float kk[NV], vv[NV], dK[NV], dV[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) dK[k] = dV[k] = 0.f;
  if (a.kv[(int64_t)b * L + j] != 0) {                   // a masked key: every probability 0
    ga_load<T, NV>(base + (int64_t)j * ld + D, Dh, lane, kk);
    ga_load<T, NV>(base + (int64_t)j * ld + 2 * D, Dh, lane, vv);
    for (int i = j; i < L; ++i) {                       // row i has key j allowed: finite lse
      const T* qr = base + (int64_t)i * ld;
      const T* dor = dctx + (int64_t)i * D;
      const float s = ga_dot<T, NV>(qr, Dh, lane, kk) * a.scale;
      const float dp = ga_dot<T, NV>(dor, Dh, lane, vv);
      const int64_t wi = bh * L + i;
      const float p = expf(s - a.lse[wi]);
      const float kap = ga_keep(dk, (uint32_t)wi * (uint32_t)L + (uint32_t)j);
      const float ds = p * (kap * dp - a.dsum[wi]);
      const float pk = p * kap;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int d = lane + 64 * k;
        if (d < Dh) {
          dK[k] += ds * ldf<T>(qr, d);
          dV[k] += pk * ldf<T>(dor, d);
        }
      }
    }
  }
  T* dst = static_cast<T*>(a.dqkv) + ((int64_t)b * L + j) * ld + h * Dh;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int d = lane + 64 * k;
    if (d < Dh) {
      stf<T>(dst + D, d, dK[k] * a.scale);
      stf<T>(dst + 2 * D, d, dV[k]);
    }
  }
}

int ga_check(const char* fn, int dtype, int B, int L, int H, int Dh, const void* qkv, const int64_t* kv,
             float drop_p) {
  TTMI_REQUIRE(dtype == TTMI_F32 || dtype == TTMI_BF16, "%s: bad dtype", fn);
  TTMI_REQUIRE(B >= 0 && L > 0 && H > 0 && Dh > 0 && Dh <= 512, "%s: need L > 0, H > 0, 0 < Dh <= 512", fn);
  TTMI_REQUIRE(qkv && kv, "%s: null argument", fn);
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "%s: drop_p out of [0,1)", fn);
  TTMI_REQUIRE(drop_p == 0.f || (int64_t)B * H * L * L < (1LL << 32),
               "%s: with dropout on, B*H*L*L must stay below 2^32 (32-bit mask index); split the batch", fn);
  TTMI_REQUIRE((int64_t)B * H * L < (1LL << 31) / 4 * 4, "%s: too many rows", fn);
  return TTMI_OK;
}

}  // namespace

extern "C" int ttmi_mha_generic_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                                    const int64_t* key_valid, float drop_p, const uint64_t* drop_seed,
                                    void* ctx, float* lse, hipStream_t s) {
  static const char* fn = "ttmi_mha_generic_fwd";
  int rc = ga_check(fn, dtype, B, L, H, Dh, qkv, key_valid, drop_p);
  if (rc) return rc;
  TTMI_REQUIRE(ctx && lse, "%s: null output", fn);
  if (B == 0) return TTMI_OK;
  GaArgs a{};
  a.B = B; a.L = L; a.H = H; a.Dh = Dh; a.qkv = qkv; a.kv = key_valid;
  a.scale = 1.f / sqrtf((float)Dh); a.drop = make_drop(drop_p, drop_seed);
  a.ctx = ctx; a.lse = lse;
  const dim3 grid((unsigned)(((int64_t)B * H * L + 3) / 4));
#define TTMI_GA(T, NV) hipLaunchKernelGGL((ga_fwd_kernel<T, NV>), grid, dim3(256), 0, s, a)
#define TTMI_GA_NV(T) do { if (Dh <= 64) TTMI_GA(T, 1); else if (Dh <= 128) TTMI_GA(T, 2); \
                           else if (Dh <= 256) TTMI_GA(T, 4); else TTMI_GA(T, 8); } while (0)
  if (dtype == TTMI_BF16) TTMI_GA_NV(bf16_t);
  else TTMI_GA_NV(float);
#undef TTMI_GA_NV
#undef TTMI_GA
  return ttmi_check_launch(fn);
}

extern "C" int ttmi_mha_generic_bwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                                    const int64_t* key_valid, const float* lse, const void* ctx,
                                    const void* dctx, float drop_p, const uint64_t* drop_seed, float* dsum_ws,
                                    void* dqkv, hipStream_t s) {
  static const char* fn = "ttmi_mha_generic_bwd";
  int rc = ga_check(fn, dtype, B, L, H, Dh, qkv, key_valid, drop_p);
  if (rc) return rc;
  TTMI_REQUIRE(lse && ctx && dctx && dsum_ws && dqkv, "%s: null argument", fn);
  if (B == 0) return TTMI_OK;
  GaArgs a{};
  a.B = B; a.L = L; a.H = H; a.Dh = Dh; a.qkv = qkv; a.kv = key_valid;
  a.scale = 1.f / sqrtf((float)Dh); a.drop = make_drop(drop_p, drop_seed);
  a.ctx = const_cast<void*>(ctx); a.lse = const_cast<float*>(lse);
  a.dctx = dctx; a.dsum = dsum_ws; a.dqkv = dqkv;
  const dim3 grid((unsigned)(((int64_t)B * H * L + 3) / 4));
#define TTMI_GB(KN, T, NV) hipLaunchKernelGGL((KN<T, NV>), grid, dim3(256), 0, s, a)
#define TTMI_GB_NV(KN, T) do { if (Dh <= 64) TTMI_GB(KN, T, 1); else if (Dh <= 128) TTMI_GB(KN, T, 2); \
                               else if (Dh <= 256) TTMI_GB(KN, T, 4); else TTMI_GB(KN, T, 8); } while (0)
  if (dtype == TTMI_BF16) TTMI_GB_NV(ga_bwd_q_kernel, bf16_t);
  else TTMI_GB_NV(ga_bwd_q_kernel, float);
  rc = ttmi_check_launch(fn);
  if (rc) return rc;
  if (dtype == TTMI_BF16) TTMI_GB_NV(ga_bwd_kv_kernel, bf16_t);
  else TTMI_GB_NV(ga_bwd_kv_kernel, float);
#undef TTMI_GB_NV
#undef TTMI_GB
  return ttmi_check_launch(fn);
}
