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
#include "ttmi_q1.h"

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

// The one-query kernels: 4 waves per workgroup, one (sequence, head) per wave (ttmi_q1.h).
// Wave w of block x owns bh = 4x + w; the H heads of a sequence (H <= 4 divides 4) share a
// workgroup, so the 64-byte head slices of the same 768-byte QKV rows meet in one L1.
template <typename T, bool GATHER>
__global__ __launch_bounds__(256) void mha_q1_fwd_kernel(Q1Args a) {
  __shared__ Q1Lds S[4];
  const int w = threadIdx.x >> 6, bh = blockIdx.x * 4 + w;
  if (bh >= a.B * a.H) return;                       // whole wave: wave-level syncs only
  q1_fwd_wave<T, GATHER>(a, bh, S[w]);
}

template <typename T>
__global__ __launch_bounds__(256) void mha_q1_bwd_kernel(Q1Args a) {
  __shared__ Q1Lds S[4];
  const int w = threadIdx.x >> 6, bh = blockIdx.x * 4 + w;
  if (bh >= a.B * a.H) return;
  q1_bwd_wave<T>(a, bh, S[w]);
}

// The one-query backward with the item head's BatchNorm1d backward on the same grid
// (ttmi_mha_q1_bnr_bwd): workgroups [0, nbn) run bnr_bwd_body (4 columns x 64 row groups,
// independent of the attention), the rest the (sequence, head) waves.
constexpr int CO_BN_COLS = 4, CO_BN_RG = 64;
template <typename T, typename TB, int RPT>
__global__ __launch_bounds__(256) void mha_q1_bnr_bwd_kernel(Q1Args a, BnrBwdArgs bn, int nbn) {
  __shared__ union U {
    Q1Lds q[4];
    BnrLds<CO_BN_COLS, CO_BN_RG> b;
  } S;
  if ((int)blockIdx.x < nbn) {
    bnr_bwd_body<TB, CO_BN_COLS, CO_BN_RG, RPT>(bn, blockIdx.x, S.b);
    return;
  }
  const int w = threadIdx.x >> 6, bh = ((int)blockIdx.x - nbn) * 4 + w;
  if (bh >= a.B * a.H) return;
  q1_bwd_wave<T>(a, bh, S.q[w]);
}

// ttmi_mha_q1_kv_bwd (ABI 21; cfg 2: bf16, H = 4, Dh = 32, so workgroup x is sequence x): the
// one-query backward leaving dqkv's Q columns alone, then, from the four heads' dQ_p in LDS,
//   dq_rows[b] = bf16(dQ_p)   (the gathered rows' in_proj Q-row gradient operand)
//   a_rows[b]  = a_in[rows[b]]
//   dyq[b][d]  = Σ_j bf16(dQ_p)[j]·W_q[j][d]   (fp32; W_q = in_proj rows [0, D), read through the
//                transposed mirror wqt = in_projᵀ [D, 3D]: row d is contiguous over j)
// which the LN1-backward panel adds to that row's dY (ttmi_linear_ln_bwd dy_add).
struct Q1Kv {
  const bf16_t* wqt; int64_t ld_wqt;
  const bf16_t* a_in; bf16_t* dq_rows; bf16_t* a_rows; float* dyq;
};
TTMI_DEV void q1_kv_tail(const Q1Args& a, const Q1Kv& k, int b, const float* sdq) {
  constexpr int D = 128;
  const int tid = threadIdx.x;
  __syncthreads();                                   // the four heads' dQ_p are in sdq
  const int64_t r = a.rows[b];
  if (tid < D / 8) {                                 // 16-byte chunks: dq_rows, a_rows
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = sdq[8 * tid + e];
    *reinterpret_cast<uint4*>(k.dq_rows + (int64_t)b * D + 8 * tid) = pack8(v);
    *reinterpret_cast<uint4*>(k.a_rows + (int64_t)b * D + 8 * tid) =
        *reinterpret_cast<const uint4*>(k.a_in + r * D + 8 * tid);
  }
  // dyq: thread (d, half) dots the bf16-rounded dq with 64 of W_q's column d (row d of wqt)
  const int d = tid >> 1, hf = tid & 1;
  const uint4* wr = reinterpret_cast<const uint4*>(k.wqt + (int64_t)d * k.ld_wqt + 64 * hf);
  uint4 wv[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) wv[c] = wr[c];
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const uint32_t wx[4] = {wv[c].x, wv[c].y, wv[c].z, wv[c].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = 64 * hf + 8 * c + 2 * e;
      const float q0 = bf2f(f2bf(sdq[j])), q1 = bf2f(f2bf(sdq[j + 1]));
      acc = fmaf(q0, __uint_as_float(wx[e] << 16), acc);
      acc = fmaf(q1, __uint_as_float(wx[e] & 0xFFFF0000u), acc);
    }
  }
  acc += __shfl_xor(acc, 1, 64);
  if (hf == 0) k.dyq[(int64_t)b * D + d] = acc;
}

template <typename TB, int RPT, bool BN>
__global__ __launch_bounds__(256) void mha_q1_kv_bwd_kernel(Q1Args a, Q1Kv k, BnrBwdArgs bn, int nbn) {
  __shared__ union U {
    Q1Lds q[4];
    BnrLds<CO_BN_COLS, CO_BN_RG> b;
  } S;
  __shared__ float sdq[128];
  if (BN && (int)blockIdx.x < nbn) {
    bnr_bwd_body<TB, CO_BN_COLS, CO_BN_RG, RPT>(bn, blockIdx.x, S.b);
    return;
  }
  const int x = (int)blockIdx.x - (BN ? nbn : 0);
  const int w = threadIdx.x >> 6;
  q1_bwd_wave<bf16_t, true>(a, x * 4 + w, S.q[w], sdq);
  q1_kv_tail(a, k, x, sdq);
}

Q1Args q1_args(int B, int L, int H, int Dh, const void* qkv, const int64_t* kv, int32_t* rows,
               const float* x, float* x_rows, DropParams dp, void* ctx, float* lse, const void* dctx,
               void* dqkv) {
  Q1Args a{};
  a.B = B; a.L = L; a.H = H; a.Dh = Dh; a.scale = 1.f / sqrtf((float)Dh);
  a.qkv = qkv; a.kvalid = kv; a.rows = rows; a.x = x; a.x_rows = x_rows; a.dp = dp;
  a.ctx = ctx; a.lse = lse; a.dctx = dctx; a.dqkv = dqkv;
  return a;
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

// Shared argument check of the one-query entry points.  The dropout element index
// (bh·L + p)·L + j is 32-bit, so B·H·L² < 2^32 is needed only when dropout is on (eval and
// inference encodes, p = 0, take any batch).
int q1_validate(const char* who, int dtype, int B, int L, int H, int Dh, const void* qkv, float drop_p,
                const uint64_t* drop_seed) {
  TTMI_REQUIRE(dtype == TTMI_F32 || dtype == TTMI_BF16, "%s: bad dtype", who);
  TTMI_REQUIRE(B >= 0 && L > 0 && L <= TTMI_ATTN_LMAX && H > 0 && Dh > 0 && Dh <= 64 && Dh % 8 == 0,
               "%s: need L <= %d, Dh <= 64, Dh %% 8 == 0", who, TTMI_ATTN_LMAX);
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || drop_seed), "%s: bad dropout", who);
  TTMI_REQUIRE(drop_p == 0.f || (int64_t)B * H * L * L < (1LL << 32),
               "%s: with dropout on, B*H*L*L must stay below 2^32 (32-bit mask index); "
               "split the batch (B = %d, H = %d, L = %d)", who, B, H, L);
  TTMI_REQUIRE(((uintptr_t)qkv & 15) == 0, "%s: qkv must be 16-byte aligned", who);
  return TTMI_OK;
}

namespace {
template <typename T, bool GATHER>
void q1_fwd_launch(const Q1Args& a, hipStream_t s) {
  hipLaunchKernelGGL((mha_q1_fwd_kernel<T, GATHER>), dim3((a.B * a.H + 3) / 4), dim3(256), 0, s, a);
}
}  // namespace

extern "C" int ttmi_mha_q1_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                               const int64_t* key_valid, const int32_t* rows, float drop_p,
                               const uint64_t* drop_seed, void* ctx, float* lse, hipStream_t s) {
  int rc = q1_validate("ttmi_mha_q1_fwd", dtype, B, L, H, Dh, qkv, drop_p, drop_seed);
  if (rc) return rc;
  TTMI_REQUIRE(qkv && key_valid && rows && ctx && lse, "ttmi_mha_q1_fwd: null argument");
  if (B == 0) return TTMI_OK;
  DropParams dp = make_drop(drop_p, drop_seed);
  int32_t* rw = const_cast<int32_t*>(rows);          // read only (GATHER = false)
  if (L > 64) return attn_long_q1_fwd(dtype, B, L, H, Dh, qkv, key_valid, rw, nullptr, nullptr, false, dp, ctx, lse, s);
  const Q1Args a = q1_args(B, L, H, Dh, qkv, key_valid, rw, nullptr, nullptr, dp, ctx, lse, nullptr, nullptr);
  if (dtype == TTMI_BF16) q1_fwd_launch<bf16_t, false>(a, s);
  else q1_fwd_launch<float, false>(a, s);
  return ttmi_check_launch("ttmi_mha_q1_fwd");
}

extern "C" int ttmi_mha_q1_gather_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                                      const int64_t* key_valid, const float* x, int32_t* rows,
                                      float* x_rows, float drop_p, const uint64_t* drop_seed,
                                      void* ctx, float* lse, hipStream_t s) {
  int rc = q1_validate("ttmi_mha_q1_gather_fwd", dtype, B, L, H, Dh, qkv, drop_p, drop_seed);
  if (rc) return rc;
  TTMI_REQUIRE(qkv && key_valid && x && rows && x_rows && ctx && lse, "ttmi_mha_q1_gather_fwd: null argument");
  if (B == 0) return TTMI_OK;
  DropParams dp = make_drop(drop_p, drop_seed);
  if (L > 64) return attn_long_q1_fwd(dtype, B, L, H, Dh, qkv, key_valid, rows, x, x_rows, true, dp, ctx, lse, s);
  const Q1Args a = q1_args(B, L, H, Dh, qkv, key_valid, rows, x, x_rows, dp, ctx, lse, nullptr, nullptr);
  if (dtype == TTMI_BF16) q1_fwd_launch<bf16_t, true>(a, s);
  else q1_fwd_launch<float, true>(a, s);
  return ttmi_check_launch("ttmi_mha_q1_gather_fwd");
}

extern "C" int ttmi_mha_q1_bwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                               const int64_t* key_valid, const int32_t* rows, const float* lse,
                               const void* dctx, float drop_p, const uint64_t* drop_seed,
                               void* dqkv, hipStream_t s) {
  return ttmi_mha_q1_bnr_bwd(dtype, B, L, H, Dh, qkv, key_valid, rows, lse, dctx, drop_p, drop_seed,
                             dqkv, nullptr, s);
}

extern "C" int ttmi_mha_q1_bnr_bwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                                   const int64_t* key_valid, const int32_t* rows, const float* lse,
                                   const void* dctx, float drop_p, const uint64_t* drop_seed,
                                   void* dqkv, const ttmi_bn_bwd_desc* bn, hipStream_t s) {
  int rc = q1_validate("ttmi_mha_q1_bwd", dtype, B, L, H, Dh, qkv, drop_p, drop_seed);
  if (rc) return rc;
  TTMI_REQUIRE(qkv && key_valid && rows && lse && dctx && dqkv, "ttmi_mha_q1_bwd: null argument");
  TTMI_REQUIRE(((uintptr_t)dqkv & 15) == 0, "ttmi_mha_q1_bwd: dqkv must be 16-byte aligned");
  // the BatchNorm backward rides on the grid when the register path takes its batch
  const int rpt = bn ? (bn->B <= 4 * CO_BN_RG ? 4 : bn->B <= 8 * CO_BN_RG ? 8 : bn->B <= 16 * CO_BN_RG ? 16 : 0) : 0;
  const bool co = bn && rpt && L <= 64 && B > 0;
  if (bn && !co) {
    rc = ttmi_batchnorm_bwd(bn->dtype, bn->B, bn->C, bn->dy, bn->z, bn->w, bn->mean, bn->rstd, bn->y,
                            bn->gate_scale, bn->gated, bn->dz, bn->dw, bn->db, bn->dz16, s);
    if (rc) return rc;
  }
  if (B == 0) return TTMI_OK;
  DropParams dp = make_drop(drop_p, drop_seed);
  if (L > 64) return attn_long_q1_bwd(dtype, B, L, H, Dh, qkv, key_valid, rows, lse, dctx, dp, dqkv, s);
  const Q1Args a = q1_args(B, L, H, Dh, qkv, key_valid, const_cast<int32_t*>(rows), nullptr, nullptr, dp,
                           nullptr, const_cast<float*>(lse), dctx, dqkv);
  const unsigned nq = (unsigned)((B * H + 3) / 4);
  if (!co) {
    if (dtype == TTMI_BF16) hipLaunchKernelGGL(mha_q1_bwd_kernel<bf16_t>, dim3(nq), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(mha_q1_bwd_kernel<float>, dim3(nq), dim3(256), 0, s, a);
    return ttmi_check_launch("ttmi_mha_q1_bwd");
  }
  TTMI_REQUIRE(bn->dtype == TTMI_F32 || bn->dtype == TTMI_BF16, "ttmi_mha_q1_bnr_bwd: bad BatchNorm dtype");
  TTMI_REQUIRE(bn->B > 1 && bn->C > 0 && bn->dy && bn->z && bn->w && bn->mean && bn->rstd && bn->dz &&
                   (!bn->gated || bn->y),
               "ttmi_mha_q1_bnr_bwd: bad BatchNorm descriptor");
  BnrBwdArgs b{};
  b.B = bn->B; b.C = bn->C; b.dy = bn->dy; b.z = bn->z; b.w = bn->w; b.mean = bn->mean; b.rstd = bn->rstd;
  b.y = bn->y; b.gate_scale = bn->gate_scale; b.gated = bn->gated; b.dz = bn->dz; b.dw = bn->dw; b.db = bn->db;
  b.dz16 = (bf16_t*)bn->dz16;
  const int nbn = (bn->C + CO_BN_COLS - 1) / CO_BN_COLS;
  const dim3 grid(nq + (unsigned)nbn);
#define TTMI_Q1BN(T, TB, R) hipLaunchKernelGGL((mha_q1_bnr_bwd_kernel<T, TB, R>), grid, dim3(256), 0, s, a, b, nbn)
#define TTMI_Q1BN_R(T, TB) do { if (rpt == 4) TTMI_Q1BN(T, TB, 4); else if (rpt == 8) TTMI_Q1BN(T, TB, 8); else TTMI_Q1BN(T, TB, 16); } while (0)
  if (dtype == TTMI_BF16) {
    if (bn->dtype == TTMI_BF16) TTMI_Q1BN_R(bf16_t, bf16_t); else TTMI_Q1BN_R(bf16_t, float);
  } else {
    if (bn->dtype == TTMI_BF16) TTMI_Q1BN_R(float, bf16_t); else TTMI_Q1BN_R(float, float);
  }
#undef TTMI_Q1BN_R
#undef TTMI_Q1BN
  return ttmi_check_launch("ttmi_mha_q1_bnr_bwd");
}

extern "C" int ttmi_mha_q1_kv_bwd(const ttmi_q1_kv_bwd_desc* d, hipStream_t s) {
  static const char* fn = "ttmi_mha_q1_kv_bwd";
  TTMI_REQUIRE(d != nullptr, "%s: null descriptor", fn);
  int rc = q1_validate(fn, TTMI_BF16, d->B, d->L, d->H, d->Dh, d->qkv, d->drop_p, d->drop_seed);
  if (rc) return rc;
  TTMI_REQUIRE(d->H == 4 && d->Dh == 32 && d->L <= 64, "%s: serves bf16, H = 4, Dh = 32, L <= 64", fn);
  TTMI_REQUIRE(d->qkv && d->key_valid && d->rows && d->lse && d->dctx && d->dqkv && d->wqt && d->a_in &&
                   d->dq_rows && d->a_rows && d->dyq, "%s: null argument", fn);
  TTMI_REQUIRE((((uintptr_t)d->dqkv | (uintptr_t)d->wqt | (uintptr_t)d->a_in | (uintptr_t)d->dq_rows |
                 (uintptr_t)d->a_rows) & 15) == 0 && d->ld_wqt % 8 == 0 && d->ld_wqt >= 128,
               "%s: operands must be 16-byte aligned", fn);
  const ttmi_bn_bwd_desc* bn = d->bn;
  const int rpt = bn ? (bn->B <= 4 * CO_BN_RG ? 4 : bn->B <= 8 * CO_BN_RG ? 8 : bn->B <= 16 * CO_BN_RG ? 16 : 0) : 0;
  const bool co = bn && rpt && d->B > 0;
  if (bn && !co) {
    rc = ttmi_batchnorm_bwd(bn->dtype, bn->B, bn->C, bn->dy, bn->z, bn->w, bn->mean, bn->rstd, bn->y,
                            bn->gate_scale, bn->gated, bn->dz, bn->dw, bn->db, bn->dz16, s);
    if (rc) return rc;
  }
  if (d->B == 0) return TTMI_OK;
  const Q1Args a = q1_args(d->B, d->L, d->H, d->Dh, d->qkv, d->key_valid, const_cast<int32_t*>(d->rows), nullptr,
                           nullptr, make_drop(d->drop_p, d->drop_seed), nullptr, const_cast<float*>(d->lse),
                           d->dctx, d->dqkv);
  Q1Kv k{(const bf16_t*)d->wqt, d->ld_wqt, (const bf16_t*)d->a_in, (bf16_t*)d->dq_rows, (bf16_t*)d->a_rows, d->dyq};
  if (!co) {
    hipLaunchKernelGGL((mha_q1_kv_bwd_kernel<float, 4, false>), dim3(d->B), dim3(256), 0, s, a, k, BnrBwdArgs{}, 0);
    return ttmi_check_launch(fn);
  }
  TTMI_REQUIRE(bn->dtype == TTMI_F32 || bn->dtype == TTMI_BF16, "%s: bad BatchNorm dtype", fn);
  TTMI_REQUIRE(bn->B > 1 && bn->C > 0 && bn->dy && bn->z && bn->w && bn->mean && bn->rstd && bn->dz &&
                   (!bn->gated || bn->y), "%s: bad BatchNorm descriptor", fn);
  BnrBwdArgs b{};
  b.B = bn->B; b.C = bn->C; b.dy = bn->dy; b.z = bn->z; b.w = bn->w; b.mean = bn->mean; b.rstd = bn->rstd;
  b.y = bn->y; b.gate_scale = bn->gate_scale; b.gated = bn->gated; b.dz = bn->dz; b.dw = bn->dw; b.db = bn->db;
  b.dz16 = (bf16_t*)bn->dz16;
  const int nbn = (bn->C + CO_BN_COLS - 1) / CO_BN_COLS;
  const dim3 grid((unsigned)d->B + (unsigned)nbn);
#define TTMI_Q1KV(TB, R) hipLaunchKernelGGL((mha_q1_kv_bwd_kernel<TB, R, true>), grid, dim3(256), 0, s, a, k, b, nbn)
#define TTMI_Q1KV_R(TB) do { if (rpt == 4) TTMI_Q1KV(TB, 4); else if (rpt == 8) TTMI_Q1KV(TB, 8); else TTMI_Q1KV(TB, 16); } while (0)
  if (bn->dtype == TTMI_BF16) TTMI_Q1KV_R(bf16_t); else TTMI_Q1KV_R(float);
#undef TTMI_Q1KV_R
#undef TTMI_Q1KV
  return ttmi_check_launch(fn);
}
