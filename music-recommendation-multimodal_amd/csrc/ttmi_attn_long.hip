// ttmi_attn_long.hip — the SASRec causal self-attention (reference user_tower.py:111-116) for
// sequences longer than one 64-row tile: 64 < L <= TTMI_ATTN_LMAX.  ttmi_attn.hip / ttmi_rows.hip
// keep a whole sequence in one wave's LDS image and take L <= 64 (the benchmarked L = 50); the
// reference accepts any max_seq_len, so longer histories run here, tiled over 64-key blocks.
//
// Same contract as the short kernels, bit for bit where it is observable: qkv [B, L, 3D],
// key_valid [B, L], causal + key padding, lse[bh·L + r] = m + ln Σ (INFINITY for a fully masked
// row), dropout on the normalised probabilities with element index bh·L·L + r·L + c.
//  * forward: one 256-thread workgroup per (sequence, head, 64-query block); online softmax
//    over the key blocks up to the diagonal; a thread owns (query row, a quarter of the keys /
//    head columns), rows reduce over 4 adjacent lanes;
//  * backward: one workgroup per (sequence, head): per query block D_r = Σ_c p·dP (recomputed,
//    no workspace) and dQ; then per key block dK, dV over the query blocks at or below it;
//  * one-query variants for the pruned last layer (the last valid row only), keys strided
//    over 256 threads.
// Operand tiles are fp32 [64][65] LDS images (odd pitch: the column walks are conflict-free);
// the products are VALU FMAs — this is the long-sequence fallback, not the benchmarked path.
#include "ttmi_common.h"

namespace {

constexpr int LB = 64, PT = 65;
constexpr int LMAX = TTMI_ATTN_LMAX;

// rows r0 .. r0+63 of a head slice (row stride ld elements, Dh columns) -> dst[r][d], zero-padded
template <typename T>
TTMI_DEV void lt_load(float* dst, const T* __restrict__ src, int64_t ld, int r0, int L, int Dh, int tid) {
  for (int i = tid; i < LB * 64; i += 256) {
    const int r = i >> 6, d = i & 63;
    float v = 0.f;
    if (r0 + r < L && d < Dh) v = ldf<T>(src, (int64_t)(r0 + r) * ld + d);
    dst[r * PT + d] = v;
  }
}

// s[k] = Σ_d A[row][d] · B[kq + 4k][d], k < 16
TTMI_DEV void lt_dots(const float* A, const float* Bm, int row, int kq, int Dh, float* s) {
#pragma unroll
  for (int k = 0; k < 16; ++k) s[k] = 0.f;
  for (int d = 0; d < Dh; ++d) {
    const float a = A[row * PT + d];
#pragma unroll
    for (int k = 0; k < 16; ++k) s[k] += a * Bm[(kq + 4 * k) * PT + d];
  }
}

TTMI_DEV float quad_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 1, 64));
  return fmaxf(v, __shfl_xor(v, 2, 64));
}
TTMI_DEV float quad_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  return v + __shfl_xor(v, 2, 64);
}

template <typename T>
__global__ __launch_bounds__(256) void mha_long_fwd_kernel(int L, int H, int Dh, const T* __restrict__ qkv,
                                                           const int64_t* __restrict__ kvalid, DropParams dp,
                                                           T* __restrict__ ctx, float* __restrict__ lse,
                                                           float scale) {
  __shared__ float sQ[LB * PT], sK[LB * PT], sV[LB * PT], sP[LB * PT], sKv[LB];
  const int tid = threadIdx.x, row = tid >> 2, kq = tid & 3;
  const int bh = blockIdx.x, qb = blockIdx.y, b = bh / H, h = bh % H;
  const int D = H * Dh;
  const int64_t ld = 3LL * D;
  const T* base = qkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  const int q0 = qb * LB, r = q0 + row;
  lt_load<T>(sQ, base, ld, q0, L, Dh, tid);
  const DropKeys dk = resolve_drop(dp);
  const uint32_t pbase = (uint32_t)((int64_t)bh * L * L);
  float m = -INFINITY, sum = 0.f, o[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) o[i] = 0.f;
  for (int kb = 0; kb <= qb; ++kb) {                  // causal: key blocks up to the diagonal
    const int k0 = kb * LB;
    __syncthreads();                                  // the previous block's tiles are consumed
    lt_load<T>(sK, base + D, ld, k0, L, Dh, tid);
    lt_load<T>(sV, base + 2 * D, ld, k0, L, Dh, tid);
    if (tid < LB) sKv[tid] = (k0 + tid < L && kvalid[(int64_t)b * L + k0 + tid] != 0) ? 1.f : 0.f;
    __syncthreads();
    float s[16];
    lt_dots(sQ, sK, row, kq, Dh, s);
    float bm = -INFINITY;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int cl = kq + 4 * k, c = k0 + cl;
      const bool ok = r < L && c <= r && sKv[cl] > 0.f;
      s[k] = ok ? s[k] * scale : -INFINITY;
      bm = fmaxf(bm, s[k]);
    }
    bm = quad_max(bm);
    const float mn = fmaxf(m, bm);
    const float alpha = m == -INFINITY ? 0.f : expf(m - mn);
    float ls = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int cl = kq + 4 * k;
      const float p = s[k] == -INFINITY ? 0.f : expf(s[k] - mn);
      ls += p;
      sP[row * PT + cl] = (dk.on && p != 0.f) ? drop_apply(dk, pbase + (uint32_t)(r * L + k0 + cl), p) : p;
    }
    sum = sum * alpha + quad_sum(ls);
#pragma unroll
    for (int i = 0; i < 16; ++i) o[i] *= alpha;
    m = mn;
    __syncthreads();
    for (int c = 0; c < LB; ++c) {
      const float pc = sP[row * PT + c];
#pragma unroll
      for (int i = 0; i < 16; ++i) o[i] += pc * sV[c * PT + kq + 4 * i];
    }
  }
  if (r < L) {
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
    T* dst = ctx + ((int64_t)b * L + r) * D + (int64_t)h * Dh;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (kq + 4 * i < Dh) stf<T>(dst, kq + 4 * i, o[i] * inv);
    if (kq == 0) lse[(int64_t)bh * L + r] = m == -INFINITY ? INFINITY : m + logf(sum);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void mha_long_bwd_kernel(int L, int H, int Dh, const T* __restrict__ qkv,
                                                           const int64_t* __restrict__ kvalid,
                                                           const float* __restrict__ lse,
                                                           const T* __restrict__ dctx, DropParams dp,
                                                           T* __restrict__ dqkv, float scale) {
  __shared__ float sQ[LB * PT], sO[LB * PT], sK[LB * PT], sV[LB * PT], sS[LB * PT], sU[LB * PT];
  __shared__ float sD[LMAX], sL[LMAX], sKv[LMAX];
  const int tid = threadIdx.x, me = tid >> 2, qq = tid & 3;
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int D = H * Dh;
  const int64_t ld = 3LL * D;
  const T* base = qkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  const T* dob = dctx + (int64_t)b * L * D + (int64_t)h * Dh;
  T* gq = dqkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  const int nb = (L + LB - 1) / LB;
  for (int i = tid; i < L; i += 256) {
    sKv[i] = kvalid[(int64_t)b * L + i] != 0 ? 1.f : 0.f;
    sL[i] = lse[(int64_t)bh * L + i];
  }
  const DropKeys dk = resolve_drop(dp);
  const uint32_t pbase = (uint32_t)((int64_t)bh * L * L);
  // p, dP of score (r, c) from the dots s = q_r·k_c and dpd = dO_r·v_c
  auto probs = [&](int r, int c, float s, float dpd, float& p, float& dP, float& ks) {
    const bool ok = r < L && c < L && c <= r && sKv[c] > 0.f;
    p = ok ? expf(s * scale - sL[r]) : 0.f;
    ks = 1.f;
    if (dk.on && ok) ks = drop_keep(dk, pbase + (uint32_t)(r * L + c)) ? dk.scale : 0.f;
    dP = ok ? dpd * ks : 0.f;
  };
  // ---- per query block: D_r = Σ_c p·dP, then dQ_r = Σ_c dS_rc k_c
  for (int qb = 0; qb < nb; ++qb) {
    const int q0 = qb * LB, r = q0 + me;
    __syncthreads();
    lt_load<T>(sQ, base, ld, q0, L, Dh, tid);
    lt_load<T>(sO, dob, D, q0, L, Dh, tid);
    __syncthreads();
    float dpart = 0.f;
    for (int kb = 0; kb <= qb; ++kb) {
      const int k0 = kb * LB;
      __syncthreads();
      lt_load<T>(sK, base + D, ld, k0, L, Dh, tid);
      lt_load<T>(sV, base + 2 * D, ld, k0, L, Dh, tid);
      __syncthreads();
      float s[16], dpd[16];
      lt_dots(sQ, sK, me, qq, Dh, s);
      lt_dots(sO, sV, me, qq, Dh, dpd);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        float p, dP, ks;
        probs(r, k0 + qq + 4 * k, s[k], dpd[k], p, dP, ks);
        dpart += p * dP;
      }
    }
    const float Dr = quad_sum(dpart);
    if (qq == 0 && r < L) sD[r] = Dr;
    float dq[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[i] = 0.f;
    for (int kb = 0; kb <= qb; ++kb) {
      const int k0 = kb * LB;
      __syncthreads();
      lt_load<T>(sK, base + D, ld, k0, L, Dh, tid);
      lt_load<T>(sV, base + 2 * D, ld, k0, L, Dh, tid);
      __syncthreads();
      float s[16], dpd[16];
      lt_dots(sQ, sK, me, qq, Dh, s);
      lt_dots(sO, sV, me, qq, Dh, dpd);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        float p, dP, ks;
        probs(r, k0 + qq + 4 * k, s[k], dpd[k], p, dP, ks);
        sS[me * PT + qq + 4 * k] = p * (dP - Dr) * scale;
      }
      __syncthreads();
      for (int c = 0; c < LB; ++c) {
        const float ds = sS[me * PT + c];
#pragma unroll
        for (int i = 0; i < 16; ++i) dq[i] += ds * sK[c * PT + qq + 4 * i];
      }
    }
    if (r < L) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (qq + 4 * i < Dh) stf<T>(gq, (int64_t)r * ld + qq + 4 * i, dq[i]);
    }
  }
  // ---- per key block: dK_c = Σ_r dS_rc q_r, dV_c = Σ_r Pd_rc dO_r over the query blocks >= it
  for (int kb = 0; kb < nb; ++kb) {
    const int k0 = kb * LB, c = k0 + me;
    __syncthreads();
    lt_load<T>(sK, base + D, ld, k0, L, Dh, tid);
    lt_load<T>(sV, base + 2 * D, ld, k0, L, Dh, tid);
    float dkk[16], dvv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) dkk[i] = dvv[i] = 0.f;
    for (int qb = kb; qb < nb; ++qb) {
      const int q0 = qb * LB;
      __syncthreads();
      lt_load<T>(sQ, base, ld, q0, L, Dh, tid);
      lt_load<T>(sO, dob, D, q0, L, Dh, tid);
      __syncthreads();
      float s[16], dpd[16];
      lt_dots(sK, sQ, me, qq, Dh, s);                 // s[k] = k_c · q_{q0 + qq + 4k}
      lt_dots(sV, sO, me, qq, Dh, dpd);               // dpd[k] = v_c · dO_{q0 + qq + 4k}
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int rl = qq + 4 * k, r = q0 + rl;
        float p, dP, ks;
        probs(r, c, s[k], dpd[k], p, dP, ks);
        sS[me * PT + rl] = r < L ? p * (dP - sD[r]) * scale : 0.f;
        sU[me * PT + rl] = p * ks;
      }
      __syncthreads();
      for (int rl = 0; rl < LB; ++rl) {
        const float ds = sS[me * PT + rl], pd = sU[me * PT + rl];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          dkk[i] += ds * sQ[rl * PT + qq + 4 * i];
          dvv[i] += pd * sO[rl * PT + qq + 4 * i];
        }
      }
    }
    if (c < L) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (qq + 4 * i < Dh) {
          stf<T>(gq + D, (int64_t)c * ld + qq + 4 * i, dkk[i]);
          stf<T>(gq + 2 * D, (int64_t)c * ld + qq + 4 * i, dvv[i]);
        }
    }
  }
}

// ---------------------------------------------------------------- one query row (pruned layer)
// 256 threads per (sequence, head); keys c = tid + 256·t.  GATHER as mha_q1_fwd_kernel: the
// workgroup finds its sequence's last valid row and the head-0 workgroup writes rows[b] and
// x_rows[b] = x[rows[b]].
TTMI_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}
TTMI_DEV float block_max(float v, float* red) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}
template <typename T>
TTMI_DEV float row_dot(const float* q, const T* __restrict__ k, int Dh) {
  float s = 0.f;
  for (int d = 0; d < Dh; ++d) s += q[d] * ldf<T>(k, d);
  return s;
}
// out[d] (d = tid & 63 < Dh) = Σ_{c < n} coef[c] · rows[c][d]: four key phases, LDS combine
template <typename T>
TTMI_DEV float q1_combine(const float* coef, const T* __restrict__ rows, int64_t ld, int n, int Dh,
                          float* red4) {
  const int d = threadIdx.x & 63, g = threadIdx.x >> 6;
  float a = 0.f;
  if (d < Dh)
    for (int c = g; c < n; c += 4) a += coef[c] * ldf<T>(rows, (int64_t)c * ld + d);
  red4[g * 64 + d] = a;
  __syncthreads();
  return red4[d] + red4[64 + d] + red4[128 + d] + red4[192 + d];
}

template <typename T, bool GATHER>
__global__ __launch_bounds__(256) void mha_long_q1_fwd_kernel(int L, int H, int Dh, const T* __restrict__ qkv,
                                                              const int64_t* __restrict__ kvalid,
                                                              int32_t* __restrict__ rows,
                                                              const float* __restrict__ x,
                                                              float* __restrict__ x_rows, DropParams dp,
                                                              T* __restrict__ ctx, float* __restrict__ lse,
                                                              float scale) {
  __shared__ float sq[64], sp[LMAX], red[4], red4[256];
  const int tid = threadIdx.x;
  const int bh = xcd_contiguous(blockIdx.x, gridDim.x), b = bh / H, h = bh % H;
  const int D = H * Dh;
  const int64_t ld = 3LL * D;
  int64_t r;
  if constexpr (GATHER) {
    float cnt = 0.f;
    for (int c = tid; c < L; c += 256) cnt += kvalid[(int64_t)b * L + c] != 0 ? 1.f : 0.f;
    const int len = (int)(block_sum(cnt, red) + 0.5f);
    r = (int64_t)b * L + max(len - 1, 0);
    if (h == 0) {
      if (tid == 0) rows[b] = (int32_t)r;
      for (int c = tid; c < D; c += 256) x_rows[(int64_t)b * D + c] = x[r * D + c];
    }
  } else {
    r = rows[b];
  }
  const int p = (int)(r - (int64_t)b * L);
  const T* seq = qkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  if (tid < Dh) sq[tid] = ldf<T>(qkv, r * ld + (int64_t)h * Dh + tid);
  __syncthreads();
  float sc[LMAX / 256];
  float mloc = -INFINITY;
#pragma unroll
  for (int t = 0; t < LMAX / 256; ++t) {
    const int c = tid + 256 * t;
    const bool ok = c < L && c <= p && kvalid[(int64_t)b * L + c] != 0;
    sc[t] = ok ? row_dot<T>(sq, seq + (int64_t)c * ld + D, Dh) * scale : -INFINITY;
    mloc = fmaxf(mloc, sc[t]);
  }
  const float m = block_max(mloc, red);
  float eloc = 0.f;
#pragma unroll
  for (int t = 0; t < LMAX / 256; ++t) {
    sc[t] = (sc[t] == -INFINITY) ? 0.f : expf(sc[t] - m);
    eloc += sc[t];
  }
  const float sum = block_sum(eloc, red);
  const DropKeys dk = resolve_drop(dp);
#pragma unroll
  for (int t = 0; t < LMAX / 256; ++t) {
    const int c = tid + 256 * t;
    if (c >= L) continue;
    float pc = sum > 0.f ? sc[t] / sum : 0.f;
    if (dk.on && pc != 0.f) pc = drop_apply(dk, (uint32_t)((((int64_t)bh * L) + p) * L + c), pc);
    sp[c] = pc;
  }
  if (tid == 0) lse[bh] = m == -INFINITY ? INFINITY : m + logf(sum);
  __syncthreads();
  const float acc = q1_combine<T>(sp, seq + 2 * D, ld, min(p, L - 1) + 1, Dh, red4);
  if (tid < Dh) stf<T>(ctx, (int64_t)b * D + (int64_t)h * Dh + tid, acc);
}

template <typename T>
__global__ __launch_bounds__(256) void mha_long_q1_bwd_kernel(int L, int H, int Dh, const T* __restrict__ qkv,
                                                              const int64_t* __restrict__ kvalid,
                                                              const int32_t* __restrict__ rows,
                                                              const float* __restrict__ lse,
                                                              const T* __restrict__ dctx, DropParams dp,
                                                              T* __restrict__ dqkv, float scale) {
  __shared__ float sq[64], sdo[64], sds[LMAX], spd[LMAX], red[4], red4[256];
  const int tid = threadIdx.x;
  const int bh = xcd_contiguous(blockIdx.x, gridDim.x), b = bh / H, h = bh % H;
  const int D = H * Dh;
  const int64_t ld = 3LL * D;
  const int64_t r = rows[b];
  const int p = (int)(r - (int64_t)b * L);
  const T* seq = qkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  T* dseq = dqkv + (int64_t)b * L * ld + (int64_t)h * Dh;
  if (tid < Dh) {
    sq[tid] = ldf<T>(qkv, r * ld + (int64_t)h * Dh + tid);
    sdo[tid] = ldf<T>(dctx, (int64_t)b * D + (int64_t)h * Dh + tid);
  }
  __syncthreads();
  const DropKeys dk = resolve_drop(dp);
  float pj[LMAX / 256], dP[LMAX / 256], kp[LMAX / 256];
  float part = 0.f;
#pragma unroll
  for (int t = 0; t < LMAX / 256; ++t) {
    const int c = tid + 256 * t;
    const bool ok = c < L && c <= p && kvalid[(int64_t)b * L + c] != 0;
    pj[t] = 0.f; dP[t] = 0.f; kp[t] = 1.f;
    if (ok) {
      const float sd = row_dot<T>(sq, seq + (int64_t)c * ld + D, Dh);
      const float dv = row_dot<T>(sdo, seq + (int64_t)c * ld + 2 * D, Dh);
      pj[t] = expf(sd * scale - lse[bh]);
      if (dk.on) kp[t] = drop_keep(dk, (uint32_t)((((int64_t)bh * L) + p) * L + c)) ? dk.scale : 0.f;
      dP[t] = dv * kp[t];
    }
    part += pj[t] * dP[t];
  }
  const float Dsum = block_sum(part, red);
#pragma unroll
  for (int t = 0; t < LMAX / 256; ++t) {
    const int c = tid + 256 * t;
    if (c < L) {
      sds[c] = pj[t] * (dP[t] - Dsum) * scale;
      spd[c] = pj[t] * kp[t];
    }
  }
  __syncthreads();
  // rows: dQ slice zero except the query row, dK_c = dS_c q, dV_c = Pd_c dO
  for (int i = tid; i < L * 64; i += 256) {
    const int c = i >> 6, d = i & 63;
    if (d >= Dh) continue;
    T* row = dseq + (int64_t)c * ld;
    if (c != p) stf<T>(row, d, 0.f);
    stf<T>(row + D, d, sds[c] * sq[d]);
    stf<T>(row + 2 * D, d, spd[c] * sdo[d]);
  }
  __syncthreads();
  const float acc = q1_combine<T>(sds, seq + D, ld, min(p, L - 1) + 1, Dh, red4);
  if (tid < Dh) stf<T>(dseq + (int64_t)p * ld, tid, acc);
}

}  // namespace

int attn_long_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv, const int64_t* kv, DropParams dp,
                  void* ctx, float* lse, hipStream_t s) {
  const dim3 grid((unsigned)(B * H), (unsigned)((L + LB - 1) / LB));
  const float sc = 1.f / sqrtf((float)Dh);
  if (dtype == TTMI_BF16)
    hipLaunchKernelGGL(mha_long_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, L, H, Dh, (const bf16_t*)qkv, kv, dp,
                       (bf16_t*)ctx, lse, sc);
  else
    hipLaunchKernelGGL(mha_long_fwd_kernel<float>, grid, dim3(256), 0, s, L, H, Dh, (const float*)qkv, kv, dp,
                       (float*)ctx, lse, sc);
  return ttmi_check_launch("ttmi_mha_fwd/long");
}

int attn_long_bwd(int dtype, int B, int L, int H, int Dh, const void* qkv, const int64_t* kv, const float* lse,
                  const void* dctx, DropParams dp, void* dqkv, hipStream_t s) {
  const float sc = 1.f / sqrtf((float)Dh);
  if (dtype == TTMI_BF16)
    hipLaunchKernelGGL(mha_long_bwd_kernel<bf16_t>, dim3((unsigned)(B * H)), dim3(256), 0, s, L, H, Dh,
                       (const bf16_t*)qkv, kv, lse, (const bf16_t*)dctx, dp, (bf16_t*)dqkv, sc);
  else
    hipLaunchKernelGGL(mha_long_bwd_kernel<float>, dim3((unsigned)(B * H)), dim3(256), 0, s, L, H, Dh,
                       (const float*)qkv, kv, lse, (const float*)dctx, dp, (float*)dqkv, sc);
  return ttmi_check_launch("ttmi_mha_bwd/long");
}

int attn_long_q1_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv, const int64_t* kv, int32_t* rows,
                     const float* x, float* x_rows, bool gather, DropParams dp, void* ctx, float* lse,
                     hipStream_t s) {
  const float sc = 1.f / sqrtf((float)Dh);
  const dim3 grid((unsigned)(B * H));
  if (dtype == TTMI_BF16) {
    if (gather)
      hipLaunchKernelGGL((mha_long_q1_fwd_kernel<bf16_t, true>), grid, dim3(256), 0, s, L, H, Dh,
                         (const bf16_t*)qkv, kv, rows, x, x_rows, dp, (bf16_t*)ctx, lse, sc);
    else
      hipLaunchKernelGGL((mha_long_q1_fwd_kernel<bf16_t, false>), grid, dim3(256), 0, s, L, H, Dh,
                         (const bf16_t*)qkv, kv, rows, x, x_rows, dp, (bf16_t*)ctx, lse, sc);
  } else {
    if (gather)
      hipLaunchKernelGGL((mha_long_q1_fwd_kernel<float, true>), grid, dim3(256), 0, s, L, H, Dh,
                         (const float*)qkv, kv, rows, x, x_rows, dp, (float*)ctx, lse, sc);
    else
      hipLaunchKernelGGL((mha_long_q1_fwd_kernel<float, false>), grid, dim3(256), 0, s, L, H, Dh,
                         (const float*)qkv, kv, rows, x, x_rows, dp, (float*)ctx, lse, sc);
  }
  return ttmi_check_launch("ttmi_mha_q1_fwd/long");
}

int attn_long_q1_bwd(int dtype, int B, int L, int H, int Dh, const void* qkv, const int64_t* kv,
                     const int32_t* rows, const float* lse, const void* dctx, DropParams dp, void* dqkv,
                     hipStream_t s) {
  const float sc = 1.f / sqrtf((float)Dh);
  const dim3 grid((unsigned)(B * H));
  if (dtype == TTMI_BF16)
    hipLaunchKernelGGL(mha_long_q1_bwd_kernel<bf16_t>, grid, dim3(256), 0, s, L, H, Dh, (const bf16_t*)qkv, kv,
                       rows, lse, (const bf16_t*)dctx, dp, (bf16_t*)dqkv, sc);
  else
    hipLaunchKernelGGL(mha_long_q1_bwd_kernel<float>, grid, dim3(256), 0, s, L, H, Dh, (const float*)qkv, kv,
                       rows, lse, (const float*)dctx, dp, (float*)dqkv, sc);
  return ttmi_check_launch("ttmi_mha_q1_bwd/long");
}
