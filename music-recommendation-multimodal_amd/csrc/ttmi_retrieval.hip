// ttmi_retrieval.hip — global retrieval evaluation and serving top-K (reference
// src/evaluate_metrics.py:107-192 calculate_metrics_global; src/inference.py recommend):
// scores = û·Îᵀ over the whole catalogue (ttmi_gemm), score[:, 0] = -inf (padding item), the
// top-K item indices per user, and the rank of each user's target in that list (Recall@k =
// rank < k, NDCG@k = 1/log2(rank + 2)).
//
//   topk_rows_kernel   one workgroup per row: exact K-th largest key by MSB-first radix select
//                      (four 8-bit histogram passes over the row in LDS), then the keys above it
//                      plus the lowest-index ties, sorted by (score desc, index asc) in one wave.
//                      Rows up to 16,384 scores are read from HBM once into LDS (as order keys);
//                      longer rows are re-read per pass (L2-resident for V <= ~100k).
//   rank_kernel        first position of target[b] in idx[b, :K] (K if absent).
#include "ttmi_common.h"

namespace {

constexpr int TK_MAX = 64;              // K <= 64

TTMI_DEV uint32_t fkey(float f) {       // order-preserving float -> uint32
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
TTMI_DEV float funkey(uint32_t k) {
  const uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
  return __uint_as_float(u);
}

constexpr int TK_LDS_MAX = 16384;      // rows up to this length are staged once in LDS (64 KB)
constexpr int TK_NT = 512;              // threads per row (8 waves)

// Block-wide exclusive prefix sum of one value per thread (TK_NT threads).
TTMI_DEV uint32_t block_exclusive_scan(uint32_t v, uint32_t* wtot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wtot[wave] = inc;
  __syncthreads();
  uint32_t base = 0;
  for (int w = 0; w < wave; ++w) base += wtot[w];
  return base + inc - v;
}

// Histogram increment of `bin` for the lanes with `take`: the lanes sharing the first taking
// lane's bin add once through that lane (in the first radix pass the scores of a row share
// one or two exponents, so most of a wave lands in one bin and serialised LDS atomics on a
// single address were the kernel's bound); the other lanes add individually.
TTMI_DEV void hist_add(uint32_t* hist, bool take, uint32_t bin) {
  const int lane = threadIdx.x & 63;
  const uint64_t act = __ballot(take);
  if (!act) return;
  const int leader = __ffsll((unsigned long long)act) - 1;
  const uint32_t lb = (uint32_t)__builtin_amdgcn_readlane((int)bin, leader);   // leader is uniform
  const uint64_t same = __ballot(take && bin == lb);
  if (lane == leader) atomicAdd(&hist[lb], (uint32_t)__popcll(same));
  if (take && bin != lb) atomicAdd(&hist[bin], 1u);
}

// One workgroup (8 waves) per row.  LDSROW: the row is read from HBM once (16-byte loads when
// the row is 16-byte aligned) and kept in LDS as order keys, padded to a multiple of 4; the four
// radix passes and the collection read it 4 keys per LDS instruction.  Otherwise every pass
// re-reads the row from global memory (L2-resident for moderate V).
template <bool LDSROW>
__global__ __launch_bounds__(TK_NT) void topk_rows_kernel(int V, int K, const float* __restrict__ scores,
                                                          int64_t ld, int skip0, float* __restrict__ out_val,
                                                          int64_t* __restrict__ out_idx) {
  extern __shared__ uint4 skeys4[];
  uint32_t* skeys = reinterpret_cast<uint32_t*>(skeys4);
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_prefix, s_mask, s_rem;
  __shared__ uint32_t s_wtot[TK_NT / 64];
  __shared__ uint32_t s_ngt;
  __shared__ uint32_t ck[TK_MAX];
  __shared__ int32_t ci[TK_MAX];
  const int tid = threadIdx.x, lane = tid & 63;
  const float* row = scores + (int64_t)blockIdx.x * ld;
  const int chunk = (V + TK_NT - 1) / TK_NT;
  const int lo = min(V, tid * chunk), hi = min(V, lo + chunk);   // contiguous slice per thread
  const int V4 = (V + 3) >> 2;                                    // key quads (LDSROW)
  auto gkey = [&](int i) -> uint32_t {
    return (skip0 && i == 0) ? fkey(-INFINITY) : fkey(row[i]);
  };
  auto key_at = [&](int i) -> uint32_t {
    if constexpr (LDSROW) return skeys[i];
    else return gkey(i);
  };
  if constexpr (LDSROW) {
    if ((reinterpret_cast<uintptr_t>(row) & 15) == 0) {
      const int full = V >> 2;
      for (int j = tid; j < full; j += TK_NT) {
        const float4 f = reinterpret_cast<const float4*>(row)[j];
        skeys4[j] = make_uint4(fkey(f.x), fkey(f.y), fkey(f.z), fkey(f.w));
      }
      for (int i = full * 4 + tid; i < V; i += TK_NT) skeys[i] = fkey(row[i]);
    } else {
      for (int i = tid; i < V; i += TK_NT) skeys[i] = fkey(row[i]);
    }
    if (tid == 0) {                        // same thread as the writes of key 0: no race
      if (skip0) skeys[0] = fkey(-INFINITY);
      for (int i = V; i < 4 * V4; ++i) skeys[i] = 0u;   // pad (never counted: i >= V)
    }
  }
  if (tid == 0) { s_prefix = 0; s_mask = 0; s_rem = (uint32_t)K; }
  // -- radix select of the K-th largest key
  for (int shift = 24; shift >= 0; shift -= 8) {
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix, mask = s_mask;
    if constexpr (LDSROW) {
      for (int j = tid; j < V4; j += TK_NT) {
        const uint4 q = skeys4[j];
        const uint32_t k4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          hist_add(hist, 4 * j + e < V && (k4[e] & mask) == prefix, (k4[e] >> shift) & 255u);
      }
    } else {
      for (int i = tid; i < V; i += TK_NT) {                // coalesced
        const uint32_t u = gkey(i);
        hist_add(hist, (u & mask) == prefix, (u >> shift) & 255u);
      }
    }
    __syncthreads();
    if (tid < 64) {
      // the digit d: keys with a larger digit number < rem <= those with digit >= d.  Lane l
      // holds digits 255-4l .. 252-4l; a wave prefix sum over lanes = descending digits.
      uint32_t h[4], tot = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) { h[j] = hist[255 - 4 * lane - j]; tot += h[j]; }
      uint32_t inc = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o, 64);
        if (lane >= o) inc += u;
      }
      const uint32_t rem = s_rem, excl = inc - tot;
      if (excl < rem && rem <= inc) {                       // exactly one lane
        uint32_t above = excl;
        int d = 255 - 4 * lane;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          if (above + h[j] >= rem) break;
          above += h[j];
          --d;
        }
        s_rem = rem - above;               // how many keys equal to the prefix we still need
        s_prefix = prefix | ((uint32_t)d << shift);
        s_mask = mask | (255u << shift);
      }
    }
    __syncthreads();
  }
  const uint32_t T = s_prefix;             // the K-th largest key
  const uint32_t need_eq = s_rem;          // ties at T to take (lowest indices first)
  // -- collect: keys > T anywhere, keys == T in index order
  uint32_t n_eq = 0;
  for (int i = lo; i < hi; ++i) n_eq += key_at(i) == T ? 1u : 0u;
  if (tid == 0) s_ngt = 0;
  uint32_t before = block_exclusive_scan(n_eq, s_wtot);   // tie counts of the slices before
  const uint32_t n_gt_total = (uint32_t)K - need_eq;
  if constexpr (LDSROW) {
    for (int j = tid; j < V4; j += TK_NT) {                 // keys above T: any order
      const uint4 q = skeys4[j];
      const uint32_t k4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (k4[e] > T && 4 * j + e < V) {
          const uint32_t p = atomicAdd(&s_ngt, 1u);
          ck[p] = k4[e]; ci[p] = 4 * j + e;
        }
    }
  } else {
    for (int i = tid; i < V; i += TK_NT) {
      const uint32_t u = gkey(i);
      if (u > T) {
        const uint32_t p = atomicAdd(&s_ngt, 1u);
        ck[p] = u; ci[p] = i;
      }
    }
  }
  for (int i = lo; i < hi && before < need_eq; ++i) {       // ties at T: lowest indices first
    if (key_at(i) == T) {
      ck[n_gt_total + before] = T; ci[n_gt_total + before] = i;
      ++before;
    }
  }
  __syncthreads();
  // -- sort the K candidates (score desc, index asc): rank by counting, one wave
  if (tid < K) {
    const uint32_t u = ck[tid];
    const int ix = ci[tid];
    int r = 0;
    for (int j = 0; j < K; ++j) {
      const uint32_t v = ck[j];
      r += (v > u || (v == u && ci[j] < ix)) ? 1 : 0;
    }
    out_val[(int64_t)blockIdx.x * K + r] = funkey(u);
    out_idx[(int64_t)blockIdx.x * K + r] = ix;
  }
}

__global__ __launch_bounds__(256) void rank_kernel(int B, int K, const int64_t* __restrict__ idx,
                                                   const int64_t* __restrict__ target,
                                                   int32_t* __restrict__ rank) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int r = K;
  for (int j = K - 1; j >= 0; --j)
    if (idx[(int64_t)b * K + j] == target[b]) r = j;
  rank[b] = r;
}

// scores[r, ids[r, j]] = -inf for every listed item (the user's history, inference.py:294-303)
__global__ __launch_bounds__(256) void mask_items_kernel(int R, int V, float* __restrict__ scores, int64_t ld,
                                                         const int64_t* __restrict__ ids, int Lh) {
  const int64_t n = (int64_t)R * Lh;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / Lh;
    const int64_t id = ids[t];
    if (id >= 0 && id < V) scores[r * ld + id] = -INFINITY;
  }
}

}  // namespace

// Catalogue index rows (evaluate_metrics.py:58-104, inference.py:175-201): per item row
// e = get_item_embedding's F.normalize(x) (eps 1e-12); NaN -> 0 (nan_to_num, :76-78); e /
// max(|e|, 1e-8) (:82); dense[ids[r]] = e.  One wave per row.
__global__ __launch_bounds__(256) void catalogue_rows_kernel(int n, int D, const float* __restrict__ x,
                                                             int64_t ldx, const int64_t* __restrict__ ids,
                                                             int64_t V, float* __restrict__ dense,
                                                             int32_t* __restrict__ id_err) {
  const int lane = threadIdx.x & 63;
  const int r = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (r >= n) return;
  const int64_t id = ids[r];
  if (id < 0 || id >= V) {                 // skipped; the host raises IndexError (ABI 20)
    raise_id_err(id_err, TTMI_IDERR_CATALOGUE);
    return;
  }
  const float* xr = x + (int64_t)r * ldx;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) s += xr[c] * xr[c];
  const float inv1 = 1.f / fmaxf(sqrtf(wave_sum(s)), 1e-12f);
  float s2 = 0.f;
  for (int c = lane; c < D; c += 64) {
    float e = xr[c] * inv1;
    if (e != e) e = 0.f;
    s2 += e * e;
  }
  const float inv2 = 1.f / fmaxf(sqrtf(wave_sum(s2)), 1e-8f);
  float* dr = dense + id * (int64_t)D;
  for (int c = lane; c < D; c += 64) {
    float e = xr[c] * inv1;
    if (e != e) e = 0.f;
    dr[c] = e * inv2;
  }
}

extern "C" int ttmi_catalogue_rows(int n, int D, const float* x, int64_t ldx, const int64_t* ids,
                                   int64_t V, float* dense, int32_t* id_err, hipStream_t s) {
  TTMI_REQUIRE(n >= 0 && D > 0 && ldx >= D && V > 0, "ttmi_catalogue_rows: bad sizes");
  if (n == 0) return TTMI_OK;
  TTMI_REQUIRE(x && ids && dense, "ttmi_catalogue_rows: null argument");
  hipLaunchKernelGGL(catalogue_rows_kernel, dim3((n + 3) / 4), dim3(256), 0, s, n, D, x, ldx, ids,
                     V, dense, id_err);
  return ttmi_check_launch("ttmi_catalogue_rows");
}

extern "C" int ttmi_mask_items(int R, int V, float* scores, int64_t ld, const int64_t* ids, int Lh,
                               hipStream_t s) {
  TTMI_REQUIRE(R > 0 && V > 0 && Lh > 0 && ld >= V && scores && ids, "ttmi_mask_items: bad argument");
  const int64_t n = (int64_t)R * Lh;
  hipLaunchKernelGGL(mask_items_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0, s,
                     R, V, scores, ld, ids, Lh);
  return ttmi_check_launch("ttmi_mask_items");
}

extern "C" int ttmi_topk_rows(int R, int V, int K, const float* scores, int64_t ld, int skip_first,
                              float* out_val, int64_t* out_idx, hipStream_t s) {
  TTMI_REQUIRE(R > 0 && V > 0 && K > 0 && K <= TK_MAX && K <= V && ld >= V,
               "ttmi_topk_rows: need 0 < K <= min(V, %d), ld >= V", TK_MAX);
  TTMI_REQUIRE(scores && out_val && out_idx, "ttmi_topk_rows: null argument");
  if (V <= TK_LDS_MAX)
    hipLaunchKernelGGL(topk_rows_kernel<true>, dim3((unsigned)R), dim3(TK_NT), (size_t)((V + 3) / 4) * 16, s, V,
                       K, scores, ld, skip_first, out_val, out_idx);
  else
    hipLaunchKernelGGL(topk_rows_kernel<false>, dim3((unsigned)R), dim3(TK_NT), 0, s, V, K, scores, ld,
                       skip_first, out_val, out_idx);
  return ttmi_check_launch("ttmi_topk_rows");
}

extern "C" int ttmi_rank_of(int B, int K, const int64_t* idx, const int64_t* target, int32_t* rank,
                            hipStream_t s) {
  TTMI_REQUIRE(B > 0 && K > 0 && idx && target && rank, "ttmi_rank_of: bad argument");
  hipLaunchKernelGGL(rank_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, B, K, idx, target, rank);
  return ttmi_check_launch("ttmi_rank_of");
}
