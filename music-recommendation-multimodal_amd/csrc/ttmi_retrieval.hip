// ttmi_retrieval.hip — global retrieval evaluation and serving top-K (reference
// src/evaluate_metrics.py:107-192 calculate_metrics_global; src/inference.py recommend):
// scores = û·Îᵀ over the whole catalogue (ttmi_gemm), score[:, 0] = -inf (padding item), the
// top-K item indices per user, and the rank of each user's target in that list (Recall@k =
// rank < k, NDCG@k = 1/log2(rank + 2)).
//
//   topk_rows_kernel   one workgroup per row: exact K-th largest key by MSB-first radix select
//                      (four 8-bit histogram passes over the row in LDS), then the keys above it
//                      plus the lowest-index ties, sorted by (score desc, index asc) in one wave.
//                      HBM-bound: the row is read 5 times (L2-resident for V <= ~100k).
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

__global__ __launch_bounds__(256) void topk_rows_kernel(int V, int K, const float* __restrict__ scores,
                                                        int64_t ld, int skip0, float* __restrict__ out_val,
                                                        int64_t* __restrict__ out_idx) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_prefix, s_mask, s_rem;
  __shared__ uint32_t s_cnt[256];
  __shared__ uint32_t s_ngt;
  __shared__ uint32_t ck[TK_MAX];
  __shared__ int32_t ci[TK_MAX];
  const int tid = threadIdx.x;
  const float* row = scores + (int64_t)blockIdx.x * ld;
  const int chunk = (V + 255) / 256;
  const int lo = min(V, tid * chunk), hi = min(V, lo + chunk);   // contiguous slice per thread
  auto key_at = [&](int i) -> uint32_t {
    return (skip0 && i == 0) ? fkey(-INFINITY) : fkey(row[i]);
  };
  if (tid == 0) { s_prefix = 0; s_mask = 0; s_rem = (uint32_t)K; }
  // -- radix select of the K-th largest key
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix, mask = s_mask;
    for (int i = tid; i < V; i += 256) {                    // coalesced
      const uint32_t u = key_at(i);
      if ((u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t rem = s_rem, above = 0;
      int d = 255;
      for (; d > 0; --d) {
        if (above + hist[d] >= rem) break;
        above += hist[d];
      }
      s_rem = rem - above;                 // how many keys equal to the prefix we still need
      s_prefix = prefix | ((uint32_t)d << shift);
      s_mask = mask | (255u << shift);
    }
    __syncthreads();
  }
  const uint32_t T = s_prefix;             // the K-th largest key
  const uint32_t need_eq = s_rem;          // ties at T to take (lowest indices first)
  // -- collect: keys > T anywhere, keys == T in index order
  uint32_t n_eq = 0;
  for (int i = lo; i < hi; ++i) n_eq += key_at(i) == T ? 1u : 0u;
  s_cnt[tid] = n_eq;
  if (tid == 0) s_ngt = 0;
  __syncthreads();
  uint32_t before = 0;                     // exclusive scan of tie counts (contiguous slices)
  for (int t = 0; t < tid; ++t) before += s_cnt[t];
  const uint32_t n_gt_total = (uint32_t)K - need_eq;
  for (int i = tid; i < V; i += 256) {                      // keys above T: any order
    const uint32_t u = key_at(i);
    if (u > T) {
      const uint32_t p = atomicAdd(&s_ngt, 1u);
      ck[p] = u; ci[p] = i;
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
  hipLaunchKernelGGL(topk_rows_kernel, dim3((unsigned)R), dim3(256), 0, s, V, K, scores, ld, skip_first,
                     out_val, out_idx);
  return ttmi_check_launch("ttmi_topk_rows");
}

extern "C" int ttmi_rank_of(int B, int K, const int64_t* idx, const int64_t* target, int32_t* rank,
                            hipStream_t s) {
  TTMI_REQUIRE(B > 0 && K > 0 && idx && target && rank, "ttmi_rank_of: bad argument");
  hipLaunchKernelGGL(rank_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, B, K, idx, target, rank);
  return ttmi_check_launch("ttmi_rank_of");
}
