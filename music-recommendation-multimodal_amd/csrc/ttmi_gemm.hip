// ttmi_gemm.hip — MFMA GEMM with fused epilogue for every nn.Linear on the hot path.
//
// C[m,n] = epi(alpha * Σ_k A(m,k) B(n,k)).  One 256-thread workgroup (4 waves, 2x2)
// owns a BM x BN tile; each wave a (BM/2) x (BN/2) block of 16x16 MFMA tiles.  K is
// walked in 128-byte tiles (64 bf16 / 32 f32) staged through LDS as [row][k] with a
// 144-byte row pitch (16-byte pad: the 16 rows one ds_read_b128 lane-group touches land on
// distinct 4-bank slots).  A k-major operand is copied 16 B per lane; a non-k-major one
// (the weight-gradient operands dYᵀ and Xᵀ, or Wᵀ for dX = dY·W) is loaded 16 B along m/n
// and transposed on the LDS write.  The next K-tile is prefetched into registers while
// the current one feeds the MFMAs (register double-buffering, two barriers per K-tile).
//
// Epilogue order (ttmi.h): bias -> act -> dropout -> gate -> colsum -> residual -> store.
#include "ttmi_common.h"

namespace {

constexpr int ROWB = 144;

struct GemmArgs {
  int64_t M, N, K;
  const char* A; int64_t lda;
  const char* B; int64_t ldb;
  void* C; int64_t ldc; int c_f32; int c_mode;
  float alpha;
  const float* bias; int act;
  DropParams drop; int64_t ld_drop;
  const void* gate; int gate_f32; int64_t ld_gate; float gate_scale;
  const float* residual; int64_t ld_res;
  float* colsum;
  int64_t k_split;   // K elements per split (multiple of the K tile)
};

template <typename T, int ROWS, bool KMAJ>
struct TileLoader {
  static constexpr int E = 16 / sizeof(T);
  static constexpr int BKE = 128 / sizeof(T);
  static constexpr int PER = ROWS / 32;           // 16-byte chunks per thread
  uint4 r[PER];

  TTMI_DEV void load(const char* base, int64_t ld, int64_t row0, int64_t nrows, int64_t k0,
                     int64_t kend, int tid) {
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int idx = tid + c * 256;
      int64_t row, k;
      if constexpr (KMAJ) {
        row = row0 + (idx >> 3);
        k = k0 + (idx & 7) * E;
      } else {
        constexpr int CPR = ROWS / E;               // chunks per k-row
        k = k0 + idx / CPR;
        row = row0 + (idx % CPR) * E;
      }
      if (row < nrows && k < kend) {
        const int64_t off = KMAJ ? (row * ld + k) : (k * ld + row);
        r[c] = *reinterpret_cast<const uint4*>(base + off * (int64_t)sizeof(T));
      } else {
        r[c] = make_uint4(0, 0, 0, 0);
      }
    }
  }

  TTMI_DEV void store(char* s, int tid) const {
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int idx = tid + c * 256;
      if constexpr (KMAJ) {
        *reinterpret_cast<uint4*>(s + (idx >> 3) * ROWB + (idx & 7) * 16) = r[c];
      } else {
        constexpr int CPR = ROWS / E;
        const int kk = idx / CPR;
        const int rr = (idx % CPR) * E;
        const T* v = reinterpret_cast<const T*>(&r[c]);
#pragma unroll
        for (int e = 0; e < E; ++e)
          *reinterpret_cast<T*>(s + (rr + e) * ROWB + kk * (int)sizeof(T)) = v[e];
      }
    }
  }
};

template <typename T, int BM, int BN, bool AK, bool BKM>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
  constexpr int BKE = 128 / sizeof(T);
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  __shared__ __attribute__((aligned(16))) char smem[(BM + BN) * ROWB];
  char* sA = smem;
  char* sB = smem + BM * ROWB;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t n0 = (int64_t)blockIdx.x * BN;
  const int64_t m0 = (int64_t)blockIdx.y * BM;
  const int64_t kbeg = (int64_t)blockIdx.z * g.k_split;
  const int64_t kend = min(g.K, kbeg + g.k_split);
  const DropKeys dk = resolve_drop(g.drop);

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  TileLoader<T, BM, AK> la;
  TileLoader<T, BN, BKM> lb;
  if (kbeg < kend) {
    la.load(g.A, g.lda, m0, g.M, kbeg, kend, tid);
    lb.load(g.B, g.ldb, n0, g.N, kbeg, kend, tid);
    la.store(sA, tid);
    lb.store(sB, tid);
  }
  __syncthreads();

  const int arow = wm * WTM + (lane & 15);
  const int brow = wn * WTN + (lane & 15);
  const int kq = (lane >> 4) * 16;
  for (int64_t k0 = kbeg; k0 < kend; k0 += BKE) {
    const bool more = k0 + BKE < kend;
    if (more) {
      la.load(g.A, g.lda, m0, g.M, k0 + BKE, kend, tid);
      lb.load(g.B, g.ldb, n0, g.N, k0 + BKE, kend, tid);
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      uint4 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = lds16(sA + (arow + i * 16) * ROWB + c * 64 + kq);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = lds16(sB + (brow + j * 16) * ROWB + c * 64 + kq);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) Mma<T>::run(acc[i][j], af[i], bfr[j]);
    }
    __syncthreads();
    if (more) {
      la.store(sA, tid);
      lb.store(sB, tid);
    }
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  const bool first = blockIdx.z == 0;
  const int rq = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int64_t n = n0 + wn * WTN + j * 16 + (lane & 15);
    const bool nok = n < g.N;
    const float bias = (g.bias && first && nok) ? g.bias[n] : 0.f;
    float csum = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t m = m0 + wm * WTM + i * 16 + rq + e;
        if (!(nok && m < g.M)) continue;
        float v = g.alpha * acc[i][j][e] + bias;
        if (g.act == 1) v = fmaxf(v, 0.f);
        if (dk.on) v = drop_apply(dk, (uint32_t)(m * g.ld_drop + n), v);
        if (g.gate) v = ld_dyn(g.gate, m * g.ld_gate + n, g.gate_f32) > 0.f ? v * g.gate_scale : 0.f;
        csum += v;
        if (g.residual && first) v += g.residual[m * g.ld_res + n];
        const int64_t o = m * g.ldc + n;
        if (g.c_mode == 1) atomicAdd(reinterpret_cast<float*>(g.C) + o, v);
        else st_dyn(g.C, o, v, g.c_f32);
      }
    }
    if (g.colsum) {
      csum += __shfl_xor(csum, 16, 64);
      csum += __shfl_xor(csum, 32, 64);
      if (lane < 16 && nok) atomicAdd(g.colsum + n, csum);
    }
  }
}

template <typename T, int BM, int BN>
void launch_layout(const GemmArgs& a, bool ak, bool bk, dim3 grid, hipStream_t s) {
  if (ak && bk) hipLaunchKernelGGL((gemm_kernel<T, BM, BN, true, true>), grid, dim3(256), 0, s, a);
  else if (ak) hipLaunchKernelGGL((gemm_kernel<T, BM, BN, true, false>), grid, dim3(256), 0, s, a);
  else if (bk) hipLaunchKernelGGL((gemm_kernel<T, BM, BN, false, true>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((gemm_kernel<T, BM, BN, false, false>), grid, dim3(256), 0, s, a);
}

template <typename T>
void launch_typed(const GemmArgs& a, bool ak, bool bk, int bm, int bn, dim3 grid, hipStream_t s) {
  if (bm == 128) launch_layout<T, 128, 128>(a, ak, bk, grid, s);
  else if (bn == 128) launch_layout<T, 64, 128>(a, ak, bk, grid, s);
  else launch_layout<T, 64, 64>(a, ak, bk, grid, s);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int ttmi_gemm(const ttmi_gemm_desc* d, hipStream_t stream) {
  TTMI_REQUIRE(d != nullptr, "ttmi_gemm: null descriptor");
  TTMI_REQUIRE(d->dtype == TTMI_F32 || d->dtype == TTMI_BF16, "ttmi_gemm: bad dtype %d", d->dtype);
  TTMI_REQUIRE(d->M >= 0 && d->N >= 0 && d->K >= 0, "ttmi_gemm: negative size");
  if (d->M == 0 || d->N == 0) return TTMI_OK;
  const int es = d->dtype == TTMI_F32 ? 4 : 2;
  const int E = 16 / es;
  TTMI_REQUIRE(d->A && d->B && d->C, "ttmi_gemm: null operand");
  TTMI_REQUIRE(aligned16(d->A) && aligned16(d->B), "ttmi_gemm: A/B must be 16-byte aligned");
  TTMI_REQUIRE((d->lda * es) % 16 == 0 && (d->ldb * es) % 16 == 0,
               "ttmi_gemm: lda/ldb must be multiples of 16 bytes");
  if (d->a_kmajor) TTMI_REQUIRE(d->K % E == 0 && d->lda >= d->K, "ttmi_gemm: k-major A needs K %% %d == 0, lda >= K", E);
  else TTMI_REQUIRE(d->M % E == 0 && d->lda >= d->M, "ttmi_gemm: m-major A needs M %% %d == 0, lda >= M", E);
  if (d->b_kmajor) TTMI_REQUIRE(d->K % E == 0 && d->ldb >= d->K, "ttmi_gemm: k-major B needs K %% %d == 0, ldb >= K", E);
  else TTMI_REQUIRE(d->N % E == 0 && d->ldb >= d->N, "ttmi_gemm: n-major B needs N %% %d == 0, ldb >= N", E);
  TTMI_REQUIRE(d->ldc >= d->N, "ttmi_gemm: ldc < N");
  TTMI_REQUIRE(d->c_mode == 0 || d->c_mode == 1, "ttmi_gemm: bad c_mode");
  TTMI_REQUIRE(d->c_mode == 0 || d->c_dtype == TTMI_F32, "ttmi_gemm: accumulate needs an f32 C");
  TTMI_REQUIRE(d->act == 0 || d->act == 1, "ttmi_gemm: bad act");
  TTMI_REQUIRE(d->drop_p >= 0.f && d->drop_p < 1.f, "ttmi_gemm: drop_p out of [0,1)");
  TTMI_REQUIRE(d->drop_p == 0.f || d->drop_seed, "ttmi_gemm: dropout needs a seed pointer");
  TTMI_REQUIRE(!d->gate || d->ld_gate >= d->N, "ttmi_gemm: ld_gate < N");
  TTMI_REQUIRE(!d->residual || d->ld_res >= d->N, "ttmi_gemm: ld_res < N");

  const int bke = 128 / es;
  int bm, bn;
  const int64_t t128 = ((d->M + 127) / 128) * ((d->N + 127) / 128);
  const int64_t t64x128 = ((d->M + 63) / 64) * ((d->N + 127) / 128);
  if (d->N > 64 && t128 >= 256) { bm = 128; bn = 128; }
  else if (d->N > 64 && t64x128 >= 128) { bm = 64; bn = 128; }
  else { bm = 64; bn = 64; }
  const int64_t gx = (d->N + bn - 1) / bn, gy = (d->M + bm - 1) / bm;
  TTMI_REQUIRE(gy <= 65535 && gx <= 2147483647LL, "ttmi_gemm: grid too large");

  int split = d->split_k;
  const int64_t ktiles = (d->K + bke - 1) / bke;
  if (split <= 0) {                      // auto: only when accumulating and linear epilogue
    split = 1;
    if (d->c_mode == 1 && d->act == 0) {
      const int64_t want = (512 + gx * gy - 1) / (gx * gy);
      split = (int)std::max<int64_t>(1, std::min<int64_t>(want, ktiles / 2));
    }
  }
  TTMI_REQUIRE(split == 1 || (d->c_mode == 1 && d->act == 0),
               "ttmi_gemm: split_k > 1 needs c_mode 1 and act 0");
  const int64_t tiles_per_split = (ktiles + split - 1) / std::max(split, 1);
  const int64_t kspl = std::max<int64_t>(tiles_per_split, 1) * bke;
  split = (int)std::max<int64_t>(1, (d->K + kspl - 1) / kspl);
  TTMI_REQUIRE(split <= 65535, "ttmi_gemm: too many splits");

  GemmArgs a;
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.A = static_cast<const char*>(d->A); a.lda = d->lda;
  a.B = static_cast<const char*>(d->B); a.ldb = d->ldb;
  a.C = d->C; a.ldc = d->ldc; a.c_f32 = d->c_dtype == TTMI_F32; a.c_mode = d->c_mode;
  a.alpha = d->alpha;
  a.bias = d->bias; a.act = d->act;
  a.drop = make_drop(d->drop_p, d->drop_seed); a.ld_drop = d->ld_drop ? d->ld_drop : d->N;
  a.gate = d->gate; a.gate_f32 = d->gate_dtype == TTMI_F32; a.ld_gate = d->ld_gate;
  a.gate_scale = d->gate_scale;
  a.residual = d->residual; a.ld_res = d->ld_res;
  a.colsum = d->colsum;
  a.k_split = kspl;

  dim3 grid((unsigned)gx, (unsigned)gy, (unsigned)split);
  if (d->dtype == TTMI_BF16) launch_typed<bf16_t>(a, d->a_kmajor, d->b_kmajor, bm, bn, grid, stream);
  else launch_typed<float>(a, d->a_kmajor, d->b_kmajor, bm, bn, grid, stream);
  return ttmi_check_launch("ttmi_gemm");
}
