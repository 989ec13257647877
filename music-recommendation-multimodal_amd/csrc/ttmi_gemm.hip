// ttmi_gemm.hip — MFMA GEMM with fused epilogue for every nn.Linear on the hot path.
//
// C[m,n] = epi(alpha * Σ_k A(m,k) B(n,k)).  One 256-thread workgroup (4 waves, 2x2) owns
// a BM x BN tile, each wave a (BM/2) x (BN/2) block of 16x16 MFMA tiles.  K is walked in
// 128-byte tiles (64 bf16 / 32 f32), double-buffered in LDS with register prefetch (one
// barrier per K-tile).
//
// Operand staging (bf16):
//   k-major operand  -> LDS [row][k], 144-byte pitch, fragments by two ds_read_b64;
//   row-major operand (the weight-gradient operands dYᵀ / Xᵀ and the Wᵀ of dX = dY·W)
//                    -> LDS [k][row] exactly as it sits in HBM (16-byte copies, no
//                       transpose), fragments by two ds_read_b64_tr_b16 (gfx950 transpose
//                       read), pitch = rowbytes + 32 so the 8 k-rows a 32-lane half reads
//                       land in disjoint 8-bank windows.
//   Both read paths feed the 16x16x32 MFMA the same k-permutation (lane group g holds
//   k = 4g..4g+3 and 16+4g..16+4g+3 of each 32-wide chunk), which is what makes both
//   conflict-free.  fp32 operands use the 16x16x4 f32 MFMA; a row-major fp32 operand is
//   transposed on its LDS write.
// The MFMA is issued with the B tile as its row operand, so each lane ends up holding four
// CONSECUTIVE output columns of one row: the epilogue reads bias/gate/residual and writes C
// with 8-byte (bf16) / 16-byte (f32) vector accesses.
//
// Epilogue order (ttmi.h): bias -> act -> dropout -> gate -> colsum -> residual -> store.
#include "ttmi_common.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4_t;

struct GemmArgs {
  int64_t M, N, K;
  const char* A; int64_t lda;
  const char* B; int64_t ldb;
  void* C; int64_t ldc; int c_f32; int c_mode;
  float alpha;
  const float* bias; int act;
  DropParams drop; int64_t ld_drop; const int32_t* drop_rows;
  const void* gate; int gate_f32; int64_t ld_gate; float gate_scale;
  const float* residual; int64_t ld_res;
  float* colsum;
  int64_t k_split;   // K elements per split (multiple of the K tile)
  int vec;           // 1: all row strides allow 4-wide vector epilogue accesses
  float* rowsum_a;   // rowsum_a[m] += Σ_k A(m,k)  (bias grad of a weight-gradient GEMM)
  bf16_t* pre_out;   // act 2: the pre-activation (after bias) is also stored here (row stride ldc)
  int wdma;          // panel kernel: stage W by LDS-DMA (set by launch_panel_t)
  int wrot;          // panel kernel: rotate the W DMA order per workgroup (TTMI_PANEL_WROT)
  int nslice, rgroups;   // panel kernel: N split into nslice column panels over rgroups row groups
};

// Sum of the 8 bf16 / 4 f32 operand values a lane holds in one fragment.
template <typename T> TTMI_DEV float frag_sum(const uint4& f);
template <> TTMI_DEV float frag_sum<bf16_t>(const uint4& f) {
  const uint32_t w[4] = {f.x, f.y, f.z, f.w};
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) s += __uint_as_float(w[i] << 16) + __uint_as_float(w[i] & 0xFFFF0000u);
  return s;
}
template <> TTMI_DEV float frag_sum<float>(const uint4& f) {
  return __uint_as_float(f.x) + __uint_as_float(f.y) + __uint_as_float(f.z) + __uint_as_float(f.w);
}

TTMI_DEV uint2 lds8(const char* p) { return *reinterpret_cast<const uint2*>(p); }
TTMI_DEV uint2 lds_tr8(const char* p) {
  const s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4_t*)(p));
  return __builtin_bit_cast(uint2, v);
}

// One operand's K-tile: global -> registers -> LDS, and LDS -> MFMA fragments.
template <typename T, int ROWS, bool KMAJ>
struct Operand {
  static constexpr int E = 16 / sizeof(T);            // elements per 16-byte chunk
  static constexpr int BKE = 128 / sizeof(T);         // k per tile
  static constexpr bool TR = !KMAJ && sizeof(T) == 2; // natural [k][row] image + tr reads
  static constexpr int PITCH = TR ? ROWS * 2 + 32 : 144;
  static constexpr int BYTES = TR ? BKE * PITCH : ROWS * 144;
  static constexpr int PER = ROWS / 32;               // 16-byte chunks per thread
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
        constexpr int CPR = ROWS / E;
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
        *reinterpret_cast<uint4*>(s + (idx >> 3) * PITCH + (idx & 7) * 16) = r[c];
      } else if constexpr (TR) {
        constexpr int CPR = ROWS / E;
        *reinterpret_cast<uint4*>(s + (idx / CPR) * PITCH + (idx % CPR) * 16) = r[c];
      } else {                                         // f32 row-major: transpose on write
        constexpr int CPR = ROWS / E;
        const int kk = idx / CPR;
        const int rr = (idx % CPR) * E;
        const T* v = reinterpret_cast<const T*>(&r[c]);
#pragma unroll
        for (int e = 0; e < E; ++e)
          *reinterpret_cast<T*>(s + (rr + e) * PITCH + kk * (int)sizeof(T)) = v[e];
      }
    }
  }

  // Fragment of the 16-row tile starting at `row0` for 64-byte k-chunk `c`.
  TTMI_DEV uint4 frag(const char* s, int row0, int c, int lane) const {
    const int i = lane & 15, g = lane >> 4;
    if constexpr (sizeof(T) == 4) {
      return lds16(s + (row0 + i) * PITCH + c * 64 + g * 16);
    } else if constexpr (!TR) {
      const char* p = s + (row0 + i) * PITCH + c * 64 + g * 8;
      const uint2 lo = lds8(p), hi = lds8(p + 32);
      return make_uint4(lo.x, lo.y, hi.x, hi.y);
    } else {
      const int q = i >> 2, pp = i & 3;
      const char* p = s + (c * 32 + 4 * g + q) * PITCH + (row0 + 4 * pp) * 2;
      const uint2 lo = lds_tr8(p), hi = lds_tr8(p + 16 * PITCH);
      return make_uint4(lo.x, lo.y, hi.x, hi.y);
    }
  }
};

template <typename T, int BM, int BN, bool AK, bool BKM>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
  using OA = Operand<T, BM, AK>;
  using OB = Operand<T, BN, BKM>;
  constexpr int BKE = 128 / sizeof(T);
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int STAGE = OA::BYTES + OB::BYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

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
  float asum[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) asum[i] = 0.f;
  const bool do_asum = g.rowsum_a != nullptr && wn == 0 && blockIdx.x == 0;   // one N-tile

  OA la;
  OB lb;
  if (kbeg < kend) {
    la.load(g.A, g.lda, m0, g.M, kbeg, kend, tid);
    lb.load(g.B, g.ldb, n0, g.N, kbeg, kend, tid);
    la.store(smem, tid);
    lb.store(smem + OA::BYTES, tid);
  }
  __syncthreads();

  int buf = 0;
  for (int64_t k0 = kbeg; k0 < kend; k0 += BKE) {
    const bool more = k0 + BKE < kend;
    if (more) {
      la.load(g.A, g.lda, m0, g.M, k0 + BKE, kend, tid);
      lb.load(g.B, g.ldb, n0, g.N, k0 + BKE, kend, tid);
    }
    const char* sA = smem + buf * STAGE;
    const char* sB = sA + OA::BYTES;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      uint4 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = la.frag(sA, wm * WTM + i * 16, c, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = lb.frag(sB, wn * WTN + j * 16, c, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) Mma<T>::run(acc[i][j], bfr[j], af[i]);   // Cᵀ tile
      if (do_asum) {
#pragma unroll
        for (int i = 0; i < TM; ++i) asum[i] += frag_sum<T>(af[i]);
      }
    }
    if (more) {
      char* nA = smem + (buf ^ 1) * STAGE;
      la.store(nA, tid);
      lb.store(nA + OA::BYTES, tid);
    }
    __syncthreads();
    buf ^= 1;
  }

  // ------------------------------------------------------------------ epilogue
  // lane holds C[m][n..n+3]: m = tile row + (lane&15), n = tile col + 4*(lane>>4)
  const bool first = blockIdx.z == 0;
  const int li = lane & 15, lg = lane >> 4;
  if (do_asum) {                     // Σ over this split's k of A(m, k): reduce the 4 k-groups
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float v = asum[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int64_t m = m0 + wm * WTM + i * 16 + li;
      if (lg == 0 && m < g.M) atomicAdd(g.rowsum_a + m, v);
    }
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int64_t n = n0 + wn * WTN + j * 16 + 4 * lg;
    float bias[4] = {0.f, 0.f, 0.f, 0.f};
    if (g.bias && first) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bias[e] = (n + e < g.N) ? g.bias[n + e] : 0.f;
    }
    float cs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int64_t m = m0 + wm * WTM + i * 16 + li;
      if (m >= g.M || n >= g.N) continue;
      const bool full = g.vec && (n + 3 < g.N);
      const int64_t drow = g.drop_rows ? (int64_t)g.drop_rows[m] : m;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = g.alpha * acc[i][j][e] + bias[e];
      if (g.pre_out) {
        const int64_t o = m * g.ldc + n;
        if (full) {
          ushort4 q;
          q.x = f2bf(v[0]); q.y = f2bf(v[1]); q.z = f2bf(v[2]); q.w = f2bf(v[3]);
          *reinterpret_cast<ushort4*>(g.pre_out + o) = q;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) if (n + e < g.N) g.pre_out[o + e] = f2bf(v[e]);
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (g.act == 1) v[e] = fmaxf(v[e], 0.f);
        if (g.act == 2) v[e] = gelu_erf(v[e]);
      }
      drop_apply_vec<4>(dk, (uint32_t)(drow * g.ld_drop + n), v);
      if (g.gate) {
        const int64_t o = m * g.ld_gate + n;
        float gv[4];
        if (full && !g.gate_f32) {
          const ushort4 q = *reinterpret_cast<const ushort4*>((const bf16_t*)g.gate + o);
          gv[0] = bf2f(q.x); gv[1] = bf2f(q.y); gv[2] = bf2f(q.z); gv[3] = bf2f(q.w);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) gv[e] = (n + e < g.N) ? ld_dyn(g.gate, o + e, g.gate_f32) : 0.f;
        }
        if (g.act == 3) {                         // GELU backward: gate = pre-activation
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= gelu_erf_grad(gv[e]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = gv[e] > 0.f ? v[e] * g.gate_scale : 0.f;
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) cs[e] += (n + e < g.N) ? v[e] : 0.f;
      if (g.residual && first) {
        const float* rp = g.residual + m * g.ld_res + n;
        if (full) {
          const float4 rv = *reinterpret_cast<const float4*>(rp);
          v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) if (n + e < g.N) v[e] += rp[e];
        }
      }
      const int64_t o = m * g.ldc + n;
      if (g.c_mode == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n + e < g.N) atomicAdd(reinterpret_cast<float*>(g.C) + o + e, v[e]);
      } else if (full && g.c_f32) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(g.C) + o) = make_float4(v[0], v[1], v[2], v[3]);
      } else if (full) {
        ushort4 q;
        q.x = f2bf(v[0]); q.y = f2bf(v[1]); q.z = f2bf(v[2]); q.w = f2bf(v[3]);
        *reinterpret_cast<ushort4*>(reinterpret_cast<bf16_t*>(g.C) + o) = q;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) if (n + e < g.N) st_dyn(g.C, o + e, v[e], g.c_f32);
      }
    }
    if (g.colsum) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float s = cs[e];
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        s += __shfl_xor(s, 8, 64);
        if (li == 0 && n + e < g.N) atomicAdd(g.colsum + n + e, s);
      }
    }
  }
}


template <int N_>
TTMI_DEV void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory"); }

// ------------------------------------------------ row-panel GEMM (skinny K, whole N per WG)
// C[m, :] = epi(alpha * A[m, :K] · Wᵀ) for M >> N with N in {128,..,512}, K <= 512, both
// operands k-major (nn.Linear forward; input grads through a transposed weight mirror).
// The generic tile kernel pays two serial K-tile load latencies per 128x128 tile here and
// reaches ~1 TB/s.  Instead (measured on MI355X against hipBLASLt, tools/gemm_variants.py):
//  * W is stationary in LDS (N x K, pitch 2K+16 so the 16 rows a ds_read_b128 lane group
//    reads fall in distinct bank slots), loaded once per CU; the bias row sits beside it;
//  * 8 waves per workgroup each own whole 16-row tiles across all N columns (column groups
//    of 128 bound the live state); two waves per SIMD hide each other's latency and nothing
//    synchronises after the W load;
//  * k is permuted so every fragment is a contiguous 16-byte read: lane group g of chunk c
//    holds k = g*K/4 + 8c .. +7 on both operands, so A fragments come straight from HBM
//    into VGPRs (each A row read once), the first tile's under the W load;
//  * W fragment columns are paired (tile 2p slot 4q+r <-> column 32p+8q+r, tile 2p+1 <->
//    32p+8q+4+r), so each lane owns 8 consecutive output columns: 16-byte stores and
//    16-byte bias / gate / residual loads; dropout hashes once per column pair.
enum PanelEpi { PE_NONE = 0, PE_RES = 1, PE_GATE_BF16 = 2, PE_GATE_F32 = 3, PE_LNBWD = 4, PE_RESLN = 5 };

// PE_LNBWD: the GEMM output dY (N = 128 = LayerNorm width, never stored) feeds the
// LayerNorm backward of the rows it completes:
//   xh = (x - mean) * rstd,  g = dY * w,  dx = rstd * (g - mean(g) - xh * mean(g * xh)) + res,
//   dw += Σ_rows dY * xh,  db += Σ_rows dY,  next = bf16(dropout(dx))  (optional),
// i.e. ttmi_layernorm_bwd + ttmi_dropout_bwd fused into the input-grad GEMM.
struct LnBwdArgs {
  const float* x; int64_t ldx;
  const float* mean; const float* rstd; const float* w;
  const float* res; int64_t ld_res;
  const int32_t* res_rows; int64_t res_L;   // res row b feeds row res_rows[b] (b = m / res_L) only
  const float* dy_add; int64_t ld_add;      // row b added to dY of row res_rows[b] (before the LN)
  float* dx; int64_t lddx;
  bf16_t* next; int64_t ld_next;
  DropParams drop; int64_t ld_drop; const int32_t* drop_rows;
  float* dw; float* db;
  float* sum_ws;   // non-NULL: per-workgroup dw / db sums to sum_ws[blockIdx][2][N] (no atomics)
  // PE_RESLN (forward): y = LN(C row) * w + lnb -> bf16 y, per-row mean / rstd
  const float* lnb; float eps; bf16_t* y; int64_t ldy; float* mean_out; float* rstd_out;
};

// Sum over the 16 lanes of a DPP row (GFX9 quad_perm / row_half_mirror / row_mirror).
template <int CTRL>
TTMI_DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
TTMI_DEV float row16_sum(float v) {
  v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);   // row_half_mirror
  v += dpp_f<0x140>(v);   // row_mirror
  return v;
}


// The LayerNorm-backward epilogue's row operands (x, residual, mean, rstd), loaded at the
// start of the tile so their latency hides under the MFMAs (rows clamped: unconditional).
struct LnBwdRow {
  float4 x[8];
  float4 r[8];
  float4 a[8];              // dy_add's row (zero unless this is the gathered row)
  float mu, rs;
};

TTMI_DEV void panel_ln_bwd_load(const LnBwdArgs& ln, int64_t m, int64_t M, int lg, LnBwdRow& o) {
  const int64_t mc = std::min<int64_t>(m, M - 1);
  o.mu = ln.mean[mc];
  o.rs = ln.rstd[mc];
  // gathered residual: row b = m / res_L of res, added only at row res_rows[b] (the pruned
  // layer's last-valid rows); the select follows the unconditional clamped load
  int64_t rr = mc;
  bool rhit = true;
  if (ln.res_rows) {
    rr = mc / ln.res_L;
    rhit = (int64_t)ln.res_rows[rr] == mc;
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int n = 32 * p + 8 * lg;
    o.x[2 * p] = *reinterpret_cast<const float4*>(ln.x + mc * ln.ldx + n);
    o.x[2 * p + 1] = *reinterpret_cast<const float4*>(ln.x + mc * ln.ldx + n + 4);
    if (ln.res) {
      o.r[2 * p] = *reinterpret_cast<const float4*>(ln.res + rr * ln.ld_res + n);
      o.r[2 * p + 1] = *reinterpret_cast<const float4*>(ln.res + rr * ln.ld_res + n + 4);
    }
  }
  if (ln.res && !rhit) {
#pragma unroll
    for (int q = 0; q < 8; ++q) o.r[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (ln.dy_add) {          // (the launcher requires res_rows with it)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int n = 32 * p + 8 * lg;
      o.a[2 * p] = *reinterpret_cast<const float4*>(ln.dy_add + rr * ln.ld_add + n);
      o.a[2 * p + 1] = *reinterpret_cast<const float4*>(ln.dy_add + rr * ln.ld_add + n + 4);
    }
    if (!rhit) {
#pragma unroll
      for (int q = 0; q < 8; ++q) o.a[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// LayerNorm-backward epilogue of one 16-row tile (N = 128): lane (li, lg) holds row li,
// columns 32p + 8lg + e (p < 4, e < 8) of dY in acc (column-paired tiles 2p, 2p+1).
TTMI_DEV void panel_ln_bwd_epilogue(const GemmArgs& g, const LnBwdArgs& ln, const f32x4_t (&acc)[8],
                                    int64_t m, bool mok, int li, int lg, const float* sw,
                                    float* sdw, float* sdb, const DropKeys& dk2,
                                    const LnBwdRow& pre) {
  const float mu = mok ? pre.mu : 0.f, rs = mok ? pre.rs : 0.f;
  float dy[32], xh[32];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int n = 32 * p + 8 * lg;
    float xr[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (mok) {
      const float4 x0 = pre.x[2 * p], x1 = pre.x[2 * p + 1];
      xr[0] = x0.x; xr[1] = x0.y; xr[2] = x0.z; xr[3] = x0.w;
      xr[4] = x1.x; xr[5] = x1.y; xr[6] = x1.z; xr[7] = x1.w;
    }
    float ad[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (ln.dy_add) {
      const float4 a0 = pre.a[2 * p], a1 = pre.a[2 * p + 1];
      ad[0] = a0.x; ad[1] = a0.y; ad[2] = a0.z; ad[3] = a0.w;
      ad[4] = a1.x; ad[5] = a1.y; ad[6] = a1.z; ad[7] = a1.w;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float d = mok ? g.alpha * (e < 4 ? acc[2 * p][e] : acc[2 * p + 1][e - 4]) : 0.f;
      if (ln.dy_add && mok) d += ad[e];
      const float h = (xr[e] - mu) * rs;
      const float gg = d * sw[n + e];
      dy[8 * p + e] = d;
      xh[8 * p + e] = h;
      s1 += gg;
      s2 += gg * h;
    }
  }
  // the row's 128 columns live in the 4 lanes li, li+16, li+32, li+48
  s1 += __shfl_xor(s1, 16, 64);
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 16, 64);
  s2 += __shfl_xor(s2, 32, 64);
  const float c1 = s1 * (1.f / 128.f), c2 = s2 * (1.f / 128.f);
  if (mok) {
    const int64_t drow = ln.drop_rows ? (int64_t)ln.drop_rows[m] : m;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int n = 32 * p + 8 * lg;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = rs * (dy[8 * p + e] * sw[n + e] - c1 - xh[8 * p + e] * c2);
      if (ln.res) {
        const float4 r0 = pre.r[2 * p], r1 = pre.r[2 * p + 1];
        o[0] += r0.x; o[1] += r0.y; o[2] += r0.z; o[3] += r0.w;
        o[4] += r1.x; o[5] += r1.y; o[6] += r1.z; o[7] += r1.w;
      }
      float* dp = ln.dx + m * ln.lddx + n;
      *reinterpret_cast<float4*>(dp) = make_float4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<float4*>(dp + 4) = make_float4(o[4], o[5], o[6], o[7]);
      if (ln.next) {
        drop_apply_vec<8>(dk2, (uint32_t)(drow * ln.ld_drop + n), o);
        uint4 q;
        q.x = pk_bf2(o[0], o[1]);
        q.y = pk_bf2(o[2], o[3]);
        q.z = pk_bf2(o[4], o[5]);
        q.w = pk_bf2(o[6], o[7]);
        *reinterpret_cast<uint4*>(ln.next + m * ln.ld_next + n) = q;
      }
    }
  }
  // dw / db: sum the tile's 16 rows (one DPP row) into this wave's own LDS row (sdw / sdb
  // point at it): one adder per column, tiles in the wave's program order (deterministic;
  // the waves' rows are summed in wave order at the end)
#pragma unroll
  for (int p = 0; p < 4; ++p) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float a = row16_sum(dy[8 * p + e] * xh[8 * p + e]);
      const float b = row16_sum(dy[8 * p + e]);
      if (li == 0) {          // ds_add on the wave's own row: program order, no read stall
        atomicAdd(sdw + 32 * p + 8 * lg + e, a);
        atomicAdd(sdb + 32 * p + 8 * lg + e, b);
      }
    }
  }
}

template <int NT, int KC, int EPI, int CS>
__global__ __launch_bounds__(512 * CS) void panel_kernel(GemmArgs g, int tiles_per_wg, LnBwdArgs ln) {
  constexpr int K = KC * 32, N = NT * 16, WP = 2 * K + 16;
  constexpr bool LNB = EPI == PE_LNBWD, LNF = EPI == PE_RESLN;
  static_assert(NT % 8 == 0, "column groups of 128");
  static_assert(!(LNB || LNF) || NT == 8, "LayerNorm epilogues need N = 128");
  // CS = 2: 16 waves, a pair per row tile, each wave one half of the column groups (twice the
  // waves per SIMD to hide latency; the LayerNorm epilogues need whole rows: CS = 1)
  static_assert(CS == 1 || ((NT / 8) % CS == 0 && !(LNB || LNF)), "column split");
  constexpr int NTH = 512 * CS, CGW = NT / 8 / CS;
  constexpr int SROWS = LNB ? 8 : 1;                            // LNB: one row per wave
  __shared__ __attribute__((aligned(16))) char smem[N * WP + N * 4 + ((LNB || LNF) ? 2 * SROWS * N * 4 : 0)];
  float* sbias = reinterpret_cast<float*>(smem + N * WP);     // bias, or the LN weight
  float* sdw = sbias + N;                                       // LNB: per-wave dw / db sums
  float* sdb = sdw + SROWS * N;                                 // LNF: LN weight / bias
  TTMI_TSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rwave = wave / CS, cg0 = (wave % CS) * CGW;      // row-tile slot, first column group
  const int li = lane & 15, lg = lane >> 4;
  // column slices (g.nslice > 1: the output is nslice panels of N columns, one per workgroup;
  // the slices of one row group sit on one XCD, consecutive, so its A rows are read from HBM
  // once and from that XCD's L2 after)
  int rg = blockIdx.x, dn0 = 0;
  if (!(LNB || LNF) && g.nslice > 1) {
    const int k = blockIdx.x / 8, sl = k % g.nslice;
    rg = (k / g.nslice) * 8 + blockIdx.x % 8;
    if (rg >= g.rgroups) return;                                  // grid padding (uniform)
    dn0 = sl * N;
    g.B += (int64_t)dn0 * g.ldb * 2;
    g.C = static_cast<char*>(g.C) + (int64_t)dn0 * (g.c_f32 ? 4 : 2);
    if (g.bias) g.bias += dn0;
    if (g.gate) g.gate = static_cast<const char*>(g.gate) + (int64_t)dn0 * (g.gate_f32 ? 4 : 2);
    if (g.residual) g.residual += dn0;
  }
  const int64_t tile_beg = (int64_t)rg * tiles_per_wg;
  const int64_t tile_end = std::min<int64_t>((g.M + 15) / 16, tile_beg + tiles_per_wg);
  const int64_t tile0 = tile_beg + rwave;
  // A fragments.  K <= 256 (AFULL): the wave's whole first tile of A (16 rows x K: KC 16-byte
  // fragments per lane) is loaded BEFORE the W staging and stays in registers across the column
  // groups (QKV 11.7 -> 10.7 us, FFN1 15.6 -> ~14.5 us in the cfg-2 step).  K >= 384: one k group
  // (4 fragments) in flight ahead of the MFMAs; loading the whole A row up front there measured
  // slower (FFN1 dgrad + LN 21.0 -> 22.4 us): the extra 16 KB per wave competes with the W image
  // for the CU's ingest and the MFMA phase stays LDS / issue bound (tools/stamp_phases.py).
  constexpr bool AFULL = KC <= 8;
  constexpr int AR = AFULL ? KC : 4;
  uint4 af[AR];
  auto load_af = [&](int64_t tile) {   // rows clamped into range: unconditional loads
    const int64_t m = std::min<int64_t>(tile * 16 + li, g.M - 1);
    const char* ap = g.A + (m * g.lda + lg * (K / 4)) * 2;
#pragma unroll
    for (int c = 0; c < AR; ++c) af[c] = *reinterpret_cast<const uint4*>(ap + 16 * c);
  };
  load_af(tile0);
  if (g.wdma) {
    // W -> LDS by LDS-DMA, every chunk in flight at once (no VGPR round trip): the image is
    // a run of 16-byte chunks, K/8 + 1 per row (the last one is the row pad, filled with the
    // buffer's out-of-range zeros); wave-instruction ii writes chunks [64 ii, 64 ii + 64)
    constexpr int CPRP = K / 8 + 1, INSTR = N * CPRP / 64;
    static_assert((N * CPRP) % 64 == 0, "whole DMA instructions");
    const uint32_t wbytes = (uint32_t)(((int64_t)(N - 1) * g.ldb + K) * 2);
    const i32x4_t rw = make_rsrc(g.B, wbytes);
    const uint32_t base = lds_addr(smem);
    // every workgroup fetches the same image: start each at its own point of it (a rotation
    // of the instruction order) so the CUs of an XCD do not queue on the same L2 channel
    const int rot = g.wrot ? (int)((blockIdx.x * 5u + blockIdx.x / 8u) % INSTR) : 0;
#pragma unroll
    for (int t = 0; t < (INSTR + 8 * CS - 1) / (8 * CS); ++t) {
      const int i0 = wave + 8 * CS * t;
      if (i0 >= INSTR) break;                   // wave-uniform
      const int ii = i0 + rot < INSTR ? i0 + rot : i0 + rot - INSTR;
      const int q = ii * 64 + lane, n = q / CPRP, c = q % CPRP;
      const uint32_t voff = c == K / 8 ? wbytes : (uint32_t)(((int64_t)n * g.ldb + 8 * c) * 2);
      dma16(rw, voff, base + ii * 1024);
    }
  } else {   // W -> LDS, coalesced 16-byte chunks, 8 loads in flight per thread before the LDS
      // writes (a load -> wait -> write loop pays one memory round trip per chunk: 16 round
      // trips for a 128 KB W image, which used to be most of the kernel's time)
    constexpr int CPR = K / 8, TOT = N * CPR, PER = (TOT + NTH - 1) / NTH, BATCH = PER <= 16 ? PER : 8;
#pragma unroll
    for (int j0 = 0; j0 < PER; j0 += BATCH) {
      uint4 wv[BATCH];
#pragma unroll
      for (int j = 0; j < BATCH; ++j) {
        if (j0 + j < PER) {            // compile-time; the chunk index is clamped, not branched
          const int i = min(tid + NTH * (j0 + j), TOT - 1);    // (a branch here spilled wv)
          const int n = i / CPR, c = i % CPR;
          wv[j] = *reinterpret_cast<const uint4*>(g.B + ((int64_t)n * g.ldb + 8 * c) * 2);
        }
      }
#pragma unroll
      for (int j = 0; j < BATCH; ++j) {
        const int i = tid + NTH * (j0 + j);
        if (j0 + j < PER && i < TOT) {
          const int n = i / CPR, c = i % CPR;
          *reinterpret_cast<uint4*>(smem + n * WP + c * 16) = wv[j];
        }
      }
    }
  }
  {
    if constexpr (LNB) {
      for (int i = tid; i < N; i += NTH) sbias[i] = ln.w[i];
      for (int i = tid; i < SROWS * N; i += NTH) { sdw[i] = 0.f; sdb[i] = 0.f; }
    } else if constexpr (LNF) {
      for (int i = tid; i < N; i += NTH) {
        sbias[i] = g.bias ? g.bias[i] : 0.f;
        sdw[i] = ln.w[i];
        sdb[i] = ln.lnb[i];
      }
    } else {
      for (int i = tid; i < N; i += NTH) sbias[i] = g.bias ? g.bias[i] : 0.f;
    }
  }
  const DropKeys dk = resolve_drop(g.drop);
  const DropKeys dk2 = resolve_drop(ln.drop);
  TTMI_TSTAMP(1);
  if (g.wdma) wait_vm<0>();          // this wave's W DMAs landed (the barrier covers the rest)
  __syncthreads();
  TTMI_TSTAMP(2);
  bool first_tile = true;

  // W fragment base for this lane (column-paired: tile 2p slot 4q+r <-> column 32p+8q+r)
  const int wrow = 8 * (li >> 2) + (li & 3);
  for (int64_t tile = tile_beg + rwave; tile < tile_end; tile += 8) {
    const int64_t m = tile * 16 + li;
    const bool mok = m < g.M;
    const char* ap = g.A + (std::min<int64_t>(m, g.M - 1) * g.lda + lg * (K / 4)) * 2;
    // the next tile's rows (clamped: past the last tile the prefetch is a harmless re-load)
    const char* ap_next = g.A + (std::min<int64_t>(m + 128, g.M - 1) * g.lda + lg * (K / 4)) * 2;
    if (AFULL && !first_tile) load_af(tile);   // (one tile per wave at M = 25,600)
    // column groups of 128 (8 MFMA tiles) keep the accumulator and W fragment state bounded
#pragma unroll 1
    for (int cg = cg0; cg < cg0 + CGW; ++cg) {
      f32x4_t acc[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const char* wb = smem + (cg * 128 + wrow) * WP + lg * (K / 2);
      LnBwdRow pre;
      if constexpr (LNB) panel_ln_bwd_load(ln, m, g.M, lg, pre);
      // the epilogue's other row operands (the residual rows, the ReLU / dropout gate) are
      // loaded before the MFMAs too: read in the epilogue they were one more memory round trip
      // after the last MFMA of every tile (rows clamped: unconditional loads)
      constexpr bool RPRE = EPI == PE_RES || LNF, GPRE = EPI == PE_GATE_BF16;
      float4 rpre[RPRE ? 8 : 1];
      uint4 gpre[GPRE ? 4 : 1];
      {
        const int64_t mcl = std::min<int64_t>(m, g.M - 1);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int n = cg * 128 + 32 * p + 8 * lg;
          if constexpr (RPRE) {
            const float* rp = g.residual + mcl * g.ld_res + n;
            rpre[2 * p] = *reinterpret_cast<const float4*>(rp);
            rpre[2 * p + 1] = *reinterpret_cast<const float4*>(rp + 4);
          }
          if constexpr (GPRE) gpre[p] = *reinterpret_cast<const uint4*>((const bf16_t*)g.gate + mcl * g.ld_gate + n);
        }
      }
      if constexpr (AFULL) {
#pragma unroll
        for (int cq = 0; cq < KC / 4; ++cq) {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const uint4 wf = lds16(wb + (32 * (t >> 1) + 4 * (t & 1)) * WP + 64 * cq + 16 * c);
              Mma<bf16_t>::run(acc[t], wf, af[4 * cq + c]);
            }
            // bound the scheduler's window to one 16-byte k chunk: hoisting every W fragment
            // read of the unrolled loop ahead of the MFMAs spilled
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      } else {
        // k groups of 4 fragments, the next group's (or the next column group's / next tile's
        // first group's) loads in flight under this group's MFMAs
#pragma unroll 1
        for (int cq = 0; cq < KC / 4; ++cq) {
          uint4 an[4];
          const char* src = cq + 1 < KC / 4 ? ap + 64 * (cq + 1) : (cg + 1 < cg0 + CGW ? ap : ap_next);
#pragma unroll
          for (int c = 0; c < 4; ++c) an[c] = *reinterpret_cast<const uint4*>(src + 16 * c);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const uint4 wf = lds16(wb + (32 * (t >> 1) + 4 * (t & 1)) * WP + 64 * cq + 16 * c);
              Mma<bf16_t>::run(acc[t], wf, af[c]);
            }
          }
#pragma unroll
          for (int c = 0; c < 4; ++c) af[c] = an[c];
        }
      }
      if (first_tile && cg == cg0) TTMI_TSTAMP(3);
      if constexpr (LNB) {
        panel_ln_bwd_epilogue(g, ln, acc, m, mok, li, lg, sbias, sdw + wave * N, sdb + wave * N, dk2, pre);
        continue;
      }
      if (!mok) continue;
      float vr[LNF ? 32 : 1];                     // LNF: the lane's 32 values of row m
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int n = cg * 128 + 32 * p + 8 * lg;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = g.alpha * acc[2 * p][e] + sbias[n + e];
          v[4 + e] = g.alpha * acc[2 * p + 1][e] + sbias[n + 4 + e];
        }
        if (g.act == 1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        drop_apply_vec<8>(dk, (uint32_t)(m * g.ld_drop + dn0 + n), v);
        if constexpr (EPI == PE_GATE_BF16) {
          const uint4 q = gpre[p];
          const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] = __uint_as_float(qw[e] << 16) > 0.f ? v[2 * e] * g.gate_scale : 0.f;
            v[2 * e + 1] = __uint_as_float(qw[e] & 0xFFFF0000u) > 0.f ? v[2 * e + 1] * g.gate_scale : 0.f;
          }
        }
        if constexpr (EPI == PE_GATE_F32) {
          const float* gp = (const float*)g.gate + m * g.ld_gate + n;
          const float4 q0 = *reinterpret_cast<const float4*>(gp), q1 = *reinterpret_cast<const float4*>(gp + 4);
          const float gv[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gv[e] > 0.f ? v[e] * g.gate_scale : 0.f;
        }
        if constexpr (EPI == PE_RES || LNF) {
          const float4 r0 = rpre[2 * p], r1 = rpre[2 * p + 1];
          v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w;
          v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
        }
        if (g.c_f32) {
          float* cp = reinterpret_cast<float*>(g.C) + m * g.ldc + n;
          *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
        } else {
          uint4 q;
          q.x = pk_bf2(v[0], v[1]);
          q.y = pk_bf2(v[2], v[3]);
          q.z = pk_bf2(v[4], v[5]);
          q.w = pk_bf2(v[6], v[7]);
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(g.C) + m * g.ldc + n) = q;
        }
        if constexpr (LNF) {
#pragma unroll
          for (int e = 0; e < 8; ++e) vr[8 * p + e] = v[e];
        }
      }
      if constexpr (LNF) {   // LayerNorm of the finished row: its 128 columns live in lanes
        float s1 = 0.f;      // li, li+16, li+32, li+48 (two-pass mean / variance, as ln_fwd)
#pragma unroll
        for (int e = 0; e < 32; ++e) s1 += vr[e];
        s1 += __shfl_xor(s1, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        const float mu = s1 * (1.f / 128.f);
        float s2 = 0.f;
#pragma unroll
        for (int e = 0; e < 32; ++e) s2 += (vr[e] - mu) * (vr[e] - mu);
        s2 += __shfl_xor(s2, 16, 64);
        s2 += __shfl_xor(s2, 32, 64);
        const float rs = 1.f / sqrtf(s2 * (1.f / 128.f) + ln.eps);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int n = 32 * p + 8 * lg;
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (vr[8 * p + e] - mu) * rs * sdw[n + e] + sdb[n + e];
          uint4 q;
          q.x = pk_bf2(o[0], o[1]);
          q.y = pk_bf2(o[2], o[3]);
          q.z = pk_bf2(o[4], o[5]);
          q.w = pk_bf2(o[6], o[7]);
          *reinterpret_cast<uint4*>(ln.y + m * ln.ldy + n) = q;
        }
        if (lg == 0) {
          ln.mean_out[m] = mu;
          ln.rstd_out[m] = rs;
        }
      }
    }
    if (first_tile) TTMI_TSTAMP(4);
    first_tile = false;
  }
  TTMI_TSTAMP(5);
  if constexpr (LNB) {
    __syncthreads();
    for (int i = tid; i < N; i += NTH) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w = 0; w < SROWS; ++w) { a += sdw[w * N + i]; b += sdb[w * N + i]; }
      if (ln.sum_ws) {          // deterministic: folded later in workgroup order (ttmi_fold)
        float* o = ln.sum_ws + (int64_t)blockIdx.x * 2 * N;
        o[i] = a;
        o[N + i] = b;
      } else {                  // legacy ABI callers without a workspace: float atomics
        if (ln.dw) atomicAdd(ln.dw + i, a);
        if (ln.db) atomicAdd(ln.db + i, b);
      }
    }
  }
  TTMI_TSTAMP(6);
}

// ------------------------------------- N = 256 LayerNorm-epilogue panels, W and A streamed
// The D = 256 encoder (the reference's default width, user_tower.py:9) ends its residual
// sub-blocks with GEMMs of N = 256 columns and K up to 1,024 (FFN2 forward; the QKV and FFN1
// input grads), whose W image (up to 512 KB) does not fit in LDS.  Here:
//  * 8 waves, one 16-row tile each (one tile group per workgroup: tiles_per_wg <= 8);
//  * W and A stream through 3-slot LDS rings of 64-wide k chunks by LDS-DMA (W 256 rows x
//    128 B, A 8 waves x 16 rows x 128 B per chunk), two chunks in flight under the MFMAs and
//    one barrier per chunk.  Everything in the loop is DMA: no compiler-visible global load,
//    so hipcc inserts no vmcnt(0) that would drain the ring (the counts are explicit);
//  * both images are unpadded with the 16-byte pieces of row r XOR-swizzled by
//    swz(r) = ((r >> 1) ^ r) & 7 (on the DMA source: the destination is lane-linear), which
//    puts the 16 rows each ds_read_b128 lane group reads into distinct bank windows for the
//    A tile and for every W column tile of the column-paired layout;
//  * k order: lane group g of chunk ch holds k = 64 ch + 16 g + 8 c .. +7 (c < 2) of both
//    operands; output layout and epilogues as the N = 128 panel over two column groups, the
//    LayerNorm statistics over 256 columns (residual + LayerNorm forward, PE_RESLN; the
//    LayerNorm backward, PE_LNBWD, its per-wave dw / db rows in a drained W slot).
TTMI_DEV int swz8(int r) { return ((r >> 1) ^ r) & 7; }

template <int KCH, int EPI>
__global__ __launch_bounds__(512) void panel256_kernel(GemmArgs g, int tiles_per_wg, LnBwdArgs ln) {
  constexpr int N = 256, KW = 64, K = KW * KCH;
  constexpr int WSLOT = N * KW * 2, ASLOT = 8 * 16 * KW * 2;      // 32 KB, 16 KB
  constexpr int WI = WSLOT / 1024 / 8, AI = 2;                     // DMA instructions per wave
  constexpr bool LNB = EPI == PE_LNBWD;
  static_assert(EPI == PE_LNBWD || EPI == PE_RESLN, "LayerNorm epilogues only");
  static_assert(KCH >= 2, "K >= 128");
  __shared__ __attribute__((aligned(16))) char smem[3 * WSLOT + 3 * ASLOT + 3 * N * 4];
  float* sw = reinterpret_cast<float*>(smem + 3 * WSLOT + 3 * ASLOT);   // bias (RESLN) / LN w (LNBWD)
  float* slw = sw + N;                                                // RESLN: LN weight, bias
  float* slb = slw + N;
  TTMI_TSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const int64_t tiles = (g.M + 15) / 16;
  const int64_t tile_beg = (int64_t)blockIdx.x * tiles_per_wg;
  const int64_t tile_end = std::min<int64_t>(tiles, tile_beg + tiles_per_wg);
  const int64_t tile = tile_beg + wave;
  const int64_t m = tile * 16 + li;
  const bool mok = tile < tile_end && m < g.M;
  const int64_t mc = std::min<int64_t>(m, g.M - 1);
  // ---- DMA sources
  const i32x4_t rw = make_rsrc(g.B, (uint32_t)(((int64_t)(N - 1) * g.ldb + K) * 2));
  const i32x4_t ra = make_rsrc(g.A, (uint32_t)(g.M * g.lda * 2));
  const uint32_t wbase = lds_addr(smem), abase = wbase + 3 * WSLOT + wave * (ASLOT / 8);
  // every workgroup streams the same W: each starts at its own point of the chunk
  const int rot = g.wrot ? (int)((blockIdx.x * 5u + blockIdx.x / 8u) % (WI * 8)) : 0;
  uint32_t woff[WI], aoff[AI];        // chunk-0 source offsets; chunk ch adds 128 ch bytes
#pragma unroll
  for (int u = 0; u < WI; ++u) {
    int ii = wave + 8 * u + rot;
    ii = ii < WI * 8 ? ii : ii - WI * 8;
    const int n = ii * 8 + (lane >> 3), q = (lane & 7) ^ swz8(n);
    woff[u] = (uint32_t)(((int64_t)n * g.ldb + 8 * q) * 2);
  }
#pragma unroll
  for (int u = 0; u < AI; ++u) {      // the wave's 16 rows (clamped) of A
    const int r = u * 8 + (lane >> 3), q = (lane & 7) ^ swz8(r);
    const int64_t row = std::min<int64_t>(tile * 16 + r, g.M - 1);
    aoff[u] = (uint32_t)((row * g.lda + 8 * q) * 2);
  }
  auto stage = [&](int ch, int slot) {
#pragma unroll
    for (int u = 0; u < WI; ++u) {
      int ii = wave + 8 * u + rot;
      ii = ii < WI * 8 ? ii : ii - WI * 8;
      dma16(rw, woff[u] + ch * KW * 2, wbase + slot * WSLOT + ii * 1024);
    }
#pragma unroll
    for (int u = 0; u < AI; ++u) dma16(ra, aoff[u] + ch * KW * 2, abase + slot * ASLOT + u * 1024);
  };
  // the per-column parameters (1 KB each) by DMA too, ahead of chunk 0 (a compiler-visible
  // load here would make hipcc drain every DMA before its LDS store); a null bias reads zeros
  if (wave < (LNB ? 1 : 3)) {
    const float* src = LNB ? ln.w : wave == 0 ? g.bias : wave == 1 ? ln.w : ln.lnb;
    dma16(make_rsrc(src, src ? N * 4 : 0), lane * 16, lds_addr(sw + wave * N));
  }
  stage(0, 0);
  stage(1, 1);
  TTMI_TSTAMP(1);
  // W fragment: column tile t of group cg at row n = 128 cg + 32 (t >> 1) + 4 (t & 1) + wrow;
  // swz8(n) depends on n & 15 only, i.e. on t & 1 and the lane
  const int wrow = 8 * (li >> 2) + (li & 3);
  const int key[2] = {swz8(wrow), swz8(wrow + 4)};
  const int akey = swz8(li);
  f32x4_t acc[2][8];
#pragma unroll
  for (int cg = 0; cg < 2; ++cg)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[cg][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ch = 0; ch < KCH; ++ch) {
    // this wave's chunk-ch pieces landed (ch + 1's in flight) and its LDS reads returned, then
    // the barrier: everyone's chunk ch landed, everyone is done with ch - 1 (one asm statement,
    // not __syncthreads, whose release fence would drain vmcnt to 0)
    if (ch + 1 < KCH) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(WI + AI) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (ch + 2 < KCH) stage(ch + 2, (ch + 2) % 3);
    const char* ws = smem + (ch % 3) * WSLOT;
    const char* as = smem + 3 * WSLOT + (ch % 3) * ASLOT + wave * (ASLOT / 8) + li * (KW * 2);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int q = 2 * lg + c;
      const uint4 a = lds16(as + ((q ^ akey) << 4));
#pragma unroll
      for (int cg = 0; cg < 2; ++cg) {
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int n = 128 * cg + 32 * (t >> 1) + 4 * (t & 1) + wrow;
          const uint4 wf = lds16(ws + n * (KW * 2) + ((q ^ key[t & 1]) << 4));
          Mma<bf16_t>::run(acc[cg][t], wf, a);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  TTMI_TSTAMP(2);
  // ---- epilogues: lane (li, lg) holds row li, columns 128 cg + 32 p + 8 lg + e
  const DropKeys dk = resolve_drop(g.drop);
  const DropKeys dk2 = resolve_drop(ln.drop);
  if constexpr (!LNB) {
    float vr[64];
#pragma unroll
    for (int cg = 0; cg < 2; ++cg) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int n = 128 * cg + 32 * p + 8 * lg;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = g.alpha * acc[cg][2 * p][e] + sw[n + e];
          v[4 + e] = g.alpha * acc[cg][2 * p + 1][e] + sw[n + 4 + e];
        }
        drop_apply_vec<8>(dk, (uint32_t)(m * g.ld_drop + n), v);
        const float* rp = g.residual + mc * g.ld_res + n;
        const float4 r0 = *reinterpret_cast<const float4*>(rp), r1 = *reinterpret_cast<const float4*>(rp + 4);
        v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w;
        v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
        if (mok) {
          float* cp = reinterpret_cast<float*>(g.C) + m * g.ldc + n;
          *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) vr[32 * cg + 8 * p + e] = v[e];
      }
    }
    float s1 = 0.f;                    // two-pass mean / variance over the 256 columns (ln_fwd)
#pragma unroll
    for (int e = 0; e < 64; ++e) s1 += vr[e];
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    const float mu = s1 * (1.f / 256.f);
    float s2 = 0.f;
#pragma unroll
    for (int e = 0; e < 64; ++e) s2 += (vr[e] - mu) * (vr[e] - mu);
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    const float rs = 1.f / sqrtf(s2 * (1.f / 256.f) + ln.eps);
    if (mok) {
#pragma unroll
      for (int cg = 0; cg < 2; ++cg) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int n = 128 * cg + 32 * p + 8 * lg;
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (vr[32 * cg + 8 * p + e] - mu) * rs * slw[n + e] + slb[n + e];
          uint4 qv;
          qv.x = pk_bf2(o[0], o[1]);
          qv.y = pk_bf2(o[2], o[3]);
          qv.z = pk_bf2(o[4], o[5]);
          qv.w = pk_bf2(o[6], o[7]);
          *reinterpret_cast<uint4*>(ln.y + m * ln.ldy + n) = qv;
        }
      }
      if (lg == 0) {
        ln.mean_out[m] = mu;
        ln.rstd_out[m] = rs;
      }
    }
  } else {
    const float mu = mok ? ln.mean[mc] : 0.f, rs = mok ? ln.rstd[mc] : 0.f;
    int64_t rr = mc;
    bool rhit = ln.res != nullptr;
    if (ln.res && ln.res_rows) {
      rr = mc / ln.res_L;
      rhit = (int64_t)ln.res_rows[rr] == mc;
    }
    float dy[64], xh[64];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int cg = 0; cg < 2; ++cg) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int n = 128 * cg + 32 * p + 8 * lg;
        const float4 x0 = *reinterpret_cast<const float4*>(ln.x + mc * ln.ldx + n);
        const float4 x1 = *reinterpret_cast<const float4*>(ln.x + mc * ln.ldx + n + 4);
        const float xr[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = mok ? g.alpha * (e < 4 ? acc[cg][2 * p][e] : acc[cg][2 * p + 1][e - 4]) : 0.f;
          const float h = mok ? (xr[e] - mu) * rs : 0.f;
          const float gg = d * sw[n + e];
          dy[32 * cg + 8 * p + e] = d;
          xh[32 * cg + 8 * p + e] = h;
          s1 += gg;
          s2 += gg * h;
        }
      }
    }
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    const float c1 = s1 * (1.f / 256.f), c2 = s2 * (1.f / 256.f);
    const int64_t drow = ln.drop_rows ? (int64_t)ln.drop_rows[mc] : m;
#pragma unroll
    for (int cg = 0; cg < 2; ++cg) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int n = 128 * cg + 32 * p + 8 * lg;
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          o[e] = rs * (dy[32 * cg + 8 * p + e] * sw[n + e] - c1 - xh[32 * cg + 8 * p + e] * c2);
        if (ln.res) {
          const float4 r0 = *reinterpret_cast<const float4*>(ln.res + rr * ln.ld_res + n);
          const float4 r1 = *reinterpret_cast<const float4*>(ln.res + rr * ln.ld_res + n + 4);
          if (rhit) {
            o[0] += r0.x; o[1] += r0.y; o[2] += r0.z; o[3] += r0.w;
            o[4] += r1.x; o[5] += r1.y; o[6] += r1.z; o[7] += r1.w;
          }
        }
        if (mok) {
          float* dp = ln.dx + m * ln.lddx + n;
          *reinterpret_cast<float4*>(dp) = make_float4(o[0], o[1], o[2], o[3]);
          *reinterpret_cast<float4*>(dp + 4) = make_float4(o[4], o[5], o[6], o[7]);
          if (ln.next) {
            drop_apply_vec<8>(dk2, (uint32_t)(drow * ln.ld_drop + n), o);
            uint4 qv;
            qv.x = pk_bf2(o[0], o[1]);
            qv.y = pk_bf2(o[2], o[3]);
            qv.z = pk_bf2(o[4], o[5]);
            qv.w = pk_bf2(o[6], o[7]);
            *reinterpret_cast<uint4*>(ln.next + m * ln.ld_next + n) = qv;
          }
        }
      }
    }
    // dw / db: the tile's 16 rows summed per column (one DPP row), stored into this wave's
    // own row of a drained W slot (the last iteration's barrier retired every read of it),
    // then the waves' rows summed in wave order: deterministic, no atomics
    float* srow = reinterpret_cast<float*>(smem + ((KCH + 1) % 3) * WSLOT) + wave * 2 * N;
#pragma unroll
    for (int cg = 0; cg < 2; ++cg) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i = 32 * cg + 8 * p + e;
          const float a = row16_sum(dy[i] * xh[i]);
          const float b = row16_sum(dy[i]);
          if (li == 0) {
            srow[128 * cg + 32 * p + 8 * lg + e] = a;
            srow[N + 128 * cg + 32 * p + 8 * lg + e] = b;
          }
        }
      }
    }
    __syncthreads();
    const float* rows = reinterpret_cast<const float*>(smem + ((KCH + 1) % 3) * WSLOT);
    for (int i = tid; i < 2 * N; i += 512) {
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) a += rows[w * 2 * N + i];
      if (ln.sum_ws) {          // folded later in workgroup order (ttmi_fold)
        ln.sum_ws[(int64_t)blockIdx.x * 2 * N + i] = a;
      } else {
        float* dst = i < N ? ln.dw : ln.db;
        if (dst) atomicAdd(dst + (i < N ? i : i - N), a);
      }
    }
  }
  TTMI_TSTAMP(3);
}

// ------------------------------------------------------------ weight-gradient GEMM (bf16)
// C[m,n] += alpha * Σ_r A[r,m] B[r,n]: A = dY [R][lda], B = X [R][ldb], both row-major with
// the reduction over rows (R = B*L tokens), C fp32.  This shape (output <= 512 x 512, R up
// to 25,600) is latency-bound in the generic kernel: one 16 KB stage in flight per CU.  Here:
//  * each workgroup owns a BM x BN tile and a contiguous row split; splits of one tile are
//    combined with fp32 atomics, reshaped through LDS so every atomic wave-instruction adds
//    256 contiguous bytes;
//  * rows are staged by LDS-DMA (buffer_load ... lds, 16 B/lane) into an NS-deep ring of
//    64-row stages, NS-1 stages in flight; the buffer descriptor's range is the split, so
//    rows past it read as zero;
//  * the LDS image is [64 k][W cols] unpadded with 32-byte chunks XOR-swizzled by k (the DMA
//    destination is lane-linear, so the swizzle goes on the source address); the 8 k-rows a
//    half-wave's ds_read_b64_tr_b16 touches land in 8 distinct bank windows;
//  * splits of one row range are grouped on one XCD (blockIdx % 8) so the tiles that re-read
//    the same rows share that XCD's L2.
struct WgradArgs {
  int64_t M, N, R;
  const char* A; int64_t lda;
  const char* B; int64_t ldb;
  float* C; int64_t ldc;
  float alpha;
  float* rowsum_a;
  int64_t rows_per_split;   // multiple of 64
  int tiles_m, tiles_n, splits, xcd_remap;
  // epilogue: WG_ATOMIC adds into C (legacy ttmi_gemm path); WG_SLAB stores the split's
  // partial tile to part[split][M][N] (and the row sums to part_rs[split][M]) with plain
  // stores, folded in split order by wgrad_fold_kernel; WG_DIRECT (one split) writes C itself
  int mode, accumulate;
  float* part; float* part_rs;
};
enum { WG_ATOMIC = 0, WG_SLAB = 1, WG_DIRECT = 2 };

template <int W>
struct WImg {
  static constexpr int PB = W * 2;                       // k-row pitch, bytes
  static constexpr int CPR = PB / 32;                    // 32-byte chunks per k-row
  static constexpr int RPB = PB >= 256 ? 1 : 256 / PB;   // k-rows per 256-byte bank row
  static constexpr int BYTES = 64 * PB;
  static constexpr int INSTR = BYTES / 1024;             // DMA wave-instructions per stage
  static TTMI_DEV int swz(int k) { return (k / RPB) % CPR; }

  // Issue this wave's share of one 64-row stage: rows [r0, r0+64) of the descriptor's range,
  // into the LDS image at byte address `img` (wave-uniform).
  static TTMI_DEV void issue(const i32x4_t& rs, int64_t ld, int col0, int r0, uint32_t img,
                             int wave, int lane) {
    static_assert(INSTR % 4 == 0, "stage must split evenly over 4 waves");
#pragma unroll
    for (int t = 0; t < INSTR / 4; ++t) {
      const int ii = wave + 4 * t;
      const int o = ii * 1024 + lane * 16;
      const int k = o / PB, pb = o % PB;
      const int lc = (pb >> 5) ^ swz(k);
      const uint32_t voff = (uint32_t)((int64_t)(r0 + k) * ld * 2 + col0 * 2 + lc * 32 + (pb & 16));
      dma16(rs, voff, img + ii * 1024);
    }
  }

  // MFMA fragment of the 16 columns at `row0` for 32-k chunk `c` (same k-permutation as
  // Operand<bf16, *, false>::frag).
  static TTMI_DEV uint4 frag(const char* img, int row0, int c, int lane) {
    const int i = lane & 15, g = lane >> 4;
    const int k = c * 32 + 4 * g + (i >> 2);
    const char* p = img + k * PB + ((((row0 >> 4)) ^ swz(k)) << 5) + 8 * (i & 3);
    const uint2 lo = lds_tr8(p), hi = lds_tr8(p + 16 * PB);
    return make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
};

// This wave's DMAs but the N_ youngest have landed and its LDS reads have returned; then
// the workgroup barrier (one asm statement: no memory access moves across it).
template <int N_>
TTMI_DEV void wait_vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N_) : "memory");
}

template <int BM, int BN, int NS>
TTMI_DEV void wgrad_body(const WgradArgs& g, const int bid) {
  using IA = WImg<BM>;
  using IB = WImg<BN>;
  constexpr int STAGE = IA::BYTES + IB::BYTES;
  constexpr int P = (IA::INSTR + IB::INSTR) / 4;          // DMA instructions per wave per stage
  constexpr int TP = BN + 16;                              // epilogue fp32 tile pitch (floats)
  static_assert(NS * STAGE >= BM * TP * 4, "epilogue tile must fit the ring");
  static_assert((NS - 2) * P <= 63, "vmcnt range");
  constexpr int WTM = BM / 2, WTN = BN / 2, TM = WTM / 16, TN = WTN / 16;
  __shared__ __attribute__((aligned(1024))) char ring[NS * STAGE];

  TTMI_TSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int T = g.tiles_m * g.tiles_n;
  int tile, split;
  if (g.xcd_remap == 2) {     // split-major (split, tile) pairs dealt to the 8 XCDs in
    // contiguous runs: the tiles of one split (which re-read the same operand rows) run side
    // by side on one XCD and share its L2.  The entry's first block sits at a multiple of 8
    // and its grid is 8 * ceil(P / 8) blocks; the surplus slots exit.
    const int x = bid & 7, j = bid >> 3;
    const int P = T * g.splits;
    const int lo = (int)((int64_t)P * x / 8), hi = (int)((int64_t)P * (x + 1) / 8);
    if (lo + j >= hi) return;
    split = (lo + j) / T;
    tile = (lo + j) % T;
  } else if (g.xcd_remap) {   // splits % 8 == 0: one XCD per (split mod 8)
    const int x = bid & 7, j = bid >> 3;
    tile = j % T;
    split = (j / T) * 8 + x;
  } else {
    tile = bid % T;
    split = bid / T;
  }
  const int tm = tile / g.tiles_n, tn = tile % g.tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)split * g.rows_per_split;
  if (kbeg >= g.R) return;
  const int rows = (int)min(g.R - kbeg, g.rows_per_split);
  const int nst = (rows + 63) >> 6;
  // the descriptor ends at the last valid element ((rows-1)·ld + extent): a column view of a
  // wider buffer (ld > extent) must not read past its allocation in the last row
  const i32x4_t ra = make_rsrc(g.A + kbeg * g.lda * 2, (uint32_t)(((int64_t)(rows - 1) * g.lda + g.M) * 2));
  const i32x4_t rb = make_rsrc(g.B + kbeg * g.ldb * 2, (uint32_t)(((int64_t)(rows - 1) * g.ldb + g.N) * 2));
  const uint32_t ring_lds = lds_addr(ring);

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float asum[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) asum[i] = 0.f;
  const bool do_asum = g.rowsum_a != nullptr && wn == 0 && tn == 0;

#pragma unroll
  for (int s = 0; s < NS - 1; ++s) {
    if (s < nst) {
      IA::issue(ra, g.lda, (int)m0, s * 64, ring_lds + s * STAGE, wave, lane);
      IB::issue(rb, g.ldb, (int)n0, s * 64, ring_lds + s * STAGE + IA::BYTES, wave, lane);
    }
  }
  TTMI_TSTAMP(1);
  uint64_t waited = 0, issued = 0;   // (diagnostic build) realtime ticks in the ring waits / DMA issue
  for (int t = 0; t < nst; ++t) {
    // stage t landed for every wave; every wave is done reading slot (t-1) % NS
    const uint64_t w0 = TTMI_TNOW();
    if (t + NS - 2 < nst) wait_vm_barrier<(NS - 2) * P>();
    else wait_vm_barrier<0>();
    waited += TTMI_TNOW() - w0;
    const int tn_ = t + NS - 1;
    const uint64_t i0 = TTMI_TNOW();
    if (tn_ < nst) {
      const uint32_t dst = ring_lds + (tn_ % NS) * STAGE;
      IA::issue(ra, g.lda, (int)m0, tn_ * 64, dst, wave, lane);
      IB::issue(rb, g.ldb, (int)n0, tn_ * 64, dst + IA::BYTES, wave, lane);
    }
    issued += TTMI_TNOW() - i0;
    const char* sA = ring + (t % NS) * STAGE;
    const char* sB = sA + IA::BYTES;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      uint4 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = IA::frag(sA, wm * WTM + i * 16, c, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = IB::frag(sB, wn * WTN + j * 16, c, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) Mma<bf16_t>::run(acc[i][j], bfr[j], af[i]);
      if (do_asum) {
#pragma unroll
        for (int i = 0; i < TM; ++i) asum[i] += frag_sum<bf16_t>(af[i]);
      }
    }
  }

  TTMI_TSTAMP(2);
  TTMI_TSTAMP_VAL(3, waited);
  TTMI_TSTAMP_VAL(4, nst);
  TTMI_TSTAMP_VAL(5, issued);
  (void)waited;
  (void)issued;
  const int li = lane & 15, lg = lane >> 4;
  if (do_asum) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float v = asum[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int64_t m = m0 + wm * WTM + i * 16 + li;
      if (lg == 0 && m < g.M) {
        if (g.mode == WG_ATOMIC) atomicAdd(g.rowsum_a + m, v);
        else if (g.mode == WG_SLAB) g.part_rs[(int64_t)split * g.M + m] = v;
        else g.rowsum_a[m] = g.accumulate ? g.rowsum_a[m] + v : v;
      }
    }
  }
  if (g.mode != WG_ATOMIC) {
    // deterministic epilogues: every (split, tile) element has exactly one writer; the lane
    // holds 4 consecutive columns of one row per accumulator (16-byte stores, N % 4 == 0)
    wait_vm<0>();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int64_t m = m0 + wm * WTM + i * 16 + li, n = n0 + wn * WTN + j * 16 + 4 * lg;
        if (m >= g.M || n >= g.N) continue;
        float4 v = make_float4(g.alpha * acc[i][j][0], g.alpha * acc[i][j][1],
                               g.alpha * acc[i][j][2], g.alpha * acc[i][j][3]);
        if (g.mode == WG_SLAB) {
          *reinterpret_cast<float4*>(g.part + ((int64_t)split * g.M + m) * g.N + n) = v;
        } else {
          float4* cp = reinterpret_cast<float4*>(g.C + m * g.ldc + n);
          if (g.accumulate) {
            const float4 c = *cp;
            v.x += c.x; v.y += c.y; v.z += c.z; v.w += c.w;
          }
          *cp = v;
        }
      }
    return;
  }
  // reshape through LDS: every atomic wave-instruction then covers 64 consecutive columns
  wait_vm<0>();
  __syncthreads();
  float* tl = reinterpret_cast<float*>(ring);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int m = wm * WTM + i * 16 + li, n = wn * WTN + j * 16 + 4 * lg;
      *reinterpret_cast<float4*>(tl + m * TP + n) =
          make_float4(g.alpha * acc[i][j][0], g.alpha * acc[i][j][1], g.alpha * acc[i][j][2],
                      g.alpha * acc[i][j][3]);
    }
  __syncthreads();
#pragma unroll 4
  for (int r = wave; r < BM; r += 4) {
    const int64_t m = m0 + r;
    if (m >= g.M) break;
#pragma unroll
    for (int c0 = 0; c0 < BN; c0 += 64) {
      const int64_t n = n0 + c0 + lane;
      if (n < g.N) atomicAdd(g.C + m * g.ldc + n, tl[r * TP + c0 + lane]);
    }
  }
}

template <int BM, int BN, int NS>
__global__ __launch_bounds__(256) void wgrad_kernel(WgradArgs g) {
  wgrad_body<BM, BN, NS>(g, blockIdx.x);
}

// Grouped weight gradients: several GEMMs' (tile, split) workgroups in one launch (the
// step's deferred weight gradients: one launch instead of one per Linear, and the short
// 512-row reductions fill the gaps the long ones leave).  Entry k owns workgroups
// [wg_begin[k], wg_begin[k+1]); its arguments are read from the kernel-argument segment at a
// uniform offset (no scratch copy of the table).
constexpr int WG_GROUP = 16;
struct WgradGroup { WgradArgs e[WG_GROUP]; int wg_begin[WG_GROUP + 1]; int n; };
typedef const __attribute__((address_space(4))) WgradGroup* KWgradGroup;

template <int BM, int BN, int NS>
__global__ __launch_bounds__(256) void wgrad_group_kernel(WgradGroup grp) {
  (void)grp;
  KWgradGroup kg = (KWgradGroup)__builtin_amdgcn_kernarg_segment_ptr();
  const int bid = blockIdx.x;
  int k = 0;                 // the last entry with wg_begin[k] <= bid (binary search)
  for (int lo = 0, hi = kg->n - 1; lo <= hi;) {
    const int mid = (lo + hi) >> 1;
    if (kg->wg_begin[mid] <= bid) { k = mid; lo = mid + 1; } else { hi = mid - 1; }
  }
  const auto& e = kg->e[k];
  WgradArgs g;
  g.M = e.M; g.N = e.N; g.R = e.R;
  g.A = e.A; g.lda = e.lda; g.B = e.B; g.ldb = e.ldb; g.C = e.C; g.ldc = e.ldc;
  g.alpha = e.alpha; g.rowsum_a = e.rowsum_a; g.rows_per_split = e.rows_per_split;
  g.tiles_m = e.tiles_m; g.tiles_n = e.tiles_n; g.splits = e.splits; g.xcd_remap = e.xcd_remap;
  g.mode = e.mode; g.accumulate = e.accumulate; g.part = e.part; g.part_rs = e.part_rs;
  wgrad_body<BM, BN, NS>(g, bid - kg->wg_begin[k]);
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
  if (bm == 128 && bn == 128) launch_layout<T, 128, 128>(a, ak, bk, grid, s);
  else if (bm == 128) launch_layout<T, 128, 64>(a, ak, bk, grid, s);
  else if (bn == 128) launch_layout<T, 64, 128>(a, ak, bk, grid, s);
  else if (bm == 32) launch_layout<T, 32, 32>(a, ak, bk, grid, s);
  else launch_layout<T, 64, 64>(a, ak, bk, grid, s);
}


// Weight-gradient dispatch (bf16, both operands row-major over the reduction, accumulate into
// an fp32 C, no epilogue extras).
bool wgrad_applies(const ttmi_gemm_desc* d) {
  return d->dtype == TTMI_BF16 && !d->a_kmajor && !d->b_kmajor && d->c_mode == 1 &&
         d->c_dtype == TTMI_F32 && !d->bias && !d->act && d->drop_p == 0.f && !d->gate &&
         !d->residual && !d->colsum && !d->drop_rows;
}


// Tile / ring-depth choice: 64x64 tiles, 4-deep ring (64 KB LDS: two workgroups per CU).
// Measured on MI355X (tools/wgrad_sweep.sh, R = 25,600): a CU ingests ~33 GB/s from the
// Infinity Cache whether staged by LDS-DMA or registers and whatever the ring depth, so the
// time is ~ re-read input bytes / (#CUs x 33 GB/s) + atomic bytes / 1.3 TB/s; 64x64 tiles
// with ~1.1 workgroups per CU minimise that sum (128x128 tiles halve the reads but
// quadruple the atomic bytes per workgroup).  TTMI_WGRAD="BMxBNxNS[:noremap]" overrides the
// tile for tuning runs.
struct WgradCfg { int bm, bn, ns, remap; };

WgradCfg wgrad_cfg() {
  static const WgradCfg cfg = [] {
    WgradCfg c{64, 64, 4, 1};
    if (const char* e = getenv("TTMI_WGRAD")) {
      int bm = 0, bn = 0, ns = 0;
      if (sscanf(e, "%dx%dx%d", &bm, &bn, &ns) == 3) c = WgradCfg{bm, bn, ns, 1};
      if (strstr(e, "noremap")) c.remap = 0;
    }
    return c;
  }();
  return cfg;
}

template <int BM, int BN, int NS>
int launch_wgrad_t(const ttmi_gemm_desc* d, int remap, hipStream_t stream) {
  const int tiles_m = (int)((d->M + BM - 1) / BM), tiles_n = (int)((d->N + BN - 1) / BN);
  const int T = tiles_m * tiles_n;
  const int64_t stages = (d->K + 63) / 64;
  int S = d->split_k;
  if (S <= 0) {                              // ~320 workgroups, splits a multiple of 8
    static const int target = [] {           // TTMI_WGRAD_WG: tuning runs only
      const char* e = getenv("TTMI_WGRAD_WG");
      const int v = e ? atoi(e) : 0;
      return v > 0 ? v : 320;
    }();
    S = (target / T + 4) & ~7;
    if (S < 8) S = std::max(1, target / T);
  }
  S = (int)std::max<int64_t>(1, std::min<int64_t>(S, stages));
  int64_t sps = (stages + S - 1) / S;        // stages per split
  const int64_t ldmax = std::max(d->lda, d->ldb);
  while (sps > 1 && sps * 64 * ldmax * 2 >= (int64_t)1 << 31) sps = (sps + 1) / 2;
  TTMI_REQUIRE(sps * 64 * ldmax * 2 < ((int64_t)1 << 31), "ttmi_gemm: split range exceeds 2 GiB");
  S = (int)((stages + sps - 1) / sps);
  WgradArgs a;
  a.M = d->M; a.N = d->N; a.R = d->K;
  a.A = static_cast<const char*>(d->A); a.lda = d->lda;
  a.B = static_cast<const char*>(d->B); a.ldb = d->ldb;
  a.C = static_cast<float*>(d->C); a.ldc = d->ldc;
  a.alpha = d->alpha;
  a.rowsum_a = d->rowsum_a;
  a.rows_per_split = sps * 64;
  a.tiles_m = tiles_m; a.tiles_n = tiles_n; a.splits = S;
  a.xcd_remap = remap && (S % 8 == 0);
  a.mode = WG_ATOMIC; a.accumulate = 1; a.part = nullptr; a.part_rs = nullptr;
  const int64_t nwg = (int64_t)T * S;
  TTMI_REQUIRE(nwg <= 2147483647LL, "ttmi_gemm: grid too large");
  hipLaunchKernelGGL((wgrad_kernel<BM, BN, NS>), dim3((unsigned)nwg), dim3(256), 0, stream, a);
  return ttmi_check_launch("ttmi_gemm");
}

int launch_wgrad(const ttmi_gemm_desc* d, hipStream_t stream) {
  const WgradCfg c = wgrad_cfg();
  if (c.bm == 128 && c.bn == 128) return launch_wgrad_t<128, 128, 4>(d, c.remap, stream);
  if (c.ns == 8) return launch_wgrad_t<64, 64, 8>(d, c.remap, stream);
  return launch_wgrad_t<64, 64, 4>(d, c.remap, stream);
}


bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// --------------------------------------------- deterministic weight gradient (ttmi_wgrad)
// Same 64x64 tiles, ring and split geometry as the atomic path (about 320 workgroups, splits
// a multiple of 8 so the tiles re-reading one row range share an XCD's L2), but the split
// partials are plain 16-byte stores into a caller workspace, summed in split order by
// wgrad_fold_kernel: bit-reproducible, and the partial bytes leave at store rate (~6 TB/s)
// instead of the memory-side float-atomic rate (~1.3 TB/s, MI355X_MICROARCH §Global float
// atomics).  One split (short R) writes C directly.  Folds of several GEMMs share one launch.
struct WgradPlan { int tiles_m, tiles_n, S, tile; int64_t sps; };

WgradPlan wgrad_plan64(int64_t R, int64_t M, int64_t N, int64_t ldmax, bool allow32) {
  WgradPlan p;
  p.tile = 64;
  p.tiles_m = (int)((M + 63) / 64);
  p.tiles_n = (int)((N + 63) / 64);
  const int T = p.tiles_m * p.tiles_n;
  const int64_t stages = std::max<int64_t>(1, (R + 63) / 64);
  static const int target = [] {
    const char* e = getenv("TTMI_WGRAD_WG");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 320;
  }();
  int S = (target / T + 4) & ~7;
  if (S < 8) S = std::max(1, target / T);
  // at least MIN_STAGES 64-row stages per split: below that a split's partial tile costs more
  // bytes (written, then folded) than the rows it reduces (R = 512 -> one split, direct)
  static const int min_stages = [] {
    const char* e = getenv("TTMI_WGRAD_MIN_STAGES");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 6;
  }();
  S = (int)std::max<int64_t>(1, std::min<int64_t>(S, stages / min_stages));
  int64_t sps = (stages + S - 1) / S;
  while (sps > 1 && sps * 64 * ldmax * 2 >= (int64_t)1 << 31) sps = (sps + 1) / 2;
  p.S = (int)((stages + sps - 1) / sps);
  p.sps = sps;
  if (allow32 && p.S == 1 && T < 128) {   // one split: 32x32 tiles, 4x the workgroups
    p.tile = 32;
    p.tiles_m = (int)((M + 31) / 32);
    p.tiles_n = (int)((N + 31) / 32);
  }
  return p;
}

// Grouped launches (ttmi_wgrad_batch) may use larger tiles: a 128 x 128 tile reads each
// operand row slice once for twice the outputs of a 64 x 64 one, halving what the CUs ingest
// (the family is bound by per-CU ingest from L2 / Infinity Cache), at one workgroup per CU
// (128 KB ring).  TTMI_WGRAD_GROUP="T:S" (T = 64 or 128, S = splits per long-GEMM tile, 0 =
// the 64-tile default sizing) selects it.  Default 128:14: the cfg-2 step's group is 14
// long-GEMM tiles x S splits + ~33 short-GEMM workgroups, and a workgroup holds a CU (128 KB
// ring), so the launch takes one round only while that sum stays <= 256 CUs: per GEMM
// 128:12 4.05 us, 128:14 3.80, 128:15 5.04 (a second round), 128:16 4.95 (tools/ab.sh, three
// pairs each; round 2: 64:0 4.73, 128:8 5.11, 128:24 4.83, 128:32 5.01).
struct WgradGroupCfg { int tile, splits; };

WgradGroupCfg wgrad_group_cfg() {
  static const WgradGroupCfg cfg = [] {
    WgradGroupCfg c{128, 14};
    if (const char* e = getenv("TTMI_WGRAD_GROUP")) {
      int t = 0, sp = 0;
      if (sscanf(e, "%d:%d", &t, &sp) >= 1 && (t == 64 || t == 128)) c = WgradGroupCfg{t, std::max(sp, 0)};
    }
    return c;
  }();
  return cfg;
}

// TTMI_WGRAD_CHUNK=0 restores the tile-major block order of the grouped launch (A/B runs).
bool wgrad_group_chunked() {
  static const bool on = [] {
    const char* e = getenv("TTMI_WGRAD_CHUNK");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

WgradPlan wgrad_group_plan(int64_t R, int64_t M, int64_t N, int64_t ldmax) {
  const WgradGroupCfg c = wgrad_group_cfg();
  if (c.tile == 64) return wgrad_plan64(R, M, N, ldmax, false);
  WgradPlan p;
  p.tile = c.tile;
  p.tiles_m = (int)((M + c.tile - 1) / c.tile);
  p.tiles_n = (int)((N + c.tile - 1) / c.tile);
  const int T = p.tiles_m * p.tiles_n;
  const int64_t stages = std::max<int64_t>(1, (R + 63) / 64);
  // at most ~64 workgroups per GEMM (every split one CU-resident 128 KB ring): the D = 256
  // encoder's four long weight gradients have 12-16 tiles each, and 12 splits of them made
  // 576 workgroups = 2.25 rounds on 256 CUs (117 us); the D = 128 shapes (<= 4 tiles) keep 12
  int S = c.splits > 0 ? std::min(c.splits, std::max(1, 64 / T)) : std::max(1, 256 / T);
  S = (int)std::max<int64_t>(1, std::min<int64_t>(S, stages / 6));
  int64_t sps = (stages + S - 1) / S;
  while (sps > 1 && sps * 64 * ldmax * 2 >= (int64_t)1 << 31) sps = (sps + 1) / 2;
  p.S = (int)((stages + sps - 1) / sps);
  p.sps = sps;
  return p;
}

// The standalone ttmi_wgrad uses the grouped launch's split boundaries (so a deferred,
// grouped weight gradient and an immediate one are bit-identical: the result depends on the
// splits, not on the tile shape that computes them), executed with 64 x 64 tiles (32 x 32 for
// a single split of a small output: 4x the workgroups).
WgradPlan wgrad_plan(int64_t R, int64_t M, int64_t N, int64_t ldmax, bool allow32 = true) {
  WgradPlan p = wgrad_group_plan(R, M, N, ldmax);
  p.tile = 64;
  p.tiles_m = (int)((M + 63) / 64);
  p.tiles_n = (int)((N + 63) / 64);
  if (allow32 && p.S == 1 && p.tiles_m * p.tiles_n < 128) {
    p.tile = 32;
    p.tiles_m = (int)((M + 31) / 32);
    p.tiles_n = (int)((N + 31) / 32);
  }
  return p;
}

int64_t al256(int64_t b) { return (b + 255) / 256 * 256; }

int64_t wgrad_ws_bytes(const WgradPlan& p, int64_t M, int64_t N) {
  if (p.S <= 1) return 0;
  return al256((int64_t)p.S * M * N * 4) + al256((int64_t)p.S * M * 4);
}

constexpr int FOLD_SEGS = 32;   // kernarg: 32 x 100 B (a cfg-2 step folds ~24 segments)
struct FoldSeg {
  const void* part; const float* part_rs; float* C; float* rs;
  int64_t M, N, ldc, units, base, s_stride;   // s_stride: elements between split slabs
  int S, acc, fx;                             // fx > 0: int64 fixed-point partials, 2^-fx
};
struct FoldArgs { FoldSeg seg[FOLD_SEGS]; int blk_begin[FOLD_SEGS + 1]; int n; int64_t total; };

// The segment is read straight from the kernel-argument segment at the uniform offset
// blockIdx.y (scalar loads); copying the argument array to a local and indexing it
// dynamically would put it in scratch memory.
typedef const __attribute__((address_space(4))) FoldArgs* KFoldArgs;

// The S partials of one 4-column unit, summed in split order: fp32 partials in float, int64
// fixed-point partials exactly (integer adds) and converted once.  `consume` zeroes them.
TTMI_DEV float4 fold_unit(const FoldSeg& sg, int64_t off, int s_lo, int s_hi, bool consume) {
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (sg.fx) {
    const int64_t* p = static_cast<const int64_t*>(sg.part) + off;
    long long q[4] = {0, 0, 0, 0};
    for (int s0 = s_lo; s0 < s_hi; s0 += 4) {
      longlong2 w[4][2];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int s = min(s0 + j, s_hi - 1);     // clamped: unconditional loads
        w[j][0] = *reinterpret_cast<const longlong2*>(p + s * sg.s_stride);
        w[j][1] = *reinterpret_cast<const longlong2*>(p + s * sg.s_stride + 2);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (s0 + j < s_hi) {
          q[0] += w[j][0].x; q[1] += w[j][0].y; q[2] += w[j][1].x; q[3] += w[j][1].y;
          if (consume) {
            int64_t* z = const_cast<int64_t*>(p) + (s0 + j) * sg.s_stride;
            *reinterpret_cast<longlong2*>(z) = make_longlong2(0, 0);
            *reinterpret_cast<longlong2*>(z + 2) = make_longlong2(0, 0);
          }
        }
    }
    v = make_float4(fx_to_f(q[0], sg.fx), fx_to_f(q[1], sg.fx), fx_to_f(q[2], sg.fx), fx_to_f(q[3], sg.fx));
    return v;
  }
  const float* p = static_cast<const float*>(sg.part) + off;
  if (s_hi <= s_lo) return v;
  for (int s0 = s_lo; s0 < s_hi; s0 += 8) {
    float4 w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {          // clamped: unconditional loads, all in flight
      const int s = min(s0 + j, s_hi - 1);
      w[j] = *reinterpret_cast<const float4*>(p + s * sg.s_stride);
    }
    if (consume) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (s0 + j < s_hi)
          *reinterpret_cast<float4*>(const_cast<float*>(p) + (s0 + j) * sg.s_stride) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (s0 + j < s_hi) { v.x += w[j].x; v.y += w[j].y; v.z += w[j].z; v.w += w[j].w; }
  }
  return v;
}

TTMI_DEV void fold_store(const FoldSeg& sg, int64_t u, int64_t nq, float4 v) {
  const int64_t m = u / nq, n = (u % nq) * 4;
  float4* cp = reinterpret_cast<float4*>(sg.C + m * sg.ldc + n);
  if (sg.acc & 1) {
    const float4 c = *cp;
    v.x = c.x + v.x; v.y = c.y + v.y; v.z = c.z + v.z; v.w = c.w + v.w;
  }
  *cp = v;
}

// P partitions of the S partials x 256/P units per block pass: partition q sums its splits in
// split order, the P partition sums are added in partition order through LDS (deterministic
// for a given S).  P = 4 for a weight gradient's ~12 splits; P = 16 for the many-partial
// slabs (a LayerNorm's per-workgroup column sums, S ~ 229, 32-64 units), where 4 partitions
// meant ~57 dependent loads per thread in 4 serial batches.
constexpr int FOLD_WIDE_S = 32;
// Up to FOLD_NARROW_S partials (a weight gradient's ~14 splits) a thread owns whole units and
// sums all their partials itself, in split order: the partitioned form left 3 of 4 threads idle
// in the update and padded each thread's 3-4 loads to a batch of 8.
#ifndef TTMI_FOLD_NARROW_S
#define TTMI_FOLD_NARROW_S 16
#endif
constexpr int FOLD_NARROW_S = TTMI_FOLD_NARROW_S < 2 ? 2 : TTMI_FOLD_NARROW_S;
static_assert(FOLD_NARROW_S < FOLD_WIDE_S, "fold regimes");
// The fold of one segment's units over this block's share [bx, nbx), handing each finished
// unit to store4(u, float4 sum) (a 4-column weight unit) or store1(m, sum) (a bias row):
// wgrad_fold_kernel stores them into the gradient, adamw_fold_kernel updates the parameters.
template <int P, class S4, class S1>
TTMI_DEV void fold_parts(const FoldSeg& sg, int bx, int nbx, bool consume, int64_t nel, int64_t nq,
                         S4& store4, S1& store1) {
  constexpr int U = 256 / P;
  __shared__ float4 red[256];
  const int ul = threadIdx.x % U, q = threadIdx.x / U;
  const int s_lo = (int)((int64_t)sg.S * q / P), s_hi = (int)((int64_t)sg.S * (q + 1) / P);
  for (int64_t ub = (int64_t)bx * U; ub < sg.units; ub += (int64_t)nbx * U) {
    const int64_t u = ub + ul;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (u < nel) {
      const int64_t m = u / nq, n = (u % nq) * 4;
      v = fold_unit(sg, m * sg.N + n, s_lo, s_hi, consume);
    } else if (u < sg.units) {
      const int64_t m = u - nel;
      for (int s0 = s_lo; s0 < s_hi; s0 += 8) {
        float w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = sg.part_rs[min(s0 + j, s_hi - 1) * sg.M + m];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (s0 + j < s_hi) v.x += w[j];
      }
    }
    red[q * U + ul] = v;
    __syncthreads();
    if (q == 0 && u < sg.units) {
#pragma unroll
      for (int k = 1; k < P; ++k) {
        const float4 w = red[k * U + ul];
        v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
      }
      if (u < nel) store4(u, v);
      else store1(u - nel, v.x);
    }
    __syncthreads();
  }
}

template <class S4, class S1>
TTMI_DEV void fold_segment(const FoldSeg& sg, int bx, int nbx, S4& store4, S1& store1) {
  const int64_t nq = sg.N / 4, nel = sg.M * nq;
  const bool consume = (sg.acc & 2) != 0;
  if (sg.S <= FOLD_NARROW_S) {   // few partials (fixed-point accumulators, split slabs): one unit a thread
    for (int64_t u = (int64_t)bx * 256 + threadIdx.x; u < sg.units; u += (int64_t)nbx * 256) {
      if (u < nel) {
        const int64_t m = u / nq, n = (u % nq) * 4;
        store4(u, fold_unit(sg, m * sg.N + n, 0, sg.S, consume));
      } else {                // a weight gradient's bias: the split row sums
        const int64_t m = u - nel;
        float v = 0.f;
        for (int s0 = 0; s0 < sg.S; s0 += 8) {     // batches of 8 loads in flight, split order
          float w[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) w[j] = sg.part_rs[(int64_t)min(s0 + j, sg.S - 1) * sg.M + m];
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (s0 + j < sg.S) v += w[j];
        }
        store1(m, v);
      }
    }
    return;
  }
  if (sg.S > FOLD_WIDE_S) fold_parts<16>(sg, bx, nbx, consume, nel, nq, store4, store1);
  else fold_parts<4>(sg, bx, nbx, consume, nel, nq, store4, store1);
}

// The last k < n with begin[k] <= b, by binary search over a kernel-argument array (dependent
// scalar loads: 5 for 32 entries instead of a walk)
template <class KA>
TTMI_DEV int find_job(KA begin, int n, int b) {
  int k = 0;
  for (int lo = 0, hi = n - 1; lo <= hi;) {
    const int mid = (lo + hi) >> 1;
    if (begin[mid] <= b) { k = mid; lo = mid + 1; } else { hi = mid - 1; }
  }
  return k;
}

TTMI_DEV FoldSeg load_seg(const __attribute__((address_space(4))) FoldSeg& sgk) {
  FoldSeg sg;
  sg.part = sgk.part; sg.part_rs = sgk.part_rs; sg.C = sgk.C; sg.rs = sgk.rs;
  sg.M = sgk.M; sg.N = sgk.N; sg.ldc = sgk.ldc; sg.units = sgk.units; sg.base = 0;
  sg.s_stride = sgk.s_stride;
  sg.S = sgk.S; sg.acc = sgk.acc; sg.fx = sgk.fx;
  return sg;
}

__global__ __launch_bounds__(256) void wgrad_fold_kernel(FoldArgs a) {
  (void)a;
  // segment k owns blocks [blk_begin[k], blk_begin[k+1]) of the flat grid (each sized to its
  // units: launching the largest segment's block count for every segment dispatched tens of
  // thousands of empty blocks)
  const KFoldArgs ka = (KFoldArgs)__builtin_amdgcn_kernarg_segment_ptr();
  const int k = find_job(ka->blk_begin, ka->n, (int)blockIdx.x);
  const int bx = (int)blockIdx.x - ka->blk_begin[k], nbx = ka->blk_begin[k + 1] - ka->blk_begin[k];
  const FoldSeg sg = load_seg(ka->seg[k]);
  const int64_t nq = sg.N / 4;
  auto store4 = [&](int64_t u, float4 v) { fold_store(sg, u, nq, v); };
  auto store1 = [&](int64_t m, float v) { sg.rs[m] = (sg.acc & 1) ? sg.rs[m] + v : v; };
  fold_segment(sg, bx, nbx, store4, store1);
}

// ----------------------------------------------------- AdamW with the gradient fold fused
// One process (no gradient all-reduce between the fold and the update): the fold's segments
// (weight-gradient split partials, LayerNorm per-workgroup sums, fixed-point accumulators) are
// summed in the fold's order and applied by AdamW right there, instead of stored into the flat
// gradient by wgrad_fold_kernel and read back by adamw_kernel: one launch and one round trip of
// those gradients less per step.  The grid is jobs: plain AdamW over the flat ranges no segment
// covers (float4 units, 256·AF_U per block, the fixed-point range read from fx as adamw_kernel does),
// then one job per segment.
constexpr int AF_SEGS = FOLD_SEGS, AF_PLAIN = 40;
#ifndef TTMI_AF_U
#define TTMI_AF_U 4
#endif
constexpr int AF_U = TTMI_AF_U;                 // float4 units a thread of a plain job updates
struct AdamFoldArgs {
  float* p; float* g; float* m; float* v; bf16_t* pb;
  const double* hyper; const int32_t* step;
  int64_t* fx; int64_t fx_lo, fx_hi; int fx_shift, zero_grad;
  const int32_t* skip_if;                       // ABI 22: bad-id step, no update
  int nplain, nseg;
  int blk_begin[AF_PLAIN + AF_SEGS + 1];
  int plo[AF_PLAIN], phi[AF_PLAIN];             // float4 units
  FoldSeg seg[AF_SEGS];
};
typedef const __attribute__((address_space(4))) AdamFoldArgs* KAdamFoldArgs;

__global__ __launch_bounds__(256) void adamw_fold_kernel(AdamFoldArgs a) {
  (void)a;
  const KAdamFoldArgs ka = (KAdamFoldArgs)__builtin_amdgcn_kernarg_segment_ptr();
  const int nj = ka->nplain + ka->nseg;
  const int k = find_job(ka->blk_begin, nj, (int)blockIdx.x);
  const int bx = (int)blockIdx.x - ka->blk_begin[k], nbx = ka->blk_begin[k + 1] - ka->blk_begin[k];
  float* __restrict__ p = ka->p;
  float* __restrict__ g = ka->g;
  float* __restrict__ mo = ka->m;
  float* __restrict__ vo = ka->v;
  bf16_t* __restrict__ pb = ka->pb;
  const int zero_grad = ka->zero_grad;
  const AdamScalars as = adam_scalars(ka->hyper, ka->step);
  const bool keep = !id_err_raised(ka->skip_if);
  auto upd4 = [&](int64_t q, float4 gg) {
    float4 pp = reinterpret_cast<const float4*>(p)[q];
    float4 mm = reinterpret_cast<const float4*>(mo)[q];
    float4 vv = reinterpret_cast<const float4*>(vo)[q];
    adam_upd(as, pp.x, gg.x, mm.x, vv.x);
    adam_upd(as, pp.y, gg.y, mm.y, vv.y);
    adam_upd(as, pp.z, gg.z, mm.z, vv.z);
    adam_upd(as, pp.w, gg.w, mm.w, vv.w);
    if (!keep) return;
    reinterpret_cast<float4*>(p)[q] = pp;
    reinterpret_cast<float4*>(mo)[q] = mm;
    reinterpret_cast<float4*>(vo)[q] = vv;
    if (pb) {
      ushort4 o;
      o.x = f2bf(pp.x); o.y = f2bf(pp.y); o.z = f2bf(pp.z); o.w = f2bf(pp.w);
      reinterpret_cast<ushort4*>(pb)[q] = o;
    }
  };
  if (k < ka->nplain) {
    const int64_t lo = ka->plo[k], hi = ka->phi[k];
    int64_t* fx = ka->fx;
    const int64_t fx_lo = ka->fx_lo, fx_hi = ka->fx_hi;
    const int fx_shift = ka->fx_shift;
    constexpr int U = AF_U;
    float4 gg[U];
    int64_t q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      q[u] = lo + (int64_t)bx * (256 * U) + u * 256 + threadIdx.x;
      const int64_t qc = min(q[u], hi - 1);
      if (fx != nullptr && qc >= fx_lo && qc < fx_hi) {
        const longlong2 x0 = reinterpret_cast<const longlong2*>(fx)[2 * (qc - fx_lo)];
        const longlong2 x1 = reinterpret_cast<const longlong2*>(fx)[2 * (qc - fx_lo) + 1];
        gg[u] = make_float4(fx_to_f(x0.x, fx_shift), fx_to_f(x0.y, fx_shift), fx_to_f(x1.x, fx_shift),
                            fx_to_f(x1.y, fx_shift));
      } else {
        gg[u] = reinterpret_cast<const float4*>(g)[qc];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (q[u] >= hi) break;
      upd4(q[u], gg[u]);
      if (fx != nullptr && q[u] >= fx_lo && q[u] < fx_hi) {
        reinterpret_cast<longlong2*>(fx)[2 * (q[u] - fx_lo)] = make_longlong2(0, 0);
        reinterpret_cast<longlong2*>(fx)[2 * (q[u] - fx_lo) + 1] = make_longlong2(0, 0);
      } else if (zero_grad) {
        reinterpret_cast<float4*>(g)[q[u]] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    return;
  }
  const FoldSeg sg = load_seg(ka->seg[k - ka->nplain]);
  const int64_t nq = sg.N / 4;
  auto store4 = [&](int64_t u, float4 v) {       // fold_store's sum, then the update
    const int64_t mr = u / nq, n = (u % nq) * 4;
    float* cp = sg.C + mr * sg.ldc + n;
    if (sg.acc & 1) {
      const float4 c = *reinterpret_cast<const float4*>(cp);
      v.x = c.x + v.x; v.y = c.y + v.y; v.z = c.z + v.z; v.w = c.w + v.w;
    }
    upd4((cp - g) / 4, v);
    if (zero_grad) *reinterpret_cast<float4*>(cp) = make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto store1 = [&](int64_t mr, float v) {
    float* rp = sg.rs + mr;
    if (sg.acc & 1) v = *rp + v;
    const int64_t e = rp - g;
    float P = p[e], Mv = mo[e], Vv = vo[e];
    adam_upd(as, P, v, Mv, Vv);
    if (keep) {
      p[e] = P; mo[e] = Mv; vo[e] = Vv;
      if (pb) pb[e] = f2bf(P);
    }
    if (zero_grad) *rp = 0.f;
  };
  fold_segment(sg, bx, nbx, store4, store1);
}

// ------------------------------------------- large token GEMM: 256x256x64 tiles, 8 waves
// C[M,N] = epi(alpha · A[M,K] · B[N,K]ᵀ) for the mDeBERTa token GEMMs (M = B·S = 65,536,
// N, K in {768, 832, 2304, 3072}): bf16, both operands k-major, K % 64 == 0.
//  * 8 waves as 2 (rows) x 4 (cols); a wave owns 128 x 64 outputs = 8 x 4 MFMA tiles (128
//    accumulator registers).  Per 64-deep K-tile each wave runs 4 phases, one per 64 x 32
//    quadrant of its block (16 v_mfma_f32_16x16x32_bf16 each).
//  * Operands are staged by LDS-DMA (buffer_load_dwordx4 ... lds) into two 64 KB K-tile
//    buffers, [row][128 B] images whose 16-byte chunks are XOR-swizzled per row on the SOURCE
//    address (the DMA writes lane-linearly), so the 16 rows a ds_read_b128 lane group reads
//    fall in 16 distinct bank slots.
//  * The two wave groups (rows 0-127 / 128-255) run one barrier apart: while one group's
//    waves issue their ds_reads and DMAs, the other group's waves, on the same SIMDs, run
//    their MFMA cluster.  Every phase is {ds_read [+ DMA issue]; barrier; MFMA x16; barrier}.
//  * DMA schedule of K-tile t+1 (buffer (t+1)&1, which held t-1): A/B rows 0-127 at phase 3
//    of tile t-1 (after the last reads of those rows), rows 128-255 at phase 1 of tile t;
//    all of t+1 is waited for (counted vmcnt, never in flight across the read) at phase 3
//    of tile t, two barriers before any wave reads it.
//  * B fragment rows are paired (tile 2p row 4q+r <-> column 32p+8q+r, tile 2p+1 <->
//    32p+8q+4+r), so each lane owns 8 consecutive output columns: 16-byte epilogue accesses.
//  * blockIdx is remapped so each XCD owns a contiguous run of tiles (row panels shared in
//    its L2).
namespace big {
constexpr int BMN = 256;
constexpr int HALF = 128 * 128;     // bytes: 128 rows x 64 bf16
constexpr int IMG = 2 * HALF;       // one operand's K-tile image
constexpr int STAGE = 2 * IMG;      // A + B
TTMI_DEV int swz_a(int r) { return (r >> 1) & 7; }
TTMI_DEV int swz_b(int r) { return ((r >> 1) & 1) | (((r >> 3) & 3) << 1); }
TTMI_DEV void barrier() { asm volatile("s_barrier" ::: "memory"); }
TTMI_DEV void wait_lgkm0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
}  // namespace big

struct BigArgs {
  GemmArgs g;
  int tiles_n, tiles;
};

// One 128-row half of a K-tile image: this wave's 2 of its 16 DMA wave-instructions.
template <bool ISB>
TTMI_DEV void big_issue(const i32x4_t& rs, int64_t ld, int half, int k0, uint32_t img, int wave,
                        int lane) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int ii = wave + 8 * u;
    const int r = half * 128 + ii * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ (ISB ? big::swz_b(r) : big::swz_a(r));
    const uint32_t voff = (uint32_t)(((int64_t)r * ld + k0) * 2 + ch * 16);
    dma16(rs, voff, img + half * big::HALF + ii * 1024);
  }
}

TTMI_DEV uint4 big_frag_a(const char* img, int row, int c, int lane) {
  const int ch = (4 * c + (lane >> 4)) ^ big::swz_a(row);
  return lds16(img + row * 128 + ch * 16);
}
// B tile j of the wave's 64 columns (paired mapping), row-operand lane i = lane & 15
TTMI_DEV int big_brow(int wc, int j, int lane) {
  const int i = lane & 15;
  return wc * 64 + 32 * (j >> 1) + 8 * (i >> 2) + 4 * (j & 1) + (i & 3);
}
TTMI_DEV uint4 big_frag_b(const char* img, int row, int c, int lane) {
  const int ch = (4 * c + (lane >> 4)) ^ big::swz_b(row);
  return lds16(img + row * 128 + ch * 16);
}

// Epilogue families, specialised at compile time (EPI >= 0) so each instantiation's
// straight-line epilogue stays small; EPI_ANY reads every flag at run time.
enum BigEpi {
  BE_BIAS = 1, BE_RELU = 2, BE_GELU = 4, BE_DROP = 8, BE_GELU_GRAD = 16, BE_RELU_GATE = 32,
  BE_RES = 64, BE_F32 = 128, BE_ACC = 256, BE_PRE = 512, BE_ANY = -1
};

template <int EPI>
TTMI_DEV void big_epi8(const GemmArgs& g, const DropKeys& dk, int64_t m, int64_t n, float* v) {
  constexpr bool RT = EPI < 0;
  const bool bias = RT ? g.bias != nullptr : (EPI & BE_BIAS);
  const bool relu = RT ? g.act == 1 : (EPI & BE_RELU);
  const bool gelu = RT ? g.act == 2 : (EPI & BE_GELU);
  const bool drop = RT ? true : (EPI & BE_DROP);
  const bool gate = RT ? g.gate != nullptr : (EPI & (BE_GELU_GRAD | BE_RELU_GATE));
  const bool ggrad = RT ? g.act == 3 : (EPI & BE_GELU_GRAD);
  const bool res = RT ? g.residual != nullptr : (EPI & BE_RES);
  const bool f32 = RT ? g.c_f32 != 0 : (EPI & BE_F32);
  const bool accum = RT ? g.c_mode == 1 : (EPI & BE_ACC);
  const bool pre = RT ? g.pre_out != nullptr : (EPI & BE_PRE);
  const bool full = n + 7 < g.N;
  if (bias) {
    if (full) {
      const float4 b0 = *reinterpret_cast<const float4*>(g.bias + n);
      const float4 b1 = *reinterpret_cast<const float4*>(g.bias + n + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
      v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += (n + e < g.N) ? g.bias[n + e] : 0.f;
    }
  }
  if (pre) {                                   // pre-activation copy (bf16, C's row stride)
    const int64_t o = m * g.ldc + n;
    if (full) {
      *reinterpret_cast<uint4*>(g.pre_out + o) = pack8(v);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) if (n + e < g.N) g.pre_out[o + e] = f2bf(v[e]);
    }
  }
  if (relu) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
  } else if (gelu) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
  }
  if (drop) drop_apply_vec<8>(dk, (uint32_t)(m * g.ld_drop + n), v);
  if (gate) {
    const int64_t o = m * g.ld_gate + n;
    float gv[8];
    if (full) {
      unpack8(*reinterpret_cast<const uint4*>((const bf16_t*)g.gate + o), gv);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) gv[e] = (n + e < g.N) ? bf2f(((const bf16_t*)g.gate)[o + e]) : 0.f;
    }
    if (ggrad) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= gelu_erf_grad(gv[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = gv[e] > 0.f ? v[e] * g.gate_scale : 0.f;
    }
  }
  if (res) {
    const float* rp = g.residual + m * g.ld_res + n;
    if (full) {
      const float4 r0 = *reinterpret_cast<const float4*>(rp);
      const float4 r1 = *reinterpret_cast<const float4*>(rp + 4);
      v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w;
      v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) if (n + e < g.N) v[e] += rp[e];
    }
  }
  const int64_t o = m * g.ldc + n;
  if (accum) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (n + e < g.N) atomicAdd(reinterpret_cast<float*>(g.C) + o + e, v[e]);
  } else if (full && f32) {
    float* cp = reinterpret_cast<float*>(g.C) + o;
    *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else if (full) {
    *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(g.C) + o) = pack8(v);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) if (n + e < g.N) st_dyn(g.C, o + e, v[e], f32);
  }
}

// Epilogue operands of one 8-column item (bias, GELU gate, fp32 residual), loaded one item
// ahead of its use: the loads of item k+1 issue before item k's math and stores, so their
// latency hides behind them (a load right before its use waited vmcnt(0) 16 times per tile).
// Addresses are clamped into the matrix; items off its edge fall back to big_epi8.
struct EpiIn {
  float4 b0, b1, r0, r1;
  uint4 gate;
};
template <int EPI>
TTMI_DEV void big_epi_load(const GemmArgs& g, int64_t m, int64_t n, EpiIn& in) {
  const int64_t mc = min<int64_t>(m, g.M - 1), nc = min<int64_t>(n, g.N - 8);
  if (EPI & BE_BIAS) {
    in.b0 = *reinterpret_cast<const float4*>(g.bias + nc);
    in.b1 = *reinterpret_cast<const float4*>(g.bias + nc + 4);
  }
  if (EPI & (BE_GELU_GRAD | BE_RELU_GATE))
    in.gate = *reinterpret_cast<const uint4*>((const bf16_t*)g.gate + mc * g.ld_gate + nc);
  if (EPI & BE_RES) {
    const float* rp = g.residual + mc * g.ld_res + nc;
    in.r0 = *reinterpret_cast<const float4*>(rp);
    in.r1 = *reinterpret_cast<const float4*>(rp + 4);
  }
}
// big_epi8 for a full item (n + 7 < N) with its operands already in registers.
template <int EPI>
TTMI_DEV void big_epi8_pre(const GemmArgs& g, const DropKeys& dk, int64_t m, int64_t n, float* v,
                           const EpiIn& in) {
  if (EPI & BE_BIAS) {
    v[0] += in.b0.x; v[1] += in.b0.y; v[2] += in.b0.z; v[3] += in.b0.w;
    v[4] += in.b1.x; v[5] += in.b1.y; v[6] += in.b1.z; v[7] += in.b1.w;
  }
  if (EPI & BE_PRE) *reinterpret_cast<uint4*>(g.pre_out + m * g.ldc + n) = pack8(v);
  if (EPI & BE_RELU) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
  } else if (EPI & BE_GELU) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
  }
  if (EPI & BE_DROP) drop_apply_vec<8>(dk, (uint32_t)(m * g.ld_drop + n), v);
  if (EPI & (BE_GELU_GRAD | BE_RELU_GATE)) {
    float gv[8];
    unpack8(in.gate, gv);
    if (EPI & BE_GELU_GRAD) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= gelu_erf_grad(gv[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = gv[e] > 0.f ? v[e] * g.gate_scale : 0.f;
    }
  }
  if (EPI & BE_RES) {
    v[0] += in.r0.x; v[1] += in.r0.y; v[2] += in.r0.z; v[3] += in.r0.w;
    v[4] += in.r1.x; v[5] += in.r1.y; v[6] += in.r1.z; v[7] += in.r1.w;
  }
  const int64_t o = m * g.ldc + n;
  if (EPI & BE_ACC) {
#pragma unroll
    for (int e = 0; e < 8; ++e) atomicAdd(reinterpret_cast<float*>(g.C) + o + e, v[e]);
  } else if (EPI & BE_F32) {
    float* cp = reinterpret_cast<float*>(g.C) + o;
    *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(g.C) + o) = pack8(v);
  }
}

template <int EPI>
__global__ __launch_bounds__(512) void gemm_big_kernel(BigArgs ba) {
  using namespace big;
  const GemmArgs& g = ba.g;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  // XCD-contiguous tile order (bijective for any tile count)
  const int bid = blockIdx.x, nwg = ba.tiles;
  const int xcd = bid & 7, q = nwg >> 3, rem = nwg & 7;
  const int tile = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
  const int64_t m0 = (int64_t)(tile / ba.tiles_n) * BMN, n0 = (int64_t)(tile % ba.tiles_n) * BMN;
  const int nt = (int)(g.K / 64);
  // descriptors start at the tile's first row; rows past M / N read as zero
  const int64_t arows = min<int64_t>(g.M - m0, BMN), brows = min<int64_t>(g.N - n0, BMN);
  const i32x4_t ra = make_rsrc(g.A + m0 * g.lda * 2, (uint32_t)(((arows - 1) * g.lda + g.K) * 2));
  const i32x4_t rb = make_rsrc(g.B + n0 * g.ldb * 2, (uint32_t)(((brows - 1) * g.ldb + g.K) * 2));
  const uint32_t sl = lds_addr(smem);

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // prologue: all of tile 0, rows 0-127 of tile 1
  big_issue<false>(ra, g.lda, 0, 0, sl, wave, lane);
  big_issue<false>(ra, g.lda, 1, 0, sl, wave, lane);
  big_issue<true>(rb, g.ldb, 0, 0, sl + IMG, wave, lane);
  big_issue<true>(rb, g.ldb, 1, 0, sl + IMG, wave, lane);
  if (nt > 1) {
    big_issue<false>(ra, g.lda, 0, 64, sl + STAGE, wave, lane);
    big_issue<true>(rb, g.ldb, 0, 64, sl + STAGE + IMG, wave, lane);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  barrier();
  if (wr == 1) barrier();          // the second wave group runs one barrier behind

  const int arow0 = wr * 128 + (lane & 15);
  uint4 a[4][2], b0[2][2], b1[2][2];
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const char* sA = smem + cur * STAGE;
    const char* sB = sA + IMG;
    const uint32_t nxt = sl + (cur ^ 1) * STAGE;
    // phase 0: quadrant (rows 0-63, cols 0-31)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int c = 0; c < 2; ++c) a[i][c] = big_frag_a(sA, arow0 + 16 * i, c, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int c = 0; c < 2; ++c) b0[j][c] = big_frag_b(sB, big_brow(wc, j, lane), c, lane);
    barrier();
    wait_lgkm0();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) Mma<bf16_t>::run(acc[i][j], b0[j][c], a[i][c]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    barrier();
    // phase 1: quadrant (rows 0-63, cols 32-63); DMA rows 128-255 of tile t+1
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int c = 0; c < 2; ++c) b1[j][c] = big_frag_b(sB, big_brow(wc, 2 + j, lane), c, lane);
    if (t + 1 < nt) {
      big_issue<false>(ra, g.lda, 1, 64 * (t + 1), nxt, wave, lane);
      big_issue<true>(rb, g.ldb, 1, 64 * (t + 1), nxt + IMG, wave, lane);
    }
    barrier();
    wait_lgkm0();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) Mma<bf16_t>::run(acc[i][2 + j], b1[j][c], a[i][c]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    barrier();
    // phase 2: quadrant (rows 64-127, cols 32-63)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int c = 0; c < 2; ++c) a[i][c] = big_frag_a(sA, arow0 + 64 + 16 * i, c, lane);
    barrier();
    wait_lgkm0();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) Mma<bf16_t>::run(acc[4 + i][2 + j], b1[j][c], a[i][c]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    barrier();
    // phase 3: quadrant (rows 64-127, cols 0-31) from registers; tile t+1 complete; DMA
    // rows 0-127 of tile t+2 into this buffer (their last reads were phases 0-2)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (t + 2 < nt) {
      const uint32_t here = sl + cur * STAGE;
      big_issue<false>(ra, g.lda, 0, 64 * (t + 2), here, wave, lane);
      big_issue<true>(rb, g.ldb, 0, 64 * (t + 2), here + IMG, wave, lane);
    }
    barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) Mma<bf16_t>::run(acc[4 + i][j], b0[j][c], a[i][c]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    barrier();
  }
  if (wr == 0) barrier();          // balance the barrier count of the two groups

  // epilogue: lane holds rows 16i + (lane&15), columns 32p + 8(lane>>4) .. +7
  const DropKeys dk = resolve_drop(g.drop);
  const int li = lane & 15, lg = lane >> 4;
  if constexpr (EPI >= 0 && (EPI & (BE_BIAS | BE_GELU_GRAD | BE_RELU_GATE | BE_RES))) {
    // 16 items (i, p), operands DEPTH items ahead (a ring of registers once the loop is
    // unrolled).  One item ahead left each item waiting out most of an HBM round trip: with
    // one workgroup per CU the epilogue is not hidden behind another tile's main loop.
    constexpr int DEPTH = (EPI & BE_RES) ? 4 : 8;
    EpiIn buf[16];
#pragma unroll
    for (int it = 0; it < DEPTH; ++it)
      big_epi_load<EPI>(g, m0 + wr * 128 + 16 * (it >> 1) + li, n0 + wc * 64 + 32 * (it & 1) + 8 * lg, buf[it]);
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int i = it >> 1, p = it & 1;
      if (it + DEPTH < 16)
        big_epi_load<EPI>(g, m0 + wr * 128 + 16 * ((it + DEPTH) >> 1) + li,
                          n0 + wc * 64 + 32 * ((it + DEPTH) & 1) + 8 * lg, buf[it + DEPTH]);
      const int64_t m = m0 + wr * 128 + 16 * i + li;
      const int64_t n = n0 + wc * 64 + 32 * p + 8 * lg;
      if (m < g.M && n < g.N) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = g.alpha * acc[i][2 * p][e];
          v[4 + e] = g.alpha * acc[i][2 * p + 1][e];
        }
        if (n + 7 < g.N) big_epi8_pre<EPI>(g, dk, m, n, v, buf[it]);
        else big_epi8<EPI>(g, dk, m, n, v);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t m = m0 + wr * 128 + 16 * i + li;
      if (m >= g.M) continue;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int64_t n = n0 + wc * 64 + 32 * p + 8 * lg;
        if (n >= g.N) continue;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = g.alpha * acc[i][2 * p][e];
          v[4 + e] = g.alpha * acc[i][2 * p + 1][e];
        }
        big_epi8<EPI>(g, dk, m, n, v);
      }
    }
  }
}

// Big-tile dispatch: bf16 k-major operands, K % 64 == 0, enough 256x256 tiles to fill the
// chip, no split-K / colsum / row sums / row-mapped dropout, 16-byte epilogue rows.
bool big_applies(const ttmi_gemm_desc* d) {
  if (getenv("TTMI_NO_BIG")) return false;          // tuning runs only
  if (d->dtype != TTMI_BF16 || !d->a_kmajor || !d->b_kmajor || d->K % 64 || d->K == 0) return false;
  if (d->colsum || d->rowsum_a || d->drop_rows || d->split_k > 1) return false;
  if (d->N < 256 || ((d->M + 255) / 256) * ((d->N + 255) / 256) < 256) return false;
  if (!al16(d->A) || !al16(d->B) || d->lda % 8 || d->ldb % 8) return false;
  const int cb = d->c_dtype == TTMI_F32 ? 4 : 2;
  if (!al16(d->C) || (d->ldc * cb) % 16) return false;
  if (d->bias && !al16(d->bias)) return false;
  if (d->residual && (!al16(d->residual) || d->ld_res % 4)) return false;
  if (d->gate && (!al16(d->gate) || d->ld_gate % 8 || d->gate_dtype == TTMI_F32)) return false;
  // 32-bit buffer offsets within one 256-row panel
  if ((int64_t)256 * std::max(d->lda, d->ldb) * 2 >= ((int64_t)1 << 31)) return false;
  return true;
}

int big_epi_code(const ttmi_gemm_desc* d) {
  if (d->drop_p > 0.f && d->drop_rows) return BE_ANY;
  int e = 0;
  if (d->bias) e |= BE_BIAS;
  if (d->act == 1 && !d->gate) e |= BE_RELU;
  if (d->act == 2) e |= BE_GELU;
  if (d->drop_p > 0.f) e |= BE_DROP;
  if (d->gate) e |= d->act == 3 ? BE_GELU_GRAD : BE_RELU_GATE;
  if (d->residual) e |= BE_RES;
  if (d->c_dtype == TTMI_F32) e |= BE_F32;
  if (d->c_mode == 1) e |= BE_ACC;
  if (d->pre_out) e |= BE_PRE;
  return e;
}

int launch_big(const ttmi_gemm_desc* d, const GemmArgs& a, hipStream_t s) {
  BigArgs ba;
  ba.g = a;
  ba.tiles_n = (int)((a.N + 255) / 256);
  const int64_t tiles = ((a.M + 255) / 256) * (int64_t)ba.tiles_n;
  TTMI_REQUIRE(tiles < (1ll << 31), "ttmi_gemm: grid too large");
  ba.tiles = (int)tiles;
  const dim3 grid((unsigned)tiles), blk(512);
  switch (big_epi_code(d)) {
    case BE_BIAS: hipLaunchKernelGGL(gemm_big_kernel<BE_BIAS>, grid, blk, 0, s, ba); break;
    case 0: hipLaunchKernelGGL(gemm_big_kernel<0>, grid, blk, 0, s, ba); break;
    case BE_BIAS | BE_DROP | BE_RES | BE_F32:
      hipLaunchKernelGGL((gemm_big_kernel<BE_BIAS | BE_DROP | BE_RES | BE_F32>), grid, blk, 0, s, ba); break;
    case BE_RES | BE_F32: hipLaunchKernelGGL((gemm_big_kernel<BE_RES | BE_F32>), grid, blk, 0, s, ba); break;
    case BE_BIAS | BE_RES | BE_F32:
      hipLaunchKernelGGL((gemm_big_kernel<BE_BIAS | BE_RES | BE_F32>), grid, blk, 0, s, ba); break;
    case BE_GELU_GRAD: hipLaunchKernelGGL(gemm_big_kernel<BE_GELU_GRAD>, grid, blk, 0, s, ba); break;
    case BE_BIAS | BE_GELU | BE_PRE:
      hipLaunchKernelGGL((gemm_big_kernel<BE_BIAS | BE_GELU | BE_PRE>), grid, blk, 0, s, ba); break;
    // D = 256 SASRec FFN (linear1 + ReLU + dropout; its gated input grad): compiled epilogues
    // keep the operand prefetch of big_epi_load (the run-time BE_ANY form took 72 vs ~30 µs)
    case BE_BIAS | BE_RELU | BE_DROP:
      hipLaunchKernelGGL((gemm_big_kernel<BE_BIAS | BE_RELU | BE_DROP>), grid, blk, 0, s, ba); break;
    case BE_BIAS | BE_RELU: hipLaunchKernelGGL((gemm_big_kernel<BE_BIAS | BE_RELU>), grid, blk, 0, s, ba); break;
    case BE_RELU_GATE: hipLaunchKernelGGL(gemm_big_kernel<BE_RELU_GATE>, grid, blk, 0, s, ba); break;
    default: hipLaunchKernelGGL(gemm_big_kernel<BE_ANY>, grid, blk, 0, s, ba); break;
  }
  return ttmi_check_launch("ttmi_gemm");
}

int num_cus() {
  static const int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return cus > 0 ? cus : 256;
  }();
  return n;
}

int panel_epi(const ttmi_gemm_desc* d) {
  if (d->residual && d->gate) return -1;
  if (d->residual) return PE_RES;
  if (d->gate) return d->gate_dtype == TTMI_F32 ? PE_GATE_F32 : PE_GATE_BF16;
  return PE_NONE;
}

// Row-panel dispatch: bf16, both operands k-major, plain store, N in {128,..,512} with the
// W image in LDS, K % 128 == 0, many rows, 16-byte aligned epilogue operands.
bool panel_applies(const ttmi_gemm_desc* d) {
  if (getenv("TTMI_NO_PANEL")) return false;       // tuning runs only
  if (d->dtype != TTMI_BF16 || !d->a_kmajor || !d->b_kmajor || d->c_mode != 0) return false;
  if (d->colsum || d->split_k > 1 || d->drop_rows || d->M < 2048 || d->act >= 2) return false;
  if (d->N % 128 || d->N > 512 || d->K % 128 || d->K > 512) return false;
  if (d->N * (2 * d->K + 16) + d->N * 4 > 150 * 1024 || panel_epi(d) < 0) return false;
  if (d->ldc % 8 || !al16(d->C) || !al16(d->A) || !al16(d->B) || d->lda % 8 || d->ldb % 8) return false;
  if (d->bias && !al16(d->bias)) return false;
  const int64_t lim = (int64_t)INT_MAX;
  if (d->M * d->lda * 2 >= lim) return false;
  if (d->residual && (d->ld_res % 4 || !al16(d->residual) || d->M * d->ld_res * 4 >= lim)) return false;
  if (d->gate && (d->ld_gate % 8 || !al16(d->gate) || d->M * d->ld_gate * 4 >= lim)) return false;
  return true;
}

template <int NT, int KC, int EPI>
void launch_panel_t(const GemmArgs& a, hipStream_t s, const LnBwdArgs& ln = LnBwdArgs{}) {
  constexpr bool split = EPI != PE_LNBWD && EPI != PE_RESLN && NT == 32;   // N = 512 (N = 256 spilled)
  // contiguous row ranges, about one workgroup per CU; fewer than 8 tiles per workgroup
  // leaves waves idle but puts a workgroup on more CUs (M = 25,600 -> 1,600 tiles -> 229
  // workgroups of 7 instead of 200 of 8 on 256 CUs)
  const int64_t tiles = (a.M + 15) / 16;
  const int S = std::max(1, a.nslice);
  // column slices: one workgroup per CU (a 135 KB W image each) in ONE round: the row groups,
  // padded to whole XCD rounds, times the slices must not exceed the CUs (264 workgroups on
  // 256 CUs ran the D = 256 QKV panel in two rounds: 38 us)
  const int64_t rg_max = S > 1 ? std::max<int64_t>(8, (int64_t)(num_cus() / S) / 8 * 8) : (int64_t)num_cus();
  const int64_t tpw = std::max<int64_t>(1, (tiles + rg_max - 1) / rg_max);
  const int64_t rgroups = (tiles + tpw - 1) / tpw;
  // column slices: row groups padded to whole XCD rounds (panel_kernel's block decode)
  const int64_t grid = S > 1 ? (rgroups + 7) / 8 * 8 * S : rgroups;
  static const int wdma = [] {            // TTMI_PANEL_WDMA=0: VGPR staging (A/B runs only)
    const char* e = getenv("TTMI_PANEL_WDMA");
    return e ? atoi(e) : 1;
  }();
  static const int wrot = [] {            // TTMI_PANEL_WROT=0: one DMA order for all (A/B runs)
    const char* e = getenv("TTMI_PANEL_WROT");
    return e ? atoi(e) : 1;
  }();
  GemmArgs b = a;
  b.wdma = wdma && a.ldb * 2 * a.N < ((int64_t)1 << 31);
  b.wrot = wrot;
  b.nslice = S;
  b.rgroups = (int)rgroups;
  static const int cs = [] {              // TTMI_PANEL_CS=1: no column split (A/B runs only)
    const char* e = getenv("TTMI_PANEL_CS");
    return e ? atoi(e) : 2;
  }();
  if (split && cs == 2)
    hipLaunchKernelGGL((panel_kernel<NT, KC, EPI, split ? 2 : 1>), dim3((unsigned)grid), dim3(split ? 1024 : 512), 0, s, b,
                       (int)tpw, ln);
  else
    hipLaunchKernelGGL((panel_kernel<NT, KC, EPI, 1>), dim3((unsigned)grid), dim3(512), 0, s, b, (int)tpw, ln);
}

// Column-sliced row panels (N a multiple of 256 past what one W image in LDS holds, K = 256:
// the D = 256 encoder's QKV / FFN1 forward and FFN2 input grad): nslice panels of 256 columns.
int panel_slices(const ttmi_gemm_desc* d) {
  if (getenv("TTMI_NO_PANEL") || getenv("TTMI_NO_PANEL_SLICE")) return 0;
  if (d->dtype != TTMI_BF16 || !d->a_kmajor || !d->b_kmajor || d->c_mode != 0) return 0;
  if (d->colsum || d->split_k > 1 || d->drop_rows || d->M < 2048 || d->act >= 2) return 0;
  if (d->K != 256 || d->N % 256 || d->N < 512 || d->N > 4096) return 0;
  const int E = panel_epi(d);
  if (E != PE_NONE && E != PE_GATE_BF16) return 0;
  if (d->ldc % 8 || !al16(d->C) || !al16(d->A) || !al16(d->B) || d->lda % 8 || d->ldb % 8) return 0;
  if (d->bias && !al16(d->bias)) return 0;
  const int64_t lim = (int64_t)INT_MAX;
  if (d->M * d->lda * 2 >= lim || d->N * d->ldb * 2 >= lim) return 0;
  if (d->gate && (d->ld_gate % 8 || !al16(d->gate) || d->M * d->ld_gate * 4 >= lim)) return 0;
  return (int)(d->N / 256);
}

bool launch_panel_sliced(const ttmi_gemm_desc* d, const GemmArgs& a0, int S, hipStream_t s) {
  GemmArgs a = a0;
  a.N = 256;
  a.nslice = S;
  if (panel_epi(d) == PE_GATE_BF16) launch_panel_t<16, 8, PE_GATE_BF16>(a, s);
  else launch_panel_t<16, 8, PE_NONE>(a, s);
  return true;
}

bool launch_panel(const ttmi_gemm_desc* d, const GemmArgs& a, hipStream_t s) {
  const int NT = (int)(a.N / 16), KC = (int)(a.K / 32), E = panel_epi(d);
#define TTMI_PANEL(nt, kc, e) if (NT == nt && KC == kc && E == e) { launch_panel_t<nt, kc, e>(a, s); return true; }
  TTMI_PANEL(8, 4, PE_NONE) TTMI_PANEL(8, 4, PE_RES) TTMI_PANEL(8, 4, PE_GATE_BF16)      // N=128
  TTMI_PANEL(8, 12, PE_NONE) TTMI_PANEL(8, 16, PE_NONE) TTMI_PANEL(8, 16, PE_RES)
  TTMI_PANEL(16, 4, PE_NONE) TTMI_PANEL(16, 8, PE_NONE) TTMI_PANEL(16, 8, PE_GATE_BF16)  // N=256
  TTMI_PANEL(24, 4, PE_NONE)                                                             // N=384
  TTMI_PANEL(32, 4, PE_NONE) TTMI_PANEL(32, 4, PE_GATE_BF16) TTMI_PANEL(32, 4, PE_GATE_F32)  // N=512
#undef TTMI_PANEL
  return false;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// panel256_kernel's grid: one tile group (<= 8 tiles) per workgroup, about one per CU
int64_t panel256_tpw(int64_t M) {
  const int64_t tiles = (M + 15) / 16;
  return std::min<int64_t>(8, std::max<int64_t>(1, (tiles + num_cus() - 1) / num_cus()));
}

template <int EPI>
int launch_panel256(const GemmArgs& a, const LnBwdArgs& ln, hipStream_t s) {
  const int64_t tiles = (a.M + 15) / 16, tpw = panel256_tpw(a.M);
  const dim3 grid((unsigned)((tiles + tpw - 1) / tpw));
  static const int wrot = [] {
    const char* e = getenv("TTMI_PANEL_WROT");
    return e ? atoi(e) : 1;
  }();
  GemmArgs b = a;
  b.wrot = wrot;
  switch (a.K) {
    case 256: hipLaunchKernelGGL((panel256_kernel<4, EPI>), grid, dim3(512), 0, s, b, (int)tpw, ln); break;
    case 512: hipLaunchKernelGGL((panel256_kernel<8, EPI>), grid, dim3(512), 0, s, b, (int)tpw, ln); break;
    case 768: hipLaunchKernelGGL((panel256_kernel<12, EPI>), grid, dim3(512), 0, s, b, (int)tpw, ln); break;
    default: hipLaunchKernelGGL((panel256_kernel<16, EPI>), grid, dim3(512), 0, s, b, (int)tpw, ln); break;
  }
  return TTMI_OK;
}

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
  TTMI_REQUIRE(d->act >= 0 && d->act <= 3, "ttmi_gemm: bad act");
  TTMI_REQUIRE(d->act != 3 || d->gate, "ttmi_gemm: act 3 (GELU backward) needs the pre-activation as gate");
  TTMI_REQUIRE(d->drop_p >= 0.f && d->drop_p < 1.f, "ttmi_gemm: drop_p out of [0,1)");
  TTMI_REQUIRE(d->drop_p == 0.f || d->drop_seed, "ttmi_gemm: dropout needs a seed pointer");
  TTMI_REQUIRE(!d->gate || d->ld_gate >= d->N, "ttmi_gemm: ld_gate < N");
  TTMI_REQUIRE(!d->residual || d->ld_res >= d->N, "ttmi_gemm: ld_res < N");
  TTMI_REQUIRE(!d->pre_out || (d->act == 2 && d->c_mode == 0 && d->c_dtype == TTMI_BF16 &&
                               d->drop_p == 0.f && !d->gate && !d->residual && !d->colsum &&
                               d->split_k <= 1 && ((uintptr_t)d->pre_out & 15) == 0),
               "ttmi_gemm: pre_out needs act 2, a bf16 C written once, no dropout/gate/residual/"
               "colsum/split, 16-byte alignment");

  if (wgrad_applies(d)) return launch_wgrad(d, stream);

  const int bke = 128 / es;
  int bm, bn;
  const int64_t tiles128 = ((d->M + 127) / 128) * ((d->N + 127) / 128);
  const int64_t tiles64x128 = ((d->M + 63) / 64) * ((d->N + 127) / 128);
  const int64_t tiles64 = ((d->M + 63) / 64) * ((d->N + 63) / 64);
  if (es == 4 && d->K <= 256 && tiles64 >= 256) { bm = 64; bn = 64; }   // short-K fp32 (catalogue
                                                                           // scores): 24 vs 30 us
  else if (d->N > 64 && tiles128 >= 256) { bm = 128; bn = 128; }
  else if (d->N > 64 && tiles64x128 >= 128) { bm = 64; bn = 128; }
  else if (tiles64 < 128 && d->c_mode == 0) { bm = 32; bn = 32; }   // small GEMMs: fill the CUs
  else { bm = 64; bn = 64; }
  if (const char* e = getenv("TTMI_GEMM_TILE")) {     // tuning runs only
    int tm = 0, tn = 0;
    if (sscanf(e, "%dx%d", &tm, &tn) == 2 && (tm == 64 || tm == 128) && (tn == 64 || tn == 128)) {
      bm = tm; bn = tn;
    }
  }
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

  GemmArgs a{};
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.A = static_cast<const char*>(d->A); a.lda = d->lda;
  a.B = static_cast<const char*>(d->B); a.ldb = d->ldb;
  a.C = d->C; a.ldc = d->ldc; a.c_f32 = d->c_dtype == TTMI_F32; a.c_mode = d->c_mode;
  a.alpha = d->alpha;
  a.bias = d->bias; a.act = d->act;
  a.drop = make_drop(d->drop_p, d->drop_seed); a.ld_drop = d->ld_drop ? d->ld_drop : d->N;
  a.drop_rows = d->drop_rows;
  a.gate = d->gate; a.gate_f32 = d->gate_dtype == TTMI_F32; a.ld_gate = d->ld_gate;
  a.gate_scale = d->gate_scale;
  a.residual = d->residual; a.ld_res = d->ld_res;
  a.colsum = d->colsum;
  a.k_split = kspl;
  a.rowsum_a = d->rowsum_a;
  a.pre_out = static_cast<bf16_t*>(d->pre_out);
  const int cbytes = a.c_f32 ? 4 : 2;
  a.vec = (d->ldc % 4 == 0) && ((uintptr_t)d->C % (4 * cbytes) == 0) &&
          (!d->residual || (d->ld_res % 4 == 0 && (uintptr_t)d->residual % 16 == 0)) &&
          (!d->gate || (d->ld_gate % 4 == 0 && (uintptr_t)d->gate % 16 == 0));

  if (panel_applies(d) && launch_panel(d, a, stream)) return ttmi_check_launch("ttmi_gemm");
  if (const int S = panel_slices(d)) {
    launch_panel_sliced(d, a, S, stream);
    return ttmi_check_launch("ttmi_gemm");
  }
  if (big_applies(d)) return launch_big(d, a, stream);
  dim3 grid((unsigned)gx, (unsigned)gy, (unsigned)split);
  if (d->dtype == TTMI_BF16) launch_typed<bf16_t>(a, d->a_kmajor, d->b_kmajor, bm, bn, grid, stream);
  else launch_typed<float>(a, d->a_kmajor, d->b_kmajor, bm, bn, grid, stream);
  return ttmi_check_launch("ttmi_gemm");
}

extern "C" int ttmi_linear_res_ln(const ttmi_linear_res_ln_desc* d, hipStream_t stream) {
  TTMI_REQUIRE(d != nullptr, "ttmi_linear_res_ln: null descriptor");
  TTMI_REQUIRE(d->M >= 0 && (d->N == 128 || d->N == 256), "ttmi_linear_res_ln: N must be 128 or 256 (got %lld)",
               (long long)d->N);
  TTMI_REQUIRE(d->N == 256 || (d->K > 0 && d->K % 128 == 0 && d->K <= 512),
               "ttmi_linear_res_ln: N = 128 needs K in {128, 256, 384, 512}");
  TTMI_REQUIRE(d->N == 128 || (d->K >= 256 && d->K % 256 == 0 && d->K <= 1024),
               "ttmi_linear_res_ln: N = 256 needs K in {256, 512, 768, 1024}");
  if (d->M == 0) return TTMI_OK;
  const int64_t NN = d->N;
  TTMI_REQUIRE(d->x && d->w && d->residual && d->out && d->ln_w && d->ln_b && d->y && d->mean && d->rstd,
               "ttmi_linear_res_ln: null argument");
  TTMI_REQUIRE(al16(d->x) && al16(d->w) && d->ldx % 8 == 0 && d->ldw % 8 == 0 && d->ldx >= d->K &&
               d->ldw >= d->K, "ttmi_linear_res_ln: x/w need 16-byte rows");
  TTMI_REQUIRE(al16(d->residual) && d->ld_res % 4 == 0 && d->ld_res >= NN && al16(d->out) &&
               d->ld_out % 4 == 0 && d->ld_out >= NN, "ttmi_linear_res_ln: residual/out need 16-byte rows");
  TTMI_REQUIRE(al16(d->y) && d->ldy % 8 == 0 && d->ldy >= NN, "ttmi_linear_res_ln: y needs 16-byte rows");
  TTMI_REQUIRE(NN == 128 || (d->M * d->ldx * 2 < ((int64_t)1 << 32) && (NN * d->ldw) * 2 < ((int64_t)1 << 32)),
               "ttmi_linear_res_ln: N = 256 needs x and w under 4 GB (32-bit DMA offsets)");
  TTMI_REQUIRE(NN == 128 || ((!d->bias || al16(d->bias)) && al16(d->ln_w) && al16(d->ln_b)),
               "ttmi_linear_res_ln: N = 256 needs 16-byte aligned bias / LayerNorm parameters");
  TTMI_REQUIRE(d->drop_p >= 0.f && d->drop_p < 1.f && (d->drop_p == 0.f || d->drop_seed),
               "ttmi_linear_res_ln: bad dropout");
  GemmArgs a{};
  a.M = d->M; a.N = NN; a.K = d->K;
  a.A = static_cast<const char*>(d->x); a.lda = d->ldx;
  a.B = static_cast<const char*>(d->w); a.ldb = d->ldw;
  a.C = d->out; a.ldc = d->ld_out; a.c_f32 = 1;
  a.alpha = 1.f;
  a.bias = d->bias;
  a.drop = make_drop(d->drop_p, d->drop_seed); a.ld_drop = d->ld_drop ? d->ld_drop : NN;
  a.residual = d->residual; a.ld_res = d->ld_res;
  LnBwdArgs ln{};
  ln.w = d->ln_w; ln.lnb = d->ln_b; ln.eps = d->eps;
  ln.y = static_cast<bf16_t*>(d->y); ln.ldy = d->ldy;
  ln.mean_out = d->mean; ln.rstd_out = d->rstd;
  if (NN == 256) {
    launch_panel256<PE_RESLN>(a, ln, stream);
    return ttmi_check_launch("ttmi_linear_res_ln");
  }
  switch (d->K) {
    case 128: launch_panel_t<8, 4, PE_RESLN>(a, stream, ln); break;
    case 256: launch_panel_t<8, 8, PE_RESLN>(a, stream, ln); break;
    case 384: launch_panel_t<8, 12, PE_RESLN>(a, stream, ln); break;
    default: launch_panel_t<8, 16, PE_RESLN>(a, stream, ln); break;
  }
  return ttmi_check_launch("ttmi_linear_res_ln");
}

extern "C" int ttmi_linear_ln_bwd(const ttmi_linear_ln_bwd_desc* d, hipStream_t stream) {
  TTMI_REQUIRE(d != nullptr, "ttmi_linear_ln_bwd: null descriptor");
  TTMI_REQUIRE(d->M >= 0 && (d->N == 128 || d->N == 256), "ttmi_linear_ln_bwd: N must be 128 or 256 (got %lld)",
               (long long)d->N);
  TTMI_REQUIRE(d->N == 256 || (d->K > 0 && d->K % 128 == 0 && d->K <= 512),
               "ttmi_linear_ln_bwd: N = 128 needs K in {128, 256, 384, 512}");
  TTMI_REQUIRE(d->N == 128 || (d->K >= 256 && d->K % 256 == 0 && d->K <= 1024),
               "ttmi_linear_ln_bwd: N = 256 needs K in {256, 512, 768, 1024}");
  if (d->M == 0) return TTMI_OK;
  const int64_t NN = d->N;
  TTMI_REQUIRE(d->dh && d->wt && d->x && d->mean && d->rstd && d->ln_w && d->dx,
               "ttmi_linear_ln_bwd: null argument");
  TTMI_REQUIRE(al16(d->dh) && al16(d->wt) && d->ld_dh % 8 == 0 && d->ld_wt % 8 == 0 &&
               d->ld_dh >= d->K && d->ld_wt >= d->K, "ttmi_linear_ln_bwd: dh/wt need 16-byte rows");
  TTMI_REQUIRE(al16(d->x) && d->ldx % 4 == 0 && d->ldx >= NN && al16(d->dx) && d->lddx % 4 == 0 &&
               d->lddx >= NN, "ttmi_linear_ln_bwd: x/dx need 16-byte rows");
  TTMI_REQUIRE(!d->res || (al16(d->res) && d->ld_res % 4 == 0 && d->ld_res >= NN),
               "ttmi_linear_ln_bwd: res needs 16-byte rows");
  TTMI_REQUIRE(NN == 128 || (d->M * d->ld_dh * 2 < ((int64_t)1 << 32) && (NN * d->ld_wt) * 2 < ((int64_t)1 << 32)
                             && al16(d->ln_w)),
               "ttmi_linear_ln_bwd: N = 256 needs dh and wt under 4 GB and an aligned LayerNorm weight");
  TTMI_REQUIRE(!d->res_rows || (d->res && d->res_L > 0), "ttmi_linear_ln_bwd: res_rows needs res and res_L > 0");
  TTMI_REQUIRE(!d->dy_add || (d->res_rows && NN == 128 && al16(d->dy_add) && d->ld_add % 4 == 0 && d->ld_add >= NN),
               "ttmi_linear_ln_bwd: dy_add needs res_rows, N = 128 and 16-byte rows");
  TTMI_REQUIRE(!d->next || (al16(d->next) && d->ld_next % 8 == 0 && d->ld_next >= NN),
               "ttmi_linear_ln_bwd: next needs 16-byte rows");
  TTMI_REQUIRE(d->drop_p >= 0.f && d->drop_p < 1.f && (d->drop_p == 0.f || d->drop_seed),
               "ttmi_linear_ln_bwd: bad dropout");
  GemmArgs a{};
  a.M = d->M; a.N = NN; a.K = d->K;
  a.A = static_cast<const char*>(d->dh); a.lda = d->ld_dh;
  a.B = static_cast<const char*>(d->wt); a.ldb = d->ld_wt;
  a.alpha = 1.f;
  a.drop = make_drop(0.f, nullptr);
  LnBwdArgs ln{};
  ln.x = d->x; ln.ldx = d->ldx; ln.mean = d->mean; ln.rstd = d->rstd; ln.w = d->ln_w;
  ln.res = d->res; ln.ld_res = d->ld_res;
  ln.res_rows = d->res_rows; ln.res_L = d->res_L;
  ln.dy_add = d->dy_add; ln.ld_add = d->ld_add;
  ln.dx = d->dx; ln.lddx = d->lddx;
  ln.next = static_cast<bf16_t*>(d->next); ln.ld_next = d->ld_next;
  ln.drop = make_drop(d->drop_p, d->drop_seed); ln.ld_drop = d->ld_drop ? d->ld_drop : NN;
  ln.drop_rows = d->drop_rows;
  ln.dw = d->ln_dw; ln.db = d->ln_db;
  ln.sum_ws = d->sum_ws;
  if (NN == 256) {
    launch_panel256<PE_LNBWD>(a, ln, stream);
    return ttmi_check_launch("ttmi_linear_ln_bwd");
  }
  switch (d->K) {
    case 128: launch_panel_t<8, 4, PE_LNBWD>(a, stream, ln); break;
    case 256: launch_panel_t<8, 8, PE_LNBWD>(a, stream, ln); break;
    case 384: launch_panel_t<8, 12, PE_LNBWD>(a, stream, ln); break;
    default: launch_panel_t<8, 16, PE_LNBWD>(a, stream, ln); break;
  }
  return ttmi_check_launch("ttmi_linear_ln_bwd");
}

namespace {
int wgrad_check(const ttmi_wgrad_desc* d) {
  TTMI_REQUIRE(d != nullptr, "ttmi_wgrad: null descriptor");
  TTMI_REQUIRE(d->R >= 0 && d->M > 0 && d->N > 0, "ttmi_wgrad: bad sizes");
  TTMI_REQUIRE(d->dy && d->x && d->dw, "ttmi_wgrad: null operand");
  TTMI_REQUIRE(d->M % 8 == 0 && d->N % 8 == 0, "ttmi_wgrad: M and N must be multiples of 8");
  TTMI_REQUIRE(d->ld_dy >= d->M && d->ld_x >= d->N && d->ld_dw >= d->N && d->ld_dw % 4 == 0,
               "ttmi_wgrad: bad leading dimensions");
  TTMI_REQUIRE(al16(d->dy) && al16(d->x) && al16(d->dw) && d->ld_dy % 8 == 0 && d->ld_x % 8 == 0,
               "ttmi_wgrad: operands must be 16-byte aligned");
  return TTMI_OK;
}

WgradArgs wgrad_args(const ttmi_wgrad_desc* d, const WgradPlan& p) {
  WgradArgs a;
  a.M = d->M; a.N = d->N; a.R = d->R;
  a.A = static_cast<const char*>(d->dy); a.lda = d->ld_dy;
  a.B = static_cast<const char*>(d->x); a.ldb = d->ld_x;
  a.C = d->dw; a.ldc = d->ld_dw;
  a.alpha = d->alpha;
  a.rowsum_a = d->db;
  a.rows_per_split = p.sps * 64;
  a.tiles_m = p.tiles_m; a.tiles_n = p.tiles_n; a.splits = p.S;
  a.xcd_remap = p.S % 8 == 0;
  a.accumulate = d->accumulate;
  a.mode = p.S > 1 ? WG_SLAB : WG_DIRECT;
  a.part = static_cast<float*>(d->workspace);
  a.part_rs = p.S > 1 ? reinterpret_cast<float*>(static_cast<char*>(d->workspace) +
                                                  al256((int64_t)p.S * d->M * d->N * 4)) : nullptr;
  return a;
}

FoldSeg fold_seg(const ttmi_wgrad_desc* d, const WgradPlan& p) {
  FoldSeg f;
  f.part = static_cast<const float*>(d->workspace);
  f.part_rs = reinterpret_cast<const float*>(static_cast<const char*>(d->workspace) +
                                             al256((int64_t)p.S * d->M * d->N * 4));
  f.C = d->dw; f.rs = d->db;
  f.M = d->M; f.N = d->N; f.ldc = d->ld_dw;
  f.units = d->M * (d->N / 4) + (d->db ? d->M : 0);
  f.base = 0;
  f.s_stride = d->M * d->N;
  f.S = p.S; f.acc = d->accumulate; f.fx = 0;
  return f;
}

int launch_fold(FoldArgs& a, hipStream_t s) {
  if (a.n == 0 || a.total == 0) return TTMI_OK;
  a.blk_begin[0] = 0;
  for (int k = 0; k < a.n; ++k) {
    const int per = a.seg[k].S <= FOLD_NARROW_S ? 256 : a.seg[k].S > FOLD_WIDE_S ? 16 : 64;   // units per block pass
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>((a.seg[k].units + per - 1) / per, 1024));
    a.blk_begin[k + 1] = a.blk_begin[k] + (int)nb;
  }
  hipLaunchKernelGGL(wgrad_fold_kernel, dim3((unsigned)a.blk_begin[a.n]), dim3(256), 0, s, a);
  return ttmi_check_launch("ttmi_wgrad_fold");
}
}  // namespace

extern "C" int64_t ttmi_wgrad_workspace(int64_t R, int64_t M, int64_t N, int64_t ld_dy,
                                        int64_t ld_x) {
  if (R <= 0 || M <= 0 || N <= 0) return 0;
  const int64_t ldmax = std::max(ld_dy, ld_x);
  return std::max(wgrad_ws_bytes(wgrad_plan(R, M, N, ldmax), M, N),
                  wgrad_ws_bytes(wgrad_group_plan(R, M, N, ldmax), M, N));
}

extern "C" int ttmi_wgrad(const ttmi_wgrad_desc* d, hipStream_t stream) {
  int rc = wgrad_check(d);
  if (rc) return rc;
  const WgradPlan p = wgrad_plan(d->R, d->M, d->N, std::max(d->ld_dy, d->ld_x));
  if (d->R == 0) {                          // empty reduction: dW (+)= 0
    if (d->accumulate) return TTMI_OK;
    if (hipMemset2DAsync(d->dw, (size_t)d->ld_dw * 4, 0, (size_t)d->N * 4, (size_t)d->M, stream) != hipSuccess ||
        (d->db && hipMemsetAsync(d->db, 0, (size_t)d->M * 4, stream) != hipSuccess)) {
      ttmi_set_error("ttmi_wgrad: memset failed");
      return TTMI_ERR_LAUNCH;
    }
    return TTMI_OK;
  }
  const int64_t need = wgrad_ws_bytes(p, d->M, d->N);
  TTMI_REQUIRE(need == 0 || (d->workspace && d->workspace_bytes >= need && al16(d->workspace)),
               "ttmi_wgrad: workspace of %lld bytes required", (long long)need);
  const WgradArgs a = wgrad_args(d, p);
  const int64_t nwg = (int64_t)p.tiles_m * p.tiles_n * p.S;
  TTMI_REQUIRE(nwg <= 2147483647LL, "ttmi_wgrad: grid too large");
  if (p.tile == 32) hipLaunchKernelGGL((wgrad_kernel<32, 32, 4>), dim3((unsigned)nwg), dim3(256), 0, stream, a);
  else hipLaunchKernelGGL((wgrad_kernel<64, 64, 4>), dim3((unsigned)nwg), dim3(256), 0, stream, a);
  rc = ttmi_check_launch("ttmi_wgrad");
  if (rc || p.S <= 1 || d->defer) return rc;
  FoldArgs f;
  f.seg[0] = fold_seg(d, p);
  f.n = 1;
  f.total = f.seg[0].units;
  return launch_fold(f, stream);
}

extern "C" int64_t ttmi_linear_ln_bwd_sum_blocks(int64_t M) {
  if (M <= 0) return 0;
  const int64_t tiles = (M + 15) / 16;
  const int64_t tpw = std::max<int64_t>(1, (tiles + num_cus() - 1) / num_cus());
  return (tiles + tpw - 1) / tpw;     // launch_panel_t's grid
}

extern "C" int64_t ttmi_linear_ln_bwd_sum_blocks_n(int64_t M, int64_t N) {
  if (N != 256) return ttmi_linear_ln_bwd_sum_blocks(M);
  if (M <= 0) return 0;
  const int64_t tiles = (M + 15) / 16, tpw = panel256_tpw(M);
  return (tiles + tpw - 1) / tpw;     // launch_panel256's grid
}

namespace {
int wgrad_fold_impl(int n, const ttmi_wgrad_desc* const* descs, int nf, const ttmi_fold_desc* folds,
                    hipStream_t stream, bool grouped, std::vector<FoldSeg>* collect = nullptr) {
  TTMI_REQUIRE(n >= 0 && (n == 0 || descs) && nf >= 0 && (nf == 0 || folds),
               "ttmi_wgrad_fold: bad arguments");
  FoldArgs f;
  f.n = 0;
  f.total = 0;
  for (int i = 0; i < nf; ++i) {
    const ttmi_fold_desc* d = folds + i;
    TTMI_REQUIRE(d->part && d->C && d->S > 0 && d->M > 0 && d->N > 0 && d->N % 4 == 0 &&
                 d->ldc % 4 == 0 && d->s_stride >= d->M * d->N && d->s_stride % 4 == 0 &&
                 al16(d->part) && al16(d->C) && d->fx_shift >= 0 && d->fx_shift < 63,
                 "ttmi_wgrad_fold: bad fold descriptor %d", i);
    if (f.n == FOLD_SEGS) {
      int rc = launch_fold(f, stream);
      if (rc) return rc;
      f.n = 0;
      f.total = 0;
    }
    FoldSeg sg;
    sg.part = d->part; sg.part_rs = nullptr; sg.C = d->C; sg.rs = nullptr;
    sg.M = d->M; sg.N = d->N; sg.ldc = d->ldc; sg.units = d->M * (d->N / 4);
    sg.base = f.total; sg.s_stride = d->s_stride;
    sg.S = (int)d->S; sg.acc = d->accumulate; sg.fx = d->fx_shift;
    if (collect) { collect->push_back(sg); continue; }
    f.seg[f.n++] = sg;
    f.total += sg.units;
  }
  for (int i = 0; i < n; ++i) {
    const ttmi_wgrad_desc* d = descs[i];
    int rc = wgrad_check(d);
    if (rc) return rc;
    const int64_t ldmax = std::max(d->ld_dy, d->ld_x);
    const WgradPlan p = grouped ? wgrad_group_plan(d->R, d->M, d->N, ldmax)
                                : wgrad_plan(d->R, d->M, d->N, ldmax);
    if (p.S <= 1 || d->R == 0) continue;     // written directly by ttmi_wgrad
    TTMI_REQUIRE(d->workspace, "ttmi_wgrad_fold: descriptor %d has no workspace", i);
    if (f.n == FOLD_SEGS) {
      rc = launch_fold(f, stream);
      if (rc) return rc;
      f.n = 0;
      f.total = 0;
    }
    FoldSeg sg = fold_seg(d, p);
    sg.base = f.total;
    if (collect) { collect->push_back(sg); continue; }
    f.seg[f.n++] = sg;
    f.total += sg.units;
  }
  return launch_fold(f, stream);
}
}  // namespace

extern "C" int ttmi_wgrad_fold(int n, const ttmi_wgrad_desc* const* descs, int nf,
                               const ttmi_fold_desc* folds, hipStream_t stream) {
  return wgrad_fold_impl(n, descs, nf, folds, stream, false);
}

namespace {
int wgrad_batch_impl(int n, const ttmi_wgrad_desc* const* descs, int nf, const ttmi_fold_desc* folds,
                     hipStream_t stream, std::vector<FoldSeg>* collect) {
  TTMI_REQUIRE(n >= 0 && (n == 0 || descs) && nf >= 0 && (nf == 0 || folds),
               "ttmi_wgrad_batch: bad arguments");
  WgradGroup grp;
  grp.n = 0;
  grp.wg_begin[0] = 0;
  const int tile = wgrad_group_cfg().tile;
  auto flush = [&]() -> int {
    if (grp.n == 0) return TTMI_OK;
    static const int ns = [] {               // TTMI_WGRAD_NS=5: 5-deep ring (tuning runs)
      const char* e = getenv("TTMI_WGRAD_NS");
      return e ? atoi(e) : 4;
    }();
    if (tile == 128 && ns == 5)
      hipLaunchKernelGGL((wgrad_group_kernel<128, 128, 5>), dim3((unsigned)grp.wg_begin[grp.n]), dim3(256), 0,
                         stream, grp);
    else if (tile == 128)
      hipLaunchKernelGGL((wgrad_group_kernel<128, 128, 4>), dim3((unsigned)grp.wg_begin[grp.n]), dim3(256), 0,
                         stream, grp);
    else
      hipLaunchKernelGGL((wgrad_group_kernel<64, 64, 4>), dim3((unsigned)grp.wg_begin[grp.n]), dim3(256), 0,
                         stream, grp);
    grp.n = 0;
    grp.wg_begin[0] = 0;
    return ttmi_check_launch("ttmi_wgrad_batch");
  };
  // entries in decreasing rows per split (longest workgroups first): when a group needs more
  // than one round of workgroups (D = 256), the long ones must not be the ones left for the
  // second round.  The order changes no result: each GEMM's splits and sums are its own.
  std::vector<int> order(n);
  std::vector<int64_t> len(n, 0);
  for (int i = 0; i < n; ++i) {
    const ttmi_wgrad_desc* d = descs[i];
    int rc = wgrad_check(d);
    if (rc) return rc;
    order[i] = i;
    if (d->R > 0) len[i] = wgrad_group_plan(d->R, d->M, d->N, std::max(d->ld_dy, d->ld_x)).sps;
  }
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return len[x] > len[y]; });
  for (int oi = 0; oi < n; ++oi) {
    const int i = order[oi];
    const ttmi_wgrad_desc* d = descs[i];
    int rc;
    if (d->R == 0) {                                   // dW (+)= 0: no reduction to group
      ttmi_wgrad_desc z = *d;
      z.defer = 1;
      rc = ttmi_wgrad(&z, stream);
      if (rc) return rc;
      continue;
    }
    const WgradPlan p = wgrad_group_plan(d->R, d->M, d->N, std::max(d->ld_dy, d->ld_x));
    const int64_t need = wgrad_ws_bytes(p, d->M, d->N);
    TTMI_REQUIRE(need == 0 || (d->workspace && d->workspace_bytes >= need && al16(d->workspace)),
                 "ttmi_wgrad_batch: descriptor %d needs a workspace of %lld bytes", i,
                 (long long)need);
    // tiles re-reading a split's rows grouped on one XCD (xcd_remap 2): the entry starts at a
    // multiple of 8 blocks and its (split, tile) pairs are padded to a multiple of 8
    const int64_t T = (int64_t)p.tiles_m * p.tiles_n;
    const bool chunk = p.S > 1 && T > 1 && wgrad_group_chunked();
    const int64_t nwg = chunk ? (T * p.S + 7) / 8 * 8 : T * p.S;
    if (grp.n == WG_GROUP || (int64_t)grp.wg_begin[grp.n] + nwg + 8 > 2147483647LL) {
      rc = flush();
      if (rc) return rc;
    }
    if (chunk) grp.wg_begin[grp.n] = (grp.wg_begin[grp.n] + 7) / 8 * 8;
    grp.e[grp.n] = wgrad_args(d, p);
    if (chunk) grp.e[grp.n].xcd_remap = 2;
    grp.wg_begin[grp.n + 1] = grp.wg_begin[grp.n] + (int)nwg;
    ++grp.n;
  }
  int rc = flush();
  if (rc) return rc;
  return wgrad_fold_impl(n, descs, nf, folds, stream, true, collect);
}

// The segments of a plan, launched as ordinary folds (the fused update's fallback).
int launch_fold_segs(const FoldSeg* segs, int n, hipStream_t s) {
  FoldArgs f;
  f.n = 0;
  f.total = 0;
  for (int i = 0; i < n; ++i) {
    if (f.n == FOLD_SEGS) {
      int rc = launch_fold(f, s);
      if (rc) return rc;
      f.n = 0;
      f.total = 0;
    }
    f.seg[f.n] = segs[i];
    f.seg[f.n].base = f.total;
    f.total += segs[i].units;
    ++f.n;
  }
  return launch_fold(f, s);
}

int fold_blocks(const FoldSeg& sg) {        // launch_fold's per-segment block count
  const int per = sg.S <= FOLD_NARROW_S ? 256 : sg.S > FOLD_WIDE_S ? 16 : 64;
  return (int)std::max<int64_t>(1, std::min<int64_t>((sg.units + per - 1) / per, 1024));
}
}  // namespace

extern "C" int ttmi_wgrad_batch(int n, const ttmi_wgrad_desc* const* descs, int nf,
                                const ttmi_fold_desc* folds, hipStream_t stream) {
  return wgrad_batch_impl(n, descs, nf, folds, stream, nullptr);
}

static_assert(sizeof(FoldSeg) * AF_SEGS <= sizeof(((ttmi_fold_plan*)nullptr)->seg), "fold plan storage");

extern "C" int ttmi_wgrad_batch_plan(int n, const ttmi_wgrad_desc* const* descs, int nf,
                                     const ttmi_fold_desc* folds, ttmi_fold_plan* plan, hipStream_t stream) {
  TTMI_REQUIRE(plan != nullptr, "ttmi_wgrad_batch_plan: null plan");
  plan->n = 0;
  std::vector<FoldSeg> segs;
  int rc = wgrad_batch_impl(n, descs, nf, folds, stream, &segs);
  if (rc) return rc;
  if ((int)segs.size() > AF_SEGS || getenv("TTMI_NO_FOLD_PLAN"))   // too many: fold them now
    return launch_fold_segs(segs.data(), (int)segs.size(), stream);
  memcpy(plan->seg, segs.data(), segs.size() * sizeof(FoldSeg));
  plan->n = (int32_t)segs.size();
  return TTMI_OK;
}

extern "C" int ttmi_fold_plan_run(const ttmi_fold_plan* plan, hipStream_t stream) {
  TTMI_REQUIRE(plan && plan->n >= 0 && plan->n <= AF_SEGS, "ttmi_fold_plan_run: bad plan");
  if (plan->n == 0) return TTMI_OK;
  return launch_fold_segs(reinterpret_cast<const FoldSeg*>(plan->seg), plan->n, stream);
}

extern "C" int ttmi_fold_plan_merge(ttmi_fold_plan* dst, const ttmi_fold_plan* src, hipStream_t stream) {
  TTMI_REQUIRE(dst && src && dst->n >= 0 && dst->n <= AF_SEGS && src->n >= 0 && src->n <= AF_SEGS,
               "ttmi_fold_plan_merge: bad plan");
  const FoldSeg* b = reinterpret_cast<const FoldSeg*>(src->seg);
  if (dst->n + src->n > AF_SEGS) return launch_fold_segs(b, src->n, stream);   // no room: fold now
  memcpy(reinterpret_cast<FoldSeg*>(dst->seg) + dst->n, b, (size_t)src->n * sizeof(FoldSeg));
  dst->n += src->n;
  return TTMI_OK;
}

extern "C" int ttmi_adamw_folded(int64_t n, float* p, float* g, float* m, float* v, uint16_t* p_bf16,
                                 const double* hyper, const int32_t* step, int zero_grad, int64_t* fx,
                                 int64_t fx_off, int64_t fx_len, int fx_shift, const ttmi_fold_plan* plan,
                                 const int32_t* skip_if, hipStream_t s) {
  return ttmi_adamw_folded_skip(n, p, g, m, v, p_bf16, hyper, step, zero_grad, fx, fx_off, fx_len, fx_shift,
                                plan, 0, 0, skip_if, s);
}

extern "C" int ttmi_adamw_folded_skip(int64_t n, float* p, float* g, float* m, float* v, uint16_t* p_bf16,
                                      const double* hyper, const int32_t* step, int zero_grad, int64_t* fx,
                                      int64_t fx_off, int64_t fx_len, int fx_shift, const ttmi_fold_plan* plan,
                                      int64_t skip_off, int64_t skip_len, const int32_t* skip_if,
                                      hipStream_t s) {
  TTMI_REQUIRE(skip_len == 0 || (!fx && skip_off >= 0 && skip_len > 0 && skip_off % 4 == 0 && skip_len % 4 == 0 &&
                                 skip_off + skip_len <= n),
               "ttmi_adamw_folded_skip: the skipped range must be float4-aligned, inside [0, n), without fx");
  if (skip_len > 0 && (!plan || plan->n <= 0 || n % 4 != 0)) {   // the plain update around it
    int rc = plan && plan->n > 0 ? launch_fold_segs(reinterpret_cast<const FoldSeg*>(plan->seg), plan->n, s) : 0;
    if (rc) return rc;
    const int64_t e = skip_off + skip_len;
    rc = ttmi_adamw(skip_off, p, g, m, v, p_bf16, hyper, step, zero_grad, skip_if, s);
    if (rc) return rc;
    return ttmi_adamw(n - e, p + e, g + e, m + e, v + e, p_bf16 ? p_bf16 + e : nullptr, hyper, step, zero_grad,
                      skip_if, s);
  }
  if (!plan || plan->n <= 0)
    return ttmi_adamw_fx(n, p, g, m, v, p_bf16, hyper, step, zero_grad, fx, fx_off, fx_len, fx_shift, skip_if, s);
  TTMI_REQUIRE(plan->n <= AF_SEGS, "ttmi_adamw_folded: bad plan");
  const FoldSeg* segs = reinterpret_cast<const FoldSeg*>(plan->seg);
  // the flat ranges the segments update (float4 units), which the plain jobs then skip
  std::vector<std::pair<int64_t, int64_t>> cov;
  bool ok = n % 4 == 0 && n / 4 < INT_MAX && ((uintptr_t)g & 15) == 0;
  for (int i = 0; ok && i < plan->n; ++i) {
    const FoldSeg& sg = segs[i];
    const int64_t c0 = sg.C - g, clen = sg.M == 1 ? sg.N : (sg.ldc == sg.N ? sg.M * sg.N : -1);
    ok = clen > 0 && c0 >= 0 && c0 % 4 == 0 && clen % 4 == 0 && c0 + clen <= n;
    if (ok) cov.push_back({c0 / 4, (c0 + clen) / 4});
    const bool has_rs = sg.units > sg.M * (sg.N / 4);
    if (ok && has_rs) {
      const int64_t r0 = sg.rs - g;
      ok = sg.rs && r0 >= 0 && r0 % 4 == 0 && sg.M % 4 == 0 && r0 + sg.M <= n;
      if (ok) cov.push_back({r0 / 4, (r0 + sg.M) / 4});
    }
  }
  if (ok && fx) cov.push_back({fx_off / 4, (fx_off + fx_len) / 4});   // must not overlap: checked below
  if (ok && skip_len > 0) cov.push_back({skip_off / 4, (skip_off + skip_len) / 4});   // updated already
  std::sort(cov.begin(), cov.end());
  for (size_t i = 1; ok && i < cov.size(); ++i) ok = cov[i].first >= cov[i - 1].second;
  AdamFoldArgs a;
  a.nplain = 0;
  if (ok) {                   // the complement of the segments' ranges (the fx range stays plain)
    int64_t at = 0;
    const int64_t fxl = fx ? fx_off / 4 : -1, fxh = fx ? (fx_off + fx_len) / 4 : -1;
    for (const auto& r : cov) {
      if (r.first == fxl && r.second == fxh) continue;
      if (r.first > at) {
        if (a.nplain == AF_PLAIN) { ok = false; break; }
        a.plo[a.nplain] = (int)at;
        a.phi[a.nplain++] = (int)r.first;
      }
      at = r.second;
    }
    if (ok && at < n / 4) {
      if (a.nplain == AF_PLAIN) ok = false;
      else { a.plo[a.nplain] = (int)at; a.phi[a.nplain++] = (int)(n / 4); }
    }
  }
  if (!ok) {                  // layout the fused form cannot take: fold, then the plain update
    int rc = launch_fold_segs(segs, plan->n, s);
    if (rc) return rc;
    if (skip_len > 0) {
      const int64_t e = skip_off + skip_len;
      rc = ttmi_adamw(skip_off, p, g, m, v, p_bf16, hyper, step, zero_grad, skip_if, s);
      if (rc) return rc;
      return ttmi_adamw(n - e, p + e, g + e, m + e, v + e, p_bf16 ? p_bf16 + e : nullptr, hyper, step,
                        zero_grad, skip_if, s);
    }
    return ttmi_adamw_fx(n, p, g, m, v, p_bf16, hyper, step, zero_grad, fx, fx_off, fx_len, fx_shift, skip_if, s);
  }
  TTMI_REQUIRE(((uintptr_t)p & 15) == 0 && ((uintptr_t)m & 15) == 0 && ((uintptr_t)v & 15) == 0 &&
               ((uintptr_t)p_bf16 & 7) == 0, "ttmi_adamw_folded: buffers must be 16-B aligned (bf16 mirror 8-B)");
  a.p = p; a.g = g; a.m = m; a.v = v; a.pb = (bf16_t*)p_bf16;
  a.hyper = hyper; a.step = step; a.zero_grad = zero_grad; a.skip_if = skip_if;
  a.fx = fx; a.fx_lo = fx ? fx_off / 4 : 0; a.fx_hi = fx ? (fx_off + fx_len) / 4 : 0; a.fx_shift = fx_shift;
  a.nseg = plan->n;
  int nb = 0;
  for (int j = 0; j < a.nplain; ++j) {
    a.blk_begin[j] = nb;
    nb += (int)((a.phi[j] - a.plo[j] + 256 * AF_U - 1) / (256 * AF_U));
  }
  for (int i = 0; i < a.nseg; ++i) {
    a.seg[i] = segs[i];
    a.blk_begin[a.nplain + i] = nb;
    nb += fold_blocks(segs[i]);
  }
  a.blk_begin[a.nplain + a.nseg] = nb;
  hipLaunchKernelGGL(adamw_fold_kernel, dim3((unsigned)nb), dim3(256), 0, s, a);
  return ttmi_check_launch("ttmi_adamw_folded");
}

TTMI_STAMP_DUMP(gemm)
