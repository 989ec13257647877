// ttmi_conv.hip — 2-D convolution as implicit GEMM on MFMA (bf16 operands, fp32 accumulate)
// for the ResNet-18 audio/visual encoders (reference item_tower.py:9-39, torchvision
// resnet18: conv1 7x7/2, BasicBlock 3x3 convs, 1x1/2 downsample).
//
// Activations are NHWC bf16 with the channel count a multiple of 8 (the 1- and 3-channel
// stems are zero-padded to 8).  One tile kernel, templated on the mode and the tile
// (BM x BN of 64/128, four waves 2x2, each wave (BM/2)x(BN/2) of 16x16x32 MFMAs, K walked in
// 64-element steps, double-buffered LDS with a register prefetch):
//   FWD   y[m, co]  = Σ_k im2col(x)[m, k] · Wf[co, k]        m = (n, ho, wo), k = (kh, kw, ci)
//         (+ BatchNorm Σy, Σy² per channel into TTMI_CONV_STAT_REPS replica rows)
//   DGRAD dx[m, ci] = Σ_k taps(dy)[m, k] · Wd[ci, k]         per stride-parity class of m
//   WGRAD dW[co, k] = Σ_m dy[m, co] · im2col(x)[m, k]        split over m, partials to a
//                                                            workspace, reduced + permuted
// Address generation: each thread's gathered rows are fixed for the whole K walk, so their
// pixel coordinates are decoded once; the per-step (tap, channel) split uses 32-bit
// magic-number division (all indices < 2^31).  Strided DGRAD runs one GEMM per output
// parity class (h mod S, w mod S): only the taps on that class's lattice are walked, so no
// MFMA work is spent on structural zeros.  WGRAD partials are plain 16-byte stores
// (deterministic; no scattered fp32 atomics into torch's [Co][Cin][KH][KW] layout).
// Wf = [Co][KH][KW][C] and Wd = [C][KH][KW][Co] are bf16 mirrors of torch's weight
// (ttmi_conv_weight_prep).  FWD also accumulates Σy, Σy² per channel for the BatchNorm.
#include "ttmi_common.h"

#include <climits>
#include <cstdio>
#include <cstdlib>

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4c_t;

TTMI_DEV uint2 c_lds8(const char* p) { return *reinterpret_cast<const uint2*>(p); }
TTMI_DEV uint2 c_lds_tr8(const char* p) {
  const s16x4c_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4c_t*)(p));
  return __builtin_bit_cast(uint2, v);
}

// q = n / d for n < 2^31 (Granlund–Montgomery round-up multiplier).
struct FDiv {
  uint32_t m, s;
};
FDiv fdiv_make(uint32_t d) {
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  const uint64_t m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
  return FDiv{(uint32_t)m, s};
}
TTMI_DEV int fq(int n, FDiv f) {
  return (int)((__umulhi((uint32_t)n, f.m) + (uint32_t)n) >> f.s);
}

constexpr int MAXCLS = 4;   // stride-parity classes (S <= 2)

struct ConvArgs {
  int N, H, W, C, Ho, Wo, Co, KH, KW, S, P, Cin;
  const bf16_t* x;          // FWD/WGRAD: input NHWC
  const bf16_t* dy;         // DGRAD/WGRAD: output grad NHWC
  const bf16_t* w;          // FWD: Wf, DGRAD: Wd
  void* out;                // FWD: y bf16 [M][Co]; DGRAD: dx bf16 [M][C]
  const bf16_t* addend;     // DGRAD: added before the store, or NULL
  int64_t* colsum;          // FWD: Σ y per channel, int64 fixed point 2^-24 (may be NULL)
  int64_t* colsumsq;
  float* ws;                // WGRAD: partials [splits][GM][GN]
  // DGRAD: fused BatchNorm-backward reduction of the layer that produced x (bn_sums != NULL)
  const bf16_t* bn_gate;    // that BN's (ReLU) output, or NULL
  const bf16_t* bn_x;       // that BN's input
  const float* bn_mean;
  const float* bn_rstd;
  int64_t* bn_sums;         // [REPS][2][GN] int64 fixed point 2^36
  int GM, GN, GK;           // GEMM sizes (DGRAD: per class below)
  int k_split;              // WGRAD: pixels per split (multiple of 64)
  FDiv fC, fKW, fWo, fHo, fCo;
  // DGRAD parity classes (ph, pw) = (cls / S, cls % S)
  int cM[MAXCLS], cK[MAXCLS], cHc[MAXCLS], cWc[MAXCLS], ckh0[MAXCLS], ckw0[MAXCLS],
      cnkw[MAXCLS], coffh[MAXCLS], coffw[MAXCLS];
  FDiv cfW[MAXCLS], cfH[MAXCLS], cfnkw[MAXCLS];
};

constexpr int PK = 144;                     // k-major LDS pitch: 64 bf16 + 16 B

// Fragment reads (same k-permutation on both operands: lane group g of each 32-wide k chunk
// holds k = 4g..4g+3 and 16+4g..16+4g+3).
TTMI_DEV uint4 frag_k(const char* s, int row0, int c, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const char* p = s + (row0 + i) * PK + c * 64 + g * 8;
  const uint2 lo = c_lds8(p), hi = c_lds8(p + 32);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}
template <int PT>
TTMI_DEV uint4 frag_t(const char* s, int row0, int c, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int q = i >> 2, pp = i & 3;
  const char* p = s + (c * 32 + 4 * g + q) * PT + (row0 + 4 * pp) * 2;
  const uint2 lo = c_lds_tr8(p), hi = c_lds_tr8(p + 16 * PT);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

TTMI_DEV uint4 ldg16(const bf16_t* p, bool ok) {
  return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
}

template <int MODE, int BM, int BN>
__global__ __launch_bounds__(256) void conv_tile_kernel(ConvArgs a) {
  constexpr bool WG = MODE == 2;
  constexpr int CA = BM / 32, CB = BN / 32;             // 16-B chunks per thread per stage
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  constexpr int PTA = BM * 2 + 32, PTB = BN * 2 + 32;   // [k][row] pitches (WGRAD)
  constexpr int SA = WG ? 64 * PTA : BM * PK;
  constexpr int SB = WG ? 64 * PTB : BN * PK;
  constexpr int STAGE = SA + SB;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // tile coordinates: blockIdx.x enumerates (n-tile, m-tile), XCD-grouped so that the
  // n-tiles of one m-row run on the same XCD (they share the gathered A rows in its L2)
  const int gx = (a.GN + BN - 1) / BN;
  int t = blockIdx.x;
  if ((gridDim.x & 7) == 0) t = (t & 7) * (gridDim.x >> 3) + (t >> 3);
  const int n0 = (t % gx) * BN, m0 = (t / gx) * BM;
  const int cls = MODE == 1 ? (int)blockIdx.y : 0;
  const int GM = MODE == 1 ? a.cM[cls] : a.GM;
  const int GK = MODE == 1 ? a.cK[cls] : a.GK;
  if (m0 >= GM) return;                                  // DGRAD: smaller parity class
  const int kbeg = WG ? (int)blockIdx.y * a.k_split : 0;
  const int kend = WG ? min(GK, kbeg + a.k_split) : GK;

  // ---- per-thread gather state, decoded once
  const int kk = (tid & 7) * 8;                          // FWD/DGRAD: k offset of my chunks
  int rh[CA], rw[CA];                                    // row coordinates (see modes)
  const bf16_t* rbase[CA];
  int bkh[CB], bkw[CB], bci[CB];                         // WGRAD: tap/channel of my B chunks
  bool bok[CB];
  if constexpr (MODE == 0) {
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int m = m0 + (tid >> 3) + 32 * c;
      rh[c] = INT_MIN / 2; rw[c] = 0; rbase[c] = a.x;
      if (m < GM) {
        const int q = fq(m, a.fWo), wo = m - q * a.Wo;
        const int n = fq(q, a.fHo), ho = q - n * a.Ho;
        rh[c] = ho * a.S - a.P;
        rw[c] = wo * a.S - a.P;
        rbase[c] = a.x + (int64_t)n * a.H * a.W * a.C;
      }
    }
  } else if constexpr (MODE == 1) {
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int m = m0 + (tid >> 3) + 32 * c;
      rh[c] = INT_MIN / 2; rw[c] = 0; rbase[c] = a.dy;
      if (m < GM) {
        const int q = fq(m, a.cfW[cls]), ww = m - q * a.cWc[cls];
        const int n = fq(q, a.cfH[cls]), hh = q - n * a.cHc[cls];
        rh[c] = hh + a.coffh[cls];
        rw[c] = ww + a.coffw[cls];
        rbase[c] = a.dy + (int64_t)n * a.Ho * a.Wo * a.Co;
      }
    }
  } else {
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int kc = n0 + ((tid + 256 * c) % (BN / 8)) * 8;
      bok[c] = kc < a.GN;
      const int tap = fq(kc, a.fC);
      bci[c] = kc - tap * a.C;
      bkh[c] = fq(tap, a.fKW);
      bkw[c] = tap - bkh[c] * a.KW;
    }
  }

  uint4 ra[CA], rb[CB];
  auto load = [&](int k0) {
    if constexpr (MODE == 0) {
      const int k = k0 + kk;
      const bool kin = k < GK;
      const int tap = fq(k, a.fC), ci = k - tap * a.C;
      const int kh = fq(tap, a.fKW), kw = tap - kh * a.KW;
#pragma unroll
      for (int c = 0; c < CA; ++c) {
        const int hi = rh[c] + kh, wi = rw[c] + kw;
        const bool ok = kin && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
        ra[c] = ldg16(rbase[c] + ((int64_t)hi * a.W + wi) * a.C + ci, ok);
      }
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        const int n = n0 + (tid >> 3) + 32 * c;
        rb[c] = ldg16(a.w + (int64_t)n * GK + k, kin && n < a.GN);
      }
    } else if constexpr (MODE == 1) {
      const int k = k0 + kk;
      const bool kin = k < GK;
      const int tt = fq(k, a.fCo), co = k - tt * a.Co;
      const int i = fq(tt, a.cfnkw[cls]), j = tt - i * a.cnkw[cls];
#pragma unroll
      for (int c = 0; c < CA; ++c) {
        const int ho = rh[c] - i, wo = rw[c] - j;
        const bool ok = kin && (unsigned)ho < (unsigned)a.Ho && (unsigned)wo < (unsigned)a.Wo;
        ra[c] = ldg16(rbase[c] + ((int64_t)ho * a.Wo + wo) * a.Co + co, ok);
      }
      const int kh = a.ckh0[cls] + a.S * i, kw = a.ckw0[cls] + a.S * j;
      const int64_t wcol = (int64_t)(kh * a.KW + kw) * a.Co + co;
      const int64_t wrow = (int64_t)a.KH * a.KW * a.Co;
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        const int n = n0 + (tid >> 3) + 32 * c;
        rb[c] = ldg16(a.w + n * wrow + wcol, kin && n < a.GN);
      }
    } else {
#pragma unroll
      for (int c = 0; c < CA; ++c) {
        const int idx = tid + 256 * c;
        const int p = k0 + idx / (BM / 8), co = m0 + (idx % (BM / 8)) * 8;
        ra[c] = ldg16(a.dy + (int64_t)p * a.Co + co, p < kend && co < a.GM);
      }
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        const int p = k0 + (tid + 256 * c) / (BN / 8);
        const int q = fq(p, a.fWo), wo = p - q * a.Wo;
        const int n = fq(q, a.fHo), ho = q - n * a.Ho;
        const int hi = ho * a.S - a.P + bkh[c], wi = wo * a.S - a.P + bkw[c];
        const bool ok = p < kend && bok[c] && (unsigned)hi < (unsigned)a.H &&
                        (unsigned)wi < (unsigned)a.W;
        rb[c] = ldg16(a.x + (((int64_t)n * a.H + hi) * a.W + wi) * a.C + bci[c], ok);
      }
    }
  };
  auto store = [&](char* s) {
    char* sa = s;
    char* sb = s + SA;
    if constexpr (!WG) {
#pragma unroll
      for (int c = 0; c < CA; ++c)
        *reinterpret_cast<uint4*>(sa + ((tid >> 3) + 32 * c) * PK + (tid & 7) * 16) = ra[c];
#pragma unroll
      for (int c = 0; c < CB; ++c)
        *reinterpret_cast<uint4*>(sb + ((tid >> 3) + 32 * c) * PK + (tid & 7) * 16) = rb[c];
    } else {
#pragma unroll
      for (int c = 0; c < CA; ++c) {
        const int idx = tid + 256 * c;
        *reinterpret_cast<uint4*>(sa + (idx / (BM / 8)) * PTA + (idx % (BM / 8)) * 16) = ra[c];
      }
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        const int idx = tid + 256 * c;
        *reinterpret_cast<uint4*>(sb + (idx / (BN / 8)) * PTB + (idx % (BN / 8)) * 16) = rb[c];
      }
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (kbeg < kend) {
    load(kbeg);
    store(smem);
  }
  __syncthreads();
  int buf = 0;
  for (int k0 = kbeg; k0 < kend; k0 += 64) {
    const bool more = k0 + 64 < kend;
    if (more) load(k0 + 64);
    const char* sa = smem + buf * STAGE;
    const char* sb = sa + SA;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      uint4 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = WG ? frag_t<PTA>(sa, wm * WM + i * 16, c, lane) : frag_k(sa, wm * WM + i * 16, c, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = WG ? frag_t<PTB>(sb, wn * WN + j * 16, c, lane) : frag_k(sb, wn * WN + j * 16, c, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) Mma<bf16_t>::run(acc[i][j], bfr[j], af[i]);
    }
    if (more) store(smem + (buf ^ 1) * STAGE);
    __syncthreads();
    buf ^= 1;
  }

  // ---- epilogue: lane holds C[m][n..n+3], m = row + (lane & 15), n = col + 4*(lane >> 4)
  const int li = lane & 15, lg = lane >> 4;
  if constexpr (MODE == 2) {
    float* ws = a.ws + (int64_t)blockIdx.y * a.GM * a.GN;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wm * WM + i * 16 + li;
      if (m >= a.GM) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * WN + j * 16 + 4 * lg;
        if (n < a.GN) *reinterpret_cast<f32x4_t*>(ws + (int64_t)m * a.GN + n) = acc[i][j];
      }
    }
    return;
  }
  int64_t orow[FM];                                       // output pixel of each row
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wm * WM + i * 16 + li;
    orow[i] = -1;
    if (m < GM) {
      if constexpr (MODE == 1) {
        const int q = fq(m, a.cfW[cls]), ww = m - q * a.cWc[cls];
        const int n = fq(q, a.cfH[cls]), hh = q - n * a.cHc[cls];
        const int ph = cls / a.S, pw = cls - ph * a.S;
        orow[i] = ((int64_t)n * a.H + hh * a.S + ph) * a.W + ww * a.S + pw;
      } else {
        orow[i] = m;
      }
    }
  }
  float cs[FN][4], cq[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * WN + j * 16 + 4 * lg;
#pragma unroll
    for (int e = 0; e < 4; ++e) cs[j][e] = cq[j][e] = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if (orow[i] < 0 || n >= a.GN) continue;
      const float* v = reinterpret_cast<const float*>(&acc[i][j]);
      float o[4] = {v[0], v[1], v[2], v[3]};
      bf16_t* dst = static_cast<bf16_t*>(a.out) + orow[i] * a.GN + n;
      if (MODE == 1 && a.addend) {
        const ushort4 q = *reinterpret_cast<const ushort4*>(a.addend + orow[i] * a.GN + n);
        o[0] += bf2f(q.x); o[1] += bf2f(q.y); o[2] += bf2f(q.z); o[3] += bf2f(q.w);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) { cs[j][e] += o[e]; cq[j][e] += o[e] * o[e]; }
      ushort4 q;
      q.x = f2bf(o[0]); q.y = f2bf(o[1]); q.z = f2bf(o[2]); q.w = f2bf(o[3]);
      *reinterpret_cast<ushort4*>(dst) = q;
    }
  }
  if (MODE == 0 && a.colsum) {
    // BatchNorm column statistics: reduce the tile's rows (registers, then the 16 row lanes,
    // then the two row-waves through LDS, a fixed order) so each column gets one Σy and one
    // Σy² add per workgroup, spread over TTMI_CONV_STAT_REPS replica rows (one hot address
    // per channel would serialise every workgroup's atomics in a single L2 channel).  The
    // adds are int64 fixed point (TTMI_FX_STAT): the statistics do not depend on the order
    // the workgroups finish in, so the whole step is bit-reproducible.
    float* red = reinterpret_cast<float*>(smem);        // [2][BN]; the K loop has drained
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          cs[j][e] += __shfl_xor(cs[j][e], off, 64);
          cq[j][e] += __shfl_xor(cq[j][e], off, 64);
        }
    if (wm == 1 && li == 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = wn * WN + j * 16 + 4 * lg + e;
          red[col] = cs[j][e];
          red[BN + col] = cq[j][e];
        }
    }
    __syncthreads();
    if (wm == 0 && li == 0) {
      const int rep = blockIdx.x % TTMI_CONV_STAT_REPS;
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = wn * WN + j * 16 + 4 * lg + e;
          const int n = n0 + col;
          if (n < a.GN) {
            fx_add(a.colsum + (int64_t)rep * a.GN + n, cs[j][e] + red[col], TTMI_FX_STAT);
            fx_add(a.colsumsq + (int64_t)rep * a.GN + n, cq[j][e] + red[BN + col], TTMI_FX_STAT);
          }
        }
    }
  }
}

// ---------------------------------------------------------------- LDS-DMA tile (FWD / DGRAD)
// The large layers: 256 x BN output tiles (BN = 64 or 128 channels), 8 waves as 4 (rows) x 2
// (cols), a wave owning 64 x BN/2 outputs (4 x BN/32 MFMA tiles of 16x16x32).  Two waves per
// SIMD: one's fragment reads and DMA issue hide under the other's MFMAs (measured: 4 waves of
// 64 x 64 on the BN = 64 tile read less LDS but ran 1.2-1.3x longer).
// Both operands go global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds, no register
// staging) into a 3-deep ring of k-step images, [row][128 B] = 64 bf16 of k per row, with
// the 16-byte chunks XOR-swizzled per row on the SOURCE side (the DMA writes lane-linearly)
// so the 16 rows one ds_read_b128 lane group reads fall in 16 distinct bank slots.  A wave
// instruction fills 8 rows x 128 B; a lane's rows are fixed for the whole K walk, so their
// pixel bases are decoded once.  Padding taps, rows past M and k past K get an offset past
// the buffer descriptor's range: the DMA writes zeros, nothing is branched around.  Two
// k-steps are in flight while the third is multiplied (counted vmcnt, one barrier a step).
namespace cdma {
constexpr uint32_t OOB = 0xFFFFFFF0u;
TTMI_DEV int swz(int r) { return (r >> 1) & 7; }
TTMI_DEV uint4 frag(const char* img, int row, int c, int lane) {
  return lds16(img + row * 128 + (((4 * c + (lane >> 4)) ^ swz(row)) << 4));
}
template <int N_>
TTMI_DEV void wait_vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N_) : "memory");
}
}  // namespace cdma

template <int MODE, int BM, int BN, int NS>
__global__ __launch_bounds__(512) void conv_dma_kernel(ConvArgs a) {
  using namespace cdma;
  constexpr int NW = 8;                                    // waves: 4 (rows) x 2 (cols)
  constexpr int SA = BM * 128, SB = BN * 128, STAGE = SA + SB;
  constexpr int IA = SA / 1024 / NW, IB = SB / 1024 / NW;  // DMA wave-instructions per wave per stage
  constexpr int P = IA + IB;
  static_assert(IA * NW * 1024 == SA && IB * NW * 1024 == SB, "stage must split over the waves");
  static_assert((NS - 2) * P <= 63, "vmcnt range");
  constexpr int WM = BM / 4, WN = BN / 2, FM = WM / 16, FN = WN / 16;   // a wave owns WM x WN
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 3, wn = wave >> 2;

  // XCD-contiguous tile order (bijective for any count): neighbouring m-tiles share input
  // rows through their taps, the n-tiles of an m-tile share all of them
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rem = nwg & 7;
  const int tile = (xcd < rem ? xcd * (q8 + 1) : rem * (q8 + 1) + (xcd - rem) * q8) + (bid >> 3);
  const int gx = a.GN / BN;
  const int n0 = (tile % gx) * BN, m0 = (tile / gx) * BM;
  const int cls = MODE == 1 ? (int)blockIdx.y : 0;
  const int GM = MODE == 1 ? a.cM[cls] : a.GM;
  const int GK = MODE == 1 ? a.cK[cls] : a.GK;
  if (m0 >= GM) return;                                   // DGRAD: smaller parity class
  const int nt = (GK + 63) / 64;

  const i32x4_t rsa = MODE == 0 ? make_rsrc(a.x, (uint32_t)((int64_t)a.N * a.H * a.W * a.C * 2))
                                : make_rsrc(a.dy, (uint32_t)((int64_t)a.N * a.Ho * a.Wo * a.Co * 2));
  const i32x4_t rsb = MODE == 0 ? make_rsrc(a.w, (uint32_t)((int64_t)a.GN * GK * 2))
                                : make_rsrc(a.w, (uint32_t)((int64_t)a.C * a.KH * a.KW * a.Co * 2));

  // ---- this lane's DMA rows: A rows (wave + NW·u) * 8 + lane / 8, its 16-byte chunk slot
  // lane % 8 holding global chunk slot ^ swz(row)
  int apix[IA], ah[IA], aw[IA], ach[IA];
#pragma unroll
  for (int u = 0; u < IA; ++u) {
    const int r = (wave + NW * u) * 8 + (lane >> 3);
    ach[u] = (lane & 7) ^ swz(r);
    const int m = m0 + r;
    ah[u] = INT_MIN / 2; aw[u] = 0; apix[u] = 0;
    if (m < GM) {
      if constexpr (MODE == 0) {
        const int q = fq(m, a.fWo), wo = m - q * a.Wo;
        const int n = fq(q, a.fHo), ho = q - n * a.Ho;
        ah[u] = ho * a.S - a.P;
        aw[u] = wo * a.S - a.P;
        apix[u] = n * a.H * a.W;
      } else {
        const int q = fq(m, a.cfW[cls]), ww = m - q * a.cWc[cls];
        const int n = fq(q, a.cfH[cls]), hh = q - n * a.cHc[cls];
        ah[u] = hh + a.coffh[cls];
        aw[u] = ww + a.coffw[cls];
        apix[u] = n * a.Ho * a.Wo;
      }
    }
  }
  int bch[IB];
  uint32_t brow[IB];
#pragma unroll
  for (int v = 0; v < IB; ++v) {
    const int r = (wave + NW * v) * 8 + (lane >> 3);
    bch[v] = (lane & 7) ^ swz(r);
    brow[v] = MODE == 0 ? (uint32_t)(n0 + r) * (uint32_t)GK * 2u
                        : (uint32_t)(n0 + r) * (uint32_t)(a.KH * a.KW * a.Co) * 2u;
  }
  const uint32_t sl = lds_addr(smem);

  auto issue = [&](int t, int slot) {
    const uint32_t img = sl + slot * STAGE;
    const int k0 = t * 64;
    if constexpr (MODE == 0) {
      const bool uni = a.C % 64 == 0;                      // the whole k-step is one tap
      const int tap0 = fq(k0, a.fC), ci0 = k0 - tap0 * a.C;
      const int kh0 = fq(tap0, a.fKW), kw0 = tap0 - kh0 * a.KW;
#pragma unroll
      for (int u = 0; u < IA; ++u) {
        const int k = k0 + ach[u] * 8;
        int kh = kh0, kw = kw0, ci = ci0 + ach[u] * 8;
        if (!uni) {
          const int tap = fq(k, a.fC);
          ci = k - tap * a.C;
          kh = fq(tap, a.fKW);
          kw = tap - kh * a.KW;
        }
        const int hi = ah[u] + kh, wi = aw[u] + kw;
        const bool ok = k < GK && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
        const uint32_t off = ((uint32_t)(apix[u] + hi * a.W + wi) * (uint32_t)a.C + (uint32_t)ci) * 2u;
        dma16(rsa, ok ? off : OOB, img + (wave + NW * u) * 1024);
      }
#pragma unroll
      for (int v = 0; v < IB; ++v) {
        const int k = k0 + bch[v] * 8;
        dma16(rsb, k < GK ? brow[v] + (uint32_t)k * 2u : OOB, img + SA + (wave + NW * v) * 1024);
      }
    } else {
      // k = (i, j, co) on this class's tap lattice; Co % 64 == 0: one tap per k-step
      const int tt = fq(k0, a.fCo), co0 = k0 - tt * a.Co;
      const int i = fq(tt, a.cfnkw[cls]), j = tt - i * a.cnkw[cls];
#pragma unroll
      for (int u = 0; u < IA; ++u) {
        const int ho = ah[u] - i, wo = aw[u] - j;
        const bool ok = (unsigned)ho < (unsigned)a.Ho && (unsigned)wo < (unsigned)a.Wo;
        const uint32_t off =
            ((uint32_t)(apix[u] + ho * a.Wo + wo) * (uint32_t)a.Co + (uint32_t)(co0 + ach[u] * 8)) * 2u;
        dma16(rsa, ok ? off : OOB, img + (wave + NW * u) * 1024);
      }
      const int kh = a.ckh0[cls] + a.S * i, kw = a.ckw0[cls] + a.S * j;
      const uint32_t wcol = (uint32_t)((kh * a.KW + kw) * a.Co + co0) * 2u;
#pragma unroll
      for (int v = 0; v < IB; ++v) dma16(rsb, brow[v] + wcol + bch[v] * 16u, img + SA + (wave + NW * v) * 1024);
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nt) issue(s, s);
  const int ar = wm * WM + (lane & 15), br = wn * WN + (lane & 15);
  for (int t = 0; t < nt; ++t) {
    // step t landed for every wave (later steps may fly); slot (t-1) % NS is free
    if (t + NS - 2 < nt) wait_vm_barrier<(NS - 2) * P>();
    else if (t + 1 < nt) wait_vm_barrier<P>();
    else wait_vm_barrier<0>();
    if (t + NS - 1 < nt) issue(t + NS - 1, (t + NS - 1) % NS);
    const char* sA = smem + (t % NS) * STAGE;
    const char* sB = sA + SA;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      uint4 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = frag(sA, ar + 16 * i, c, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = frag(sB, br + 16 * j, c, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) Mma<bf16_t>::run(acc[i][j], bfr[j], af[i]);
    }
  }

  // ---- epilogue: lane holds C[m][n..n+3], m = row + (lane & 15), n = col + 4*(lane >> 4)
  const int li = lane & 15, lg = lane >> 4;
  int64_t orow[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wm * WM + i * 16 + li;
    orow[i] = -1;
    if (m < GM) {
      if constexpr (MODE == 1) {
        const int q = fq(m, a.cfW[cls]), ww = m - q * a.cWc[cls];
        const int n = fq(q, a.cfH[cls]), hh = q - n * a.cHc[cls];
        const int ph = cls / a.S, pw = cls - ph * a.S;
        orow[i] = ((int64_t)n * a.H + hh * a.S + ph) * a.W + ww * a.S + pw;
      } else {
        orow[i] = m;
      }
    }
  }
  float cs[FN][4], cq[FN][4];
  // DGRAD + fused BN-backward reduction: g = bf16(dx) gated by the BN's ReLU output is stored,
  // and (cs, cq) collect Σg, Σg·x̂ (the FWD statistics path reuses them for Σy, Σy²)
  const bool bnf = MODE == 1 && a.bn_sums != nullptr;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * WN + j * 16 + 4 * lg;
    float mu[4], rs[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      cs[j][e] = cq[j][e] = 0.f;
      mu[e] = bnf ? a.bn_mean[n + e] : 0.f;
      rs[e] = bnf ? a.bn_rstd[n + e] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if (orow[i] < 0) continue;
      const float* v = reinterpret_cast<const float*>(&acc[i][j]);
      float o[4] = {v[0], v[1], v[2], v[3]};
      bf16_t* dst = static_cast<bf16_t*>(a.out) + orow[i] * a.GN + n;
      if (MODE == 1 && a.addend) {
        const ushort4 q = *reinterpret_cast<const ushort4*>(a.addend + orow[i] * a.GN + n);
        o[0] += bf2f(q.x); o[1] += bf2f(q.y); o[2] += bf2f(q.z); o[3] += bf2f(q.w);
      }
      if (bnf) {
        const ushort4 qx = *reinterpret_cast<const ushort4*>(a.bn_x + orow[i] * a.GN + n);
        ushort4 qg = make_ushort4(0x3F80, 0x3F80, 0x3F80, 0x3F80);          // 1.0: no gate
        if (a.bn_gate) qg = *reinterpret_cast<const ushort4*>(a.bn_gate + orow[i] * a.GN + n);
        const float xv[4] = {bf2f(qx.x), bf2f(qx.y), bf2f(qx.z), bf2f(qx.w)};
        const float gv[4] = {bf2f(qg.x), bf2f(qg.y), bf2f(qg.z), bf2f(qg.w)};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gr = gv[e] > 0.f ? bf2f(f2bf(o[e])) : 0.f;
          o[e] = gr;
          cs[j][e] += gr;
          cq[j][e] += gr * (xv[e] - mu[e]) * rs[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) { cs[j][e] += o[e]; cq[j][e] += o[e] * o[e]; }
      }
      ushort4 q;
      q.x = f2bf(o[0]); q.y = f2bf(o[1]); q.z = f2bf(o[2]); q.w = f2bf(o[3]);
      *reinterpret_cast<ushort4*>(dst) = q;
    }
  }
  if ((MODE == 0 && a.colsum) || bnf) {
    // BatchNorm column statistics (as conv_tile_kernel): rows reduced in registers, over the
    // 16 row lanes, then over the four row-waves through LDS in a fixed order; one int64
    // fixed-point add per column per workgroup into replica row blockIdx.x % REPS.
    float* red = reinterpret_cast<float*>(smem);          // [4][2][BN]
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          cs[j][e] += __shfl_xor(cs[j][e], off, 64);
          cq[j][e] += __shfl_xor(cq[j][e], off, 64);
        }
    __syncthreads();                                      // every wave is past the ring
    if (li == 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = wn * WN + j * 16 + 4 * lg + e;
          red[(wm * 2) * BN + col] = cs[j][e];
          red[(wm * 2 + 1) * BN + col] = cq[j][e];
        }
    }
    __syncthreads();
    if (tid < BN) {
      float s = 0.f, s2 = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) { s += red[(w * 2) * BN + tid]; s2 += red[(w * 2 + 1) * BN + tid]; }
      const int rep = (blockIdx.x + blockIdx.y) % TTMI_CONV_STAT_REPS;
      if (bnf) {
        int64_t* r = a.bn_sums + (int64_t)rep * 2 * a.GN + n0 + tid;
        fx_add(r, s, TTMI_FX_GRAD);
        fx_add(r + a.GN, s2, TTMI_FX_GRAD);
      } else {
        fx_add(a.colsum + (int64_t)rep * a.GN + n0 + tid, s, TTMI_FX_STAT);
        fx_add(a.colsumsq + (int64_t)rep * a.GN + n0 + tid, s2, TTMI_FX_STAT);
      }
    }
  }
}

// ---------------------------------------------------------------- LDS-DMA tile (WGRAD)
// dW[co, kc] over one split's pixel range: BM x 128 tiles (BM = 64 or 128 output channels),
// 4 waves 2 x 2, K = pixels walked in 64-pixel stages through a 4-deep LDS-DMA ring.  Both
// operands are pixel-major: the A image holds dy[p][co0 .. co0+BM), the B image the im2col
// row x[pix(p, tap)][ci ..] of each 16-byte column chunk — a lane's column chunk (so its tap
// and channel) is fixed for the whole walk, only the pixel of its k-row moves.  Images are
// [k][W·2 B] with 32-byte chunks XOR-swizzled per k-row on the source side and read as MFMA
// fragments by ds_read_b64_tr_b16 (the k-major transpose in the LDS read).  Partials go to
// the split's slab as 16-byte stores (deterministic; reduced by wgrad_reduce_kernel).
namespace cdma {
template <int W>
struct KImg {                                              // [64 k-rows][W bf16] image
  static constexpr int PB = W * 2;
  static constexpr int CPR = PB / 32;                      // 32-byte chunks per k-row
  static constexpr int RPB = PB >= 256 ? 1 : 256 / PB;     // k-rows per 256-byte bank row
  static constexpr int BYTES = 64 * PB;
  static constexpr int INSTR = BYTES / 1024;
  static TTMI_DEV int swz(int k) { return (k / RPB) % CPR; }
  // k-row and source byte (within the row's W-column window) of this lane's bytes in
  // wave-instruction ii
  static TTMI_DEV void slot(int ii, int lane, int& k, int& col_b) {
    const int o = ii * 1024 + lane * 16;
    k = o / PB;
    const int pb = o % PB;
    col_b = (((pb >> 5) ^ swz(k)) << 5) + (pb & 16);
  }
  static TTMI_DEV uint4 frag(const char* img, int row0, int c, int lane) {
    const int i = lane & 15, g = lane >> 4;
    const int k = c * 32 + 4 * g + (i >> 2);
    const char* p = img + k * PB + (((row0 >> 4) ^ swz(k)) << 5) + 8 * (i & 3);
    const uint2 lo = c_lds_tr8(p), hi = c_lds_tr8(p + 16 * PB);
    return make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
};
}  // namespace cdma

template <int BM, int NW, int NS>
__global__ __launch_bounds__(NW * 64) void conv_wgrad_dma_kernel(ConvArgs a, int tiles_n, int tiles) {
  using namespace cdma;
  constexpr int BN = 128;
  using IA = KImg<BM>;
  using IB = KImg<BN>;
  constexpr int STAGE = IA::BYTES + IB::BYTES;
  constexpr int JA = IA::INSTR / NW, JB = IB::INSTR / NW;  // per wave per stage
  constexpr int P = JA + JB;
  static_assert(JA * NW == IA::INSTR && JB * NW == IB::INSTR, "stage must split over the waves");
  static_assert((NS - 2) * P <= 63, "vmcnt range");
  constexpr int WCOL = NW / 2;                             // waves: 2 (rows) x NW/2 (cols)
  constexpr int WTM = BM / 2, WTN = BN / WCOL, TM = WTM / 16, TN = WTN / 16;
  __shared__ __attribute__((aligned(1024))) char ring[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WCOL, wn = wave % WCOL;

  // (split, tile) in XCD-contiguous order: the tiles of one split (same pixel rows) share an
  // XCD's L2
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rem = nwg & 7;
  const int L = (xcd < rem ? xcd * (q8 + 1) : rem * (q8 + 1) + (xcd - rem) * q8) + (bid >> 3);
  const int tile = L % tiles, split = L / tiles;
  const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int kbeg = split * a.k_split;
  const int kend = min(a.GK, kbeg + a.k_split);
  if (kbeg >= kend) return;
  const int nst = (kend - kbeg + 63) >> 6;

  const i32x4_t rsa = make_rsrc(a.dy, (uint32_t)((int64_t)a.GK * a.Co * 2));
  const i32x4_t rsx = make_rsrc(a.x, (uint32_t)((int64_t)a.N * a.H * a.W * a.C * 2));
  // this lane's fixed A column byte and B column chunk (tap, channel) per wave-instruction
  int ak[JA], acol[JA], bk[JB], bkh[JB], bkw[JB], bci[JB];
  bool bok[JB];
#pragma unroll
  for (int j = 0; j < JA; ++j) {
    IA::slot(wave + NW * j, lane, ak[j], acol[j]);
    acol[j] += m0 * 2;
  }
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    int cb;
    IB::slot(wave + NW * j, lane, bk[j], cb);
    const int kc = n0 + cb / 2;
    bok[j] = kc < a.GN;
    const int tap = fq(kc, a.fC);
    bci[j] = kc - tap * a.C;
    bkh[j] = fq(tap, a.fKW);
    bkw[j] = tap - bkh[j] * a.KW;
    bkh[j] -= a.P;
    bkw[j] -= a.P;
  }
  const uint32_t sl = lds_addr(ring);
  auto issue = [&](int t, int slot) {
    const uint32_t img = sl + slot * STAGE;
    const int p0 = kbeg + t * 64;
#pragma unroll
    for (int j = 0; j < JA; ++j) {
      const int p = p0 + ak[j];
      const uint32_t off = (uint32_t)p * (uint32_t)(a.Co * 2) + (uint32_t)acol[j];
      dma16(rsa, p < kend ? off : OOB, img + (wave + NW * j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const int p = p0 + bk[j];
      const int q = fq(p, a.fWo), wo = p - q * a.Wo;
      const int n = fq(q, a.fHo), ho = q - n * a.Ho;
      const int hi = ho * a.S + bkh[j], wi = wo * a.S + bkw[j];
      const bool ok = p < kend && bok[j] && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
      const uint32_t off = ((uint32_t)((n * a.H + hi) * a.W + wi) * (uint32_t)a.C + (uint32_t)bci[j]) * 2u;
      dma16(rsx, ok ? off : OOB, img + IA::BYTES + (wave + NW * j) * 1024);
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nst) issue(s, s);
  for (int t = 0; t < nst; ++t) {
    // stage t landed for every wave (later stages may fly); slot (t-1) % NS is free
    if (t + NS - 2 < nst) wait_vm_barrier<(NS - 2) * P>();
    else if (t + 1 < nst) wait_vm_barrier<P>();
    else wait_vm_barrier<0>();
    if (t + NS - 1 < nst) issue(t + NS - 1, (t + NS - 1) % NS);
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
    }
  }
  const int li = lane & 15, lg = lane >> 4;
  float* ws = a.ws + (int64_t)split * a.GM * a.GN;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * WTM + i * 16 + li;
    if (m >= a.GM) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WTN + j * 16 + 4 * lg;
      if (n < a.GN) *reinterpret_cast<f32x4_t*>(ws + (int64_t)m * a.GN + n) = acc[i][j];
    }
  }
}

// dW (torch [Co][Cin][KH][KW]) += Σ_split ws[split][co][(kh·KW + kw)·C + ci], ci < Cin, in
// split order (deterministic).  Up to WR_SPLITS splits: one pass (x over 4-column groups of
// the [GM][GN] plane; a thread's WR_SPLITS loads in flight together).  More: a first pass
// (y over chunks of WR_SPLITS splits) sums each chunk into the chunk's first slab in place,
// then the final pass sums the chunk slabs in chunk order — fixed order, no atomics.
constexpr int WR_SPLITS = 16;
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(float* __restrict__ ws, int splits,
                                                           int step, int GM, int GN, int C, int Cin,
                                                           int KW, int KHKW, int final_pass,
                                                           float* __restrict__ dw, int s2d) {
  const int64_t n4 = (int64_t)GM * GN / 4, plane = (int64_t)GM * GN;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  // this thread's slabs: s = first + j*step for j < count
  const int first = final_pass ? 0 : blockIdx.y * WR_SPLITS * step;
  const int count = final_pass ? (splits + step - 1) / step : min(WR_SPLITS, (splits - first + step - 1) / step);
  f32x4_t s = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < count; j0 += WR_SPLITS) {
    f32x4_t part[WR_SPLITS];
#pragma unroll
    for (int j = 0; j < WR_SPLITS; ++j)           // all loads in flight together
      part[j] = j0 + j < count ? reinterpret_cast<const f32x4_t*>(ws + (int64_t)(first + (j0 + j) * step) * plane)[i]
                               : f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < WR_SPLITS; ++j) s += part[j];
  }
  if (!final_pass) {                               // chunk total into the chunk's first slab
    reinterpret_cast<f32x4_t*>(ws + (int64_t)first * plane)[i] = s;
    return;
  }
  const int64_t e0 = i * 4;
  const int co = (int)(e0 / GN), kc = (int)(e0 % GN);
  const int tap = kc / C, ci0 = kc % C;
  const float* v = reinterpret_cast<const float*>(&s);
  if (s2d) {
    // space-to-depth stem (ttmi_stem_s2d): tap (a, b) of the 4x4 kernel, channel
    // (ph·2 + pw)·Cin + ci  ->  torch tap (kh, kw) = (2a + ph − 1, 2b + pw − 1) of the 7x7
    const int ta = tap >> 2, tb = tap & 3;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = (ci0 + e) / Cin, ci = (ci0 + e) - q * Cin;
      const int kh = 2 * ta + (q >> 1) - 1, kw = 2 * tb + (q & 1) - 1;
      if (q >= 4 || kh < 0 || kh >= 7 || kw < 0 || kw >= 7) continue;
      dw[(((int64_t)co * Cin + ci) * 7 + kh) * 7 + kw] += v[e];
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int ci = ci0 + e;
    if (ci >= Cin) continue;
    dw[((int64_t)co * Cin + ci) * KHKW + tap] += v[e];
  }
}

// Wf[co][kh][kw][c] = bf16(w[co][ci][kh][kw]) (c < Cp, zero for ci >= Cin);
// Wd[c][kh][kw][co] likewise (c < Cin only: the padded stem never needs its input grad).
__global__ __launch_bounds__(256) void conv_weight_prep_kernel(int Co, int Cin, int Cp, int KH, int KW,
                                                               const float* __restrict__ w,
                                                               bf16_t* __restrict__ wf,
                                                               bf16_t* __restrict__ wd) {
  const int64_t n = (int64_t)Co * KH * KW * Cp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    int64_t t = i / Cp;
    const int kw = (int)(t % KW); t /= KW;
    const int kh = (int)(t % KH);
    const int co = (int)(t / KH);
    const float v = c < Cin ? w[(((int64_t)co * Cin + c) * KH + kh) * KW + kw] : 0.f;
    wf[i] = f2bf(v);
    if (wd && c < Cin) wd[(((int64_t)c * KH + kh) * KW + kw) * Co + co] = f2bf(v);
  }
}

// x NCHW fp32 [N][Cin][H][W] -> NHWC bf16 [N][H][W][Cp] (channels zero-padded).  One thread
// per pixel: the Cin plane reads are coalesced across threads (consecutive w), the Cp-channel
// row is written as whole 16-byte chunks.
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(int N, int Cin, int H, int W, int Cp,
                                                           const float* __restrict__ x,
                                                           bf16_t* __restrict__ y) {
  const int64_t HW = (int64_t)H * W, npix = (int64_t)N * HW;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = p / HW, hw = p - b * HW;
    const float* src = x + b * Cin * HW + hw;
    uint4* dst = reinterpret_cast<uint4*>(y + p * Cp);
    for (int c0 = 0; c0 < Cp; c0 += 8) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = c0 + e < Cin ? src[(int64_t)(c0 + e) * HW] : 0.f;
      dst[c0 / 8] = pack8(v);
    }
  }
}

// 7x7/2 stem as a 4x4/1 conv on a space-to-depth input (ttmi_stem_s2d): x' [N][H/2][W/2][Cp],
// channel (ph·2 + pw)·Cin + ci = x[n][ci][2h'+ph][2w'+pw] (zero for channels >= 4·Cin), and
// W'[co][a][b][(ph, pw, ci)] = W[co][ci][2a+ph−1][2b+pw−1] (zero off the 7x7 window): with
// pad 2 top/left, y[ho][wo] = Σ_{a,b} x'[ho−2+a][wo−2+b] · W'[a][b] is exactly the 7x7/2/3
// conv, at K = 16·Cp (128 / 256 for 1 / 3 channels) instead of 49·8 = 392 padded taps.
__global__ __launch_bounds__(256) void stem_s2d_kernel(int N, int Cin, int H, int W, int Cp,
                                                       const float* __restrict__ x,
                                                       bf16_t* __restrict__ y) {
  const int Hh = H / 2, Wh = W / 2;
  const int64_t HW = (int64_t)H * W, npix = (int64_t)N * Hh * Wh;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = p / ((int64_t)Hh * Wh);
    const int r = (int)(p - b * Hh * Wh), h = r / Wh, w = r - h * Wh;
    const float* src = x + b * Cin * HW + (int64_t)(2 * h) * W + 2 * w;
    uint4* dst = reinterpret_cast<uint4*>(y + p * Cp);
    for (int c0 = 0; c0 < Cp; c0 += 8) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int q = (c0 + e) / Cin, ci = (c0 + e) - q * Cin;
        v[e] = q < 4 ? src[(int64_t)ci * HW + (q >> 1) * W + (q & 1)] : 0.f;
      }
      dst[c0 / 8] = pack8(v);
    }
  }
}
__global__ __launch_bounds__(256) void stem_weight_prep_kernel(int Co, int Cin, int Cp,
                                                               const float* __restrict__ w,
                                                               bf16_t* __restrict__ wf) {
  const int64_t n = (int64_t)Co * 16 * Cp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    const int tap = (int)((i / Cp) % 16), co = (int)(i / (16 * Cp));
    const int q = c / Cin, ci = c - q * Cin;
    const int kh = 2 * (tap >> 2) + (q >> 1) - 1, kw = 2 * (tap & 3) + (q & 1) - 1;
    const bool ok = q < 4 && kh >= 0 && kh < 7 && kw >= 0 && kw < 7;
    wf[i] = f2bf(ok ? w[(((int64_t)co * Cin + ci) * 7 + kh) * 7 + kw] : 0.f);
  }
}

// All convs' weight mirrors in one launch.  A workgroup owns a 32 (co) x TC (c) tile of one
// item: it reads w[co][c0 .. c0+TC)[KH][KW] — contiguous per co — into LDS, then writes Wf
// [co][kh][kw][c] with c fastest and Wd [c][kh][kw][co] with co fastest, both as contiguous
// runs (the per-element kernel wrote Wd 2 bytes at a stride of KH·KW·Co: one transaction per
// element).  Space-to-depth stem items (small) go element-wise.  Items are found by a scan of
// <= TTMI_WPREP_MAX prefix offsets over workgroups.
struct WPrepBatch {
  int n;
  int blk[TTMI_WPREP_MAX + 1];            // first workgroup of each item
  ttmi_conv_wprep it[TTMI_WPREP_MAX];
};
constexpr int WP_CO = 32;
TTMI_DEV int wp_tc(const ttmi_conv_wprep& t) { return t.KH * t.KW <= 9 ? 32 : 4; }
__global__ __launch_bounds__(256) void conv_weight_prep_batch_kernel(WPrepBatch b) {
  __shared__ float tile[WP_CO * (32 * 9 + 1)];
  int k = 0;
  while (k + 1 < b.n && (int)blockIdx.x >= b.blk[k + 1]) ++k;
  const ttmi_conv_wprep& t = b.it[k];
  const int j = blockIdx.x - b.blk[k];
  bf16_t* wf = reinterpret_cast<bf16_t*>(t.wf);
  if (t.s2d) {                                          // 1024 elements per workgroup
    const int64_t n = (int64_t)t.Co * 16 * t.Cp;
    for (int64_t i = (int64_t)j * 1024 + threadIdx.x; i < min(n, (int64_t)(j + 1) * 1024); i += blockDim.x) {
      const int cc = (int)(i % t.Cp);
      const int tap = (int)((i / t.Cp) % 16), co = (int)(i / (16 * t.Cp));
      const int q = cc / t.Cin, ci = cc - q * t.Cin;
      const int kh = 2 * (tap >> 2) + (q >> 1) - 1, kw = 2 * (tap & 3) + (q & 1) - 1;
      const bool ok = q < 4 && kh >= 0 && kh < 7 && kw >= 0 && kw < 7;
      wf[i] = f2bf(ok ? t.w[(((int64_t)co * t.Cin + ci) * 7 + kh) * 7 + kw] : 0.f);
    }
    return;
  }
  const int T = t.KH * t.KW, TC = wp_tc(t), P = TC * T + 1;   // LDS pitch per co (odd: no conflicts)
  const int ntc = (t.Cp + TC - 1) / TC;
  const int co0 = (j / ntc) * WP_CO, c0 = (j % ntc) * TC;
  // load: w[co0 + r][c0 + cl][tap], cl * T + tap fastest (one contiguous run per co)
  for (int f = threadIdx.x; f < WP_CO * TC * T; f += blockDim.x) {
    const int r = f / (TC * T), q = f - r * (TC * T);
    const int cl = q / T, tap = q - cl * T;
    const int co = co0 + r, cc = c0 + cl;
    tile[r * P + q] = (co < t.Co && cc < t.Cin) ? t.w[((int64_t)co * t.Cin + cc) * T + tap] : 0.f;
  }
  __syncthreads();
  // Wf[co][tap][c]: c fastest
  for (int f = threadIdx.x; f < WP_CO * T * TC; f += blockDim.x) {
    const int cl = f % TC, q = f / TC;
    const int tap = q % T, r = q / T;
    const int co = co0 + r, cc = c0 + cl;
    if (co < t.Co && cc < t.Cp) wf[((int64_t)co * T + tap) * t.Cp + cc] = f2bf(tile[r * P + cl * T + tap]);
  }
  if (t.wd) {                                           // Wd[c][tap][co]: co fastest
    bf16_t* wd = reinterpret_cast<bf16_t*>(t.wd);
    for (int f = threadIdx.x; f < TC * T * WP_CO; f += blockDim.x) {
      const int r = f % WP_CO, q = f / WP_CO;
      const int tap = q % T, cl = q / T;
      const int co = co0 + r, cc = c0 + cl;
      if (co < t.Co && cc < t.Cin) wd[((int64_t)cc * T + tap) * t.Co + co] = f2bf(tile[r * P + cl * T + tap]);
    }
  }
}

int grid1(int64_t n) { return (int)std::min<int64_t>((n + 255) / 256, 8192); }

}  // namespace

extern "C" int ttmi_conv_weight_prep(int Co, int Cin, int Cp, int KH, int KW, const float* w,
                                     uint16_t* wf, uint16_t* wd, hipStream_t s) {
  TTMI_REQUIRE(Co > 0 && Cin > 0 && Cp >= Cin && Cp % 8 == 0 && KH > 0 && KW > 0,
               "ttmi_conv_weight_prep: bad shape");
  TTMI_REQUIRE(w && wf, "ttmi_conv_weight_prep: null argument");
  hipLaunchKernelGGL(conv_weight_prep_kernel, dim3(grid1((int64_t)Co * KH * KW * Cp)), dim3(256), 0, s,
                     Co, Cin, Cp, KH, KW, w, wf, wd);
  return ttmi_check_launch("ttmi_conv_weight_prep");
}

extern "C" int ttmi_nchw_to_nhwc(int N, int Cin, int H, int W, int Cp, const float* x, uint16_t* y,
                                 hipStream_t s) {
  TTMI_REQUIRE(N >= 0 && Cin > 0 && Cp >= Cin && Cp % 8 == 0 && H > 0 && W > 0, "ttmi_nchw_to_nhwc: bad shape");
  TTMI_REQUIRE(x && y, "ttmi_nchw_to_nhwc: null argument");
  if (N == 0) return TTMI_OK;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid1((int64_t)N * H * W)), dim3(256), 0, s, N, Cin, H,
                     W, Cp, x, y);
  return ttmi_check_launch("ttmi_nchw_to_nhwc");
}

extern "C" int ttmi_conv_weight_prep_batch(int n, const ttmi_conv_wprep* items, hipStream_t s) {
  TTMI_REQUIRE(n >= 0 && (n == 0 || items), "ttmi_conv_weight_prep_batch: bad item list");
  for (int base = 0; base < n; base += TTMI_WPREP_MAX) {
    WPrepBatch b{};
    b.n = std::min(TTMI_WPREP_MAX, n - base);
    b.blk[0] = 0;
    for (int k = 0; k < b.n; ++k) {
      const ttmi_conv_wprep& t = items[base + k];
      TTMI_REQUIRE(t.Co > 0 && t.Cin > 0 && t.Cp % 8 == 0 && t.w && t.wf, "ttmi_conv_weight_prep_batch: item %d",
                   base + k);
      TTMI_REQUIRE(t.s2d ? (t.KH == 7 && t.KW == 7 && t.Cp >= 4 * t.Cin)
                         : (t.Cp >= t.Cin && t.KH > 0 && t.KW > 0 && t.KH * t.KW <= 49),
                   "ttmi_conv_weight_prep_batch: item %d shape", base + k);
      b.it[k] = t;
      const int tc = t.KH * t.KW <= 9 ? 32 : 4;
      const int64_t nb = t.s2d ? ((int64_t)t.Co * 16 * t.Cp + 1023) / 1024
                               : (int64_t)((t.Co + WP_CO - 1) / WP_CO) * ((t.Cp + tc - 1) / tc);
      TTMI_REQUIRE(b.blk[k] + nb < (1ll << 30), "ttmi_conv_weight_prep_batch: too many tiles");
      b.blk[k + 1] = b.blk[k] + (int)nb;
    }
    hipLaunchKernelGGL(conv_weight_prep_batch_kernel, dim3((unsigned)b.blk[b.n]), dim3(256), 0, s, b);
    const int rc = ttmi_check_launch("ttmi_conv_weight_prep_batch");
    if (rc) return rc;
  }
  return TTMI_OK;
}

extern "C" int ttmi_stem_s2d(int N, int Cin, int H, int W, int Cp, const float* x, uint16_t* y,
                             hipStream_t s) {
  TTMI_REQUIRE(N >= 0 && Cin > 0 && H > 0 && W > 0 && H % 2 == 0 && W % 2 == 0 && Cp >= 4 * Cin &&
                   Cp % 8 == 0, "ttmi_stem_s2d: bad shape (H, W even, Cp >= 4 Cin, Cp % 8 == 0)");
  TTMI_REQUIRE(x && y, "ttmi_stem_s2d: null argument");
  if (N == 0) return TTMI_OK;
  hipLaunchKernelGGL(stem_s2d_kernel, dim3(grid1((int64_t)N * (H / 2) * (W / 2))), dim3(256), 0, s, N, Cin,
                     H, W, Cp, x, reinterpret_cast<bf16_t*>(y));
  return ttmi_check_launch("ttmi_stem_s2d");
}

extern "C" int ttmi_stem_weight_prep(int Co, int Cin, int Cp, const float* w, uint16_t* wf, hipStream_t s) {
  TTMI_REQUIRE(Co > 0 && Cin > 0 && Cp >= 4 * Cin && Cp % 8 == 0, "ttmi_stem_weight_prep: bad shape");
  TTMI_REQUIRE(w && wf, "ttmi_stem_weight_prep: null argument");
  hipLaunchKernelGGL(stem_weight_prep_kernel, dim3(grid1((int64_t)Co * 16 * Cp)), dim3(256), 0, s, Co, Cin, Cp,
                     w, reinterpret_cast<bf16_t*>(wf));
  return ttmi_check_launch("ttmi_stem_weight_prep");
}

namespace {

// TTMI_CONV_BM=64|128 forces the FWD/DGRAD tile height (tests cover both tile shapes).
int forced_bm() {
  const char* e = getenv("TTMI_CONV_BM");
  if (!e) return 0;
  const int v = atoi(e);
  return v == 64 || v == 128 ? v : 0;
}

// TTMI_CONV_DMA=0|1 forces the kernel family; by default the LDS-DMA kernels run whenever
// the GEMM's N (output channels) is a multiple of 64: they beat the register-staged tile on
// every cfg-3 layer, the 7x7 / 4x4 stems and the 1x1 downsamples included.
// TTMI_CONV_FT=<rows>:<stages> picks the FWD/DGRAD LDS-DMA tile.  Default (measured over
// every cfg-3 layer, tools/conv_bench.py): two-stage rings, so two workgroups share a CU —
// 256 x 64 tiles for 64-channel outputs, 128 x 128 otherwise (3- and 4-stage rings, one
// workgroup per CU, ran 1.2-1.9x longer).
struct FtCfg {
  int bm, ns;
};
FtCfg ft_cfg(int bn) {
  FtCfg f{bn == 64 ? 256 : 128, 2};
  const char* e = getenv("TTMI_CONV_FT");
  int a = 0, b = 0;
  if (e && sscanf(e, "%d:%d", &a, &b) == 2 && (a == 128 || a == 256) && b >= 2 && b <= 4) f = FtCfg{a, b};
  return f;
}
// TTMI_CONV_WG=<waves>:<stages> picks the WGRAD LDS-DMA variant (default 8:2: two 64 KB
// workgroups per CU beat deeper rings, measured over every cfg-3 layer).
struct WgCfg {
  int nw, ns;
};
WgCfg wg_cfg() {
  WgCfg w{8, 2};
  const char* e = getenv("TTMI_CONV_WG");
  int a = 0, b = 0;
  if (e && sscanf(e, "%d:%d", &a, &b) == 2) w = WgCfg{a, b};
  return w;
}
int forced_dma() {
  const char* e = getenv("TTMI_CONV_DMA");
  return e ? (atoi(e) ? 1 : 0) : -1;
}
bool use_dma(int64_t, int n) {
  if (n % 64 != 0) return false;
  const int f = forced_dma();
  return f >= 0 ? f == 1 : true;
}

struct ConvPlan {
  ConvArgs a;
  int bm, bn, splits;
  bool dma;                 // on the LDS-DMA kernels (conv_dma_kernel / conv_wgrad_dma_kernel)
  int s2d;                  // space-to-depth stem (modes 3 / 4)
  int64_t ws_bytes;
};

int conv_plan(const ttmi_conv_desc* d, ConvPlan* pl) {
  TTMI_REQUIRE(d != nullptr, "ttmi_conv2d: null descriptor");
  TTMI_REQUIRE(d->mode >= 0 && d->mode <= 4, "ttmi_conv2d: bad mode");
  if (d->mode >= 3) {
    // space-to-depth stem: the descriptor states the 7x7/2/3 conv on the image; run the
    // equivalent 4x4/1 conv (pad 2 top/left) over ttmi_stem_s2d's [N][H/2][W/2][C] input
    TTMI_REQUIRE(d->KH == 7 && d->KW == 7 && d->stride == 2 && d->pad == 3 && d->H % 2 == 0 &&
                     d->W % 2 == 0 && d->C >= 4 * d->Cin && d->C % 8 == 0 && d->Co % 64 == 0,
                 "ttmi_conv2d: stem modes need a 7x7/2/3 conv, even H, W, C >= 4 Cin, Co %% 64 == 0");
    ttmi_conv_desc e = *d;
    e.mode = d->mode == 3 ? 0 : 2;
    e.H = d->H / 2; e.W = d->W / 2; e.KH = e.KW = 4; e.stride = 1; e.pad = 2; e.Cin = d->C;
    const int rc = conv_plan(&e, pl);
    if (rc) return rc;
    ConvArgs& a = pl->a;                                  // output grid of the 7x7/2 conv
    a.Ho = d->H / 2; a.Wo = d->W / 2;
    a.fWo = fdiv_make(a.Wo); a.fHo = fdiv_make(a.Ho);
    a.Cin = d->Cin;
    if (e.mode == 0) {
      a.GM = d->N * a.Ho * a.Wo;
      pl->dma = use_dma(((int64_t)a.GM + 255) / 256 * (a.GN / pl->bn), d->Co);
    } else {
      a.GK = d->N * a.Ho * a.Wo;
      const int64_t tiles = ((a.GM + pl->bm - 1) / pl->bm) * ((a.GN + 127) / 128);
      const int64_t ksteps = ((int64_t)a.GK + 63) / 64;
      const int64_t want = std::max<int64_t>(1, (1024 + tiles - 1) / tiles);
      const int64_t per = std::max<int64_t>(std::min<int64_t>(8, ksteps), (ksteps + want - 1) / want);
      a.k_split = (int)(per * 64);
      pl->splits = (int)((ksteps + per - 1) / per);
      pl->ws_bytes = (int64_t)pl->splits * a.GM * a.GN * 4;
    }
    pl->s2d = 1;
    return TTMI_OK;
  }
  TTMI_REQUIRE(d->N >= 0 && d->H > 0 && d->W > 0 && d->C > 0 && d->C % 8 == 0 && d->Co > 0 &&
                   d->Co % 8 == 0 && d->KH > 0 && d->KW > 0 && d->stride > 0 && d->pad >= 0,
               "ttmi_conv2d: bad geometry (C, Co must be multiples of 8)");
  TTMI_REQUIRE(d->Cin > 0 && d->Cin <= d->C, "ttmi_conv2d: Cin must be in (0, C]");
  const int Ho = (d->H + 2 * d->pad - d->KH) / d->stride + 1;
  const int Wo = (d->W + 2 * d->pad - d->KW) / d->stride + 1;
  TTMI_REQUIRE(Ho > 0 && Wo > 0, "ttmi_conv2d: empty output");
  const int64_t Mi = (int64_t)d->N * d->H * d->W, Mo = (int64_t)d->N * Ho * Wo;
  TTMI_REQUIRE(Mi * std::max(d->C, d->Co) < (1ll << 31) && Mo * d->Co < (1ll << 31),
               "ttmi_conv2d: tensors must have < 2^31 elements");
  ConvArgs& a = pl->a;
  a = ConvArgs{};
  a.N = d->N; a.H = d->H; a.W = d->W; a.C = d->C;
  a.Ho = Ho; a.Wo = Wo; a.Co = d->Co;
  a.KH = d->KH; a.KW = d->KW; a.S = d->stride; a.P = d->pad; a.Cin = d->Cin;
  a.x = static_cast<const bf16_t*>(d->x);
  a.dy = static_cast<const bf16_t*>(d->dy);
  a.w = static_cast<const bf16_t*>(d->w);
  a.out = d->out;
  a.addend = static_cast<const bf16_t*>(d->addend);
  a.colsum = d->colsum; a.colsumsq = d->colsumsq;
  if (d->mode == 1 && d->bn_sums) {
    TTMI_REQUIRE(d->bn_x && d->bn_mean && d->bn_rstd, "ttmi_conv2d: bn_sums needs bn_x, bn_mean, bn_rstd");
    a.bn_gate = static_cast<const bf16_t*>(d->bn_gate);
    a.bn_x = static_cast<const bf16_t*>(d->bn_x);
    a.bn_mean = d->bn_mean; a.bn_rstd = d->bn_rstd; a.bn_sums = d->bn_sums;
  }
  a.fC = fdiv_make(d->C); a.fKW = fdiv_make(d->KW);
  a.fWo = fdiv_make(Wo); a.fHo = fdiv_make(Ho); a.fCo = fdiv_make(d->Co);
  pl->splits = 1;
  pl->ws_bytes = 0;
  pl->dma = false;
  pl->s2d = 0;
  if (d->mode == 0) {
    a.GM = (int)Mo; a.GN = d->Co; a.GK = d->KH * d->KW * d->C;
    pl->bn = d->Co % 128 == 0 ? 128 : 64;
    pl->bm = 128;
    if (((a.GM + 127) / 128) * (a.GN / pl->bn) < 512) pl->bm = 64;
    if (forced_bm()) pl->bm = forced_bm();
    pl->dma = use_dma(((int64_t)a.GM + 255) / 256 * (a.GN / pl->bn), d->Co);
  } else if (d->mode == 1) {
    TTMI_REQUIRE(d->Cin == d->C, "ttmi_conv2d: DGRAD needs unpadded channels (Cin == C)");
    TTMI_REQUIRE(d->Co % 64 == 0, "ttmi_conv2d: DGRAD needs Co %% 64 == 0");
    TTMI_REQUIRE(d->stride <= 2, "ttmi_conv2d: DGRAD supports stride 1 or 2");
    const int S = d->stride;
    a.GN = d->C; a.GM = 0; a.GK = 0;
    for (int c = 0; c < S * S; ++c) {
      const int ph = c / S, pw = c % S;
      const int kh0 = (ph + d->pad) % S, kw0 = (pw + d->pad) % S;
      const int nkh = kh0 < d->KH ? (d->KH - kh0 + S - 1) / S : 0;
      const int nkw = kw0 < d->KW ? (d->KW - kw0 + S - 1) / S : 0;
      const int Hc = (d->H - ph + S - 1) / S, Wc = (d->W - pw + S - 1) / S;
      a.cHc[c] = Hc; a.cWc[c] = Wc;
      a.cM[c] = Hc > 0 && Wc > 0 ? d->N * Hc * Wc : 0;
      a.cK[c] = nkh * nkw * d->Co;
      a.ckh0[c] = kh0; a.ckw0[c] = kw0; a.cnkw[c] = std::max(nkw, 1);
      a.coffh[c] = (ph + d->pad - kh0) / S; a.coffw[c] = (pw + d->pad - kw0) / S;
      a.cfW[c] = fdiv_make(std::max(Wc, 1)); a.cfH[c] = fdiv_make(std::max(Hc, 1));
      a.cfnkw[c] = fdiv_make(std::max(nkw, 1));
      a.GM = std::max(a.GM, a.cM[c]);
    }
    pl->bn = d->C % 128 == 0 ? 128 : 64;
    pl->bm = 128;
    if (((a.GM + 127) / 128) * (a.GN / pl->bn) * S * S < 512) pl->bm = 64;
    if (forced_bm()) pl->bm = forced_bm();
    int64_t dt = 0;
    for (int c = 0; c < S * S; ++c) dt += ((int64_t)a.cM[c] + 255) / 256 * (a.GN / pl->bn);
    pl->dma = use_dma(dt, d->C);
  } else {
    a.GM = d->Co; a.GN = d->KH * d->KW * d->C; a.GK = (int)Mo;
    pl->bm = d->Co % 128 == 0 ? 128 : 64;
    pl->bn = 128;
    const int64_t tiles = ((a.GM + pl->bm - 1) / pl->bm) * ((a.GN + 127) / 128);
    const int64_t ksteps = (Mo + 63) / 64;
    const int64_t want = std::max<int64_t>(1, (1024 + tiles - 1) / tiles);
    const int64_t per = std::max<int64_t>(std::min<int64_t>(8, ksteps), (ksteps + want - 1) / want);
    a.k_split = (int)(per * 64);
    pl->splits = (int)((ksteps + per - 1) / per);
    TTMI_REQUIRE(pl->splits <= 65535, "ttmi_conv2d: too many splits");
    pl->dma = d->Co % 64 == 0 && forced_dma() != 0;
    pl->ws_bytes = (int64_t)pl->splits * a.GM * a.GN * 4;
  }
  return TTMI_OK;
}

template <int MODE>
void launch_conv(const ConvPlan& pl, hipStream_t s) {
  const ConvArgs& a = pl.a;
  if constexpr (MODE == 2) if (pl.dma) {
    const int tn = (a.GN + 127) / 128, tiles = ((a.GM + pl.bm - 1) / pl.bm) * tn;
    const dim3 grid((unsigned)((int64_t)tiles * pl.splits));
    const WgCfg w = wg_cfg();
#define TTMI_WG(BM_, NW_, NS_)                                                                    \
  if (pl.bm == BM_ && w.nw == NW_ && w.ns == NS_) {                                             \
    hipLaunchKernelGGL((conv_wgrad_dma_kernel<BM_, NW_, NS_>), grid, dim3(NW_ * 64), 0, s, a, tn, tiles); \
    return;                                                                                      \
  }
    TTMI_WG(128, 4, 4) TTMI_WG(128, 8, 4) TTMI_WG(128, 8, 3) TTMI_WG(128, 4, 2) TTMI_WG(128, 8, 2)
    TTMI_WG(64, 4, 4) TTMI_WG(64, 8, 4) TTMI_WG(64, 8, 3) TTMI_WG(64, 4, 2) TTMI_WG(64, 8, 2)
    TTMI_WG(64, 8, 6)
#undef TTMI_WG
    if (pl.bm == 128) hipLaunchKernelGGL((conv_wgrad_dma_kernel<128, 8, 2>), grid, dim3(512), 0, s, a, tn, tiles);
    else hipLaunchKernelGGL((conv_wgrad_dma_kernel<64, 8, 2>), grid, dim3(512), 0, s, a, tn, tiles);
    return;
  }
  if constexpr (MODE != 2) if (pl.dma) {
    const FtCfg f = ft_cfg(pl.bn);
    const unsigned gy = MODE == 1 ? (unsigned)(a.S * a.S) : 1u;
    const dim3 grid((unsigned)(((int64_t)a.GM + f.bm - 1) / f.bm * (a.GN / pl.bn)), gy);
#define TTMI_FT(BM_, BN_, NS_)                                                                    \
  if (f.bm == BM_ && pl.bn == BN_ && f.ns == NS_) {                                             \
    hipLaunchKernelGGL((conv_dma_kernel<MODE, BM_, BN_, NS_>), grid, dim3(512), 0, s, a);        \
    return;                                                                                      \
  }
    TTMI_FT(256, 128, 3) TTMI_FT(256, 128, 2) TTMI_FT(128, 128, 2) TTMI_FT(128, 128, 3) TTMI_FT(128, 128, 4)
    TTMI_FT(256, 64, 3) TTMI_FT(256, 64, 2) TTMI_FT(128, 64, 2) TTMI_FT(128, 64, 3) TTMI_FT(128, 64, 4)
#undef TTMI_FT
    if (pl.bn == 128) hipLaunchKernelGGL((conv_dma_kernel<MODE, 256, 128, 3>), grid, dim3(512), 0, s, a);
    else hipLaunchKernelGGL((conv_dma_kernel<MODE, 256, 64, 3>), grid, dim3(512), 0, s, a);
    return;
  }
  const int64_t tiles = (int64_t)((a.GN + pl.bn - 1) / pl.bn) * ((a.GM + pl.bm - 1) / pl.bm);
  const unsigned gy = MODE == 1 ? (unsigned)(a.S * a.S) : (unsigned)pl.splits;
  const dim3 grid((unsigned)tiles, gy);
  if (pl.bm == 128 && pl.bn == 128)
    hipLaunchKernelGGL((conv_tile_kernel<MODE, 128, 128>), grid, dim3(256), 0, s, a);
  else if (pl.bm == 128)
    hipLaunchKernelGGL((conv_tile_kernel<MODE, 128, 64>), grid, dim3(256), 0, s, a);
  else if (pl.bn == 128)
    hipLaunchKernelGGL((conv_tile_kernel<MODE, 64, 128>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((conv_tile_kernel<MODE, 64, 64>), grid, dim3(256), 0, s, a);
}

}  // namespace

extern "C" int64_t ttmi_conv2d_workspace(const ttmi_conv_desc* d) {
  ConvPlan pl;
  if (conv_plan(d, &pl) != TTMI_OK) return -1;
  return pl.ws_bytes;
}

extern "C" int ttmi_conv2d(const ttmi_conv_desc* d, hipStream_t stream) {
  ConvPlan pl;
  int rc = conv_plan(d, &pl);
  if (rc) return rc;
  if (d->N == 0) return TTMI_OK;
  const int mode = d->mode == 3 ? 0 : d->mode == 4 ? 2 : d->mode;
  if (mode == 0) {
    TTMI_REQUIRE(d->x && d->w && d->out, "ttmi_conv2d: FWD needs x, w, out");
    TTMI_REQUIRE(!d->colsum == !d->colsumsq, "ttmi_conv2d: colsum and colsumsq go together");
    launch_conv<0>(pl, stream);
  } else if (mode == 1) {
    TTMI_REQUIRE(d->dy && d->w && d->out, "ttmi_conv2d: DGRAD needs dy, w, out");
    ConvPlan pr = pl;
    if (!pl.dma) pr.a.bn_sums = nullptr;       // register tile: the reduction runs as its own pass
    launch_conv<1>(pr, stream);
    if (d->bn_sums && !pl.dma) {
      rc = ttmi_check_launch("ttmi_conv2d/dgrad");
      if (rc) return rc;
      const uint16_t* o = static_cast<const uint16_t*>(d->out);
      return ttmi_bn2d_bwd_reduce((int64_t)d->N * d->H * d->W, d->C, o, static_cast<const uint16_t*>(d->bn_gate),
                                  static_cast<const uint16_t*>(d->bn_x), d->bn_mean, d->bn_rstd, d->bn_sums,
                                  static_cast<uint16_t*>(d->out), stream);
    }
  } else {
    TTMI_REQUIRE(d->x && d->dy && d->out, "ttmi_conv2d: WGRAD needs x, dy, out");
    TTMI_REQUIRE(d->workspace && d->workspace_bytes >= pl.ws_bytes,
                 "ttmi_conv2d: WGRAD needs a workspace of ttmi_conv2d_workspace() bytes");
    pl.a.ws = static_cast<float*>(d->workspace);
    launch_conv<2>(pl, stream);
    rc = ttmi_check_launch("ttmi_conv2d/wgrad");
    if (rc) return rc;
    const int64_t n4 = (int64_t)pl.a.GM * pl.a.GN / 4;
    const unsigned gx = (unsigned)((n4 + 255) / 256);
    const int KW = pl.a.KW, KHKW = pl.a.KH * pl.a.KW;
    int step = 1;
    if (pl.splits > WR_SPLITS) {         // chunk totals first (in place), then the chunk slabs
      hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(gx, (unsigned)((pl.splits + WR_SPLITS - 1) / WR_SPLITS)),
                         dim3(256), 0, stream, pl.a.ws, pl.splits, 1, pl.a.GM, pl.a.GN, d->C, d->Cin, KW, KHKW,
                         0, static_cast<float*>(d->out), pl.s2d);
      rc = ttmi_check_launch("ttmi_conv2d/wgrad_chunks");
      if (rc) return rc;
      step = WR_SPLITS;
    }
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(gx), dim3(256), 0, stream, pl.a.ws, pl.splits, step, pl.a.GM,
                       pl.a.GN, d->C, d->Cin, KW, KHKW, 1, static_cast<float*>(d->out), pl.s2d);
  }
  return ttmi_check_launch("ttmi_conv2d");
}
