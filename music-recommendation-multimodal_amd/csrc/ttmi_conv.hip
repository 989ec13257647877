// ttmi_conv.hip — 2-D convolution as implicit GEMM on MFMA (bf16 operands, fp32 accumulate)
// for the ResNet-18 audio/visual encoders (reference item_tower.py:9-39, torchvision
// resnet18: conv1 7x7/2, BasicBlock 3x3 convs, 1x1/2 downsample).
//
// Activations are NHWC bf16 with the channel count a multiple of 8 (the 1- and 3-channel
// stems are zero-padded to 8).  Three modes share one tile kernel (64x64 output tile, four
// waves 2x2, K walked in 64-element tiles, double-buffered LDS with register prefetch):
//   FWD   y[m, co]  = Σ_k im2col(x)[m, k] · Wf[co, k]        m = (n, ho, wo), k = (kh, kw, ci)
//   DGRAD dx[m, ci] = Σ_k taps(dy)[m, k] · Wd[ci, k]         m = (n, h, w),   k = (kh, kw, co)
//   WGRAD dW[co, k] += Σ_m dy[m, co] · im2col(x)[m, k]       split over m, fp32 atomics
// Wf = [Co][KH][KW][C] and Wd = [C][KH][KW][Co] are bf16 mirrors of torch's [Co][Ci][KH][KW]
// (ttmi_conv_weight_prep); WGRAD scatters into torch's layout directly.  A 16-byte operand
// chunk is 8 consecutive channels of one tap, so every gathered load is one uint4 (zero
// outside the image / off the stride lattice).  FWD also accumulates the per-channel Σy and
// Σy² of the fp32 output for the BatchNorm that follows.
#include "ttmi_common.h"

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4c_t;

TTMI_DEV uint2 c_lds8(const char* p) { return *reinterpret_cast<const uint2*>(p); }
TTMI_DEV uint2 c_lds_tr8(const char* p) {
  const s16x4c_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4c_t*)(p));
  return __builtin_bit_cast(uint2, v);
}

struct ConvArgs {
  int mode;                 // 0 FWD, 1 DGRAD, 2 WGRAD
  int N, H, W, C;           // input  (C padded, % 8)
  int Ho, Wo, Co;           // output (Co % 8)
  int KH, KW, S, P;
  int Cin;                  // true input channels (WGRAD scatter; <= C)
  const bf16_t* x;          // FWD/WGRAD: input NHWC
  const bf16_t* dy;         // DGRAD/WGRAD: output grad NHWC
  const bf16_t* w;          // FWD: Wf, DGRAD: Wd
  void* out;                // FWD: y bf16 [M][Co]; DGRAD: dx bf16 [M][C]; WGRAD: dW f32 torch layout
  const bf16_t* addend;     // DGRAD: added before the store (the other branch's grad), or NULL
  float* colsum;            // FWD: Σ y per channel (may be NULL)
  float* colsumsq;          // FWD: Σ y² per channel
  int64_t GM, GN, GK;       // GEMM sizes
  int64_t k_split;          // WGRAD: pixels per split (multiple of 64)
};

constexpr int BM = 64, BN = 64, BKE = 64;
constexpr int PK = 144;                     // k-major pitch: 64 bf16 + 16 B
constexpr int PT = BM * 2 + 32;             // [k][row] pitch for transposed reads

// Address of the 16-byte chunk of im2col(x) at output pixel m, column k (k % 8 == 0).
TTMI_DEV const bf16_t* im2col_ptr(const ConvArgs& a, int64_t m, int64_t k) {
  if (m >= (int64_t)a.N * a.Ho * a.Wo || k >= (int64_t)a.KH * a.KW * a.C) return nullptr;
  const int wo = (int)(m % a.Wo);
  const int64_t t = m / a.Wo;
  const int ho = (int)(t % a.Ho);
  const int n = (int)(t / a.Ho);
  const int tap = (int)(k / a.C), ci = (int)(k % a.C);
  const int kh = tap / a.KW, kw = tap % a.KW;
  const int hi = ho * a.S - a.P + kh, wi = wo * a.S - a.P + kw;
  if (hi < 0 || hi >= a.H || wi < 0 || wi >= a.W) return nullptr;
  return a.x + (((int64_t)n * a.H + hi) * a.W + wi) * a.C + ci;
}

// Address of the chunk of the transposed-conv taps of dy at input pixel m, column k =
// (kh, kw, co): dy[n, (h+P-kh)/S, (w+P-kw)/S, co] when on the stride lattice.
TTMI_DEV const bf16_t* dgrad_ptr(const ConvArgs& a, int64_t m, int64_t k) {
  if (m >= (int64_t)a.N * a.H * a.W || k >= (int64_t)a.KH * a.KW * a.Co) return nullptr;
  const int w = (int)(m % a.W);
  const int64_t t = m / a.W;
  const int h = (int)(t % a.H);
  const int n = (int)(t / a.H);
  const int tap = (int)(k / a.Co), co = (int)(k % a.Co);
  const int kh = tap / a.KW, kw = tap % a.KW;
  const int th = h + a.P - kh, tw = w + a.P - kw;
  if (th < 0 || tw < 0 || th % a.S || tw % a.S) return nullptr;
  const int ho = th / a.S, wo = tw / a.S;
  if (ho >= a.Ho || wo >= a.Wo) return nullptr;
  return a.dy + (((int64_t)n * a.Ho + ho) * a.Wo + wo) * a.Co + co;
}

TTMI_DEV uint4 ld_or_zero(const bf16_t* p) {
  return p ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
}

// Fragment reads (same k-permutation on both operands: lane group g of each 32-wide k chunk
// holds k = 4g..4g+3 and 16+4g..16+4g+3).
TTMI_DEV uint4 frag_k(const char* s, int row0, int c, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const char* p = s + (row0 + i) * PK + c * 64 + g * 8;
  const uint2 lo = c_lds8(p), hi = c_lds8(p + 32);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}
TTMI_DEV uint4 frag_t(const char* s, int row0, int c, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int q = i >> 2, pp = i & 3;
  const char* p = s + (c * 32 + 4 * g + q) * PT + (row0 + 4 * pp) * 2;
  const uint2 lo = c_lds_tr8(p), hi = c_lds_tr8(p + 16 * PT);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs a) {
  // FWD/DGRAD: A k-major gathered [BM][64 k], B k-major weight rows.
  // WGRAD:     A = dy as [k=pixel][row=co] (transposed reads), B = im2col as [k=pixel][row=kcol].
  constexpr int AKM = BM * PK, AT = BKE * PT;
  constexpr int STAGE = (AKM > AT ? AKM : AT) + (BN * PK > AT ? BN * PK : AT);
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t n0 = (int64_t)blockIdx.x * BN, m0 = (int64_t)blockIdx.y * BM;
  const bool wg = a.mode == 2;
  const int64_t kbeg = wg ? (int64_t)blockIdx.z * a.k_split : 0;
  const int64_t kend = wg ? std::min<int64_t>(a.GK, kbeg + a.k_split) : a.GK;
  const int64_t Kw = (int64_t)a.KH * a.KW * a.C;        // weight row length (FWD)

  // per-thread chunk coordinates: 2 chunks per operand per stage
  uint4 ra[2], rb[2];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int idx = tid + c * 256;
      if (!wg) {
        const int r = idx >> 3, kk = (idx & 7) * 8;       // [row][k]: 8 chunks per row
        const int64_t m = m0 + r, k = k0 + kk, n = n0 + r;
        const bf16_t* pa = a.mode == 0 ? im2col_ptr(a, m, k) : dgrad_ptr(a, m, k);
        ra[c] = ld_or_zero(pa);
        const int64_t kw_len = a.mode == 0 ? Kw : (int64_t)a.KH * a.KW * a.Co;
        const bf16_t* pb = (n < a.GN && k < kw_len) ? a.w + n * kw_len + k : nullptr;
        rb[c] = ld_or_zero(pb);
      } else {
        const int kr = idx >> 3, rr = (idx & 7) * 8;      // [k][row]: 8 chunks per k row
        const int64_t pix = k0 + kr;
        const int64_t co = m0 + rr, kc = n0 + rr;
        const bf16_t* pa = (pix < kend && co < a.Co) ? a.dy + pix * a.Co + co : nullptr;
        ra[c] = ld_or_zero(pa);
        rb[c] = pix < kend ? ld_or_zero(im2col_ptr(a, pix, kc)) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store = [&](char* s) {
    char* sa = s;
    char* sb = s + (AKM > AT ? AKM : AT);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int idx = tid + c * 256;
      if (!wg) {
        *reinterpret_cast<uint4*>(sa + (idx >> 3) * PK + (idx & 7) * 16) = ra[c];
        *reinterpret_cast<uint4*>(sb + (idx >> 3) * PK + (idx & 7) * 16) = rb[c];
      } else {
        *reinterpret_cast<uint4*>(sa + (idx >> 3) * PT + (idx & 7) * 16) = ra[c];
        *reinterpret_cast<uint4*>(sb + (idx >> 3) * PT + (idx & 7) * 16) = rb[c];
      }
    }
  };

  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (kbeg < kend) {
    load(kbeg);
    store(smem);
  }
  __syncthreads();
  int buf = 0;
  for (int64_t k0 = kbeg; k0 < kend; k0 += BKE) {
    const bool more = k0 + BKE < kend;
    if (more) load(k0 + BKE);
    const char* sa = smem + buf * STAGE;
    const char* sb = sa + (AKM > AT ? AKM : AT);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      uint4 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = wg ? frag_t(sa, wm * 32 + i * 16, c, lane) : frag_k(sa, wm * 32 + i * 16, c, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = wg ? frag_t(sb, wn * 32 + j * 16, c, lane) : frag_k(sb, wn * 32 + j * 16, c, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) Mma<bf16_t>::run(acc[i][j], bfr[j], af[i]);
    }
    if (more) store(smem + (buf ^ 1) * STAGE);
    __syncthreads();
    buf ^= 1;
  }

  // epilogue: lane holds C[m][n..n+3], m = tile row + (lane & 15), n = tile col + 4*(lane >> 4)
  const int li = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t n = n0 + wn * 32 + j * 16 + 4 * lg;
    float cs[4] = {0.f, 0.f, 0.f, 0.f}, cq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t m = m0 + wm * 32 + i * 16 + li;
      if (m >= a.GM || n >= a.GN) continue;
      const float* v = reinterpret_cast<const float*>(&acc[i][j]);
      if (a.mode == 2) {
        // dW[co = m][kcol = n + e] -> torch [Co][Cin][KH][KW]
        float* dw = static_cast<float*>(a.out);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t kc = n + e;
          const int tap = (int)(kc / a.C), ci = (int)(kc % a.C);
          if (ci < a.Cin) atomicAdd(dw + ((m * a.Cin + ci) * a.KH + tap / a.KW) * a.KW + tap % a.KW, v[e]);
        }
        continue;
      }
      float o[4] = {v[0], v[1], v[2], v[3]};
      if (a.mode == 1 && a.addend) {
        const ushort4 q = *reinterpret_cast<const ushort4*>(a.addend + m * a.GN + n);
        o[0] += bf2f(q.x); o[1] += bf2f(q.y); o[2] += bf2f(q.z); o[3] += bf2f(q.w);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) { cs[e] += o[e]; cq[e] += o[e] * o[e]; }
      ushort4 q;
      q.x = f2bf(o[0]); q.y = f2bf(o[1]); q.z = f2bf(o[2]); q.w = f2bf(o[3]);
      *reinterpret_cast<ushort4*>(static_cast<bf16_t*>(a.out) + m * a.GN + n) = q;
    }
    if (a.mode == 0 && a.colsum && n < a.GN) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float s = cs[e], s2 = cq[e];
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          s += __shfl_xor(s, off, 64);
          s2 += __shfl_xor(s2, off, 64);
        }
        if (li == 0) {
          atomicAdd(a.colsum + n + e, s);
          atomicAdd(a.colsumsq + n + e, s2);
        }
      }
    }
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

// x NCHW fp32 [N][Cin][H][W] -> NHWC bf16 [N][H][W][Cp] (channels zero-padded).
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(int N, int Cin, int H, int W, int Cp,
                                                           const float* __restrict__ x,
                                                           bf16_t* __restrict__ y) {
  const int64_t n = (int64_t)N * H * W * Cp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    const int64_t p = i / Cp;
    const int w = (int)(p % W);
    const int64_t t = p / W;
    const int h = (int)(t % H);
    const int b = (int)(t / H);
    y[i] = c < Cin ? f2bf(x[(((int64_t)b * Cin + c) * H + h) * W + w]) : (bf16_t)0;
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
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid1((int64_t)N * H * W * Cp)), dim3(256), 0, s, N, Cin, H,
                     W, Cp, x, y);
  return ttmi_check_launch("ttmi_nchw_to_nhwc");
}

extern "C" int ttmi_conv2d(const ttmi_conv_desc* d, hipStream_t stream) {
  TTMI_REQUIRE(d != nullptr, "ttmi_conv2d: null descriptor");
  TTMI_REQUIRE(d->mode >= 0 && d->mode <= 2, "ttmi_conv2d: bad mode");
  TTMI_REQUIRE(d->N >= 0 && d->H > 0 && d->W > 0 && d->C > 0 && d->C % 8 == 0 && d->Co > 0 &&
                   d->Co % 8 == 0 && d->KH > 0 && d->KW > 0 && d->stride > 0 && d->pad >= 0,
               "ttmi_conv2d: bad geometry (C, Co must be multiples of 8)");
  TTMI_REQUIRE(d->Cin > 0 && d->Cin <= d->C, "ttmi_conv2d: Cin must be in (0, C]");
  const int Ho = (d->H + 2 * d->pad - d->KH) / d->stride + 1;
  const int Wo = (d->W + 2 * d->pad - d->KW) / d->stride + 1;
  TTMI_REQUIRE(Ho > 0 && Wo > 0, "ttmi_conv2d: empty output");
  if (d->N == 0) return TTMI_OK;
  ConvArgs a{};
  a.mode = d->mode;
  a.N = d->N; a.H = d->H; a.W = d->W; a.C = d->C;
  a.Ho = Ho; a.Wo = Wo; a.Co = d->Co;
  a.KH = d->KH; a.KW = d->KW; a.S = d->stride; a.P = d->pad; a.Cin = d->Cin;
  a.x = static_cast<const bf16_t*>(d->x);
  a.dy = static_cast<const bf16_t*>(d->dy);
  a.w = static_cast<const bf16_t*>(d->w);
  a.out = d->out;
  a.addend = static_cast<const bf16_t*>(d->addend);
  a.colsum = d->colsum; a.colsumsq = d->colsumsq;
  const int64_t Mo = (int64_t)d->N * Ho * Wo, Mi = (int64_t)d->N * d->H * d->W;
  int splits = 1;
  if (d->mode == 0) {
    TTMI_REQUIRE(d->x && d->w && d->out, "ttmi_conv2d: FWD needs x, w, out");
    TTMI_REQUIRE(!d->colsum == !d->colsumsq, "ttmi_conv2d: colsum and colsumsq go together");
    a.GM = Mo; a.GN = d->Co; a.GK = (int64_t)d->KH * d->KW * d->C;
  } else if (d->mode == 1) {
    TTMI_REQUIRE(d->dy && d->w && d->out, "ttmi_conv2d: DGRAD needs dy, w, out");
    TTMI_REQUIRE(d->Cin == d->C, "ttmi_conv2d: DGRAD needs unpadded channels (Cin == C)");
    a.GM = Mi; a.GN = d->C; a.GK = (int64_t)d->KH * d->KW * d->Co;
  } else {
    TTMI_REQUIRE(d->x && d->dy && d->out, "ttmi_conv2d: WGRAD needs x, dy, out");
    a.GM = d->Co; a.GN = (int64_t)d->KH * d->KW * d->C; a.GK = Mo;
    const int64_t tiles = ((a.GM + BM - 1) / BM) * ((a.GN + BN - 1) / BN);
    const int64_t ktiles = (Mo + BKE - 1) / BKE;
    int64_t want = std::max<int64_t>(1, (1024 + tiles - 1) / tiles);
    want = std::min<int64_t>(want, ktiles);
    const int64_t per = (ktiles + want - 1) / want;
    a.k_split = per * BKE;
    splits = (int)((Mo + a.k_split - 1) / a.k_split);
    TTMI_REQUIRE(splits <= 65535, "ttmi_conv2d: too many splits");
  }
  const int64_t gx = (a.GN + BN - 1) / BN, gy = (a.GM + BM - 1) / BM;
  TTMI_REQUIRE(gy <= 65535, "ttmi_conv2d: grid too large");
  hipLaunchKernelGGL(conv_gemm_kernel, dim3((unsigned)gx, (unsigned)gy, (unsigned)splits), dim3(256), 0,
                     stream, a);
  return ttmi_check_launch("ttmi_conv2d");
}
