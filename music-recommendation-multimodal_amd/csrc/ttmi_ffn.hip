// ttmi_ffn.hip — the encoder layer's feed-forward sub-block forward in one launch (ABI 21).
//
// Reference: nn.TransformerEncoderLayer(norm_first=True)'s _ff_block and its residual, then the
// next layer's norm1 (user_tower.py:37-45, 111-116):
//   h  = drop_f(relu(a2·W1ᵀ + b1))         bf16 [M, F]   (kept: the backward's gate and dW2 operand)
//   x2 = x1 + drop2(h·W2ᵀ + b2)             fp32 [M, 128]
//   y  = bf16(LN(x2)·w + b), mean / rstd    (the next layer's norm1)
// The unfused pair (the FFN1 row panel, then ttmi_linear_res_ln) writes h and reads it back
// (26 MB each way at cfg 2) and stages each weight image in its own launch.  Here h never
// leaves the wave between the two GEMMs: FFN1's MFMA output fragment — lane (li, g) holds row li,
// hidden units 32p + 8g .. +7 — is, bf16-packed, exactly the B-operand fragment of FFN2's k-step
// over hidden units [32p, 32p + 32), so it feeds straight back (and is stored once for the
// backward).  The weights stream through LDS in groups of 128 hidden units (the group's W1 rows
// and W2 columns, two 128 x 128 bf16 images, 68 KB), double-buffered by LDS-DMA under the
// previous group's MFMAs.  One 16-row tile per wave, NWV waves per workgroup.
//
// Bits: h is the FFN1 row panel's (same fragments, MFMA order, epilogue).  FFN2 sums its k-steps
// in hidden-unit order (the row panel sums lane-group-strided k): x2 / y / mean / rstd agree
// with ttmi_linear_res_ln to fp32 rounding, not bit for bit.
#include "ttmi_common.h"

namespace {

constexpr int FB_D = 128;                    // the LayerNorm width (d_model)
constexpr int FB_P = 2 * FB_D + 16;          // image row pitch (bytes): a lane group's 16 rows
                                             // fall in distinct bank slots
constexpr int FB_IMG = 128 * FB_P;           // one 128 x 128 bf16 image (34,816 B)
constexpr int FB_BUF = 2 * FB_IMG;           // a group's W1 rows + W2 columns
constexpr int FB_CPR = FB_D / 8 + 1;         // 16-byte chunks per image row (the last: pad zeros)
constexpr int FB_INS = 128 * FB_CPR / 64;    // DMA wave-instructions per image (34)
static_assert((128 * FB_CPR) % 64 == 0, "whole DMA instructions");

struct FfnArgs {
  const bf16_t* a; const bf16_t* w1; const float* b1; const bf16_t* w2; const float* b2;
  const float* res; bf16_t* h; float* x2;
  const float* lnw; const float* lnb; float eps; bf16_t* y; float* mean; float* rstd;
  DropParams df, d2;
  int M;
  // KV (ABI 22): the next layer's K / V input projection of y, kv[m, n] = y·wkvᵀ + bkv (n < 256)
  const bf16_t* wkv; const float* bkv; bf16_t* kv; int64_t ldkv;
};

template <int NWV, int NG, bool PIPE, bool DF, bool KV = false>
__global__ __launch_bounds__(NWV * 64) void ffn_block_kernel(FfnArgs g) {
  constexpr int F = NG * 128;
  // Every operand reaches LDS by LDS-DMA — the rows' A tile too, staged in buffer 1's W2 image
  // — so no compiler-counted load sits among the DMAs: a compiler wait (vmcnt(0) before a
  // register's first use) there would also wait for every DMA behind it.  Each wave issues the
  // same number of wave-instructions per image (PW; the surplus re-issues an instruction another
  // wave also issues: identical bytes), so one vmcnt immediate serves every wave.
  static_assert(NWV == 8, "the vmcnt immediates below count 8 waves");
  constexpr int PW = (FB_INS + NWV - 1) / NWV;           // 5 per 34-instruction image
  constexpr int NPI = F / 256 + 5 + (KV ? 1 : 0);        // b1 (1 KB each), b2, LN w / b, 2 seeds, bkv
  static_assert(NPI <= NWV, "one parameter instruction per wave");
  constexpr int PB = F * 4;                              // parameter slots: b1 | b2 | lnw | lnb | seeds | bkv
  __shared__ __attribute__((aligned(16))) char smem[2 * FB_BUF + PB + (KV ? 6 : 5) * 1024];
  char* const spar = smem + 2 * FB_BUF;
  TTMI_TSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int64_t r0 = (int64_t)blockIdx.x * (16 * NWV);
  const int64_t m = r0 + 16 * wave + li;
  const bool mok = m < g.M;
  const int64_t mc = mok ? m : (int64_t)g.M - 1;
  const uint32_t wbytes = (uint32_t)F * FB_D * 2;        // W1 and W2 alike
  const uint32_t abytes = (uint32_t)min<int64_t>(16 * NWV, g.M - r0) * FB_D * 2;
  const i32x4_t r1 = make_rsrc(g.w1, wbytes), r2 = make_rsrc(g.w2, wbytes);
  const i32x4_t ra = make_rsrc(g.a + r0 * FB_D, abytes);  // rows past M: zeros
  // per-lane offsets of this wave's PW slots of a 128-row image (row n, chunk c; the pad chunk
  // reads at the range end: zeros); a W group adds a uniform shift (computed once: the row /
  // chunk split was ~15 VALU a DMA)
  uint32_t oA[PW], oW1[PW], oW2[PW];
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    int ii = wv + NWV * j;
    if (ii >= FB_INS) ii -= FB_INS;
    const int q = ii * 64 + lane, n = q / FB_CPR, c = q % FB_CPR;
    const bool pad = c == FB_CPR - 1;
    oA[j] = pad ? (uint32_t)(16 * NWV * FB_D * 2) : (uint32_t)((n * FB_D + 8 * c) * 2);
    oW1[j] = pad ? wbytes : (uint32_t)((n * FB_D + 8 * c) * 2);
    // (slot c holds unit chunk 4 (c & 3) + (c >> 2): FFN2's lane group lg reads its four k-step
    // chunks 4p + lg side by side, so a ds_read_b128's lane groups hit distinct banks)
    oW2[j] = pad ? wbytes : (uint32_t)((n * F + 8 * (4 * (c & 3) + (c >> 2))) * 2);
  }
  auto slot = [&](int j) { int ii = wv + NWV * j; return ii >= FB_INS ? ii - FB_INS : ii; };
  auto issue_a = [&]() {                                 // the A tile -> buffer 1's W2 image
    const uint32_t base = lds_addr(smem + FB_BUF + FB_IMG);
#pragma unroll
    for (int j = 0; j < PW; ++j) dma16(ra, oA[j], base + slot(j) * 1024);
  };
  auto issue_w1 = [&](int grp) {                         // W1 rows [128 grp, +128)
    const uint32_t base = lds_addr(smem + (grp & 1) * FB_BUF);
#pragma unroll
    for (int j = 0; j < PW; ++j) dma16(r1, oW1[j] + (uint32_t)(grp * 128 * FB_D * 2), base + slot(j) * 1024);
  };
  auto issue_w2 = [&](int grp) {                         // W2 columns [128 grp, +128)
    const uint32_t base = lds_addr(smem + (grp & 1) * FB_BUF + FB_IMG);
#pragma unroll
    for (int j = 0; j < PW; ++j) dma16(r2, oW2[j] + (uint32_t)(grp * 128 * 2), base + slot(j) * 1024);
  };
  {                                                      // parameters and dropout seeds
    const int k = wv < NPI ? wv : wv - NPI;              // (NPI <= 8 < 2 NPI)
    const uint32_t dst = lds_addr(spar) + (uint32_t)(k * 1024);
    const uint32_t off = (uint32_t)(lane * 16);
    if (k < F / 256) dma16(make_rsrc(g.b1, PB), off + (uint32_t)(k * 1024), dst);
    else if (k == F / 256) dma16(make_rsrc(g.b2, FB_D * 4), off, dst);
    else if (k == F / 256 + 1) dma16(make_rsrc(g.lnw, FB_D * 4), off, dst);
    else if (k == F / 256 + 2) dma16(make_rsrc(g.lnb, FB_D * 4), off, dst);
    else if (k == F / 256 + 3) dma16(make_rsrc(g.df.seed, g.df.on ? 8 : 0), off, dst);
    else if (!KV || k == F / 256 + 4) dma16(make_rsrc(g.d2.seed, g.d2.on ? 8 : 0), off, dst);
    else dma16(make_rsrc(g.bkv, 2 * FB_D * 4), off, dst);   // 256 floats: one 1 KB slot
  }
  // KV: W_kv [256, 128] (two images) into the buffer the last group does not use, issued at the
  // last group's start (that buffer is free then); the row tiles' y into the other one at the end
  constexpr int KVBUF = ((NG - 1) & 1) ^ 1, ABUF = (NG - 1) & 1;
  auto issue_kv = [&]() {
    const i32x4_t rkv = make_rsrc(g.wkv, 2 * FB_D * FB_D * 2);   // pad chunks past it: zeros
    const uint32_t base = lds_addr(smem + KVBUF * FB_BUF);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int j = 0; j < PW; ++j)
        dma16(rkv, oW1[j] + (uint32_t)(hf * 128 * FB_D * 2), base + hf * FB_IMG + slot(j) * 1024);
  };
  issue_a();
  issue_w1(0);
  issue_w2(0);
  if (NG > 1) issue_w1(1);
  // in flight behind the parameters, the A tile and W1 group 0: W2 group 0 and W1 group 1
  if (NG > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PW) : "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW) : "memory");
  __syncthreads();
  TTMI_TSTAMP(1);
  const float* sb1 = reinterpret_cast<const float*>(spar);
  const float* sb2 = reinterpret_cast<const float*>(spar + PB);
  const float* slw = reinterpret_cast<const float*>(spar + PB + 1024);
  const float* slb = reinterpret_cast<const float*>(spar + PB + 2048);
  DropKeys dkf, dk2;
  {
    const uint64_t sf = *reinterpret_cast<const uint64_t*>(spar + PB + 3072);
    const uint64_t s2 = *reinterpret_cast<const uint64_t*>(spar + PB + 4096);
    dkf = DropKeys{(uint32_t)sf, (uint32_t)(sf >> 32), g.df.thresh, g.df.scale, DF};   // (DF: no branch
                                                                              // splits the group's block)
    dk2 = DropKeys{(uint32_t)s2, (uint32_t)(s2 >> 32), g.d2.thresh, g.d2.scale, g.d2.on};
  }
  // the row's FFN1 operand: lane group lg holds k = 32 lg + 8c (the row panel's permutation)
  uint4 af[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) af[c] = lds16(smem + FB_BUF + FB_IMG + (16 * wave + li) * FB_P + 64 * lg + 16 * c);
  const int wrow = 8 * (li >> 2) + (li & 3);             // column-paired rows (the panel layout)
  // h stores go through a buffer resource: rows past M are dropped by its range, so every wave
  // issues exactly 4 stores a group and the vmcnt immediates below stay exact
  const __amdgpu_buffer_rsrc_t rh =
      __builtin_amdgcn_make_buffer_rsrc(g.h, 0, (int)((int64_t)g.M * F * 2), 0x00020000);
  f32x4_t acc2[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc2[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float4 rpre[8];
  uint64_t twait = 0;                                    // (diagnostic builds) ticks at the group seams
  auto load_res_half = [&](int h) {                      // x1's row, column quarters 2h, 2h + 1
    const float* rp = g.res + mc * FB_D + 8 * lg;
#pragma unroll
    for (int p = 2 * h; p < 2 * h + 2; ++p) {
      rpre[2 * p] = *reinterpret_cast<const float4*>(rp + 32 * p);
      rpre[2 * p + 1] = *reinterpret_cast<const float4*>(rp + 32 * p + 4);
    }
  };
  auto load_res = [&]() { load_res_half(0); load_res_half(1); };
  auto ffn1 = [&](int grp, f32x4_t (&acc)[8], bool barriers) {   // 16 rows x 128 hidden units
    const char* w1b = smem + (grp & 1) * FB_BUF + wrow * FB_P + 64 * lg;
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
      for (int t = 0; t < 8; ++t)
        Mma<bf16_t>::run(acc[t], lds16(w1b + (32 * (t >> 1) + 4 * (t & 1)) * FB_P + 16 * c), af[c]);
      if (barriers) __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto epi1 = [&](int grp, const f32x4_t (&acc)[8], uint4 (&hq)[4]) {   // h = drop_f(relu(. + b1))
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int n = 128 * grp + 32 * p + 8 * lg;
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = fmaxf(acc[2 * p][e] + sb1[n + e], 0.f);
        v[4 + e] = fmaxf(acc[2 * p + 1][e] + sb1[n + 4 + e], 0.f);
      }
      drop_apply_vec<8>(dkf, (uint32_t)(m * F + n), v);
      hq[p] = pack8(v);
      const i32x4_t q = {(int)hq[p].x, (int)hq[p].y, (int)hq[p].z, (int)hq[p].w};
      __builtin_amdgcn_raw_buffer_store_b128(q, rh, (uint32_t)((m * F + n) * 2), 0, 0);
    }
  };
  auto ffn2 = [&](int grp, const uint4 (&hq)[4]) {       // FFN2's k-steps over the group's units
    const char* w2b = smem + (grp & 1) * FB_BUF + FB_IMG + wrow * FB_P + 64 * lg;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
#pragma unroll
      for (int t = 0; t < 8; ++t)
        Mma<bf16_t>::run(acc2[t], lds16(w2b + (32 * (t >> 1) + 4 * (t & 1)) * FB_P + 16 * p), hq[p]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  if constexpr (PIPE) {
    // Software pipeline: group k's epilogue (VALU: bias, ReLU, the dropout hash) runs beside group
    // k + 1's FFN1 MFMAs, then group k's FFN2.  W1 and W2 images keep their slots (group & 1) but
    // are re-filled on their own schedule: W1 group k + 2 as soon as FFN1 k is done (start of
    // iteration k), W2 group k + 1 as soon as FFN2 k - 1 is (start of iteration k).  Each
    // iteration starts with one wait — the images it reads landed; younger: the previous
    // iteration's 4 h stores (iteration 0: W2 group 1) — and one barrier.
    if (NG > 1) {
      __syncthreads();                                   // every wave has its A fragments
      issue_w2(1);                                       // (over the A tile)
    }
    f32x4_t acc1[8];
    ffn1(0, acc1, true);
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const uint64_t tw0 = TTMI_TNOW();
      if (k == 0) {
        if (NG > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      }
      __syncthreads();
      twait += TTMI_TNOW() - tw0;
      if (k >= 1 && k + 1 < NG) issue_w2(k + 1);
      if (k + 2 < NG) issue_w1(k + 2);
      // x1's row for the epilogue, half an iteration early (after that iteration's DMAs: the
      // next seam's vmcnt(4) covers it), half in the last
      if (NG > 1 && k == NG - 2) load_res_half(0);
      if (k == NG - 1) {
        if (NG > 1) load_res_half(1);
        else load_res();
        if constexpr (KV) issue_kv();
      }
      f32x4_t acc1n[8];
      uint4 hq[4];
      if (k + 1 < NG) {
        // group k + 1's FFN1 k-step p (8 MFMAs) beside group k's epilogue columns 32p..32p+31, in
        // fenced quarters so the MFMAs issue among the hash VALU rather than in one run
        const char* w1b = smem + ((k + 1) & 1) * FB_BUF + wrow * FB_P + 64 * lg;
#pragma unroll
        for (int t = 0; t < 8; ++t) acc1n[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int n = 128 * k + 32 * p + 8 * lg;
          float v[8];
#pragma unroll
          for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
            for (int t = 4 * hf; t < 4 * hf + 4; ++t)
              Mma<bf16_t>::run(acc1n[t], lds16(w1b + (32 * (t >> 1) + 4 * (t & 1)) * FB_P + 16 * p), af[p]);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[4 * hf + e] = fmaxf(acc1[2 * p + hf][e] + sb1[n + 4 * hf + e], 0.f);
            drop_apply_vec<4>(dkf, (uint32_t)(m * F + n + 4 * hf), v + 4 * hf);
            __builtin_amdgcn_sched_barrier(0);
          }
          hq[p] = pack8(v);
          const i32x4_t q = {(int)hq[p].x, (int)hq[p].y, (int)hq[p].z, (int)hq[p].w};
          __builtin_amdgcn_raw_buffer_store_b128(q, rh, (uint32_t)((m * F + n) * 2), 0, 0);
        }
      } else {
        epi1(k, acc1, hq);
      }
      ffn2(k, hq);
      if (k + 1 < NG) {
#pragma unroll
        for (int t = 0; t < 8; ++t) acc1[t] = acc1n[t];
      }
      TTMI_TSTAMP(2 + (k < 4 ? k : 3));
    }
  } else {
#pragma unroll
  for (int grp = 0; grp < NG; ++grp) {
    if (grp == NG - 1) {
      load_res();
      if constexpr (KV) issue_kv();
    }
    // ---- FFN1: 16 rows x the group's 128 hidden units
    f32x4_t acc1[8];
    ffn1(grp, acc1, true);
    // ---- h = drop_f(relu(. + b1)) -> bf16 fragments (stored for the backward)
    uint4 hq[4];
    epi1(grp, acc1, hq);
    if (grp == 0) {
      // W2 group 0 landed (behind it: W1 group 1, this group's 4 h stores); every wave has read
      // its A fragments, so W2 group 1 may overwrite the A tile
      if (NG > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW + 4) : "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      __syncthreads();
      if (NG > 1) issue_w2(1);
    }
    ffn2(grp, hq);
    if (grp + 1 < NG) {
      const uint64_t tw0 = TTMI_TNOW();
      __syncthreads();                                   // every wave is done with this buffer
      // group grp + 1 landed; younger: group grp + 2's DMAs and (grp >= 1) this group's h stores
      // (group 0's precede W2 group 1)
      if (grp + 2 < NG) {
        issue_w1(grp + 2);
        issue_w2(grp + 2);
        if (grp == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PW) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PW + 4) : "memory");
      } else {
        if (grp == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      }
      __syncthreads();                                   // group grp + 1's image landed
      twait += TTMI_TNOW() - tw0;
    }
    TTMI_TSTAMP(2 + (grp < 4 ? grp : 3));
  }
  }
  // ---- x2 = x1 + drop2(. + b2); y = LN(x2) (the row's 128 columns in lanes li, li+16, li+32, li+48)
  float vr[32];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int n = 32 * p + 8 * lg;
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = acc2[2 * p][e] + sb2[n + e];
      v[4 + e] = acc2[2 * p + 1][e] + sb2[n + 4 + e];
    }
    drop_apply_vec<8>(dk2, (uint32_t)(m * FB_D + n), v);
    const float4 r0 = rpre[2 * p], r1v = rpre[2 * p + 1];
    v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w;
    v[4] += r1v.x; v[5] += r1v.y; v[6] += r1v.z; v[7] += r1v.w;
    if (!KV && mok) {                                    // (KV: stored after the projection)
      float* cp = g.x2 + m * FB_D + n;
      *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) vr[8 * p + e] = v[e];
  }
  float s1 = 0.f;                                        // two-pass mean / variance (as ln_fwd)
#pragma unroll
  for (int e = 0; e < 32; ++e) s1 += vr[e];
  s1 += __shfl_xor(s1, 16, 64);
  s1 += __shfl_xor(s1, 32, 64);
  const float mu = s1 * (1.f / FB_D);
  float s2 = 0.f;
#pragma unroll
  for (int e = 0; e < 32; ++e) s2 += (vr[e] - mu) * (vr[e] - mu);
  s2 += __shfl_xor(s2, 16, 64);
  s2 += __shfl_xor(s2, 32, 64);
  const float rs = 1.f / sqrtf(s2 * (1.f / FB_D) + g.eps);
  if constexpr (KV) {
    // ---- the next layer's K / V projection of the tile's y rows, with the row panel's fragments
    // and MFMA order (ttmi_gemm's bits): y -> a row image in the last group's buffer, A
    // fragments k = 32 lg + 8 c, W_kv images in the other buffer (column-paired rows)
    uint4 yq[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int n = 32 * p + 8 * lg;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (vr[8 * p + e] - mu) * rs * slw[n + e] + slb[n + e];
      yq[p] = pack8(o);
    }
    // W_kv landed (the 4 youngest: the last group's h stores); every wave is past its last
    // FFN2 read of the buffer the row image overwrites
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    __syncthreads();
    char* const arow = smem + ABUF * FB_BUF + (16 * wave + li) * FB_P;
#pragma unroll
    for (int p = 0; p < 4; ++p) *reinterpret_cast<uint4*>(arow + 2 * (32 * p + 8 * lg)) = yq[p];
    uint4 ak[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) ak[c] = lds16(arow + 64 * lg + 16 * c);
    f32x4_t kacc[2][8];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const char* wb = smem + KVBUF * FB_BUF + hf * FB_IMG + wrow * FB_P + 64 * lg;
#pragma unroll
      for (int t = 0; t < 8; ++t) kacc[hf][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int t = 0; t < 8; ++t)
          Mma<bf16_t>::run(kacc[hf][t], lds16(wb + (32 * (t >> 1) + 4 * (t & 1)) * FB_P + 16 * c), ak[c]);
      }
    }
    const float* sbkv = reinterpret_cast<const float*>(spar + PB + 5 * 1024);
    if (mok) {
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int n = 128 * hf + 32 * p + 8 * lg;
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = kacc[hf][2 * p][e] + sbkv[n + e];
            v[4 + e] = kacc[hf][2 * p + 1][e] + sbkv[n + 4 + e];
          }
          *reinterpret_cast<uint4*>(g.kv + m * g.ldkv + n) = pack8(v);
        }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int n = 32 * p + 8 * lg;
        float* cp = g.x2 + m * FB_D + n;
        *reinterpret_cast<float4*>(cp) = make_float4(vr[8 * p], vr[8 * p + 1], vr[8 * p + 2], vr[8 * p + 3]);
        *reinterpret_cast<float4*>(cp + 4) =
            make_float4(vr[8 * p + 4], vr[8 * p + 5], vr[8 * p + 6], vr[8 * p + 7]);
        *reinterpret_cast<uint4*>(g.y + m * FB_D + n) = yq[p];
      }
      if (lg == 0) {
        g.mean[m] = mu;
        g.rstd[m] = rs;
      }
    }
  } else if (mok) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int n = 32 * p + 8 * lg;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (vr[8 * p + e] - mu) * rs * slw[n + e] + slb[n + e];
      *reinterpret_cast<uint4*>(g.y + m * FB_D + n) = pack8(o);
    }
    if (lg == 0) {
      g.mean[m] = mu;
      g.rstd[m] = rs;
    }
  }
  TTMI_TSTAMP(6);
  TTMI_TSTAMP_VAL(7, twait);
  (void)twait;
}

// ------------------------------------------------------------------------------ D = 256
// The same sub-block at the reference's default width (ABI 22): d_model 256, F = 1024
// (src/train.py:289-297; user_tower.py:37-45).  128 rows a workgroup, F2_RT 16-row tiles a wave
// (F2_NW = 8 / F2_RT waves); the weights stream through LDS in 16 groups of 64 hidden units —
// the group's W1 rows [64][256] and W2 columns [256][64], 70 KB — double-buffered by LDS-DMA
// under the previous group's MFMAs; the row tile (A, [128][256]) is staged in buffer 1 before its
// first W group lands.  Each W fragment read from LDS feeds F2_RT MFMAs (one per row tile).
// Measured at 25,600 rows (tools/ffn_time.py): RT 1 (8 waves) 58.6 us, RT 2 (4 waves, one a SIMD,
// half the LDS reads) 72 us — the lone wave exposes its own latencies — so RT 1 ships; the
// unfused pair takes 64.7 us.  FFN1's output fragment (row li, units
// 32p + 8lg .. +7 of the group) is FFN2's B operand as at D = 128, so h never leaves the wave
// between the GEMMs (it is stored once, for the backward).  The A / W1 fragments read k =
// 128 (c >> 2) + 32 lg + 8 (c & 3) (c < 8) and the W2 image holds its unit chunks permuted, so
// every ds_read_b128's lane groups hit distinct LDS banks.  x2 / y agree with the unfused row
// panels to fp32 rounding, h to bf16 rounding (another k order).
#ifndef F2B_X1SEAM
#define F2B_X1SEAM 1                                 // (backward: x1's row at the last seam; 0: in
#endif                                               // the epilogue, 1.3 us slower)
#ifndef F2_RT
#define F2_RT 1                                      // 16-row tiles a wave
#endif
#ifndef F2_PF
#define F2_PF 2                                      // W fragment stages (k-steps read ahead + 1;
#endif                                               // 2, 3, 4 within 2 %)
constexpr int F2_D = 256, F2_F = 1024, F2_GU = 64, F2_NG = F2_F / F2_GU;
constexpr int F2_PA = 2 * F2_D + 16;                 // A / W1 image pitch (33 chunks)
constexpr int F2_PW2 = 2 * F2_GU + 16;               // W2 image pitch (9 chunks)
constexpr int F2_CA = F2_PA / 16, F2_CW2 = F2_PW2 / 16;
constexpr int F2_W1IMG = F2_GU * F2_PA;              // 33,792 B
constexpr int F2_W2IMG = F2_D * F2_PW2;              // 36,864 B
constexpr int F2_BUF = F2_W1IMG + F2_W2IMG;          // 70,656 B
constexpr int F2_AIMG = 128 * F2_PA;                 // 67,584 B (in buffer 1)
constexpr int F2_IA = 128 * F2_CA / 64;              // 66 DMA wave-instructions
constexpr int F2_IW1 = F2_GU * F2_CA / 64;           // 33
constexpr int F2_IW2 = F2_D * F2_CW2 / 64;           // 36
constexpr int F2_NW = 8 / F2_RT;
constexpr int F2_PAW = (F2_IA + F2_NW - 1) / F2_NW;  // per wave (RT 1: 9, 5, 5)
constexpr int F2_P1W = (F2_IW1 + F2_NW - 1) / F2_NW;
constexpr int F2_P2W = (F2_IW2 + F2_NW - 1) / F2_NW;
constexpr int F2_PAR = 9;                            // 1 KB parameter slots: b1 x4 | b2 | lnw | lnb | 2 seeds
constexpr int F2_PPW = (F2_PAR + F2_NW - 1) / F2_NW;
static_assert(F2_AIMG <= F2_BUF, "the A tile fits buffer 1");
static_assert(F2_IA * 64 == 128 * F2_CA && F2_IW1 * 64 == F2_GU * F2_CA && F2_IW2 * 64 == F2_D * F2_CW2,
              "whole DMA instructions");
static_assert(2 * F2_RT + F2_P1W + F2_P2W <= 63, "vmcnt immediate");

template <bool DF>
__global__ __launch_bounds__(F2_NW * 64) void ffn256_block_kernel(FfnArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[2 * F2_BUF + F2_PAR * 1024];
  char* const spar = smem + 2 * F2_BUF;
  TTMI_TSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int64_t r0 = (int64_t)blockIdx.x * 128;
  int64_t m[F2_RT], mc[F2_RT];                           // row tile rt: rows 16 (RT wave + rt) + li
  bool mok[F2_RT];
#pragma unroll
  for (int rt = 0; rt < F2_RT; ++rt) {
    m[rt] = r0 + 16 * (F2_RT * wave + rt) + li;
    mok[rt] = m[rt] < g.M;
    mc[rt] = mok[rt] ? m[rt] : (int64_t)g.M - 1;
  }
  const uint32_t w1bytes = (uint32_t)F2_F * F2_D * 2, w2bytes = (uint32_t)F2_D * F2_F * 2;
  const uint32_t abytes = (uint32_t)min<int64_t>(128, g.M - r0) * F2_D * 2;
  const i32x4_t r1 = make_rsrc(g.w1, w1bytes), r2 = make_rsrc(g.w2, w2bytes);
  const i32x4_t ra = make_rsrc(g.a + r0 * F2_D, abytes);           // rows past M: zeros
  // slot j of a batch of NI wave-instructions: ii = wave + NW j (re-issued mod NI: every wave
  // issues the same count, so one vmcnt immediate serves all)
  auto slot = [&](int j, int ni) { int ii = wv + F2_NW * j; return ii >= ni ? ii - ni : ii; };
  uint32_t oW1[F2_P1W], oW2[F2_P2W];
#pragma unroll
  for (int j = 0; j < F2_P1W; ++j) {
    const int q = slot(j, F2_IW1) * 64 + lane, n = q / F2_CA, c = q % F2_CA;
    oW1[j] = c == F2_CA - 1 ? w1bytes : (uint32_t)((n * F2_D + 8 * c) * 2);
  }
#pragma unroll
  for (int j = 0; j < F2_P2W; ++j) {
    const int q = slot(j, F2_IW2) * 64 + lane, n = q / F2_CW2, c = q % F2_CW2;
    // slot c holds unit chunk 4 ((c >> 1) & 1) + 2 (c & 1) + (c >> 2) (conflict-free FFN2 reads)
    oW2[j] = c == F2_CW2 - 1 ? w2bytes
                             : (uint32_t)((n * F2_F + 8 * (4 * ((c >> 1) & 1) + 2 * (c & 1) + (c >> 2))) * 2);
  }
  auto issue_w = [&](int grp) {                          // W1 rows / W2 columns [64 grp, +64)
    const uint32_t base = lds_addr(smem + (grp & 1) * F2_BUF);
#pragma unroll
    for (int j = 0; j < F2_P1W; ++j)
      dma16(r1, oW1[j] + (uint32_t)(grp * F2_GU * F2_D * 2), base + slot(j, F2_IW1) * 1024);
#pragma unroll
    for (int j = 0; j < F2_P2W; ++j)
      dma16(r2, oW2[j] + (uint32_t)(grp * F2_GU * 2), base + F2_W1IMG + slot(j, F2_IW2) * 1024);
  };
  {                                                      // parameters
    const uint32_t off = (uint32_t)(lane * 16);
#pragma unroll
    for (int h = 0; h < F2_PPW; ++h) {
      int k = wv + F2_NW * h;
      if (k >= F2_PAR) k -= F2_PAR;
      const uint32_t dst = lds_addr(spar) + (uint32_t)(k * 1024);
      if (k < 4) dma16(make_rsrc(g.b1, F2_F * 4), off + (uint32_t)(k * 1024), dst);
      else if (k == 4) dma16(make_rsrc(g.b2, F2_D * 4), off, dst);
      else if (k == 5) dma16(make_rsrc(g.lnw, F2_D * 4), off, dst);
      else if (k == 6) dma16(make_rsrc(g.lnb, F2_D * 4), off, dst);
      else if (k == 7) dma16(make_rsrc(g.df.seed, g.df.on ? 8 : 0), off, dst);
      else dma16(make_rsrc(g.d2.seed, g.d2.on ? 8 : 0), off, dst);
    }
  }
  {
    const uint32_t base = lds_addr(smem + F2_BUF);
#pragma unroll
    for (int j = 0; j < F2_PAW; ++j) {
      const int ii = slot(j, F2_IA), q = ii * 64 + lane, n = q / F2_CA, c = q % F2_CA;
      dma16(ra, c == F2_CA - 1 ? (uint32_t)(128 * F2_D * 2) : (uint32_t)((n * F2_D + 8 * c) * 2),
            base + ii * 1024);
    }
  }
  issue_w(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  TTMI_TSTAMP(1);
  const float* sb1 = reinterpret_cast<const float*>(spar);
  const float* sb2 = reinterpret_cast<const float*>(spar + 4096);
  const float* slw = reinterpret_cast<const float*>(spar + 5120);
  const float* slb = reinterpret_cast<const float*>(spar + 6144);
  DropKeys dkf, dk2;
  {
    const uint64_t sf = *reinterpret_cast<const uint64_t*>(spar + 7168);
    const uint64_t s2 = *reinterpret_cast<const uint64_t*>(spar + 8192);
    dkf = DropKeys{(uint32_t)sf, (uint32_t)(sf >> 32), g.df.thresh, g.df.scale, DF};
    dk2 = DropKeys{(uint32_t)s2, (uint32_t)(s2 >> 32), g.d2.thresh, g.d2.scale, g.d2.on};
  }
  // k-step c, lane group lg: k = 128 (c >> 2) + 32 lg + 8 (c & 3) (the D = 128 permutation per
  // 128-k half: with the 33-chunk pitch a ds_read_b128's lane groups hit distinct banks)
  auto koff = [&](int c) { return 256 * (c >> 2) + 64 * lg + 16 * (c & 3); };
  uint4 af[F2_RT][8];
#pragma unroll
  for (int rt = 0; rt < F2_RT; ++rt)
#pragma unroll
    for (int c = 0; c < 8; ++c)
      af[rt][c] = lds16(smem + F2_BUF + (16 * (F2_RT * wave + rt) + li) * F2_PA + koff(c));
  __syncthreads();                                       // every wave has its A fragments
  issue_w(1);                                            // over the A tile
  const int wrow = 8 * (li >> 2) + (li & 3);             // column-paired rows (the panel layout)
  const __amdgpu_buffer_rsrc_t rh =
      __builtin_amdgcn_make_buffer_rsrc(g.h, 0, (int)((int64_t)g.M * F2_F * 2), 0x00020000);
  f32x4_t acc2[F2_RT][16];
#pragma unroll
  for (int rt = 0; rt < F2_RT; ++rt)
#pragma unroll
    for (int t = 0; t < 16; ++t) acc2[rt][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float4 rpre[F2_RT][16];
  // One group.  The W fragments are read F2_PF - 1 k-steps ahead of their MFMAs into explicit
  // register stages (a read, then its MFMA, back to back, exposes the LDS latency on every MFMA).
  auto group = [&](int grp, bool last) {
    const char* bufp = smem + (grp & 1) * F2_BUF;
    if (last) {                                          // x1's rows for the epilogue (behind this
#pragma unroll                                           // group's MFMAs)
      for (int rt = 0; rt < F2_RT; ++rt) {
        const float* rp = g.res + mc[rt] * F2_D + 8 * lg;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          rpre[rt][2 * q] = *reinterpret_cast<const float4*>(rp + 32 * q);
          rpre[rt][2 * q + 1] = *reinterpret_cast<const float4*>(rp + 32 * q + 4);
        }
      }
    }
    const char* w1b = bufp + wrow * F2_PA;
    const char* w2b = bufp + F2_W1IMG + wrow * F2_PW2 + 16 * (4 * (lg & 1) + (lg >> 1));
    auto ld1 = [&](int c, uint4 (&f)[4]) {
#pragma unroll
      for (int t = 0; t < 4; ++t) f[t] = lds16(w1b + (32 * (t >> 1) + 4 * (t & 1)) * F2_PA + koff(c));
    };
    auto ld2 = [&](int j, uint4 (&f)[4]) {              // FFN2 chunk j: k-step p = j >> 2, tiles 4 (j & 3) + u
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = 4 * (j & 3) + u;
        f[u] = lds16(w2b + (32 * (t >> 1) + 4 * (t & 1)) * F2_PW2 + 32 * (j >> 2));
      }
    };
    // ---- FFN1: the tiles' rows x the group's 64 hidden units
    f32x4_t acc1[F2_RT][4];
#pragma unroll
    for (int rt = 0; rt < F2_RT; ++rt)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc1[rt][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    uint4 wf[F2_PF][4];
#pragma unroll
    for (int c = 0; c < F2_PF - 1; ++c) ld1(c, wf[c]);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int c2 = c + F2_PF - 1;
      if (c2 < 8) ld1(c2, wf[c2 % F2_PF]);
      else ld2(c2 - 8, wf[c2 % F2_PF]);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int rt = 0; rt < F2_RT; ++rt) Mma<bf16_t>::run(acc1[rt][t], wf[c % F2_PF][t], af[rt][c]);
    }
    // ---- h = drop_f(relu(. + b1)), bf16: FFN2's operand and the stored activation
    uint4 hq[F2_RT][2];
#pragma unroll
    for (int rt = 0; rt < F2_RT; ++rt)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int n = F2_GU * grp + 32 * p + 8 * lg;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = fmaxf(acc1[rt][2 * p][e] + sb1[n + e], 0.f);
          v[4 + e] = fmaxf(acc1[rt][2 * p + 1][e] + sb1[n + 4 + e], 0.f);
        }
        if (DF) drop_apply_vec<8>(dkf, (uint32_t)(m[rt] * F2_F + n), v);
        hq[rt][p] = pack8(v);
        const i32x4_t q = {(int)hq[rt][p].x, (int)hq[rt][p].y, (int)hq[rt][p].z, (int)hq[rt][p].w};
        __builtin_amdgcn_raw_buffer_store_b128(q, rh, (uint32_t)((m[rt] * F2_F + n) * 2), 0, 0);
      }
    // ---- FFN2's k-steps over the group's units, 8 chunks of 4 fragments
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int j2 = j + F2_PF - 1;
      if (j2 < 8) ld2(j2, wf[(j2 + 8) % F2_PF]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int rt = 0; rt < F2_RT; ++rt)
          Mma<bf16_t>::run(acc2[rt][4 * (j & 3) + u], wf[(j + 8) % F2_PF][u], hq[rt][j >> 2]);
    }
    if (!last) {
      __syncthreads();                                   // every wave is done with this buffer
      // group grp + 1 landed; younger: this group's 2 RT h stores and group grp + 2's DMAs
      if (grp + 2 < F2_NG) {
        issue_w(grp + 2);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * F2_RT + F2_P1W + F2_P2W) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * F2_RT) : "memory");
      }
      __syncthreads();                                   // group grp + 1's images landed
    }
  };
#pragma unroll 1
  for (int grp = 0; grp < F2_NG - 1; ++grp) group(grp, false);
  group(F2_NG - 1, true);
  TTMI_TSTAMP(2);
  // ---- x2 = x1 + drop2(. + b2); y = LN(x2) (a row's 256 columns in lanes li, li+16, li+32, li+48)
#pragma unroll
  for (int rt = 0; rt < F2_RT; ++rt) {
    float vr[64];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int n = 32 * q + 8 * lg;
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc2[rt][2 * q][e] + sb2[n + e];
        v[4 + e] = acc2[rt][2 * q + 1][e] + sb2[n + 4 + e];
      }
      drop_apply_vec<8>(dk2, (uint32_t)(m[rt] * F2_D + n), v);
      const float4 a0 = rpre[rt][2 * q], a1 = rpre[rt][2 * q + 1];
      v[0] += a0.x; v[1] += a0.y; v[2] += a0.z; v[3] += a0.w;
      v[4] += a1.x; v[5] += a1.y; v[6] += a1.z; v[7] += a1.w;
      if (mok[rt]) {
        float* cp = g.x2 + m[rt] * F2_D + n;
        *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) vr[8 * q + e] = v[e];
    }
    float s1 = 0.f;                                      // two-pass mean / variance (as ln_fwd)
#pragma unroll
    for (int e = 0; e < 64; ++e) s1 += vr[e];
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    const float mu = s1 * (1.f / F2_D);
    float s2 = 0.f;
#pragma unroll
    for (int e = 0; e < 64; ++e) s2 += (vr[e] - mu) * (vr[e] - mu);
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    const float rs = 1.f / sqrtf(s2 * (1.f / F2_D) + g.eps);
    if (mok[rt]) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int n = 32 * q + 8 * lg;
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (vr[8 * q + e] - mu) * rs * slw[n + e] + slb[n + e];
        *reinterpret_cast<uint4*>(g.y + m[rt] * F2_D + n) = pack8(o);
      }
      if (lg == 0) {
        g.mean[m[rt]] = mu;
        g.rstd[m[rt]] = rs;
      }
    }
  }
  TTMI_TSTAMP(3);
}

// ------------------------------------------------------------------------------ backward
// The sub-block's input-grad half (ABI 21, ttmi_ffn_block_bwd): the same two back-to-back GEMMs
// on the transposed weight mirrors — W2ᵀ [F, D] has the forward W1's layout, W1ᵀ [D, F] the
// forward W2's — with the row panels' epilogues:
//   dz1 = (dy2·W2) ⊙ [h > 0]·sf                  bf16 [M, F] (stored: dW1's operand; the gated
//                                                 row panel's bits)
//   dY  = dz1·W1 (never stored), then norm2's backward (ttmi_linear_ln_bwd's epilogue):
//   dx1 = rstd·(dY·w − mean(dY·w) − x̂·mean(dY·w·x̂)) + res,  dy1 = bf16(drop1ᵀ(dx1)),
//   Σ_rows dY·x̂ and Σ_rows dY per workgroup -> sum_ws[blk][2][D] (folded in workgroup order).
// dY sums its k-steps in hidden-unit order: dx1 / dy1 / the sums agree with the row panels to
// fp32 rounding.  The gate rows are compiler-counted loads: each is issued right after one seam
// (behind the next images' DMAs) and read after the next seam, whose wait the compiler sees
// (a builtin s_waitcnt: vmcnt(4), the group's dz1 buffer stores left in flight).
struct FfnBwdArgs {
  const bf16_t* dy; const bf16_t* w2t; const bf16_t* w1t; const bf16_t* h; float sf;
  bf16_t* dz1;
  const float* x1; const float* m2; const float* r2; const float* lnw; const float* res;
  float* dx1; bf16_t* dy1; DropParams d1; float* sum_ws;
  int M;
};

template <int NG>
__global__ __launch_bounds__(512) void ffn_block_bwd_kernel(FfnBwdArgs g) {
  constexpr int NWV = 8, F = NG * 128;
  constexpr int PW = (FB_INS + NWV - 1) / NWV;
  __shared__ __attribute__((aligned(16))) char smem[2 * FB_BUF + 2 * 1024];   // + LN weight | seed
  __shared__ float sdw[NWV][FB_D], sdb[NWV][FB_D];
  char* const spar = smem + 2 * FB_BUF;
  TTMI_TSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int64_t r0 = (int64_t)blockIdx.x * (16 * NWV);
  const int64_t m = r0 + 16 * wave + li;
  const bool mok = m < g.M;
  const int64_t mc = mok ? m : (int64_t)g.M - 1;
  const uint32_t wbytes = (uint32_t)F * FB_D * 2;
  const uint32_t abytes = (uint32_t)min<int64_t>(16 * NWV, g.M - r0) * FB_D * 2;
  const i32x4_t r1 = make_rsrc(g.w2t, wbytes), r2 = make_rsrc(g.w1t, wbytes);
  const i32x4_t ra = make_rsrc(g.dy + r0 * FB_D, abytes);
  uint32_t oA[PW], oW1[PW], oW2[PW];
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    int ii = wv + NWV * j;
    if (ii >= FB_INS) ii -= FB_INS;
    const int q = ii * 64 + lane, n = q / FB_CPR, c = q % FB_CPR;
    const bool pad = c == FB_CPR - 1;
    oA[j] = pad ? (uint32_t)(16 * NWV * FB_D * 2) : (uint32_t)((n * FB_D + 8 * c) * 2);
    oW1[j] = pad ? wbytes : (uint32_t)((n * FB_D + 8 * c) * 2);
    // (slot c holds unit chunk 4 (c & 3) + (c >> 2): FFN2's lane group lg reads its four k-step
    // chunks 4p + lg side by side, so a ds_read_b128's lane groups hit distinct banks)
    oW2[j] = pad ? wbytes : (uint32_t)((n * F + 8 * (4 * (c & 3) + (c >> 2))) * 2);
  }
  auto slot = [&](int j) { int ii = wv + NWV * j; return ii >= FB_INS ? ii - FB_INS : ii; };
  auto issue_group = [&](int grp) {      // W2ᵀ rows [128 grp, +128), W1ᵀ columns [128 grp, +128)
    const uint32_t b1 = lds_addr(smem + (grp & 1) * FB_BUF), b2 = b1 + FB_IMG;
#pragma unroll
    for (int j = 0; j < PW; ++j) dma16(r1, oW1[j] + (uint32_t)(grp * 128 * FB_D * 2), b1 + slot(j) * 1024);
#pragma unroll
    for (int j = 0; j < PW; ++j) dma16(r2, oW2[j] + (uint32_t)(grp * 128 * 2), b2 + slot(j) * 1024);
  };
  auto load_gate = [&](int grp, uint4 (&q)[4]) {          // h[m, 128 grp + 32p + 8lg ..]
    const uint4* hp = reinterpret_cast<const uint4*>(g.h + mc * F + 128 * grp + 8 * lg);
#pragma unroll
    for (int p = 0; p < 4; ++p) q[p] = hp[4 * p];
  };
  uint4 hg[4], hn[4];
  load_gate(0, hg);                                      // (from HBM: issued ahead of the DMAs)
  {
    const uint32_t dst = lds_addr(spar) + (uint32_t)(wv * 1024), off = (uint32_t)(lane * 16);
    if (wv == 0) dma16(make_rsrc(g.lnw, FB_D * 4), off, dst);
    else if (wv == 1) dma16(make_rsrc(g.d1.seed, g.d1.on ? 8 : 0), off, dst);
  }
  {                                                      // the dy2 tile -> buffer 1's W2ᵀ image
    const uint32_t base = lds_addr(smem + FB_BUF + FB_IMG);
#pragma unroll
    for (int j = 0; j < PW; ++j) dma16(ra, oA[j], base + slot(j) * 1024);
  }
  issue_group(0);
  for (int i = tid; i < NWV * FB_D; i += 64 * NWV) { (&sdw[0][0])[i] = 0.f; (&sdb[0][0])[i] = 0.f; }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  uint4 af[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) af[c] = lds16(smem + FB_BUF + FB_IMG + (16 * wave + li) * FB_P + 64 * lg + 16 * c);
  const float* slw = reinterpret_cast<const float*>(spar);
  DropKeys dk1;
  {
    const uint64_t s1 = *reinterpret_cast<const uint64_t*>(spar + 1024);
    dk1 = DropKeys{(uint32_t)s1, (uint32_t)(s1 >> 32), g.d1.thresh, g.d1.scale, g.d1.on};
  }
  __syncthreads();                                       // every wave has its dy2 fragments
  TTMI_TSTAMP(1);
  float4 rx[8], rr[8];
  float mu = 0.f, rs = 0.f;
  // the LayerNorm backward's row operands: x1 (+ its statistics) and the residual grad, issued at
  // two different seams so no one seam queues 1 KB of loads a row behind its DMAs
  auto load_x1 = [&](int h) {                            // column quarters 2h, 2h + 1
    const float* xp = g.x1 + mc * FB_D + 8 * lg;
#pragma unroll
    for (int p = 2 * h; p < 2 * h + 2; ++p) {
      rx[2 * p] = *reinterpret_cast<const float4*>(xp + 32 * p);
      rx[2 * p + 1] = *reinterpret_cast<const float4*>(xp + 32 * p + 4);
    }
    if (h == 0) {
      mu = g.m2[mc];
      rs = g.r2[mc];
    }
  };
  auto load_res = [&](int h) {
    const float* rp = g.res + mc * FB_D + 8 * lg;
#pragma unroll
    for (int p = 2 * h; p < 2 * h + 2; ++p) {
      rr[2 * p] = *reinterpret_cast<const float4*>(rp + 32 * p);
      rr[2 * p + 1] = *reinterpret_cast<const float4*>(rp + 32 * p + 4);
    }
  };
  if (NG > 1) {
    issue_group(1);
    load_gate(1, hn);
  }
  if (NG == 1) { load_x1(0); load_x1(1); load_res(0); load_res(1); }
  const int wrow = 8 * (li >> 2) + (li & 3);
  // dz1 stores through a buffer resource (rows past M dropped by its range): exactly 4 a group
  const __amdgpu_buffer_rsrc_t rdz =
      __builtin_amdgcn_make_buffer_rsrc(g.dz1, 0, (int)((int64_t)g.M * F * 2), 0x00020000);
  f32x4_t acc2[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc2[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int grp = 0; grp < NG; ++grp) {
    const char* w1b = smem + (grp & 1) * FB_BUF + wrow * FB_P + 64 * lg;
    const char* w2b = smem + (grp & 1) * FB_BUF + FB_IMG + wrow * FB_P + 64 * lg;
    f32x4_t acc1[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc1[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
      for (int t = 0; t < 8; ++t)
        Mma<bf16_t>::run(acc1[t], lds16(w1b + (32 * (t >> 1) + 4 * (t & 1)) * FB_P + 16 * c), af[c]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- dz1 = gate(acc): the row panel's PE_GATE_BF16 epilogue (+ 0 as its absent bias)
    uint4 hq[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int n = 128 * grp + 32 * p + 8 * lg;
      const uint32_t qw[4] = {hg[p].x, hg[p].y, hg[p].z, hg[p].w};
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = 1.f * (e < 2 ? acc1[2 * p][2 * e] : acc1[2 * p + 1][2 * e - 4]) + 0.f;
        v[2 * e + 1] = 1.f * (e < 2 ? acc1[2 * p][2 * e + 1] : acc1[2 * p + 1][2 * e - 3]) + 0.f;
        v[2 * e] = __uint_as_float(qw[e] << 16) > 0.f ? v[2 * e] * g.sf : 0.f;
        v[2 * e + 1] = __uint_as_float(qw[e] & 0xFFFF0000u) > 0.f ? v[2 * e + 1] * g.sf : 0.f;
      }
      hq[p] = pack8(v);
      const i32x4_t q = {(int)hq[p].x, (int)hq[p].y, (int)hq[p].z, (int)hq[p].w};
      __builtin_amdgcn_raw_buffer_store_b128(q, rdz, (uint32_t)((m * F + n) * 2), 0, 0);
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
#pragma unroll
      for (int t = 0; t < 8; ++t)
        Mma<bf16_t>::run(acc2[t], lds16(w2b + (32 * (t >> 1) + 4 * (t & 1)) * FB_P + 16 * p), hq[p]);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (grp + 1 < NG) {
      __syncthreads();                                   // every wave is done with this buffer
      // group grp + 1's images and gate rows; younger: this group's 4 dz1 stores (vmcnt 4,
      // expcnt / lgkmcnt not waited), which stay in flight across the seam
      __builtin_amdgcn_s_waitcnt(0x0F74);
#pragma unroll
      for (int p = 0; p < 4; ++p) hg[p] = hn[p];
      if (grp + 2 < NG) {
        issue_group(grp + 2);
        load_gate(grp + 2, hn);
      }
      // 256 B a row at each of the last three seams (at NG = 2 all at the one seam)
      if (grp == (NG > 3 ? NG - 4 : 0)) load_x1(0);
      if (grp == (NG > 2 ? NG - 3 : 0)) { load_x1(1); load_res(0); }
      if (grp == NG - 2) load_res(1);
      __syncthreads();                                   // every wave's part of the images landed
    }
    TTMI_TSTAMP(2 + (grp < 4 ? grp : 3));
  }
  // ---- norm2's backward of the finished rows (ttmi_linear_ln_bwd's PE_LNBWD epilogue)
  float dy[32], xh[32];
  float s1 = 0.f, s2 = 0.f;
  if (!mok) { mu = 0.f; rs = 0.f; }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int n = 32 * p + 8 * lg;
    const float4 x0 = rx[2 * p], x1v = rx[2 * p + 1];
    const float xr[8] = {x0.x, x0.y, x0.z, x0.w, x1v.x, x1v.y, x1v.z, x1v.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = mok ? (e < 4 ? acc2[2 * p][e] : acc2[2 * p + 1][e - 4]) : 0.f;
      const float hx = ((mok ? xr[e] : 0.f) - mu) * rs;
      const float gg = d * slw[n + e];
      dy[8 * p + e] = d;
      xh[8 * p + e] = hx;
      s1 += gg;
      s2 += gg * hx;
    }
  }
  s1 += __shfl_xor(s1, 16, 64);
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 16, 64);
  s2 += __shfl_xor(s2, 32, 64);
  const float c1 = s1 * (1.f / FB_D), c2 = s2 * (1.f / FB_D);
  if (mok) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int n = 32 * p + 8 * lg;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = rs * (dy[8 * p + e] * slw[n + e] - c1 - xh[8 * p + e] * c2);
      const float4 q0 = rr[2 * p], q1 = rr[2 * p + 1];
      o[0] += q0.x; o[1] += q0.y; o[2] += q0.z; o[3] += q0.w;
      o[4] += q1.x; o[5] += q1.y; o[6] += q1.z; o[7] += q1.w;
      float* dp = g.dx1 + m * FB_D + n;
      *reinterpret_cast<float4*>(dp) = make_float4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<float4*>(dp + 4) = make_float4(o[4], o[5], o[6], o[7]);
      drop_apply_vec<8>(dk1, (uint32_t)(m * FB_D + n), o);
      *reinterpret_cast<uint4*>(g.dy1 + m * FB_D + n) = pack8(o);
    }
  }
  TTMI_TSTAMP(7);
  // LayerNorm weight / bias grads: the tile's 16 rows summed per column in row order through a
  // wave-private LDS slice (16 rows x 132 floats) of the W buffer no wave reads any more (the
  // last group used the other one): 8 ds_write_b128 + 8 ds_read_b128 a lane per quantity, where
  // DPP row sums cost 4 dependent steps per column value.  Lanes 0-31 sum rows 0-7 and lanes
  // 32-63 rows 8-15 of column group lane & 31; the halves meet in that order.
  {
    constexpr int RS = 132;                              // row stride (floats): 16 B bank shift
    float* red = reinterpret_cast<float*>(smem + (NG & 1) * FB_BUF) + wave * 16 * RS;
    const int cg = lane & 31, rh = lane >> 5;
#pragma unroll
    for (int qd = 0; qd < 2; ++qd) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int b = 8 * p + 4 * hf;
          const float4 v = qd == 0 ? make_float4(dy[b] * xh[b], dy[b + 1] * xh[b + 1], dy[b + 2] * xh[b + 2],
                                                 dy[b + 3] * xh[b + 3])
                                   : make_float4(dy[b], dy[b + 1], dy[b + 2], dy[b + 3]);
          *reinterpret_cast<float4*>(red + li * RS + 32 * p + 8 * lg + 4 * hf) = v;
        }
      }
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const float4 w = *reinterpret_cast<const float4*>(red + (8 * rh + r) * RS + 4 * cg);
        acc.x += w.x; acc.y += w.y; acc.z += w.z; acc.w += w.w;
      }
      float4 hi;
      hi.x = __shfl_down(acc.x, 32, 64); hi.y = __shfl_down(acc.y, 32, 64);
      hi.z = __shfl_down(acc.z, 32, 64); hi.w = __shfl_down(acc.w, 32, 64);
      if (rh == 0) {
        acc.x += hi.x; acc.y += hi.y; acc.z += hi.z; acc.w += hi.w;
        *reinterpret_cast<float4*>((qd == 0 ? &sdw[wave][0] : &sdb[wave][0]) + 4 * cg) = acc;
      }
    }
  }
  __syncthreads();
  if (tid < FB_D) {                                      // the waves' rows in wave order
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) { a += sdw[w][tid]; b += sdb[w][tid]; }
    float* o = g.sum_ws + (int64_t)blockIdx.x * 2 * FB_D;
    o[tid] = a;
    o[FB_D + tid] = b;
  }
  TTMI_TSTAMP(6);
}

// ---------------------------------------------------------------- backward at D = 256
// ffn_block_bwd_kernel's math at d_model 256, F = 1,024 (round 6), on ffn256_block_kernel's
// geometry: W2ᵀ rows [64][256] and W1ᵀ columns [256][64] of a 64-unit group stream through the
// forward's two 70 KB LDS buffers (same images, same conflict-free fragment orders), one 16-row
// tile per wave, 8 waves, 128 rows a workgroup; the dy2 tile is staged in buffer 1.  x1's row is
// loaded at the last seam, the residual grad's in the epilogue; norm2's weight / bias row sums go
// through wave-private LDS slices of both (then free) buffers.  Measured at 25,600 rows
// (tools/ffn_time.py): 76.1-76.6 us with its fold against 74.2-75.3 for the gated row panel +
// ttmi_linear_ln_bwd pair — the h read and dz1 write (52 MB each) dominate either way and the
// fused loop does not hide them — so the framework keeps the pair at D = 256 (functional.py);
// the entry point serves the shape and is parity-tested.
template <bool DROP1>
__global__ __launch_bounds__(512) void ffn256_block_bwd_kernel(FfnBwdArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[2 * F2_BUF + 2 * 1024];   // + LN weight | seed
  __shared__ float sdw[8][F2_D], sdb[8][F2_D];
  char* const spar = smem + 2 * F2_BUF;
  TTMI_TSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int64_t r0 = (int64_t)blockIdx.x * 128;
  const int64_t m = r0 + 16 * wave + li;
  const bool mok = m < g.M;
  const int64_t mc = mok ? m : (int64_t)g.M - 1;
  const uint32_t wbytes = (uint32_t)F2_F * F2_D * 2;     // W2ᵀ and W1ᵀ alike
  const uint32_t abytes = (uint32_t)min<int64_t>(128, g.M - r0) * F2_D * 2;
  const i32x4_t r1 = make_rsrc(g.w2t, wbytes), r2 = make_rsrc(g.w1t, wbytes);
  const i32x4_t ra = make_rsrc(g.dy + r0 * F2_D, abytes);
  auto slot = [&](int j, int ni) { int ii = wv + 8 * j; return ii >= ni ? ii - ni : ii; };
  uint32_t oW1[F2_P1W], oW2[F2_P2W];
#pragma unroll
  for (int j = 0; j < F2_P1W; ++j) {
    const int q = slot(j, F2_IW1) * 64 + lane, n = q / F2_CA, c = q % F2_CA;
    oW1[j] = c == F2_CA - 1 ? wbytes : (uint32_t)((n * F2_D + 8 * c) * 2);
  }
#pragma unroll
  for (int j = 0; j < F2_P2W; ++j) {
    const int q = slot(j, F2_IW2) * 64 + lane, n = q / F2_CW2, c = q % F2_CW2;
    oW2[j] = c == F2_CW2 - 1 ? wbytes
                             : (uint32_t)((n * F2_F + 8 * (4 * ((c >> 1) & 1) + 2 * (c & 1) + (c >> 2))) * 2);
  }
  auto issue_group = [&](int grp) {                      // W2ᵀ rows / W1ᵀ columns [64 grp, +64)
    const uint32_t base = lds_addr(smem + (grp & 1) * F2_BUF);
#pragma unroll
    for (int j = 0; j < F2_P1W; ++j)
      dma16(r1, oW1[j] + (uint32_t)(grp * F2_GU * F2_D * 2), base + slot(j, F2_IW1) * 1024);
#pragma unroll
    for (int j = 0; j < F2_P2W; ++j)
      dma16(r2, oW2[j] + (uint32_t)(grp * F2_GU * 2), base + F2_W1IMG + slot(j, F2_IW2) * 1024);
  };
  auto load_gate = [&](int grp, uint4 (&q)[2]) {         // h[m, 64 grp + 32p + 8lg ..]
    const uint4* hp = reinterpret_cast<const uint4*>(g.h + mc * F2_F + F2_GU * grp + 8 * lg);
#pragma unroll
    for (int p = 0; p < 2; ++p) q[p] = hp[4 * p];
  };
  uint4 hg[2], hn[2];
  load_gate(0, hg);                                      // (from HBM: issued ahead of the DMAs)
  {
    const uint32_t dst = lds_addr(spar) + (uint32_t)(wv * 1024), off = (uint32_t)(lane * 16);
    if (wv == 0) dma16(make_rsrc(g.lnw, F2_D * 4), off, dst);
    else if (wv == 1) dma16(make_rsrc(g.d1.seed, g.d1.on ? 8 : 0), off, dst);
  }
  {                                                      // the dy2 tile -> buffer 1
    const uint32_t base = lds_addr(smem + F2_BUF);
#pragma unroll
    for (int j = 0; j < F2_PAW; ++j) {
      const int ii = slot(j, F2_IA), q = ii * 64 + lane, n = q / F2_CA, c = q % F2_CA;
      dma16(ra, c == F2_CA - 1 ? (uint32_t)(128 * F2_D * 2) : (uint32_t)((n * F2_D + 8 * c) * 2),
            base + ii * 1024);
    }
  }
  issue_group(0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  auto koff = [&](int c) { return 256 * (c >> 2) + 64 * lg + 16 * (c & 3); };
  uint4 af[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) af[c] = lds16(smem + F2_BUF + (16 * wave + li) * F2_PA + koff(c));
  const float* slw = reinterpret_cast<const float*>(spar);
  DropKeys dk1;
  {
    const uint64_t s1 = *reinterpret_cast<const uint64_t*>(spar + 1024);
    dk1 = DropKeys{(uint32_t)s1, (uint32_t)(s1 >> 32), g.d1.thresh, g.d1.scale, DROP1};
  }
  __syncthreads();                                       // every wave has its dy2 fragments
  issue_group(1);                                        // over the dy2 tile
  load_gate(1, hn);
  TTMI_TSTAMP(1);
  const int wrow = 8 * (li >> 2) + (li & 3);
  const __amdgpu_buffer_rsrc_t rdz =
      __builtin_amdgcn_make_buffer_rsrc(g.dz1, 0, (int)((int64_t)g.M * F2_F * 2), 0x00020000);
  f32x4_t acc2[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) acc2[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  f32x4_t xh[16];                                        // x1's row, then x̂ (epilogue)
  auto group = [&](int grp, bool last) {
    const char* bufp = smem + (grp & 1) * F2_BUF;
    const char* w1b = bufp + wrow * F2_PA;
    const char* w2b = bufp + F2_W1IMG + wrow * F2_PW2 + 16 * (4 * (lg & 1) + (lg >> 1));
    auto ld1 = [&](int c, uint4 (&f)[4]) {
#pragma unroll
      for (int t = 0; t < 4; ++t) f[t] = lds16(w1b + (32 * (t >> 1) + 4 * (t & 1)) * F2_PA + koff(c));
    };
    auto ld2 = [&](int j, uint4 (&f)[4]) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = 4 * (j & 3) + u;
        f[u] = lds16(w2b + (32 * (t >> 1) + 4 * (t & 1)) * F2_PW2 + 32 * (j >> 2));
      }
    };
    // ---- dy2 · W2 over the group's 64 hidden units
    f32x4_t acc1[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc1[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // (fragments read straight into their MFMAs: the forward's register stages, with the gate
    // rows in flight beside them, spilled here)
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      uint4 wf[4];
      ld1(c, wf);
#pragma unroll
      for (int t = 0; t < 4; ++t) Mma<bf16_t>::run(acc1[t], wf[t], af[c]);
    }
    // ---- dz1 = gate(acc): the row panel's PE_GATE_BF16 epilogue
    uint4 hq[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int n = F2_GU * grp + 32 * p + 8 * lg;
      const uint32_t qw[4] = {hg[p].x, hg[p].y, hg[p].z, hg[p].w};
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = 1.f * (e < 2 ? acc1[2 * p][2 * e] : acc1[2 * p + 1][2 * e - 4]) + 0.f;
        v[2 * e + 1] = 1.f * (e < 2 ? acc1[2 * p][2 * e + 1] : acc1[2 * p + 1][2 * e - 3]) + 0.f;
        v[2 * e] = __uint_as_float(qw[e] << 16) > 0.f ? v[2 * e] * g.sf : 0.f;
        v[2 * e + 1] = __uint_as_float(qw[e] & 0xFFFF0000u) > 0.f ? v[2 * e + 1] * g.sf : 0.f;
      }
      hq[p] = pack8(v);
      const i32x4_t q = {(int)hq[p].x, (int)hq[p].y, (int)hq[p].z, (int)hq[p].w};
      __builtin_amdgcn_raw_buffer_store_b128(q, rdz, (uint32_t)((m * F2_F + n) * 2), 0, 0);
    }
    // ---- dY += dz1 · W1 over the group's units
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint4 wf[4];
      ld2(j, wf);
#pragma unroll
      for (int u = 0; u < 4; ++u) Mma<bf16_t>::run(acc2[4 * (j & 3) + u], wf[u], hq[j >> 2]);
    }
    if (!last) {
      __syncthreads();                                   // every wave is done with this buffer
      // group grp + 1's images and gate rows; younger: this group's 2 dz1 stores
      __builtin_amdgcn_s_waitcnt(0x0F72);                // vmcnt(2), expcnt / lgkmcnt not waited
#pragma unroll
      for (int p = 0; p < 2; ++p) hg[p] = hn[p];
      if (grp + 2 < F2_NG) {
        issue_group(grp + 2);
        load_gate(grp + 2, hn);
      }
      if (F2B_X1SEAM && grp + 2 == F2_NG) {              // x1's row, behind the last group's MFMAs
        const float* xp = g.x1 + mc * F2_D + 8 * lg;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float4 a0 = *reinterpret_cast<const float4*>(xp + 32 * q);
          const float4 a1 = *reinterpret_cast<const float4*>(xp + 32 * q + 4);
          xh[2 * q] = f32x4_t{a0.x, a0.y, a0.z, a0.w};
          xh[2 * q + 1] = f32x4_t{a1.x, a1.y, a1.z, a1.w};
        }
      }
      __syncthreads();                                   // every wave's part of the images landed
    }
  };
#pragma unroll 1
  for (int grp = 0; grp < F2_NG; ++grp) group(grp, grp + 1 == F2_NG);   // (a peeled last group,
                                                                         // scheduled apart, spilled)
  TTMI_TSTAMP(2);
  // ---- norm2's backward of the finished rows (ttmi_linear_ln_bwd's PE_LNBWD epilogue).  x1's
  // and the residual grad's rows are loaded here, not at the last seam: the last group's
  // fragments, accumulators and stages leave no registers for them.  In place, to stay in
  // registers: dY is acc2 (exactly 0 on rows past M: their dy2 rows arrive as zeros), x1's row
  // becomes x̂ (0 on rows past M: mean and rstd 0 there).
  __builtin_amdgcn_sched_barrier(0);
  if (!F2B_X1SEAM) {
    const float* xp = g.x1 + mc * F2_D + 8 * lg;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 a0 = *reinterpret_cast<const float4*>(xp + 32 * q);
      const float4 a1 = *reinterpret_cast<const float4*>(xp + 32 * q + 4);
      xh[2 * q] = f32x4_t{a0.x, a0.y, a0.z, a0.w};
      xh[2 * q + 1] = f32x4_t{a1.x, a1.y, a1.z, a1.w};
    }
  }
  const float mu = mok ? g.m2[mc] : 0.f, rs = mok ? g.r2[mc] : 0.f;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const int n = 32 * (t >> 1) + 8 * lg + 4 * (t & 1);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      xh[t][e] = (xh[t][e] - mu) * rs;
      const float gg = acc2[t][e] * slw[n + e];
      s1 += gg;
      s2 += gg * xh[t][e];
    }
  }
  s1 += __shfl_xor(s1, 16, 64);
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 16, 64);
  s2 += __shfl_xor(s2, 32, 64);
  const float c1 = s1 * (1.f / F2_D), c2 = s2 * (1.f / F2_D);
  __builtin_amdgcn_sched_barrier(0);
  if (mok) {
    const float* rp = g.res + m * F2_D + 8 * lg;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int n = 32 * q + 8 * lg;
      const float4 q0 = *reinterpret_cast<const float4*>(rp + 32 * q);
      const float4 q1 = *reinterpret_cast<const float4*>(rp + 32 * q + 4);
      float o[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = rs * (acc2[2 * q][e] * slw[n + e] - c1 - xh[2 * q][e] * c2);
        o[4 + e] = rs * (acc2[2 * q + 1][e] * slw[n + 4 + e] - c1 - xh[2 * q + 1][e] * c2);
      }
      o[0] += q0.x; o[1] += q0.y; o[2] += q0.z; o[3] += q0.w;
      o[4] += q1.x; o[5] += q1.y; o[6] += q1.z; o[7] += q1.w;
      float* dp = g.dx1 + m * F2_D + n;
      *reinterpret_cast<float4*>(dp) = make_float4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<float4*>(dp + 4) = make_float4(o[4], o[5], o[6], o[7]);
      if (DROP1) drop_apply_vec<8>(dk1, (uint32_t)(m * F2_D + n), o);
      *reinterpret_cast<uint4*>(g.dy1 + m * F2_D + n) = pack8(o);
    }
  }
  TTMI_TSTAMP(3);
  // LayerNorm weight / bias grads: the tile's 16 rows summed per column in row order through a
  // wave-private LDS slice (16 rows x 260 floats) of the two W buffers, free once every wave is
  // past its last group
  __syncthreads();
  {
    constexpr int RS = F2_D + 4;
    float* red = reinterpret_cast<float*>(smem) + wave * 16 * RS;
    static_assert(8 * 16 * RS * 4 <= 2 * F2_BUF, "the slices fit the W buffers");
#pragma unroll
    for (int qd = 0; qd < 2; ++qd) {
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = acc2[2 * q + hf][e];
            v[e] = qd == 0 ? d * xh[2 * q + hf][e] : d;
          }
          *reinterpret_cast<float4*>(red + li * RS + 32 * q + 8 * lg + 4 * hf) = make_float4(v[0], v[1], v[2], v[3]);
        }
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);      // column group lane: columns 4 lane .. +3
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float4 w = *reinterpret_cast<const float4*>(red + r * RS + 4 * lane);
        acc.x += w.x; acc.y += w.y; acc.z += w.z; acc.w += w.w;
      }
      *reinterpret_cast<float4*>((qd == 0 ? &sdw[wave][0] : &sdb[wave][0]) + 4 * lane) = acc;
    }
  }
  __syncthreads();
  if (tid < F2_D) {                                      // the waves' rows in wave order
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) { a += sdw[w][tid]; b += sdb[w][tid]; }
    float* o = g.sum_ws + (int64_t)blockIdx.x * 2 * F2_D;
    o[tid] = a;
    o[F2_D + tid] = b;
  }
  TTMI_TSTAMP(4);
}

template <int NG, bool KV>
void launch_ffn_kv(const FfnArgs& a, hipStream_t s) {
  const dim3 grid((unsigned)((a.M + 127) / 128));       // 8 waves, one 16-row tile each
  static const bool pipe = !getenv("TTMI_FFN_NOPIPE");  // (A/B: the unpipelined group loop)
  if (pipe && a.df.on) hipLaunchKernelGGL((ffn_block_kernel<8, NG, true, true, KV>), grid, dim3(512), 0, s, a);
  else if (pipe) hipLaunchKernelGGL((ffn_block_kernel<8, NG, true, false, KV>), grid, dim3(512), 0, s, a);
  else if (a.df.on) hipLaunchKernelGGL((ffn_block_kernel<8, NG, false, true, KV>), grid, dim3(512), 0, s, a);
  else hipLaunchKernelGGL((ffn_block_kernel<8, NG, false, false, KV>), grid, dim3(512), 0, s, a);
}
template <int NG>
void launch_ffn(const FfnArgs& a, hipStream_t s) {
  if (a.kv) launch_ffn_kv<NG, true>(a, s);
  else launch_ffn_kv<NG, false>(a, s);
}

}  // namespace

TTMI_STAMP_DUMP(ffn)

extern "C" int ttmi_ffn_block_supported(int dtype, int D, int F) {
  return dtype == TTMI_BF16 && ((D == FB_D && (F == 256 || F == 512)) || (D == F2_D && F == F2_F));
}

extern "C" int ttmi_ffn_block_bwd_supported(int dtype, int D, int F) {
  return dtype == TTMI_BF16 && ((D == FB_D && (F == 256 || F == 512)) || (D == F2_D && F == F2_F));
}

extern "C" int ttmi_ffn_block_fwd(const ttmi_ffn_block_desc* d, hipStream_t s) {
  static const char* fn = "ttmi_ffn_block_fwd";
  TTMI_REQUIRE(d != nullptr, "%s: null descriptor", fn);
  TTMI_REQUIRE(ttmi_ffn_block_supported(TTMI_BF16, d->D, d->F),
               "%s: serves D = 128 with F in {256, 512}, D = 256 with F = 1024 (got D=%d F=%d); use "
               "ttmi_linear + ttmi_linear_res_ln", fn, d->D, d->F);
  TTMI_REQUIRE(d->M >= 0, "%s: M < 0", fn);
  TTMI_REQUIRE(!d->kv || d->D == FB_D, "%s: the fused K / V projection serves D = 128", fn);
  TTMI_REQUIRE((int64_t)d->M * d->F * 2 + 16 * d->F * 2 * 8 < ((int64_t)1 << 31),
               "%s: [M, F] bf16 must stay under 2 GB (32-bit buffer offsets; got M=%d)", fn, d->M);
  TTMI_REQUIRE(d->a && d->w1 && d->b1 && d->w2 && d->b2 && d->res && d->h && d->x2 && d->lnw && d->lnb && d->y &&
                   d->mean && d->rstd, "%s: null argument", fn);
  TTMI_REQUIRE((((uintptr_t)d->a | (uintptr_t)d->w1 | (uintptr_t)d->w2 | (uintptr_t)d->res | (uintptr_t)d->h |
                 (uintptr_t)d->x2 | (uintptr_t)d->y) & 15) == 0, "%s: row operands must be 16-byte aligned", fn);
  TTMI_REQUIRE(d->dropf_p >= 0.f && d->dropf_p < 1.f && d->drop2_p >= 0.f && d->drop2_p < 1.f,
               "%s: dropout out of [0,1)", fn);
  if (d->M == 0) return TTMI_OK;
  FfnArgs a{};
  a.a = (const bf16_t*)d->a; a.w1 = (const bf16_t*)d->w1; a.b1 = d->b1; a.w2 = (const bf16_t*)d->w2; a.b2 = d->b2;
  a.res = d->res; a.h = (bf16_t*)d->h; a.x2 = d->x2;
  a.lnw = d->lnw; a.lnb = d->lnb; a.eps = d->eps; a.y = (bf16_t*)d->y; a.mean = d->mean; a.rstd = d->rstd;
  a.df = make_drop(d->dropf_p, d->dropf_seed);
  a.d2 = make_drop(d->drop2_p, d->drop2_seed);
  a.M = d->M;
  if (d->kv) {
    TTMI_REQUIRE(d->wkv && d->bkv && d->ld_kv >= 2 * FB_D && d->ld_kv % 8 == 0 &&
                     (((uintptr_t)d->kv | (uintptr_t)d->wkv | (uintptr_t)d->bkv) & 15) == 0,
                 "%s: kv needs wkv [256, 128] bf16, bkv [256], 16-byte alignment and ld_kv >= 256, %% 8 == 0", fn);
    TTMI_REQUIRE((int64_t)d->M * d->ld_kv < ((int64_t)1 << 31), "%s: kv rows past 2^31 elements", fn);
    a.wkv = (const bf16_t*)d->wkv; a.bkv = d->bkv; a.kv = (bf16_t*)d->kv; a.ldkv = d->ld_kv;
  }
  if (d->D == F2_D) {
    const dim3 grid((unsigned)((d->M + 127) / 128));
    if (a.df.on) hipLaunchKernelGGL(ffn256_block_kernel<true>, grid, dim3(F2_NW * 64), 0, s, a);
    else hipLaunchKernelGGL(ffn256_block_kernel<false>, grid, dim3(F2_NW * 64), 0, s, a);
  } else if (d->F == 512) {
    launch_ffn<4>(a, s);
  } else {
    launch_ffn<2>(a, s);
  }
  return ttmi_check_launch(fn);
}

extern "C" int ttmi_ffn_block_bwd_sum_blocks(int M) { return M > 0 ? (M + 127) / 128 : 0; }

extern "C" int ttmi_ffn_block_bwd(const ttmi_ffn_block_bwd_desc* d, hipStream_t s) {
  static const char* fn = "ttmi_ffn_block_bwd";
  TTMI_REQUIRE(d != nullptr, "%s: null descriptor", fn);
  TTMI_REQUIRE(ttmi_ffn_block_bwd_supported(TTMI_BF16, d->D, d->F),
               "%s: serves D = 128 with F in {256, 512}, D = 256 with F = 1024 (got D=%d F=%d); use "
               "ttmi_linear + ttmi_linear_ln_bwd", fn, d->D, d->F);
  TTMI_REQUIRE(d->M >= 0, "%s: M < 0", fn);
  TTMI_REQUIRE((int64_t)d->M * d->F * 2 + 16 * d->F * 2 * 8 < ((int64_t)1 << 31),
               "%s: [M, F] bf16 must stay under 2 GB (got M=%d)", fn, d->M);
  TTMI_REQUIRE(d->dy2 && d->w2t && d->w1t && d->h && d->dz1 && d->x1 && d->m2 && d->r2 && d->n2w && d->res &&
                   d->dx1 && d->dy1 && d->sum_ws, "%s: null argument", fn);
  TTMI_REQUIRE((((uintptr_t)d->dy2 | (uintptr_t)d->w2t | (uintptr_t)d->w1t | (uintptr_t)d->h | (uintptr_t)d->dz1 |
                 (uintptr_t)d->x1 | (uintptr_t)d->res | (uintptr_t)d->dx1 | (uintptr_t)d->dy1) & 15) == 0,
               "%s: row operands must be 16-byte aligned", fn);
  TTMI_REQUIRE(d->drop1_p >= 0.f && d->drop1_p < 1.f, "%s: dropout out of [0,1)", fn);
  if (d->M == 0) return TTMI_OK;
  FfnBwdArgs a{};
  a.dy = (const bf16_t*)d->dy2; a.w2t = (const bf16_t*)d->w2t; a.w1t = (const bf16_t*)d->w1t;
  a.h = (const bf16_t*)d->h; a.sf = d->gate_scale; a.dz1 = (bf16_t*)d->dz1;
  a.x1 = d->x1; a.m2 = d->m2; a.r2 = d->r2; a.lnw = d->n2w; a.res = d->res;
  a.dx1 = d->dx1; a.dy1 = (bf16_t*)d->dy1; a.d1 = make_drop(d->drop1_p, d->drop1_seed); a.sum_ws = d->sum_ws;
  a.M = d->M;
  const dim3 grid((unsigned)((d->M + 127) / 128));
  if (d->D == F2_D) {
    if (a.d1.on) hipLaunchKernelGGL(ffn256_block_bwd_kernel<true>, grid, dim3(512), 0, s, a);
    else hipLaunchKernelGGL(ffn256_block_bwd_kernel<false>, grid, dim3(512), 0, s, a);
  } else if (d->F == 512) {
    hipLaunchKernelGGL(ffn_block_bwd_kernel<4>, grid, dim3(512), 0, s, a);
  } else {
    hipLaunchKernelGGL(ffn_block_bwd_kernel<2>, grid, dim3(512), 0, s, a);
  }
  return ttmi_check_launch(fn);
}
